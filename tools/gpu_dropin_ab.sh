#!/bin/bash
# r04: the C++ drop-in cadence (examples/path_tracer, PUPIL_BENCH=2,5,8 on config 4) static and
# with a camera move before every OnRun (PUPIL_BENCH_MOVING=1), each under the default
# speculation gate, PUPIL_AHEAD=0 (no frames ahead) and PUPIL_AHEAD=2 (frames ahead on every
# render: the r03 behaviour for 1-spp renders), in alternating rounds on one box.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dropin_ab
cd $R
X=/tmp/pupil_dropin_$$/config4.xml
mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
OUT=gpurun_out/dropin_ab/ab.txt
: > $OUT
for round in 1 2; do
  for moving in 0 1; do
    for ahead in default 0 2; do
      if [ "$ahead" = default ]; then AH=""; else AH="PUPIL_AHEAD=$ahead"; fi
      line=$(env $AH PUPIL_BENCH=2,5,8 PUPIL_BENCH_MOVING=$moving timeout -k 10 300 build/pupil_path_tracer $X 2> gpurun_out/dropin_ab/err.log | tail -n 1)
      rc=$?
      [ $rc -eq 0 ] || { cat gpurun_out/dropin_ab/err.log; exit $rc; }
      echo "round $round moving $moving ahead $ahead $line" | tee -a $OUT
    done
  done
done
rm -rf $(dirname $X)
