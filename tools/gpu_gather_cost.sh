#!/bin/bash
# Fixed cost per OnRun of the C++ drop-in's tile gather (pupil/dist.h FrameGather, synchronous
# inside PTPass::OnRun): examples/path_tracer on the config-4 scene, PUPIL_BENCH=2,5,8, without
# the distributed path and with it forced on at one rank (PUPIL_DIST=1: compact tiles, an RCCL
# group with rank 0 alone, the scatter into the full "final result"), static and moving camera,
# alternating rounds on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${OUT:-gpurun_out/gather_cost}
mkdir -p $O
cd $R
X=/tmp/pupil_gather_$$/config4.xml
mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
: > $O/gather_cost.txt
for round in 1 2; do
  for moving in 0 1; do
    for dist in 0 1; do
      E="PUPIL_BENCH=2,5,8 PUPIL_BENCH_MOVING=$moving"
      [ "$dist" = 1 ] && E="$E PUPIL_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((20000 + RANDOM % 20000))"
      line=$(env $E timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
      [ -n "$line" ] || { cat $O/err.log; exit 1; }
      echo "round $round moving $moving dist $dist $line" | tee -a $O/gather_cost.txt
    done
  done
done
rm -rf $(dirname $X)
