#!/bin/bash
# Render-ahead A/B: its parity tests, then the C++ drop-in cadence (8 x 1-spp
# OnRun per frame) and the batched bench with PUPIL_AHEAD off / on, alternating.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ahead
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "render_ahead or accumulation or consecutive or camera_change or instance_update" > gpurun_out/ahead/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/ahead/pytest.log | tail -n 5
[ "$rc" -eq 0 ] || exit $rc
X=/tmp/pupil_ahead_$$/config4.xml
mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 || exit 1
for round in 1 2; do
  for a in 0 1; do
    PUPIL_AHEAD=$a PUPIL_BENCH=2,5,8 timeout -k 10 300 build/pupil_path_tracer $X > gpurun_out/ahead/dropin_$a.log 2>&1
    rc=$?; echo "dropin ahead=$a round=$round rc=$rc $(tail -n 1 gpurun_out/ahead/dropin_$a.log)"
    [ "$rc" -eq 0 ] || exit $rc
  done
done
for a in 0 2; do
  PUPIL_AHEAD=$a timeout -k 10 300 python bench.py --cpu-baseline 0 --dropin 0 > gpurun_out/ahead/bench_$a.log 2>&1
  rc=$?; echo "bench ahead=$a rc=$rc $(tail -n 1 gpurun_out/ahead/bench_$a.log | cut -c1-220)"
  [ "$rc" -eq 0 ] || exit $rc
done
rm -rf $(dirname $X)
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  for a in 0 2; do
    PUPIL_AHEAD=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ahead/prof$a -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline 0 --dropin 0 > $R/gpurun_out/ahead/prof$a.log 2>&1
    rc=$?; echo "rocprof ahead=$a rc=$rc"
    [ "$rc" -eq 0 ] || exit $rc
  done
fi
