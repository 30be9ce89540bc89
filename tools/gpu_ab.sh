#!/bin/bash
# GPU parity tests, then the bench for each BVH width (A/B), optional profile.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|rel_L2|Error" gpurun_out/pytest_gpu.log | tail -n 20
[ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || exit $rc
for w in ${WIDTHS:-4 2}; do
  PUPIL_BVH_WIDTH=$w timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/bench_w$w.log 2>&1
  rc=$?; echo "bench width $w rc=$rc"; tail -n 1 gpurun_out/bench_w$w.log | cut -c1-700
  [ "$rc" -eq 0 ] || exit $rc
done
