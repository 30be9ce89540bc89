#!/bin/bash
# GPU parity tests, then the bench once per configuration (A/B).
# CONFIGS: space-separated "WIDTH:REFILL" pairs (PUPIL_BVH_WIDTH / PUPIL_REFILL).
set -u
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|rel_L2|Error|assert" gpurun_out/pytest_gpu.log | tail -n 20
  [ "$rc" -eq 0 ] || exit $rc
fi
for c in ${CONFIGS:-4:16 4:0}; do
  w=${c%%:*}; r=${c##*:}
  PUPIL_BVH_WIDTH=$w PUPIL_REFILL=$r timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/bench_${w}_${r}.log 2>&1
  rc=$?; echo "bench width $w refill $r rc=$rc"; tail -n 1 gpurun_out/bench_${w}_${r}.log | cut -c1-420
  [ "$rc" -eq 0 ] || exit $rc
done
