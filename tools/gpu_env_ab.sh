#!/bin/bash
# Parity tests under $TEST_ENV (e.g. "PUPIL_STATIC_PCT=60"), then alternating config-4
# bench runs for each value of $VAR in $VALUES (same build).  BENCH_ARGS adds args.
set -u
mkdir -p gpurun_out/envab
if [ -n "${TEST_ENV:-}" ]; then
  env $TEST_ENV timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/envab/pytest.log 2>&1
  rc=$?; echo "pytest ($TEST_ENV) rc=$rc $(tail -n 1 gpurun_out/envab/pytest.log)"
  [ "$rc" -eq 0 ] || exit $rc
fi
for i in ${ROUNDS:-1 2}; do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 ${BENCH_ARGS:-} > gpurun_out/envab/b_${v}_$i.log 2>&1 || exit 1
    echo "$VAR=$v $(tail -n1 gpurun_out/envab/b_${v}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
