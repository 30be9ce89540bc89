#!/bin/bash
# r03: pipelined frames -- focused GPU parity tests, then a default bench run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "shade_list" > gpurun_out/r03a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r03a_pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 4 > gpurun_out/r03a_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/r03a_bench.log
