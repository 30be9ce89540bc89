#!/bin/bash
# r03: the full GPU suite (hot-path parity files first, tests/conftest.py), then smoke()
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r03_smoke.log
[ $rc -eq 0 ] || exit $rc
# the spilled 6-wave BVH8 build (r02's lost-batch anomaly): queue accounting + the repro
PUPIL_LIB=build/ab_w8s6/libpupil_pt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 \
  --timeout-method thread -k "queue_accounting" > gpurun_out/r03_w8s6_pytest.log 2>&1
rc=$?; echo "w8s6 pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r03_w8s6_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
PUPIL_LIB=build/ab_w8s6/libpupil_pt.so timeout -k 10 300 python tools/dbg/w8_any.py > gpurun_out/r03_w8s6_repro.log 2>&1
rc=$?; echo "w8s6 repro rc=$rc"; tail -12 gpurun_out/r03_w8s6_repro.log
