#!/bin/bash
# GPU suite on the current build, then again with the environment in $SUITE_ENV (an A/B switch
# that must stay bit-exact), then an alternating same-box bench A/B (tools/gpu_lib_sweep.sh, $LIBS)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${SUITE_ENV:-}" ]; then
  env $SUITE_ENV timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_pytest_env.log 2>&1
  rc=$?; echo "pytest ($SUITE_ENV) rc=$rc"; tail -3 gpurun_out/ab_pytest_env.log
  [ $rc -eq 0 ] || exit $rc
fi
bash tools/gpu_lib_sweep.sh
