#!/bin/bash
# r04 band-major path ids (PUPIL_BANDS): the GPU suite, the parity files again with
# PUPIL_BANDS=8 (must stay bit-exact), then alternating same-box A/Bs on configs 5 and 4
# against the build before the change (build/ab_base).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04i
SUITE_ENV="PUPIL_BANDS=8" LIBS="" bash -c '
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04i/pytest.log; [ $rc -eq 0 ] || exit $rc
env $SUITE_ENV timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i/pytest_bands.log 2>&1
rc=$?; echo "pytest ($SUITE_ENV) rc=$rc"; tail -3 gpurun_out/r04i/pytest_bands.log; [ $rc -eq 0 ] || exit $rc
' || exit 1
LIBS="default default,PUPIL_BANDS=8 default,PUPIL_BANDS=32 build/ab_base/libpupil_pt.so" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-220 || exit 1
LIBS="default default,PUPIL_BANDS=8 default,PUPIL_BANDS=32 build/ab_base/libpupil_pt.so" ROUNDS=2 bash tools/gpu_lib_sweep.sh | cut -c1-220
