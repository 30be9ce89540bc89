#!/bin/bash
# r04: single-material shading through k_shade_one<MAT> (miss + that material compiled: 101-105
# VGPRs for diffuse instead of 126) at 4 waves (default build) and 5 waves per SIMD
# (build/ab_s5) against the all-material kernel (PUPIL_SHADE_ONE=0); parity file through both
# builds, then alternating same-box A/B on config 4 (3 rounds).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04v
for L in "" "PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_s5/libpupil_pt.so"; do
  env $L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04v/pytest.log 2>&1
  rc=$?; echo "pytest ($L) rc=$rc"; tail -1 gpurun_out/r04v/pytest.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="default,PUPIL_SHADE_ONE=0 default build/ab_s5/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-150
