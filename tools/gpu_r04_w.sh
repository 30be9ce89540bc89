#!/bin/bash
# r04: single-material diffuse shading at 5 waves per SIMD (default build) vs 6 waves
# (build/ab_s6d) vs the all-material kernel (PUPIL_SHADE_ONE=0); the whole GPU suite on the
# default build, the parity files through ab_s6d, then alternating same-box A/B on config 4
# (3 rounds) and config 3 (1 round).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04w/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04w/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_s6d/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04w/pytest_s6d.log 2>&1
rc=$?; echo "pytest (s6d) rc=$rc"; tail -1 gpurun_out/r04w/pytest_s6d.log; [ $rc -eq 0 ] || exit $rc
LIBS="default,PUPIL_SHADE_ONE=0 default build/ab_s6d/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-150 || exit 1
LIBS="default,PUPIL_SHADE_ONE=0 default" ROUNDS=1 BENCH_ARGS="--config 3" bash tools/gpu_lib_sweep.sh | cut -c1-150
