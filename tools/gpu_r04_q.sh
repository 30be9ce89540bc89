#!/bin/bash
# r04: the shade launch reads the hit record once (for the bin check) and hands it to the shade
# (build/ab_sh1) instead of the bin check's read plus a second read inside the shade; parity
# files through it, then alternating same-box A/B on config 4 (3 rounds) and config 5 (1 round)
# against build/ab_base.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04q
PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_sh1/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04q/pytest_sh1.log 2>&1
rc=$?; echo "pytest (sh1) rc=$rc"; tail -1 gpurun_out/r04q/pytest_sh1.log; [ $rc -eq 0 ] || exit $rc
LIBS="build/ab_base/libpupil_pt.so build/ab_sh1/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-150 || exit 1
LIBS="build/ab_base/libpupil_pt.so build/ab_sh1/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-150
