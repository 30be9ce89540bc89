#!/bin/bash
# r04: shade with the hit-independent draws and the emitter guide lookup ahead of the hit
# reconstruction (build/ab_early, -DPUPIL_SHADE_EARLY=1): parity files through it (bit-exact),
# then alternating same-box A/B on config 4 (3 rounds) and config 5 (1 round).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04m
PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_early/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m/pytest_early.log 2>&1
rc=$?; echo "pytest (ab_early) rc=$rc"; tail -3 gpurun_out/r04m/pytest_early.log; [ $rc -eq 0 ] || exit $rc
LIBS="default build/ab_early/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-200 || exit 1
LIBS="default build/ab_early/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-200
