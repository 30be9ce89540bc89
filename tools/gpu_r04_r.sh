#!/bin/bash
# r04: 64-B record slots with every leaf on a 128-B line (pt_scene.h kRecF4) -- the in-tree build;
# the whole GPU suite on it, then alternating same-box A/B on config 4 (3 rounds) and config 5
# (2 rounds) against the build before (build/ab_base: 48-B records).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04r/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04r/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
LIBS="build/ab_base/libpupil_pt.so default" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-150 || exit 1
LIBS="build/ab_base/libpupil_pt.so default" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-150
