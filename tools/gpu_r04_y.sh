#!/bin/bash
# r04: renders that start no frame ahead use one slot of one frame (the ring is sized only once a
# render speculates): the GPU suite, then the C++ drop-in cadence A/B (static / moving camera x
# speculation settings) on this build, then the default bench against the build before.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04y
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04y/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r04y/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_dropin_ab.sh | cut -c1-200 || exit 1
LIBS="build/ab_base/libpupil_pt.so default" ROUNDS=2 bash tools/gpu_lib_sweep.sh | cut -c1-120
