#!/bin/bash
# r04: node phase ends early once enough lanes are idle (PUPIL_REFILL_BREAK), so refills come
# sooner: parity file with the switch (bit-exact), then alternating same-box A/B on config 4
# (2 rounds) against the build before the switch (build/ab_base), then config 5 (1 round).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04l
PUPIL_REFILL_BREAK=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04l/pytest_rb.log 2>&1
rc=$?; echo "pytest (PUPIL_REFILL_BREAK=32) rc=$rc"; tail -3 gpurun_out/r04l/pytest_rb.log; [ $rc -eq 0 ] || exit $rc
LIBS="default default,PUPIL_REFILL_BREAK=24 default,PUPIL_REFILL_BREAK=32 default,PUPIL_REFILL_BREAK=40 default,PUPIL_REFILL_BREAK=48 build/ab_base/libpupil_pt.so" ROUNDS=2 bash tools/gpu_lib_sweep.sh | cut -c1-200 || exit 1
LIBS="default default,PUPIL_REFILL_BREAK=32 default,PUPIL_REFILL_BREAK=48 build/ab_base/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-200
