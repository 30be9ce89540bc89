#!/bin/bash
# r04: traversal diagnostics (PUPIL_TRACE_DIAG) on the default build, then the dequeue-ahead
# build (build/ab_dq, -DPUPIL_DQ_AHEAD=1): parity files through it (bit-exact), alternating
# same-box A/B on config 4 (3 rounds) and config 5 (1 round).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04k
PUPIL_TRACE_DIAG=1 timeout -k 10 300 python bench.py --steps 2 --warmup 2 --cpu-baseline 0 --dropin 0 > gpurun_out/r04k/diag4.log 2>&1 || { tail -5 gpurun_out/r04k/diag4.log; exit 1; }
grep "pupil\]" gpurun_out/r04k/diag4.log | head -20
PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_dq/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04k/pytest_dq.log 2>&1
rc=$?; echo "pytest (ab_dq) rc=$rc"; tail -3 gpurun_out/r04k/pytest_dq.log; [ $rc -eq 0 ] || exit $rc
LIBS="default build/ab_dq/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-200 || exit 1
LIBS="default build/ab_dq/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-200
