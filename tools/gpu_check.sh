#!/bin/bash
# One GPU session: parity tests, a short bench, a rocprofv3 kernel-trace profile.
# Stops at the first crash / abort / timeout (exit codes other than 0 or 1).
set -u
mkdir -p gpurun_out
STEP_OK() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 30 gpurun_out/pytest_gpu.log
STEP_OK $rc || exit $rc
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_ARGS:-} --save gpurun_out/bench.png > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 5 gpurun_out/bench.log
[ "$rc" -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -n 3 $GRAFT_REPO_ROOT/gpurun_out/prof.log
  find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
fi
