#!/bin/bash
# Parity tests (hot path first), smoke, the default bench and a rocprofv3
# kernel-trace --stats run of the same bench.  Stops at the first failure.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -n 5
[ "$rc" -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke.log
[ "$rc" -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 1 gpurun_out/bench.log | cut -c1-600
[ "$rc" -eq 0 ] || exit $rc
[ "${PROFILE:-1}" = "1" ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --cpu-baseline 0 ${BENCH_ARGS:-} > $R/gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -n 1 $R/gpurun_out/prof.log | cut -c1-200
exit $rc
