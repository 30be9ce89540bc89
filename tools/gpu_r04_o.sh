#!/bin/bash
# r04 after the trimmed traversal state became the default: the whole GPU suite + smoke, then
# the default bench line (CPU baseline, drop-in, timed-frame check).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04o
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04o/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04o/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04o/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r04o/smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r04o/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/r04o/bench.log | tail -1 > gpurun_out/r04o/bench.json; cut -c1-400 gpurun_out/r04o/bench.json
