#!/bin/bash
# Full GPU suite, then config 5 (two-level world mode, default for config 5) and config 4 benches.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -n 8
[ "$rc" -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config 5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_c5.log 2>&1 || exit 1
tail -n1 gpurun_out/bench_c5.log | cut -c1-700
timeout -k 10 500 python bench.py --config 3 --cpu-baseline 0 --dropin 0 > gpurun_out/bench_c3.log 2>&1 || exit 1
tail -n1 gpurun_out/bench_c3.log | cut -c1-300
timeout -k 10 500 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -n1 gpurun_out/bench.log | cut -c1-300
