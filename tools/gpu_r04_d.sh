#!/bin/bash
# r04: GPU suite (frame groups, fused traversal), the 1-spp OnRun shard probe (frame groups on),
# the drop-in cadence, then the same-box A/B (tools/gpu_r04_c.sh).
set -u
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu_d.txt 2>&1
rc=$?; tail -3 gpurun_out/r04/pytest_gpu_d.txt; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/shard_probe.py --onrun 1 --progressive 1 --warmup 24 --frames 24 > gpurun_out/r04/shard_onrun_d.txt 2>&1 || exit 1
cut -c1-150 gpurun_out/r04/shard_onrun_d.txt
timeout -k 10 300 python tools/shard_probe.py --progressive 1 --warmup 8 --frames 8 > gpurun_out/r04/shard_prog_d.txt 2>&1 || exit 1
cut -c1-150 gpurun_out/r04/shard_prog_d.txt
bash tools/gpu_r04_c.sh
