#!/bin/bash
# r03: 8-way shard probes (progressive batched and the 1-spp OnRun cadence) with pipelined frames
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/shard_probe.py --progressive 1 --frames 5 > gpurun_out/r03_shard_probe_progressive.txt 2>&1
rc=$?; echo "progressive rc=$rc"; cat gpurun_out/r03_shard_probe_progressive.txt | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/shard_probe.py --onrun 1 --frames 5 > gpurun_out/r03_shard_probe_onrun.txt 2>&1
rc=$?; echo "onrun rc=$rc"; cat gpurun_out/r03_shard_probe_onrun.txt | cut -c1-200
[ $rc -eq 0 ] || exit $rc
PUPIL_PIPE=1 timeout -k 10 300 python tools/shard_probe.py --progressive 1 --frames 5 > gpurun_out/r03_shard_probe_nopipe.txt 2>&1
rc=$?; echo "nopipe rc=$rc"; cat gpurun_out/r03_shard_probe_nopipe.txt | cut -c1-200
