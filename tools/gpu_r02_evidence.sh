#!/bin/bash
# Round evidence on one box: full GPU suite, smoke, default bench, rocprofv3 kernel
# stats, PMC passes (tools/gpu_round.sh), then the C++ drop-in cadence with its kernel
# trace (tools/gpu_dropin.sh) and the strong-scaling shard probe.
set -u
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round.sh || exit $?
cd $R
PROFILE=1 bash tools/gpu_dropin.sh || exit $?
cd $R
timeout -k 10 300 python tools/shard_probe.py > gpurun_out/shard_probe.txt 2>&1 && timeout -k 10 300 python tools/shard_probe.py --progressive 1 > gpurun_out/shard_probe_prog.txt 2>&1
rc=$?; echo "shard probe rc=$rc"; tail -n 1 gpurun_out/shard_probe.txt | cut -c1-200
exit $rc
