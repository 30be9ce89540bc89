#!/bin/bash
# r04 second check: GPU suite (threading, coalesced updates, deep renders, moving camera),
# the drop-in A/B, the 1-spp OnRun shard probe and the default bench line.
set -u
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu_b.txt 2>&1
rc=$?; tail -3 gpurun_out/r04/pytest_gpu_b.txt; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_dropin_ab.sh || exit 1
timeout -k 10 300 python tools/shard_probe.py --onrun 1 --progressive 1 > gpurun_out/r04/shard_onrun.txt 2>&1 || exit 1
cat gpurun_out/r04/shard_onrun.txt | cut -c1-200
timeout -k 10 400 python bench.py > gpurun_out/r04/bench4_b.log 2>&1
rc=$?; echo "bench4 rc=$rc"; grep '^{' gpurun_out/r04/bench4_b.log | tail -1 | cut -c1-400
# kernel timeline of one rank's 1-spp OnRun cadence at N = 8 (where the fixed per-OnRun cost goes)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04/tl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/shard_probe.py --onrun 1 --progressive 1 --worlds 8 --only-rank 0 --frames 3 > $GRAFT_REPO_ROOT/gpurun_out/r04/tl.log 2>&1
rc=$?; echo "timeline rc=$rc"; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] && python3 tools/timeline.py gpurun_out/r04/tl/run_kernel_trace.csv 120 --list 40 > gpurun_out/r04/timeline_onrun8.txt && tail -20 gpurun_out/r04/timeline_onrun8.txt
rm -f gpurun_out/r04/tl/run_kernel_trace.csv.gz
