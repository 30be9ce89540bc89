#!/bin/bash
# Round evidence (second pass): tools/gpu_r02_evidence.sh plus bench lines of configs 3 and 5.
set -u
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_r02_evidence.sh || exit $?
cd $R
timeout -k 10 300 python bench.py --config 3 --cpu-baseline 0 --dropin 0 > gpurun_out/bench_config3.log 2>&1
rc=$?; echo "config 3 rc=$rc $(tail -n 1 gpurun_out/bench_config3.log | cut -c1-160)"
[ "$rc" -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config 5 --cpu-baseline 0 --dropin 0 --steps 3 --warmup 1 > gpurun_out/bench_config5.log 2>&1
rc=$?; echo "config 5 rc=$rc $(tail -n 1 gpurun_out/bench_config5.log | cut -c1-160)"
[ "$rc" -eq 0 ] || exit $rc
PUPIL_AHEAD=0 timeout -k 10 300 python bench.py --cpu-baseline 0 --dropin 0 > gpurun_out/bench_noahead.log 2>&1
rc=$?; echo "config 4, PUPIL_AHEAD=0 rc=$rc $(tail -n 1 gpurun_out/bench_noahead.log | cut -c1-160)"
exit $rc
