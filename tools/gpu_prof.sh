#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench, then the PMC passes (tools/gpu_pmc.sh).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps ${BENCH_STEPS:-5} --warmup 4 --cpu-baseline 0 --dropin 0 ${BENCH_ARGS:-} > $R/gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -n 1 $R/gpurun_out/prof.log | cut -c1-300
[ "$rc" -eq 0 ] || exit $rc
if [ "${PMC:-1}" = "1" ]; then cd $R && bash tools/gpu_pmc.sh; fi
