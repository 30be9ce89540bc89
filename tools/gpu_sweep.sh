#!/bin/bash
# Env-knob sweep on the default config-4 bench (VARS: ';'-separated env settings).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
IFS=';' read -r -a V <<< "${VARS:?}"
for v in "${V[@]}"; do
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 2 --cpu-baseline 0 --dropin 0 ${BENCH_ARGS:-} > gpurun_out/sweep/b.log 2>&1 || { echo "$v failed"; tail -n 5 gpurun_out/sweep/b.log; exit 1; }
  echo "$v $(tail -n1 gpurun_out/sweep/b.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stage_ms_per_frame": {[^}]*}' | tr '\n' ' ')"
done
