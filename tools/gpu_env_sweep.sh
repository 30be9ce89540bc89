#!/bin/bash
# Alternating same-box A/B of environment settings on the default config-4 bench.
# usage: SETS="PUPIL_NODE_MIN=8 PUPIL_NODE_MIN=12 ..." bash tools/gpu_env_sweep.sh   ("base" = no setting;
# several variables in one set are joined with '+')
set -u
mkdir -p gpurun_out/sweep
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for s in $SETS; do
    envs=""; [ "$s" != "base" ] && envs="${s//+/ }"
    env $envs timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 ${BENCH_ARGS:-} > gpurun_out/sweep/run.log 2>&1 || { echo "$s failed"; tail -5 gpurun_out/sweep/run.log; exit 1; }
    echo "$r $s $(grep '^{' gpurun_out/sweep/run.log | tail -1 | grep -o '"ms_per_step": [0-9.]*') $(grep '^{' gpurun_out/sweep/run.log | tail -1 | grep -o '"ms_per_launch": [0-9.]*')"
  done
done
