#!/bin/bash
# Alternating same-box A/B of several builds of libpupil_pt.so on the default config-4 bench.
# usage: LIBS="default build/ab_base/libpupil_pt.so build/ab_x/libpupil_pt.so,PUPIL_NODE_MIN=16 ..." bash tools/gpu_lib_sweep.sh
set -u
mkdir -p gpurun_out/sweep
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for l in $LIBS; do
    # token: <lib path or "default">[,VAR=value...]
    IFS=',' read -r path extra <<< "$l"
    if [ "$path" = "default" ]; then lib=""; else lib="PUPIL_LIB=$path"; fi
    env $lib ${extra//,/ } timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 ${BENCH_ARGS:-} > gpurun_out/sweep/run.log 2>&1 || { echo "$l failed"; tail -5 gpurun_out/sweep/run.log; exit 1; }
    line=$(grep '^{' gpurun_out/sweep/run.log | tail -1)
    echo "$r $l $(echo "$line" | grep -o '"ms_per_step": [0-9.]*') $(echo "$line" | grep -o '"ms_per_launch": [0-9.]*') $(echo "$line" | grep -o '"avg_node_visits_per_ray": [0-9.]*') $(echo "$line" | grep -o '"bvh_build_ms": [0-9.]*') $(echo "$line" | grep -o '"instance_update_ms": [^}]*}')"
  done
done
