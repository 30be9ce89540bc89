#!/bin/bash
# Strong-scaling A/B on one GPU: tools/shard_probe.py (N = 1 and the 8-way
# shard) once per environment setting.  VARIANTS as in gpu_ab_env.sh.
set -u
mkdir -p gpurun_out
for v in ${VARIANTS:-NONE}; do
  tag=${v//=/_}
  if [ "$v" = "NONE" ]; then envs=""; else envs="${v//,/ }"; fi
  env $envs timeout -k 10 300 python tools/shard_probe.py --worlds ${WORLDS:-1 8} --frames ${FRAMES:-5} > gpurun_out/shard_$tag.log 2>&1
  rc=$?; [ "$rc" -eq 0 ] || { echo "probe $v rc=$rc"; tail -n 5 gpurun_out/shard_$tag.log; exit $rc; }
  python3 -c "
import json
for l in open('gpurun_out/shard_$tag.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$v', d['world'], d['ms_max'], d['pred_speedup'], d['rank0']['trace_ms'], d['rank0']['shade_ms'])"
done
