#!/bin/bash
# Strong-scaling probe (N = 1 and the 8-way shard) over several builds of the
# engine library, alternating: LIBS="name=path ..." (PUPIL_LIB per run).
set -u
mkdir -p gpurun_out
for i in ${ROUNDS:-1 2}; do
  for nl in $LIBS; do
    n=${nl%%=*}; l=${nl#*=}
    PUPIL_LIB=$l timeout -k 10 300 python tools/shard_probe.py --worlds ${WORLDS:-1 8} --frames ${FRAMES:-5} > gpurun_out/shardlib_$n$i.log 2>&1
    rc=$?; [ "$rc" -eq 0 ] || { echo "probe $n rc=$rc"; tail -n 5 gpurun_out/shardlib_$n$i.log; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/shardlib_$n$i.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$n$i', d['world'], d['ms_max'], d['pred_speedup'], d['rank0']['trace_ms'], d['rank0']['shade_ms'])"
  done
done
