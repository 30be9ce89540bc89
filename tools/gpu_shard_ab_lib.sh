#!/bin/bash
# Strong-scaling A/B of two builds on one box: tools/shard_probe.py (N = 1 and
# the 8-way shard), alternating A = pupiloptixlab_amd/lib and B = $B_LIB.
set -u
mkdir -p gpurun_out
B=${B_LIB:-build/ab/libpupil_pt.so}
for i in ${ROUNDS:-1 2 3}; do
  for ab in A B; do
    if [ $ab = A ]; then lib=""; else lib="PUPIL_LIB=$B"; fi
    env $lib timeout -k 10 300 python tools/shard_probe.py --worlds ${WORLDS:-1 8} --frames ${FRAMES:-5} > gpurun_out/shardab_$ab$i.log 2>&1
    rc=$?; [ "$rc" -eq 0 ] || { echo "probe $ab rc=$rc"; tail -n 5 gpurun_out/shardab_$ab$i.log; exit $rc; }
    python3 -c "
import json
for l in open('gpurun_out/shardab_$ab$i.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$ab$i', d['world'], d['ms_max'], d['pred_speedup'], d['rank0']['trace_ms'], d['rank0']['shade_ms'])"
  done
done
