#!/bin/bash
# Bench sweep over traversal knobs: SWEEP="refill:node_min ..." (PUPIL_REFILL / PUPIL_NODE_MIN)
set -u
mkdir -p gpurun_out
for c in ${SWEEP:-32:1}; do
  r=${c%%:*}; nm=${c##*:}
  PUPIL_REFILL=$r PUPIL_NODE_MIN=$nm timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/sw_${r}_${nm}.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/sw_${r}_${nm}.log').read().strip().splitlines()[-1]); print('refill $r node_min $nm', d['value'], d['ms_per_step'], d['config']['stage_ms_per_frame'])"
done
