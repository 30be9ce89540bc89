#!/bin/bash
# Ring-size sweep (PUPIL_PIPE = most frames in flight) on one config, same box.
# usage: CONFIG=5 PIPES="1 2 3 4 6" bash tools/gpu_pipe_sweep.sh
set -u
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp
for k in ${PIPES:-1 2 3 4 6}; do
  PUPIL_PIPE=$k timeout -k 10 400 python bench.py --config ${CONFIG:-5} --steps ${STEPS:-6} --warmup ${WARMUP:-8} \
    --cpu-baseline 0 --dropin 0 > gpurun_out/pipe/k$k.log 2>&1 || { echo "PUPIL_PIPE=$k failed"; tail -5 gpurun_out/pipe/k$k.log; exit 1; }
  grep '^{' gpurun_out/pipe/k$k.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; r=d['roofline']
print('PUPIL_PIPE=$k', d['value'], d['ms_per_step'], c['pipeline'], r['ms_per_launch'], r['rays_per_launch'], c['stage_ms_per_frame'])"
done
