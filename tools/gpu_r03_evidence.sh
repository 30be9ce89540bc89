#!/bin/bash
# r03 evidence: default bench (config 4), 2-rank rehearsal of the N > 1 path (roofline fractions),
# config 5 (two-level, cpu_baseline stride 16 + timed-frame check), config 3.
set -u
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/ev/bench4.log 2>&1
rc=$?; echo "bench4 rc=$rc"; grep '^{' gpurun_out/ev/bench4.log | tail -1 | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 2 --warmup 4 --cpu-baseline 0 --dropin 0 --dump gpurun_out/ev/frame1.npy > gpurun_out/ev/r1.log 2>&1 || exit 1
PUPIL_BENCH_DEVICES=1 PUPIL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 4 \
  --dump gpurun_out/ev/frame2.npy > gpurun_out/ev/r2.log 2>&1
rc=$?; echo "rehearsal rc=$rc"
[ $rc -eq 0 ] || { tail -20 gpurun_out/ev/r2.log; exit $rc; }
python -c "
import json, numpy as np
a=np.load('gpurun_out/ev/frame1.npy'); b=np.load('gpurun_out/ev/frame2.npy')
print('ranks 2: frame bit-identical to 1 GPU:', a.shape == b.shape and bool((a.view(np.uint32) == b.view(np.uint32)).all()))
line=[l for l in open('gpurun_out/ev/r2.log') if l.startswith('{')][-1]
r=json.loads(line)['roofline']
print('ranks 2 roofline:', r['bound'], r['frac'], {k: v['frac'] for k, v in r['ceilings'].items()})
"
timeout -k 10 900 python bench.py --config 5 --steps 3 --warmup 6 > gpurun_out/ev/bench5.log 2>&1
rc=$?; echo "bench5 rc=$rc"; grep '^{' gpurun_out/ev/bench5.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['cpu_baseline'], d['timed_frame_bit_exact'], d['config']['accel'], d['config']['pipeline'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 3 --dropin 0 > gpurun_out/ev/bench3.log 2>&1
rc=$?; echo "bench3 rc=$rc"; grep '^{' gpurun_out/ev/bench3.log | tail -1 | cut -c1-300
