#!/bin/bash
# r04: GPU suite, then the plain `bench.py --gpus 2` launcher rehearsal (2 ranks sharing this
# box's one GPU over gloo) against the 1-GPU frame, then the default bench line.
set -u
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r04/pytest_gpu.txt; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 2 --warmup 4 --cpu-baseline 0 --dropin 0 --dump gpurun_out/r04/frame1.npy > gpurun_out/r04/r1.log 2>&1 || exit 1
PUPIL_BENCH_DEVICES=1 PUPIL_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 2 --warmup 4 \
  --dump gpurun_out/r04/frame2.npy > gpurun_out/r04/r2.log 2>&1
rc=$?; echo "plain --gpus 2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04/r2.log; exit $rc; }
python -c "
import json, numpy as np
a=np.load('gpurun_out/r04/frame1.npy'); b=np.load('gpurun_out/r04/frame2.npy')
print('ranks 2: frame bit-identical to 1 GPU:', a.shape == b.shape and bool((a.view(np.uint32) == b.view(np.uint32)).all()))
line=[l for l in open('gpurun_out/r04/r2.log') if l.startswith('{')][-1]
d=json.loads(line); print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'])
"
rm -f gpurun_out/r04/*.npy
timeout -k 10 400 python bench.py > gpurun_out/r04/bench4.log 2>&1
rc=$?; echo "bench4 rc=$rc"; grep '^{' gpurun_out/r04/bench4.log | tail -1 | cut -c1-600
