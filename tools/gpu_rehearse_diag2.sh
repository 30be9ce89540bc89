#!/bin/bash
# bench.py --dump at 1 and 2 ranks for a few warmup/steps combinations.
set -u
mkdir -p gpurun_out/diag
D=/tmp/pupil_diag_$$
mkdir -p $D
for ws in "0 1" "1 1" "0 2"; do
  set -- $ws
  timeout -k 10 200 python bench.py --warmup $1 --steps $2 --cpu-baseline 0 --dropin 0 --dump $D/f1.npy > gpurun_out/diag/q1.log 2>&1 || exit 1
  PUPIL_BENCH_DEVICES=1 PUPIL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --warmup $1 --steps $2 \
    --dump $D/f2.npy > gpurun_out/diag/q2.log 2>&1 || exit 1
  python -c "
import numpy as np; a=np.load('$D/f1.npy').reshape(-1,4); b=np.load('$D/f2.npy').reshape(-1,4)
d=np.any(a.view(np.uint32)!=b.view(np.uint32),axis=1); print('warmup $1 steps $2: differing', int(d.sum()), 'means', a[:,:3].mean(), b[:,:3].mean())"
done
rm -rf $D
