#!/bin/bash
# Diagnose N-rank rehearsal differences: 1 and 2 ranks, with and without render-ahead.
set -u
mkdir -p gpurun_out/diag
D=/tmp/pupil_diag_$$
mkdir -p $D
for a in 1 0; do
  PUPIL_AHEAD=$a timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --dropin 0 --dump $D/f1_$a.npy > gpurun_out/diag/r1_$a.log 2>&1 || exit 1
  PUPIL_AHEAD=$a PUPIL_BENCH_DEVICES=1 PUPIL_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 2 --warmup 1 \
    --dump $D/f2_$a.npy > gpurun_out/diag/r2_$a.log 2>&1 || exit 1
done
python - <<PY
import numpy as np
f = {k: np.load(f"$D/{k}.npy").reshape(-1, 4) for k in ("f1_1", "f2_1", "f1_0", "f2_0")}
for a, b in (("f1_1", "f2_1"), ("f1_0", "f2_0"), ("f1_1", "f1_0"), ("f2_1", "f2_0")):
    x, y = f[a], f[b]
    d = np.any(x.view(np.uint32) != y.view(np.uint32), axis=1)
    idx = np.nonzero(d)[0]
    print(a, b, "differing pixels", int(d.sum()), "of", len(d), "first", idx[:8].tolist(),
          "max abs", float(np.abs(x - y).max()), "mean x", float(x[:, :3].mean()), "mean y", float(y[:, :3].mean()))
PY
rm -rf $D
