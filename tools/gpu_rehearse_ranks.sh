# Rehearsal of bench.py's N-rank path on a 1-GPU box: N ranks share GPU 0 (PUPIL_BENCH_DEVICES=1),
# collectives over gloo (PUPIL_BENCH_BACKEND=gloo); the frame assembled on rank 0 must equal the
# 1-GPU frame bit for bit.  (The driver's scaling runs use one rank per GPU over RCCL.)
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --dump gpurun_out/frame1.npy > gpurun_out/r1.log 2>&1 || exit 1
for n in ${RANKS:-2 8}; do
  PUPIL_BENCH_DEVICES=1 PUPIL_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 2 --warmup 1 \
    --dump gpurun_out/frame$n.npy > gpurun_out/r$n.log 2>&1 || exit 1
  python -c "
import numpy as np; a=np.load('gpurun_out/frame1.npy'); b=np.load('gpurun_out/frame$n.npy')
print('ranks $n: frame bit-identical to 1 GPU:', a.shape == b.shape and (a.view(np.uint32) == b.view(np.uint32)).all())
import json; l=[json.loads(x) for x in open('gpurun_out/r$n.log') if x.startswith('{')][-1]
print('ranks $n: comm', json.dumps(l['comm'])); print('ranks $n: per rank', json.dumps(l['ranks']))"
done
rm -f gpurun_out/frame*.npy
