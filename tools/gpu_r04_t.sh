#!/bin/bash
# r04 final build: the plain `bench.py --gpus 2` and `--gpus 4` launcher rehearsals (ranks sharing
# this box's one GPU over gloo) against the 1-GPU frame, then config 3's bench line.
set -u
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 2 --warmup 4 --cpu-baseline 0 --dropin 0 --dump $O/frame1.npy > $O/r1.log 2>&1 || exit 1
for N in 2 4; do
  PUPIL_BENCH_DEVICES=1 PUPIL_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $N --steps 2 --warmup 4 \
    --dump $O/frame$N.npy > $O/r$N.log 2>&1
  rc=$?; echo "plain --gpus $N rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/r$N.log; exit $rc; }
  python -c "
import json, numpy as np
a=np.load('$O/frame1.npy'); b=np.load('$O/frame$N.npy')
print('ranks $N: frame bit-identical to 1 GPU:', a.shape == b.shape and bool((a.view(np.uint32) == b.view(np.uint32)).all()))
line=[l for l in open('$O/r$N.log') if l.startswith('{')][-1]
d=json.loads(line); print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'])
"
done
rm -f $O/*.npy
timeout -k 10 400 python bench.py --config 3 > $O/bench3.log 2>&1
rc=$?; echo "bench3 rc=$rc"; grep '^{' $O/bench3.log | tail -1 > $O/bench3.json; cut -c1-300 $O/bench3.json
