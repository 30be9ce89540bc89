#!/bin/bash
# r04 config 5: the full bench line (sampled CPU check, timed-frame check, instance update), then
# an environment sweep of the traversal / build knobs on config 5 (one round each).
set -u
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --config 5 --steps 3 --warmup 6 > gpurun_out/r04f/bench5.log 2>&1 || { tail -5 gpurun_out/r04f/bench5.log; exit 1; }
grep '^{' gpurun_out/r04f/bench5.log | tail -1 > gpurun_out/r04f/bench5.json; cut -c1-300 gpurun_out/r04f/bench5.json
LIBS="default default,PUPIL_LEAF_SIZE=1 default,PUPIL_LEAF_SIZE=3 default,PUPIL_NODE_MIN=16 default,PUPIL_REFILL=32 default,PUPIL_TL_BRAID=7 default,PUPIL_TL_BRAID=9 default,PUPIL_TL_BRAID=10" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-160
