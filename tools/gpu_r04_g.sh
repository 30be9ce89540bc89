#!/bin/bash
# r04 config 5: TLAS braid depth 8 / 10 / 11 / 12, two alternating rounds.
set -u
export TMPDIR=/tmp
LIBS="default default,PUPIL_TL_BRAID=10 default,PUPIL_TL_BRAID=11 default,PUPIL_TL_BRAID=12" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-300
