#!/bin/bash
# r04 final build: TLAS braid depth re-swept on config 5 (record slots changed the record
# traffic), two alternating rounds.
set -u
export TMPDIR=/tmp
LIBS="default default,PUPIL_TL_BRAID=9 default,PUPIL_TL_BRAID=11" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-200
