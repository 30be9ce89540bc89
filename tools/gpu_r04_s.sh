#!/bin/bash
# r04 final build: traversal knobs re-swept (refill threshold, node-phase exit, leaf size), two
# alternating rounds on config 4.
set -u
export TMPDIR=/tmp
LIBS="default default,PUPIL_REFILL=12 default,PUPIL_REFILL=24 default,PUPIL_NODE_MIN=6 default,PUPIL_NODE_MIN=12 default,PUPIL_LEAF_SIZE=3" ROUNDS=2 bash tools/gpu_lib_sweep.sh | cut -c1-140
