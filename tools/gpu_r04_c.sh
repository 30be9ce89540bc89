#!/bin/bash
# r04 A/B: the r03 final library, this round's build (while-while and fused traversal) and this
# round's build without in-kernel camera rays (PUPIL_CAMGEN=0), alternating on one box (default
# config-4 bench, 10 steps); then config 5 while-while vs fused.
set -u
export TMPDIR=/tmp
LIBS="build/ab_r03/libpupil_pt.so default default,PUPIL_TRAVERSAL=fused build/ab_camgen0/libpupil_pt.so build/ab_camgen2/libpupil_pt.so build/ab_camgen2/libpupil_pt.so,PUPIL_TRAVERSAL=fused" ROUNDS=2 bash tools/gpu_lib_sweep.sh || exit 1
LIBS="default default,PUPIL_TRAVERSAL=fused" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh
