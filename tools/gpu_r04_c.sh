#!/bin/bash
# r04 A/B: the r03 final library, this round's build and this round's build without in-kernel
# camera rays (PUPIL_CAMGEN=0), alternating on one box (default config-4 bench, 10 steps).
set -u
export TMPDIR=/tmp
LIBS="build/ab_r03/libpupil_pt.so default build/ab_camgen0/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh
