#!/bin/bash
# r04 trimmed traversal state (-DPUPIL_TRIM=1: path id, best hit index and barycentrics in LDS,
# ray direction reloaded for sphere tests / instance entries, overflow column recomputed on
# spill): 7 waves (build/ab_W7T) and 8 waves per SIMD (build/ab_W8T, <= 64 VGPRs); parity file
# through both (bit-exact), then alternating same-box A/B on configs 4 (3 rounds) and 5 (1 round)
# against the current build (build/ab_base).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04n
for b in W7T W8T; do
  PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_$b/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04n/pytest_$b.log 2>&1
  rc=$?; echo "pytest ($b) rc=$rc"; tail -2 gpurun_out/r04n/pytest_$b.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="build/ab_base/libpupil_pt.so build/ab_W7T/libpupil_pt.so build/ab_W8T/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-170 || exit 1
LIBS="build/ab_base/libpupil_pt.so build/ab_W7T/libpupil_pt.so build/ab_W8T/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-170
