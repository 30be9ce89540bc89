#!/bin/bash
# r04: shear axes packed into one register (-DPUPIL_KPACK=1) on the trimmed traversal, at
# 7 waves (build/ab_W7K) and 8 waves per SIMD (build/ab_W8K); parity file through both, then
# alternating same-box A/B on configs 4 (3 rounds) and 5 (1 round) against build/ab_base.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r04p
for b in W7K W8K; do
  PUPIL_LIB=$GRAFT_REPO_ROOT/build/ab_$b/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04p/pytest_$b.log 2>&1
  rc=$?; echo "pytest ($b) rc=$rc"; tail -1 gpurun_out/r04p/pytest_$b.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="build/ab_base/libpupil_pt.so build/ab_W7K/libpupil_pt.so build/ab_W8K/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-150 || exit 1
LIBS="build/ab_base/libpupil_pt.so build/ab_W7K/libpupil_pt.so build/ab_W8K/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh | cut -c1-150
