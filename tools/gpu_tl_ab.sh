#!/bin/bash
# Two-level traversal A/B on config 5: builds of libpupil_pt.so with the TL kernel at
# 4 / 5 / 6 waves per SIMD (build/ab/tl<w>), two-level parity tests on each, then
# alternating config-5 benches (PUPIL_ACCEL=two_level) and one flattened bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for w in ${WAVES:-4 5 6}; do
  PUPIL_LIB=build/ab/tl$w/libpupil_pt.so PUPIL_ACCEL=two_level timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -q -x -k "two_level or instanced" --timeout 300 > gpurun_out/tl_par_$w.log 2>&1 || { echo "parity tl$w failed"; tail -n 20 gpurun_out/tl_par_$w.log; exit 1; }
  echo "tl$w parity: $(tail -n 1 gpurun_out/tl_par_$w.log)"
done
for i in 1 2; do for w in ${WAVES:-4 5 6}; do
  PUPIL_LIB=build/ab/tl$w/libpupil_pt.so PUPIL_ACCEL=two_level timeout -k 10 400 python bench.py --config 5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/tl_b_$w.log 2>&1 || exit 1
  echo "tl$w $(tail -n1 gpurun_out/tl_b_$w.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stage_ms_per_frame": {[^}]*}' | tr '\n' ' ')"
done; done
timeout -k 10 400 python bench.py --config 5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/tl_b_flat.log 2>&1 || exit 1
echo "flat $(tail -n1 gpurun_out/tl_b_flat.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stage_ms_per_frame": {[^}]*}' | tr '\n' ' ')"
