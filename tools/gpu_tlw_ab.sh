#!/bin/bash
# Two-level "world" mode (world-space BLAS copies + braided TLAS, flat kernels):
# two-level parity tests, then config-5 benches over PUPIL_TL_BRAID and the object mode.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PUPIL_ACCEL=two_level timeout -k 10 500 python -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -q -x -k "two_level or instanced" --timeout 300 > gpurun_out/tlw_par.log 2>&1 || { echo "parity failed"; tail -n 30 gpurun_out/tlw_par.log; exit 1; }
echo "world parity: $(tail -n 1 gpurun_out/tlw_par.log)"
for v in ${VARIANTS:-"PUPIL_TL_BRAID=0" "PUPIL_TL_BRAID=1" "PUPIL_TL_BRAID=2" "PUPIL_TL_BRAID=3" "PUPIL_TL_MODE=object"}; do
  env $v PUPIL_ACCEL=two_level timeout -k 10 400 python bench.py --config 5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/tlw_$v.log 2>&1 || { echo "$v failed"; tail -n 5 gpurun_out/tlw_$v.log; exit 1; }
  echo "$v $(tail -n1 gpurun_out/tlw_$v.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bvh_build_ms": [0-9.]*\|"avg_node_visits_per_ray": [0-9.]*\|"stage_ms_per_frame": {[^}]*}' | tr '\n' ' ')"
done
if [ "${FLAT:-0}" = "1" ]; then
  timeout -k 10 400 python bench.py --config 5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/tlw_flat.log 2>&1 || exit 1
  echo "flat $(tail -n1 gpurun_out/tlw_flat.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bvh_build_ms": [0-9.]*\|"avg_node_visits_per_ray": [0-9.]*\|"stage_ms_per_frame": {[^}]*}' | tr '\n' ' ')"
fi
