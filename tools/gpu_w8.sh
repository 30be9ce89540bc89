#!/bin/bash
# BVH8 (PUPIL_BVH_WIDTH=8): width-8 parity tests, then config-4 benches, BVH4 vs BVH8.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w8
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "${TESTS:-8 or all_traversals or flat8}" > gpurun_out/w8/par.log 2>&1 || { echo "parity failed"; grep -E "PASS|FAIL|Error|assert" gpurun_out/w8/par.log | tail -n 30; exit 1; }
echo "parity: $(tail -n 1 gpurun_out/w8/par.log)"
for W in ${WIDTHS:-4 8}; do
  PUPIL_BVH_WIDTH=$W timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-baseline 0 --dropin 0 > gpurun_out/w8/bench_$W.log 2>&1 || { echo "bench $W failed"; tail -n 5 gpurun_out/w8/bench_$W.log; exit 1; }
  echo "W=$W $(tail -n1 gpurun_out/w8/bench_$W.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"bvh_nodes": [0-9]*\|"avg_node_visits_per_ray": [0-9.]*\|"avg_prim_tests_per_ray": [0-9.]*\|"stage_ms_per_frame": {[^}]*}\|"bvh_build_ms": [0-9.]*' | tr '\n' ' ')"
done
