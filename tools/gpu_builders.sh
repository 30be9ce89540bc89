#!/bin/bash
# Parity tests, then the bench for each BVH builder (PUPIL_BVH_BUILDER=ploc|lbvh).
set -u
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -n 2 gpurun_out/pytest_gpu.log; [ "$rc" -eq 0 ] || exit $rc
fi
for b in ${BUILDERS:-ploc lbvh}; do
  PUPIL_BVH_BUILDER=$b timeout -k 10 600 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/bench_$b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_$b.log').read().strip().splitlines()[-1]); c=d['config']; print('$b', d['value'], d['ms_per_step'], c['stage_ms_per_frame'], 'build', c['bvh_build_ms'], 'nodes', c['bvh_nodes'], 'ext', c['extend_rays_nodes_prims'], 'sh', c['shadow_rays_nodes_prims'])"
done
