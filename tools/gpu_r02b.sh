#!/bin/bash
# Parity tests, then the emissive-mesh selection A/B (guide table vs binary search,
# 1 and 8 emissive sphere groups = 125k / 1M emitter triangles), then the default bench.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -n 12
[ "$rc" -eq 0 ] || exit $rc
for g in 1 8; do for m in guide binary guide binary; do
  PUPIL_EMITTER_SELECT=$m timeout -k 10 300 python bench.py --cpu-baseline 0 --dropin 0 --steps 5 --emissive-groups $g > gpurun_out/em_${g}_$m.log 2>&1 || exit 1
  echo "groups $g $m $(tail -n1 gpurun_out/em_${g}_$m.log | grep -o '"ms_per_step": [0-9.]*\|"area_emitters": [0-9]*\|"shade": [0-9.]*' | tr '\n' ' ')"
done; done
