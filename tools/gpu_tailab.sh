#!/bin/bash
# Tail-helping A/B: GPU parity tests on the new build, then alternating config-4
# benches: A = new build (tail helping), A0 = new build with PUPIL_TAIL_HELP=0,
# B = $B_LIB (previous build); then the drop-in cadence and the shard probe.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B=${B_LIB:-build/ab/libpupil_pt.so}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -n 12
  [ "$rc" -eq 0 ] || exit $rc
fi
for i in 1 2; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 > gpurun_out/abA$i.log 2>&1 || exit 1
  echo "A  $(tail -n1 gpurun_out/abA$i.log | grep -o '"ms_per_step": [0-9.]*')"
  PUPIL_TAIL_HELP=0 timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 > gpurun_out/abA0$i.log 2>&1 || exit 1
  echo "A0 $(tail -n1 gpurun_out/abA0$i.log | grep -o '"ms_per_step": [0-9.]*')"
  PUPIL_LIB=$B timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 > gpurun_out/abB$i.log 2>&1 || exit 1
  echo "B  $(tail -n1 gpurun_out/abB$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 300 python3 tools/shard_probe.py --worlds 1 8 > gpurun_out/shard_probe.log 2>&1 || exit 1
cut -c1-140 gpurun_out/shard_probe.log | grep world
PUPIL_TAIL_HELP=0 timeout -k 10 300 python3 tools/shard_probe.py --worlds 1 8 > gpurun_out/shard_probe0.log 2>&1 || exit 1
cut -c1-140 gpurun_out/shard_probe0.log | grep world
PROFILE=0 bash tools/gpu_dropin.sh
