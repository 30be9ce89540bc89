#!/bin/bash
# Hot-path parity tests of the new build, then A/B of two builds of libpupil_pt.so on
# one box: A = pupiloptixlab_amd/lib (new), B = $B_LIB (default build/ab/libpupil_pt.so),
# alternating config-4 bench runs (no CPU baseline, no drop-in leg).  BENCH_ARGS adds args.
set -u
mkdir -p gpurun_out/ab
B=${B_LIB:-build/ab/libpupil_pt.so}
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc $(tail -n 1 gpurun_out/ab/pytest.log)"
  [ "$rc" -eq 0 ] || exit $rc
fi
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 ${BENCH_ARGS:-} > gpurun_out/ab/A$i.log 2>&1 || exit 1
  echo "A $(tail -n1 gpurun_out/ab/A$i.log | grep -o '"ms_per_step": [0-9.]*')"
  PUPIL_LIB=$B timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 10 ${BENCH_ARGS:-} > gpurun_out/ab/B$i.log 2>&1 || exit 1
  echo "B $(tail -n1 gpurun_out/ab/B$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
