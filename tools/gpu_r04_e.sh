#!/bin/bash
# r04 evidence on one box: GPU suite + smoke, the default bench (CPU baseline, timed-frame and
# drop-in checks), a same-box A/B against the r03 library, the drop-in static / moving-camera
# cadences with frame groups, the OnRun shard probe, rocprofv3 kernel stats of the bench.
set -u
mkdir -p gpurun_out/r04e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04e/pytest_gpu.txt 2>&1
rc=$?; tail -2 gpurun_out/r04e/pytest_gpu.txt; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04e/smoke.txt 2>&1 || exit 1
tail -1 gpurun_out/r04e/smoke.txt
timeout -k 10 500 python bench.py > gpurun_out/r04e/bench4.log 2>&1 || { tail -5 gpurun_out/r04e/bench4.log; exit 1; }
grep '^{' gpurun_out/r04e/bench4.log | tail -1 > gpurun_out/r04e/bench4.json; cut -c1-300 gpurun_out/r04e/bench4.json
LIBS="build/ab_r03/libpupil_pt.so default" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-120 || exit 1
bash tools/gpu_dropin_ab.sh | cut -c1-200 || exit 1
timeout -k 10 400 python tools/shard_probe.py --onrun 1 --progressive 1 --warmup 24 --frames 24 > gpurun_out/r04e/shard_onrun.txt 2>&1 || exit 1
cut -c1-120 gpurun_out/r04e/shard_onrun.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04e/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 4 --cpu-baseline 0 --dropin 0 > $GRAFT_REPO_ROOT/gpurun_out/r04e/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; cd $GRAFT_REPO_ROOT; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py gpurun_out/r04e/prof/run_kernel_stats.csv > gpurun_out/r04e/kernel_stats.txt
python3 tools/timed_kernels.py gpurun_out/r04e/prof/run_kernel_trace.csv "k_trace4<4, false, false>" 5 > gpurun_out/r04e/timed_kernels.txt
grep '^{' gpurun_out/r04e/prof.log | tail -1 > gpurun_out/r04e/prof_bench.json
cat gpurun_out/r04e/timed_kernels.txt | tail -1
rm -rf gpurun_out/r04e/prof/*.csv.gz gpurun_out/test_scenes gpurun_out/test_images gpurun_out/test_scene
