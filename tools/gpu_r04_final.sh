#!/bin/bash
# r04 final evidence on one box: GPU suite + smoke; config-4 and config-5 PMC passes of this
# build (per-ray VALU / HBM bytes the bench's roofline reads, copied into profiles/ before the
# benches); the default bench (CPU baseline, timed-frame and drop-in checks); config 5; a same-box
# A/B against the r03 library; the OnRun shard probe; rocprofv3 kernel stats and the timed-launch
# check.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04f5
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "${SKIP_SUITE:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
tail -1 $O/smoke.txt
if [ "${SKIP_PMC:-0}" != "1" ]; then
CONFIG=4 PUPIL_ROUND=r04 bash tools/gpu_pmc.sh > $O/pmc4.log 2>&1 || { tail -5 $O/pmc4.log; exit 1; }
cd $R
cp gpurun_out/pmc_config4.json $O/pmc_config4.json && cp gpurun_out/pmc_config4.json profiles/pmc_config4.json
mv gpurun_out/pmc_summary.txt $O/pmc_summary4.txt; rm -rf gpurun_out/pmc
python3 -c "import json; d=json.load(open('$O/pmc_config4.json')); print('pmc4', round(d['traffic_bytes_per_ray'],1), 'B/ray', round(d['valu_insts_per_ray'],2), 'VALU/ray')"
CONFIG=5 PUPIL_ROUND=r04 bash tools/gpu_pmc.sh > $O/pmc5.log 2>&1 || { tail -5 $O/pmc5.log; exit 1; }
cd $R
cp gpurun_out/pmc_config5.json $O/pmc_config5.json && cp gpurun_out/pmc_config5.json profiles/pmc_config5.json
mv gpurun_out/pmc_summary.txt $O/pmc_summary5.txt; rm -rf gpurun_out/pmc
python3 -c "import json; d=json.load(open('$O/pmc_config5.json')); print('pmc5', round(d['traffic_bytes_per_ray'],1), 'B/ray', round(d['valu_insts_per_ray'],2), 'VALU/ray')"
fi
timeout -k 10 500 python bench.py > $O/bench4.log 2>&1 || { tail -5 $O/bench4.log; exit 1; }
grep '^{' $O/bench4.log | tail -1 > $O/bench4.json; cut -c1-300 $O/bench4.json
timeout -k 10 900 python bench.py --config 5 --steps 3 --warmup 6 > $O/bench5.log 2>&1 || { tail -5 $O/bench5.log; exit 1; }
grep '^{' $O/bench5.log | tail -1 > $O/bench5.json; cut -c1-300 $O/bench5.json
LIBS="build/ab_r03/libpupil_pt.so default" ROUNDS=3 bash tools/gpu_lib_sweep.sh | cut -c1-120 || exit 1
timeout -k 10 400 python tools/shard_probe.py --onrun 1 --progressive 1 --warmup 24 --frames 24 > $O/shard_onrun.txt 2>&1 || exit 1
cut -c1-120 $O/shard_onrun.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 4 --cpu-baseline 0 --dropin 0 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; cd $R; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kernel_stats.txt
python3 tools/timed_kernels.py $O/prof/run_kernel_trace.csv "k_trace4<4, false, false>" 5 > $O/timed_kernels.txt
grep '^{' $O/prof.log | tail -1 > $O/prof_bench.json
tail -1 $O/timed_kernels.txt
rm -rf $O/prof/*.csv.gz gpurun_out/test_scenes gpurun_out/test_images gpurun_out/test_scene
