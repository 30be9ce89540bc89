#!/bin/bash
# One GPU session of evidence steps, run in order; stops at the first failure and starts
# nothing more on the GPU after it.  Replaces the per-round gpu_r0x_*.sh scripts.
#
# usage (on the box, from the repo root):
#   STEPS="suite smoke pmc4 bench4" OUT=gpurun_out/r05a bash tools/gpu_session.sh
# steps:
#   suite          pytest -m gpu (all GPU tests)             -> $OUT/pytest_gpu.txt
#   parity         only the hot-path parity files           -> $OUT/pytest_parity.txt
#   smoke          __graft_entry__.smoke()                  -> $OUT/smoke.txt
#   pmc<k>         PMC passes of config k (tools/gpu_pmc.sh) -> $OUT/pmc_config<k>.json (+ profiles/ when COMMIT_PMC=1)
#   bench<k>       bench.py --config k (k = 4: the default line with its CPU / drop-in checks)
#   ab             alternating same-box A/B of builds / env (tools/gpu_lib_sweep.sh, $LIBS, $ROUNDS)
#   probe          OnRun shard probe (tools/shard_probe.py; PROBE_ARGS)
#   dropin         C++ drop-in cadence A/B (tools/gpu_dropin_ab.sh)
#   pacing         C++ drop-in OnRun p50/p99/max per frame-group size + speculation waste (tools/gpu_pacing.sh)
#   prof           rocprofv3 --kernel-trace --stats of a short default bench + the timed-launch check
#   ranks          bench.py N-rank rehearsal over gloo on this one GPU (tools/gpu_rehearse_ranks.sh)
#   cppranks       C++ drop-in with 2 ranks on this GPU over the host-staged test transport
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${OUT:-gpurun_out/session}
mkdir -p $O
export TMPDIR=/tmp
cd $R
for step in ${STEPS:-suite smoke}; do
  echo "== $step"
  case $step in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
    rc=$?; tail -2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc ;;
  parity)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py tests/test_gpu_fullsize.py -m gpu -x -q \
      --timeout 300 --timeout-method thread > $O/pytest_parity.txt 2>&1
    rc=$?; tail -2 $O/pytest_parity.txt; [ $rc -eq 0 ] || exit $rc ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
    tail -1 $O/smoke.txt ;;
  pmc[0-9])
    k=${step#pmc}
    CONFIG=$k bash tools/gpu_pmc.sh > $O/pmc$k.log 2>&1 || { tail -5 $O/pmc$k.log; exit 1; }
    cp gpurun_out/pmc_config$k.json $O/pmc_config$k.json
    [ "${COMMIT_PMC:-0}" = "1" ] && cp gpurun_out/pmc_config$k.json profiles/pmc_config$k.json
    [ -f gpurun_out/pmc_shade_config$k.json ] && mv gpurun_out/pmc_shade_config$k.json $O/pmc_shade_config$k.json
    mv gpurun_out/pmc_summary.txt $O/pmc_summary$k.txt; rm -rf gpurun_out/pmc
    python3 -c "import json; d=json.load(open('$O/pmc_config$k.json')); print('pmc$k', round(d['traffic_bytes_per_ray'],1), 'B/ray', round(d['valu_insts_per_ray'],2), 'VALU/ray')" ;;
  bench4)
    timeout -k 10 500 python bench.py ${BENCH4_ARGS:-} > $O/bench4.log 2>&1 || { tail -5 $O/bench4.log; exit 1; }
    grep '^{' $O/bench4.log | tail -1 > $O/bench4.json; cut -c1-300 $O/bench4.json ;;
  bench[0-9])
    k=${step#bench}
    timeout -k 10 900 python bench.py --config $k --steps ${BENCH_STEPS:-3} --warmup ${BENCH_WARMUP:-6} > $O/bench$k.log 2>&1 || { tail -5 $O/bench$k.log; exit 1; }
    grep '^{' $O/bench$k.log | tail -1 > $O/bench$k.json; cut -c1-300 $O/bench$k.json ;;
  ab)
    bash tools/gpu_lib_sweep.sh > $O/ab.txt 2>&1; rc=$?; cut -c1-160 $O/ab.txt; [ $rc -eq 0 ] || exit $rc ;;
  probe)
    timeout -k 10 500 python tools/shard_probe.py ${PROBE_ARGS:---onrun 1 --progressive 1 --warmup 24 --frames 24} > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
    cut -c1-160 $O/probe.txt ;;
  dropin)
    bash tools/gpu_dropin_ab.sh > $O/dropin.txt 2>&1; rc=$?; cut -c1-200 $O/dropin.txt; [ $rc -eq 0 ] || exit $rc ;;
  pacing)
    OUT=${OUT:-gpurun_out/session} bash tools/gpu_pacing.sh > $O/pacing.log 2>&1; rc=$?; cut -c1-220 $O/pacing.log; [ $rc -eq 0 ] || exit $rc ;;
  prof)
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 4 --cpu-baseline 0 --dropin 0 ${BENCH4_ARGS:-} > $O/prof.log 2>&1
    rc=$?; cd $R; [ $rc -eq 0 ] || { tail -5 $O/prof.log; exit $rc; }
    python3 tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kernel_stats.txt
    python3 tools/timed_kernels.py $O/prof/run_kernel_trace.csv "${PROF_KERNEL:-k_trace4<4, false, false, false>}" 5 > $O/timed_kernels.txt
    grep '^{' $O/prof.log | tail -1 > $O/prof_bench.json
    tail -1 $O/timed_kernels.txt; rm -f $O/prof/*.csv.gz ;;
  ranks)
    bash tools/gpu_rehearse_ranks.sh > $O/ranks.txt 2>&1; rc=$?; tail -3 $O/ranks.txt; [ $rc -eq 0 ] || exit $rc ;;
  cppranks)
    bash tools/gpu_cpp_ranks.sh > $O/cpp_ranks.txt 2>&1; rc=$?; tail -3 $O/cpp_ranks.txt; [ $rc -eq 0 ] || exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
rm -rf gpurun_out/test_scenes gpurun_out/test_images gpurun_out/test_scene
