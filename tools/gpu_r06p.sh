set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06p; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_work_counters.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.txt 2>&1; rc=$?; tail -1 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
LIBS="build/lib_base/libpupil_pt.so default" ROUNDS=3 bash tools/gpu_lib_sweep.sh > $O/ab.txt 2>&1; rc=$?; cut -c1-110 $O/ab.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 4 --cpu-baseline 0 --dropin 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/timeline.py $O/prof/run_kernel_trace.csv 80 --list 60 > $O/timeline.txt; head -12 $O/timeline.txt
rm -f $O/prof/*.csv
