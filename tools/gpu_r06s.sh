set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06s; mkdir -p $O
cd $GRAFT_REPO_ROOT
PUPIL_LIB=build/lib_dist/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/parity.txt 2>&1; rc=$?; tail -1 $O/parity.txt; [ $rc -eq 0 ] || exit $rc
PUPIL_TRACE_DIAG=1 PUPIL_LIB=build/lib_dist/libpupil_pt.so timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 5 > $O/diag.log 2>&1 || exit 1
grep "\[pupil\] traversal" $O/diag.log | head -2
LIBS="default build/lib_dist/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh > $O/ab.txt 2>&1; rc=$?; cut -c1-130 $O/ab.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default build/lib_dist/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh > $O/ab5.txt 2>&1; rc=$?; cut -c1-130 $O/ab5.txt; exit $rc
