set -u
O=gpurun_out/r06ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_scenes.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/parity.txt 2>&1; rc=$?; tail -1 $O/parity.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default build/lib_base/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-110 $O/ab4.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default build/lib_base/libpupil_pt.so" ROUNDS=1 BENCH_ARGS="--config 3" bash tools/gpu_lib_sweep.sh > $O/ab3.txt 2>&1; rc=$?; cut -c1-110 $O/ab3.txt; exit $rc
