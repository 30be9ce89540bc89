set -u
O=gpurun_out/r06ak; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.txt 2>&1; rc=$?; tail -1 $O/suite.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default build/lib_base/libpupil_pt.so" ROUNDS=3 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-110 $O/ab4.txt; exit $rc
