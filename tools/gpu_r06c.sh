set -u
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fallback or tlas_reserve or one_launch" > $O/fallback.txt 2>&1; rc=$?; tail -1 $O/fallback.txt; [ $rc -eq 0 ] || exit $rc
PUPIL_LIB=build/lib_coop2/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_coop2.txt 2>&1; rc=$?; tail -1 $O/parity_coop2.txt; [ $rc -eq 0 ] || exit $rc
PUPIL_TRACE_DIAG=1 PUPIL_LIB=build/lib_coop2/libpupil_pt.so timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 5 > $O/diag_coop2.log 2>&1 || exit 1
grep "\[pupil\] \(traversal\|coop\)" $O/diag_coop2.log | head -4
LIBS="build/lib_base/libpupil_pt.so build/lib_coop/libpupil_pt.so build/lib_coop2/libpupil_pt.so" ROUNDS=2 bash tools/gpu_lib_sweep.sh > $O/ab.txt 2>&1; rc=$?; cut -c1-120 $O/ab.txt; exit $rc
