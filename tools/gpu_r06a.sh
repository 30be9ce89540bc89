set -u
O=gpurun_out/r06a; mkdir -p $O
export PUPIL_LIB_COOP=build/lib_coop/libpupil_pt.so
PUPIL_LIB=build/lib_coop/libpupil_pt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_coop.txt 2>&1; rc=$?; tail -3 $O/parity_coop.txt; [ $rc -eq 0 ] || exit $rc
for l in build/lib_base/libpupil_pt.so build/lib_coop/libpupil_pt.so; do
  PUPIL_TRACE_DIAG=1 PUPIL_LIB=$l timeout -k 10 200 python bench.py --cpu-baseline 0 --dropin 0 --steps 5 > $O/diag_$(basename $(dirname $l)).log 2>&1 || exit 1
  grep "\[pupil\] \(traversal\|coop\)" $O/diag_$(basename $(dirname $l)).log | head -4
done
LIBS="build/lib_base/libpupil_pt.so default build/lib_coop/libpupil_pt.so" ROUNDS=2 bash tools/gpu_lib_sweep.sh > $O/ab.txt 2>&1; rc=$?; cut -c1-200 $O/ab.txt; exit $rc
