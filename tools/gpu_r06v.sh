set -u
O=gpurun_out/r06v; mkdir -p $O
STEPS="parity" OUT=$O bash tools/gpu_session.sh || exit 1
LIBS="default build/lib_pinst/libpupil_pt.so" ROUNDS=2 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh > $O/ab5.txt 2>&1; rc=$?; cut -c1-130 $O/ab5.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default build/lib_pinst/libpupil_pt.so" ROUNDS=1 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-130 $O/ab4.txt; exit $rc
