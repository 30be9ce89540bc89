set -u
O=gpurun_out/r06u; mkdir -p $O
STEPS="parity" OUT=$O bash tools/gpu_session.sh || exit 1
LIBS="default default,PUPIL_REFILL_TOP=0 default,PUPIL_REFILL_TOP=1 default,PUPIL_REFILL_TOP=5" ROUNDS=2 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-130 $O/ab4.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default default,PUPIL_REFILL_TOP=0" ROUNDS=1 BENCH_ARGS="--config 5 --steps 3 --warmup 6" bash tools/gpu_lib_sweep.sh > $O/ab5.txt 2>&1; rc=$?; cut -c1-130 $O/ab5.txt; exit $rc
