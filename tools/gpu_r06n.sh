set -u
O=gpurun_out/r06n; mkdir -p $O
SETS="base PUPIL_TL_MODE=object PUPIL_ACCEL=flat" BENCH_ARGS="--config 5 --steps 3 --warmup 6" ROUNDS=2 bash tools/gpu_env_sweep.sh > $O/sweep5.txt 2>&1; rc=$?; cat $O/sweep5.txt; exit $rc
