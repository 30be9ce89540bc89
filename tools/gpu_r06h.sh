set -u
O=gpurun_out/r06h; mkdir -p $O
VARIANTS="default: r05:PUPIL_PIPE_GROUP_PATHS=8e6;PUPIL_PIPE_GROUP_MAX=4;PUPIL_PIPE_SPLIT=0;PUPIL_PIPE_RAMP=0" PACING_BENCH=2,5,8 WASTE=8,8 OUT=gpurun_out/r06h bash tools/gpu_pacing.sh > $O/pacing.log 2>&1; rc=$?; grep waste $O/pacing.txt | cut -c1-400; [ $rc -eq 0 ] || { tail -5 $O/pacing.log; exit $rc; }
SETS="base PUPIL_NODE_MIN=12 PUPIL_NODE_MIN=16 PUPIL_REFILL=24 PUPIL_TL_BRAID=8 PUPIL_TL_BRAID=12 PUPIL_LEAF_SIZE=3" BENCH_ARGS="--config 5 --steps 3 --warmup 6" ROUNDS=1 bash tools/gpu_env_sweep.sh > $O/sweep5.txt 2>&1; rc=$?; cat $O/sweep5.txt; exit $rc
