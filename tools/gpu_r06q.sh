set -u
STEPS="suite smoke bench4 bench3 bench5 prof ranks" OUT=gpurun_out/r06q bash tools/gpu_session.sh || exit 1
VARIANTS="default:" PACING_BENCH=2,5,8 WASTE=8,8 OUT=gpurun_out/r06q bash tools/gpu_pacing.sh > gpurun_out/r06q/pacing.log 2>&1; rc=$?; cut -c1-300 gpurun_out/r06q/pacing.txt; exit $rc
