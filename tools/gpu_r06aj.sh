set -u
STEPS="suite smoke bench4 prof" OUT=gpurun_out/r06aj bash tools/gpu_session.sh
