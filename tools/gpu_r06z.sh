set -u
STEPS="suite smoke bench4 bench3 bench5 prof" OUT=gpurun_out/r06z bash tools/gpu_session.sh
