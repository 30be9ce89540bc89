set -u
STEPS="suite smoke bench4 bench5" OUT=gpurun_out/r06ae bash tools/gpu_session.sh
