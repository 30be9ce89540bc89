set -u
STEPS="suite smoke" OUT=gpurun_out/r06l bash tools/gpu_session.sh
