set -u
STEPS="pmc3 pmc5 bench4 bench3 bench5 prof" OUT=gpurun_out/r06m bash tools/gpu_session.sh
