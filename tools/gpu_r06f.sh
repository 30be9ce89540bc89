set -u
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pipelined or one_launch or moving_camera or cadence" > $O/pipe_tests.txt 2>&1; rc=$?; tail -2 $O/pipe_tests.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="default: ramp1:PUPIL_PIPE_RAMP=1 r05:PUPIL_PIPE_GROUP_PATHS=8e6;PUPIL_PIPE_GROUP_MAX=4;PUPIL_PIPE_SPLIT=0 nosplit:PUPIL_PIPE_SPLIT=0 g1:PUPIL_PIPE_GROUP_MAX=1" OUT=gpurun_out/r06f bash tools/gpu_pacing.sh > $O/pacing.log 2>&1; rc=$?; cut -c1-230 $O/pacing.txt; [ $rc -eq 0 ] || { tail -5 $O/pacing.log; exit $rc; }
bash tools/gpu_r06e.sh
