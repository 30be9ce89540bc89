set -u
O=gpurun_out/r06ad; mkdir -p $O
PUPIL_SUBSHARDS=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/parity32.txt 2>&1; rc=$?; tail -1 $O/parity32.txt; [ $rc -eq 0 ] || exit $rc
LIBS="default default,PUPIL_SUBSHARDS=4 default,PUPIL_SUBSHARDS=8 default,PUPIL_SUBSHARDS=16 default,PUPIL_SUBSHARDS=32" ROUNDS=2 bash tools/gpu_lib_sweep.sh > $O/ab4.txt 2>&1; rc=$?; cut -c1-120 $O/ab4.txt; exit $rc
