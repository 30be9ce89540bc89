set -u
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 500 --timeout-method thread -k config2 > $O/config2.txt 2>&1; rc=$?; grep -E "config2|passed|failed" $O/config2.txt | tail -3; [ $rc -eq 0 ] || exit $rc
RANKS="2 3" bash tools/gpu_rehearse_ranks.sh > $O/ranks.txt 2>&1; rc=$?; tail -6 $O/ranks.txt; [ $rc -eq 0 ] || exit $rc
PUPIL_ROUND=r06 CONFIG=4 bash tools/gpu_pmc.sh > $O/pmc4.log 2>&1 || { tail -5 $O/pmc4.log; exit 1; }
cp gpurun_out/pmc_config4.json $O/; cp gpurun_out/pmc_summary.txt $O/pmc_summary4.txt; rm -rf gpurun_out/pmc
timeout -k 10 500 python bench.py > $O/bench4.log 2>&1 || { tail -5 $O/bench4.log; exit 1; }
grep '^{' $O/bench4.log | tail -1 > $O/bench4.json; cut -c1-300 $O/bench4.json
