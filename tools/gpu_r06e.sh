set -u
O=gpurun_out/r06e; mkdir -p $O
PUPIL_ROUND=r06 CONFIG=4 bash tools/gpu_pmc.sh > $O/pmc4.log 2>&1 || { tail -5 $O/pmc4.log; exit 1; }
cp gpurun_out/pmc_config4.json $O/; cp gpurun_out/pmc_summary.txt $O/pmc_summary4.txt; rm -rf gpurun_out/pmc
cp gpurun_out/pmc_config4.json profiles/pmc_config4.json
timeout -k 10 500 python bench.py > $O/bench4.log 2>&1 || { tail -5 $O/bench4.log; exit 1; }
grep '^{' $O/bench4.log | tail -1 > $O/bench4.json; cut -c1-300 $O/bench4.json
python3 -c "import json; d=json.load(open('$O/bench4.json')); print(json.dumps(d['roofline']['ceilings'].get('td-busy')))"
