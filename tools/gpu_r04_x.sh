#!/bin/bash
# r04 final build: config-4 PMC passes (all kernels: the traversal record and the shade kernels'
# counters) and the C++ drop-in cadence A/B (static / moving camera x speculation settings).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04x
mkdir -p $O
export TMPDIR=/tmp
CONFIG=4 PUPIL_ROUND=r04 bash $R/tools/gpu_pmc.sh > $O/pmc4.log 2>&1 || { tail -5 $O/pmc4.log; exit 1; }
cd $R
mv gpurun_out/pmc_summary.txt $O/pmc_summary4.txt; mv gpurun_out/pmc_config4.json $O/pmc_config4.json; rm -rf gpurun_out/pmc
python3 -c "import json; d=json.load(open('$O/pmc_config4.json')); print('pmc4', round(d['traffic_bytes_per_ray'],1), 'B/ray', round(d['valu_insts_per_ray'],2), 'VALU/ray')"
bash tools/gpu_dropin_ab.sh | cut -c1-200
