#!/bin/bash
# r03: config 5 PMC passes (tools/gpu_pmc.sh, per-ray VALU / HBM figures of the two-level traversal),
# then the config 5 bench reading them (valu-issue / hbm ceilings beside the node-gather figure)
set -u
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
CONFIG=5 PMC_KERNELS="k_trace4<0, false, false>|k_trace4<3, false, false>|k_trace4<4, false, false>" bash tools/gpu_pmc.sh || exit 1
cp gpurun_out/pmc_config5.json profiles/pmc_config5.json
cp gpurun_out/pmc_summary.txt gpurun_out/pmc_summary_config5.txt
timeout -k 10 900 python bench.py --config 5 --steps 3 --warmup 6 --cpu-baseline 0 > gpurun_out/ev/bench5_pmc.log 2>&1
rc=$?; echo "bench5 rc=$rc"; grep '^{' gpurun_out/ev/bench5_pmc.log | tail -1 | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['bound'], r['frac'], {k: v.get('frac') for k, v in r['ceilings'].items()})"
