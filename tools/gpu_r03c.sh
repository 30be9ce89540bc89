#!/bin/bash
# r03: rocprofv3 kernel stats of the default bench + PMC passes (per-ray figures)
set -u
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_prof.sh || exit 1
cd $R
python3 tools/kstats.py gpurun_out/prof/run_kernel_stats.csv > gpurun_out/r03_kernel_stats.txt 2>&1 || true
head -20 gpurun_out/r03_kernel_stats.txt
cat gpurun_out/pmc_config4.json
