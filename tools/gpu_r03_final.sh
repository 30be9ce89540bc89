#!/bin/bash
# r03 final evidence of the final build in one session: GPU suite + smoke, rocprofv3 kernel stats
# and the PMC passes (config 4), the per-ray PMC record copied into profiles/ so the bench lines
# that follow use it, then the evidence benches (config 4 with the CPU / timed-frame / drop-in
# checks, the 2-rank rehearsal, config 5, config 3).
set -u
bash tools/gpu_r03_suite.sh || exit 1
bash tools/gpu_prof.sh || exit 1
cp gpurun_out/pmc_config4.json profiles/pmc_config4.json
bash tools/gpu_r03_evidence.sh
