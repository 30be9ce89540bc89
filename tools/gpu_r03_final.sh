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
# gpurun copies back at most 64 MiB of gpurun_out/: drop the bulky intermediates (the rehearsal's
# frames, the raw kernel traces and per-pass counter dumps; the summaries stay)
python3 tools/kstats.py gpurun_out/prof/run_kernel_stats.csv > gpurun_out/kernel_stats.txt
python3 tools/timed_kernels.py gpurun_out/prof/run_kernel_trace.csv "k_trace4<4, false, false>" 5 > gpurun_out/timed_kernels.txt
rm -rf gpurun_out/ev/*.npy gpurun_out/prof gpurun_out/pmc gpurun_out/test_scenes gpurun_out/test_images gpurun_out/test_scene
