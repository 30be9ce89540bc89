#!/bin/bash
# PMC passes over a short bench (separate passes per counter group, kernel-trace only),
# then the per-launch k_trace4 record bench.py reads (gpurun_out/pmc_config<k>.json;
# copy it to profiles/ to commit it).
set -u
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CFG=${CONFIG:-4}
ARGS="--steps 3 --warmup 4 --cpu-baseline 0 --dropin 0 --config $CFG ${BENCH_ARGS:-}"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum TA_TOTAL_WAVEFRONTS_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" ${EXTRA_SETS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${set//+/ } -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i (${set//+/ }) rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
done
cd $R
K=${PMC_KERNELS:-"k_trace4<0, false, false, false>|k_trace4<3, false, false, false>|k_trace4<4, false, false, false>|k_trace4<0, false, false, true>|k_trace4<3, false, false, true>|k_trace4<4, false, false, true>"}
PUPIL_ROUND=${PUPIL_ROUND:-r06} python3 tools/pmc_summary.py gpurun_out/pmc --json "$K" gpurun_out/pmc_config$CFG.json \
  "config $CFG default bench: all non-instrumented k_trace4 launches (primary extend, mixed extension/shadow, pipelined mixed + camera rays)"
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt
# the shade kernels of the same passes (per-path HBM bytes / VALU of the dominant non-traversal stage)
SK=$(python3 - <<'PY'
import csv, glob, re
names = set()
for f in glob.glob("gpurun_out/pmc/p1/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("pupil::(anonymous namespace)::", "").replace("pupil::", ""))
        if k.startswith("k_shade"):
            names.add(k)
print("|".join(sorted(names)))
PY
)
[ -n "$SK" ] && PUPIL_ROUND=${PUPIL_ROUND:-r06} python3 tools/pmc_summary.py gpurun_out/pmc --json "$SK" gpurun_out/pmc_shade_config$CFG.json \
  "config $CFG default bench: the shade launches (per shaded path: rays_traced here counts the traversal's rays; see shade_paths)"
