#!/bin/bash
# Extra PMC passes (one counter group per rocprofv3 run, kernel trace only) over a short
# config bench, summarised per kernel by tools/pmc_summary.py.
# usage: SETS="TA_BUSY_avr+TA_TOTAL_WAVEFRONTS_sum TD_TD_BUSY_sum+GRBM_GUI_ACTIVE" OUT=gpurun_out/x \
#        [PUPIL_LIB=build/.../libpupil_pt.so] [CONFIG=4] bash tools/gpu_pmc_sets.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${OUT:-gpurun_out/pmc_sets}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
[ -n "${PUPIL_LIB:-}" ] && case "$PUPIL_LIB" in /*) ;; *) export PUPIL_LIB=$R/$PUPIL_LIB ;; esac
ARGS="--steps 3 --warmup 4 --cpu-baseline 0 --dropin 0 --config ${CONFIG:-4}"
i=0
for set in $SETS; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${set//+/ } -d $O/p$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $O/p$i.log 2>&1
  rc=$?; echo "pass $i (${set//+/ }) rc=$rc"
  [ "$rc" -eq 0 ] || exit $rc
done
cd $R
python3 tools/pmc_summary.py $O > $O/summary.txt && rm -rf $O/p*/*.csv.gz
