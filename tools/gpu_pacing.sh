#!/bin/bash
# OnRun pacing of the C++ drop-in (examples/path_tracer on the config-4 scene): per-OnRun
# p50 / p99 / max for frame-group settings (VARIANTS: label:ENV=...;ENV=...), static and moving
# camera; then the rays a camera move discards after k static OnRuns and the heaviest OnRun of
# that stretch (PUPIL_BENCH_WASTE), per variant and with PUPIL_AHEAD=0 (nothing speculated).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${OUT:-gpurun_out/pacing}
mkdir -p $O
cd $R
X=/tmp/pupil_pacing_$$/config4.xml
mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
: > $O/pacing.txt
V=${VARIANTS:-"default: r05:PUPIL_PIPE_GROUP_PATHS=8e6;PUPIL_PIPE_GROUP_MAX=4;PUPIL_PIPE_SPLIT=0 nosplit:PUPIL_PIPE_SPLIT=0 g1:PUPIL_PIPE_GROUP_MAX=1"}
for mv in 0 1; do
  for v in $V; do
    label=${v%%:*}; E=${v#*:}; E=${E//;/ }
    [ "$mv" = 1 ] && [ "$label" != default ] && continue
    line=$(env $E PUPIL_BENCH=${PACING_BENCH:-2,5,8} PUPIL_BENCH_MOVING=$mv timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
    [ -n "$line" ] || { cat $O/err.log; exit 1; }
    echo "moving $mv $label $line" | tee -a $O/pacing.txt
  done
done
for v in $V "ahead0:PUPIL_AHEAD=0"; do
  label=${v%%:*}; E=${v#*:}; E=${E//;/ }
  line=$(env $E PUPIL_BENCH_WASTE=${WASTE:-2,8,32} timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
  [ -n "$line" ] || { cat $O/err.log; exit 1; }
  echo "waste $label $line" | tee -a $O/pacing.txt
done
rm -rf $(dirname $X)
