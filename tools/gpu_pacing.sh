#!/bin/bash
# OnRun pacing of the C++ drop-in (examples/path_tracer on the config-4 scene): per-OnRun
# p50 / p99 / max with the default frame groups (G = ceil(8 M / paths) = 4 at 1080p), G = 2 and
# G = 1 (PUPIL_PIPE_GROUP_PATHS), static and moving camera; then the rays a camera move discards
# after k static OnRuns (PUPIL_BENCH_WASTE), default vs PUPIL_AHEAD=0 (nothing speculated: the
# difference is the discarded speculation).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/${OUT:-gpurun_out/pacing}
mkdir -p $O
cd $R
X=/tmp/pupil_pacing_$$/config4.xml
mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
: > $O/pacing.txt
for mv in 0 1; do
  for g in default 4.2e6 1; do
    if [ "$g" = default ]; then E=""; else E="PUPIL_PIPE_GROUP_PATHS=$g"; fi
    line=$(env $E PUPIL_BENCH=2,5,8 PUPIL_BENCH_MOVING=$mv timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
    [ -n "$line" ] || { cat $O/err.log; exit 1; }
    echo "moving $mv group_paths $g $line" | tee -a $O/pacing.txt
  done
done
for ah in default 0; do
  if [ "$ah" = default ]; then E=""; else E="PUPIL_AHEAD=$ah"; fi
  line=$(env $E PUPIL_BENCH_WASTE=2,8,32 timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
  [ -n "$line" ] || { cat $O/err.log; exit 1; }
  echo "waste ahead $ah $line" | tee -a $O/pacing.txt
done
rm -rf $(dirname $X)
