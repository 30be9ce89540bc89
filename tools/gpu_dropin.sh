#!/bin/bash
# The C++ drop-in cadence (examples/path_tracer, PUPIL_BENCH) on config 4 and a
# rocprofv3 kernel trace of it (per-launch timeline of 8 x 1-spp OnRun).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dropin
cd $R
X=/tmp/pupil_dropin_$$/config4.xml
mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 || exit 1
PUPIL_BENCH=2,5,8 timeout -k 10 300 build/pupil_path_tracer $X > gpurun_out/dropin/bench.log 2>&1
rc=$?; echo "dropin rc=$rc"; tail -n 1 gpurun_out/dropin/bench.log
[ "$rc" -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" != "1" ]; then rm -rf $(dirname $X); exit 0; fi
cd /tmp && export TMPDIR=/tmp
PUPIL_BENCH=1,2,8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/dropin/prof -o run --output-format csv -- $R/build/pupil_path_tracer $X > $R/gpurun_out/dropin/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ "$rc" -eq 0 ] || exit $rc
rm -rf $(dirname $X)
