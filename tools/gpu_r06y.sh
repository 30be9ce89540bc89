set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06y; mkdir -p $O
cd $GRAFT_REPO_ROOT
X=/tmp/pupil_mv_$$/config4.xml; mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
export TMPDIR=/tmp
for c in 1 2; do
  PUPIL_COHORTS=$c PUPIL_BENCH=2,3,8 PUPIL_BENCH_MOVING=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/c$c -o run -- $GRAFT_REPO_ROOT/build/pupil_path_tracer $X > $O/c$c.log 2>&1 || { tail -5 $O/c$c.log; exit 1; }
  python3 tools/timeline.py $O/c$c/run_kernel_trace.csv 60 --list 60 > $O/timeline_c$c.txt; tail -25 $O/timeline_c$c.txt
  rm -f $O/c$c/*.csv.gz
done
rm -rf $(dirname $X)
