set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06x; mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "cohort" --timeout 120 --timeout-method thread > $O/cohort_tests.txt 2>&1; rc=$?; tail -3 $O/cohort_tests.txt; [ $rc -eq 0 ] || exit $rc
X=/tmp/pupil_mv_$$/config4.xml; mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
for r in 1 2; do
for v in PUPIL_COHORTS=1 base PUPIL_COHORTS=3 PUPIL_COHORTS=4; do
  E=""; [ $v != base ] && E=$v
  line=$(env $E PUPIL_BENCH=2,5,8 PUPIL_BENCH_MOVING=1 timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
  [ -n "$line" ] || { cat $O/err.log; exit 1; }
  echo "$r $v $(echo $line | cut -c1-160)" | tee -a $O/moving.txt
done
done
rm -rf $(dirname $X)
