set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06r; mkdir -p $O
cd $GRAFT_REPO_ROOT
X=/tmp/pupil_mv_$$/config4.xml; mkdir -p $(dirname $X)
python3 tools/export_xml.py $X 4 > /dev/null || exit 1
for r in 1 2; do
for v in base PUPIL_REFILL=8 PUPIL_REFILL=24 PUPIL_NODE_MIN=4 PUPIL_NODE_MIN=12 PUPIL_TRACE_GRID_WAVES=6 PUPIL_FRAME_PATHS=0; do
  E=""; [ $v != base ] && E=$v
  line=$(env $E PUPIL_BENCH=2,5,8 PUPIL_BENCH_MOVING=1 timeout -k 10 300 build/pupil_path_tracer $X 2> $O/err.log | tail -n 1)
  [ -n "$line" ] || { cat $O/err.log; exit 1; }
  echo "$r $v $(echo $line | cut -c1-120)" | tee -a $O/moving.txt
done
done
rm -rf $(dirname $X)
