set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 4 --cpu-baseline 0 --dropin 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/timeline.py $O/prof/run_kernel_trace.csv 80 --list 60 > $O/timeline.txt; head -30 $O/timeline.txt
rm -f $O/prof/*.csv
