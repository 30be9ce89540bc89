set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r06aa; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --steps 2 --warmup 2 --cpu-baseline 0 --dropin 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kernel_stats.txt
python3 tools/timeline.py $O/prof/run_kernel_trace.csv 120 --list 60 > $O/timeline.txt
rm -f $O/prof/*.csv.gz; head -25 $O/kernel_stats.txt
