set -u
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 500 python tools/shard_probe.py --onrun 1 --progressive 1 --warmup 24 --frames 24 > $O/probe_default.txt 2>&1 || { tail -5 $O/probe_default.txt; exit 1; }
cut -c1-200 $O/probe_default.txt | grep world
PUPIL_PIPE_GROUP_PATHS=8e6 PUPIL_PIPE_GROUP_MAX=64 PUPIL_PIPE_SPLIT=0 PUPIL_PIPE_RAMP=0 timeout -k 10 500 python tools/shard_probe.py --onrun 1 --progressive 1 --warmup 24 --frames 24 > $O/probe_r05.txt 2>&1 || { tail -5 $O/probe_r05.txt; exit 1; }
cut -c1-200 $O/probe_r05.txt | grep world
