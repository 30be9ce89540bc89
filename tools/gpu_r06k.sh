set -u
O=gpurun_out/r06k; mkdir -p $O
for v in "PUPIL_PIPE_GROUP_MAX=64" "PUPIL_PIPE_GROUP_MAX=64 PUPIL_PIPE_GROUP_PATHS=8e6"; do
  env $v timeout -k 10 500 python tools/shard_probe.py --onrun 1 --progressive 1 --warmup 24 --frames 24 > $O/probe.txt 2>&1 || { tail -5 $O/probe.txt; exit 1; }
  echo "== $v"; cat $O/probe.txt >> $O/probe_all.txt; grep world $O/probe.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['world'], d['ms_max'], d['pred_speedup'], d['onrun_ms'])"
done
