#!/bin/bash
# Persistent-traversal tail diagnostics: per-launch wave start / drain / exit
# distribution (PUPIL_TRACE_TAIL, STATS kernels) at the batched frame (8 spp)
# and at 1 spp (the drop-in / 8-way-shard batch size), plus the shard probe.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
cat > /tmp/tail_probe.py <<'PY'
import sys, torch
sys.path.insert(0, ".")
from pupiloptixlab_amd import scenes
from pupiloptixlab_amd.pt_pass import PTPass
desc = scenes.sphere_field(500, 1920, 1080, 4, seed=1).desc()
pt = PTPass(device=0); pt.set_scene(desc)
for spp in (8, 1):
    for rep in range(2):
        pt.mark_dirty(); pt.render(spp, collect_stats=3); torch.cuda.synchronize()
        print(f"--- spp {spp} rep {rep}", file=sys.stderr, flush=True)
        st = pt.stats()
        print(f"spp {spp}: trace_ms {st['trace_ms']:.3f} launches {st['trace_launches']} extend_ms {st['extend_ms']:.3f}", file=sys.stderr, flush=True)
PY
PUPIL_TRACE_TAIL=1 timeout -k 10 300 python3 /tmp/tail_probe.py > gpurun_out/tail.log 2>&1
rc=$?; echo "tail rc=$rc"; grep -E "tail|spp" gpurun_out/tail.log | tail -n 24
[ "$rc" -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/shard_probe.py > gpurun_out/shard_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/shard_probe.log | cut -c1-200
