set -u
cd $GRAFT_REPO_ROOT
cat > /tmp/tail_probe.py <<'PY'
import sys, torch
sys.path.insert(0, ".")
from pupiloptixlab_amd import scenes
from pupiloptixlab_amd.pt_pass import PTPass
desc = scenes.sphere_field(500, 1920, 1080, 4, seed=1).desc()
pt = PTPass(device=0); pt.set_scene(desc)
for spp in (1,):
    pt.mark_dirty(); pt.render(spp, collect_stats=3); torch.cuda.synchronize()
    st = pt.stats()
    print(f"spp {spp}: trace_ms {st['trace_ms']:.3f} nodes {st['node_visits']}", file=sys.stderr, flush=True)
PY
for h in 1 0; do PUPIL_TAIL_HELP=$h PUPIL_TRACE_TAIL=1 timeout -k 10 300 python3 /tmp/tail_probe.py > gpurun_out/tail$h.log 2>&1 || exit 1; echo "help=$h"; grep -E "tail|spp" gpurun_out/tail$h.log; done
