"""Debug: BVH8 any-hit mismatches vs the oracle for refill thresholds."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import oracle
from pupiloptixlab_amd import scenes, abi
from pupiloptixlab_amd.pt_pass import PTPass


def trace(desc, rays, any_hit):
    r8 = np.ascontiguousarray(np.concatenate([rays, np.full((len(rays), 1), 0.001, np.float32),
                                              np.full((len(rays), 1), 1e16, np.float32)], 1), np.float32)
    pt = PTPass(device=0)
    pt.set_scene(desc)
    out = np.zeros((len(rays), 4), np.float32)
    abi.check(pt._lib.pupil_pt_trace_rays(pt._pt, len(rays), r8.ctypes.data_as(abi.f32p), out.ctypes.data_as(abi.f32p), any_hit))
    pt.close_engine()
    return out


w = scenes.sphere_field(27, 64, 36, 4, seed=9)
desc = w.desc()
rng = np.random.default_rng(11)
org = rng.uniform([-7.5, 0.1, -9.5], [7.5, 13.9, 13.5], (200000, 3))
d = rng.normal(size=(200000, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.concatenate([org, d], 1).astype(np.float32)
ref = oracle.OracleScene(desc).closest(rays)
refhit = ref[:, 0] > 0
for width, refill, nmin in [("8", "1", "8"), ("8", "24", "8"), ("8", "24", "1"), ("8", "64", "8"), ("4", "24", "8")]:
    os.environ["PUPIL_BVH_WIDTH"] = width
    os.environ["PUPIL_REFILL"] = refill
    os.environ["PUPIL_NODE_MIN"] = nmin
    outa = trace(desc, rays, 1)
    occ = outa[:, 0] > 0
    fp = int((occ & ~refhit).sum()); fn = int((~occ & refhit).sum())
    print(f"w{width} refill {refill} node_min {nmin}: false occluded {fp}, missed {fn}", flush=True)
    if fn:
        idx = np.nonzero(~occ & refhit)[0][:5]
        print("  b1 marker of unwritten:", np.unique(outa[np.nonzero(~occ & refhit)[0], 1]).tolist()[:5], flush=True)
        print("  missed rays", idx.tolist(), "ref t", ref[idx, 0].tolist(), "out", outa[idx].tolist(), flush=True)
        allm = np.nonzero(~occ & refhit)[0]
        print("  unwritten (0.0):", int((outa[allm, 0] == 0).sum()), "written miss (-1):", int((outa[allm, 0] == -1).sum()),
              "runs:", np.split(allm, np.nonzero(np.diff(allm) > 8)[0] + 1)[:6], flush=True)
