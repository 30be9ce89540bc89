"""Diagnose GPU-vs-oracle differences on a reference-scene fixture: which pixels,
which sample first diverges, how large."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import oracle  # noqa: E402
from pupiloptixlab_amd import scene_io  # noqa: E402
from pupiloptixlab_amd.pt_pass import PTPass  # noqa: E402

name, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
sc = scene_io.LoadedScene(os.path.join(HERE, "tests", "golden", "ref_scenes", name + ".npz"))
d = sc.resized(w, h)
print("areas", d.num_area_emitters, "env", bool(d.env))
for i in range(d.num_area_emitters):
    e = d.area_emitters[i]
    print("  emitter", i, "type", e.type, "sel", e.select_probability, "area", e.area, "radius", e.radius)
for s in range(4):
    pt = PTPass(device=0)
    pt.set_scene(d)
    pt.dirty = False
    pt.random_seed, pt.sample_cnt = s, 0
    pt.accumulate = False
    pt.render(1)
    torch.cuda.synchronize()
    g = pt.buffers.get("pt accum buffer").cpu().numpy().reshape(-1, 4)
    pt.close_engine()
    r = oracle.OracleScene(d).render(spp=1, random_seed=s, accumulate=False)["accum"]
    bad = np.nonzero((g.view(np.uint32) != r.view(np.uint32)).any(axis=1))[0]
    print(f"sample {s}: {len(bad)} pixels differ", flush=True)
    for p in bad[:4]:
        print("   px", p, "gpu", g[p, :3], "ref", r[p, :3], "rel", np.abs(g[p, :3] - r[p, :3]).max() / max(1e-12, np.abs(r[p, :3]).max()))
