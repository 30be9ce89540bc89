"""Find non-finite pixels of a full-size config-2 render and compare them with the oracle."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import torch
import oracle
from pupiloptixlab_amd import World, scenes
from pupiloptixlab_amd.pt_pass import PTPass

res, spp = int(sys.argv[1]), int(sys.argv[2])
p = scenes.cornell_materials_xml(os.path.join(HERE, "gpurun_out", "cbmat_probe.xml"), res, res, 6)
desc = World().load_scene(p).desc()
pt = PTPass(device=0)
pt.set_scene(desc)
pt.render(spp)
torch.cuda.synchronize()
acc = pt.buffers.get("pt accum buffer").cpu().numpy().reshape(-1, 4)
bad = np.nonzero(~np.isfinite(acc).all(axis=1))[0].astype(np.uint32)
print("non-finite pixels:", len(bad), bad[:20])
if len(bad):
    ref = oracle.OracleScene(desc).render(spp=spp, pixels=bad[:200], threads=16)
    g = acc[bad[:200]]
    same = (g.view(np.uint32) == ref["accum"].view(np.uint32)).all(axis=1)
    print("oracle bit-identical on them:", int(same.sum()), "/", len(same))
    print("gpu", g[:5]); print("ref", ref["accum"][:5])
    # per-sample: which frame produces the NaN
    for s in range(spp):
        r1 = oracle.OracleScene(desc).render(spp=1, random_seed=s, pixels=bad[:1], threads=1)
        if not np.isfinite(r1["accum"]).all():
            print("first NaN sample of pixel", bad[0], "is", s, r1["accum"]); break
