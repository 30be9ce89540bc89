"""Tiled vs full-frame progressive rendering on one GPU (diagnostic): the same
sequence of batched renders, full frame vs two tile shares, compared per frame."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pupiloptixlab_amd import scenes  # noqa: E402
from pupiloptixlab_amd.pt_pass import PTPass  # noqa: E402

desc = scenes.sphere_field(60, 320, 240, 4, seed=1).desc()
frames = 3


def run(tile, continues):
    pt = PTPass(device=0)
    pt.set_scene(desc)
    if tile:
        pt.set_tiling(32, tile[0], tile[1])
    pt.mark_dirty()
    out = []
    for _ in range(frames):
        pt.render(8, continues=continues)
        torch.cuda.synchronize()
        out.append(pt.buffers.get("pt accum buffer").cpu().numpy().copy())
    pix = pt.local_pixels() if tile else None
    pt.close_engine()
    return out, pix


for cont in (False, True):
    full, _ = run(None, cont)
    parts = [run((r, 2), cont) for r in range(2)]
    for f in range(frames):
        img = np.zeros_like(full[f])
        for out, pix in parts:
            img[pix] = out[f]
        d = np.any(img.view(np.uint32) != full[f].view(np.uint32), axis=1)
        print(f"continues={cont} frame {f}: differing pixels {int(d.sum())} / {len(d)}")
