"""Regenerates the committed fixtures in tests/golden/ (run from the repo root):

    python tests/golden/make_golden.py

* rng_sequences.npz   cuda::Random streams (framework/cuda/random.h) for a
                      few (pixel, seed) pairs, from the pure-Python restatement
                      in tests/test_oracle_kat.py (independent of the oracle).
* cornell64_spp4.npz  the CPU oracle's render of the config-1 geometry
                      (data/static/cornellbox.xml transforms, 64x64, 4 spp,
                      max_depth 4) + its ray counts.  Pins the oracle against
                      regressions; the HIP engine is compared with it on the GPU.

The reference itself cannot produce these (OptiX/Windows-only),
so they are "parity unpinned" against reference outputs.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from pupiloptixlab_amd import World, scenes  # noqa: E402
from test_oracle_kat import py_random  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    keys = np.array([[0, 0], [1, 0], [640, 3], [65535, 7], [2073599, 63], [123456, 4294967295]], np.uint64)
    vals = np.stack([py_random(int(p), int(s), 32)[0] for p, s in keys])
    np.savez_compressed(os.path.join(HERE, "rng_sequences.npz"), keys=keys, values=vals)

    path = scenes.cornell_xml(os.path.join(ROOT, "gpurun_out", "golden_cb.xml"), 64, 64, 4)
    w = World().load_scene(path)
    r = oracle.OracleScene(w.desc()).render(spp=4)
    st = r["stats"]
    np.savez_compressed(os.path.join(HERE, "cornell64_spp4.npz"), accum=r["accum"],
                        rays=np.array([st["primary_rays"], st["extension_rays"], st["shadow_rays"]], np.uint64))
    print("wrote fixtures; cornell mean radiance", r["accum"][:, :3].mean(0))


if __name__ == "__main__":
    main()
