"""How far can the OptiX reference's render sit from the exact oracle?

The reference compiles its device code with -use_fast_math (CMakeLists.txt:45):
FMA contraction, approximate division / sqrt / transcendentals, flush-to-zero.  The
engine and the oracle are exact IEEE (-ffp-contract=off, correctly rounded / and
sqrt, one deterministic libm) and agree bit for bit; neither can say what the
reference's own float choices do to an image.  This tool bounds it: the same
oracle source built with that error model (oracle/Makefile liboracle_fastmath.so:
-ffp-contract=fast, -freciprocal-math, FTZ/DAZ, transcendentals displaced by their
documented CUDA fast-math error, pupil_detmath.h PUPIL_FASTMATH_EMULATION) renders
the same scenes and seeds as the exact oracle; the image difference is what
float-level choices of that magnitude do to a path-traced image -- the floor of any
"rel-L2 vs OptiX" comparison, since the real OptiX differs from both in exactly
such choices (and in its closed-source traversal / triangle test besides).

usage: python tools/fastmath_sensitivity.py [--spp 16] [--out profiles/r03_fastmath_sensitivity.json]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

SCENES = {  # name -> film size of the reference fixtures (None: a BASELINE config at its size)
    "config4_field_1m_1080p": None,
    "config2_cornell_7_materials_1024": None,
    "material_test": (320 * 2, 180 * 2),
    "mis": (320 * 2, 180 * 2),
    "cornellbox": (256, 256),
}


def load(name):
    from pupiloptixlab_amd import World, scene_io, scenes

    if name.startswith("config4"):
        return scenes.sphere_field(500, 1920, 1080, 4, seed=1).desc()
    if name.startswith("config2"):
        p = scenes.cornell_materials_xml(os.path.join(HERE, "gpurun_out", "test_scenes", "cbmat1024.xml"), 1024, 1024, 6)
        return World().load_scene(p).desc()
    w, h = SCENES[name]
    return scene_io.LoadedScene(os.path.join(HERE, "tests", "golden", "ref_scenes", name + ".npz")).resized(w, h)


def render_child(name, spp, out):
    """(subprocess) render one scene with the oracle library named by PUPIL_ORACLE_LIB."""
    import oracle

    desc = load(name)
    t0 = time.time()
    r = oracle.OracleScene(desc).render(spp=spp, threads=os.cpu_count())
    np.save(out, r["accum"])
    print(json.dumps({"seconds": time.time() - t0, "stats": r["stats"]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--out", default=os.path.join(HERE, "profiles", "r03_fastmath_sensitivity.json"))
    ap.add_argument("--scenes", nargs="*", default=list(SCENES))
    ap.add_argument("--child", nargs=3, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        render_child(a.child[0], int(a.child[1]), a.child[2])
        return
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "oracle"), "all", "_build/liboracle_fastmath.so"], check=True)
    libs = {"exact": os.path.join(HERE, "oracle", "_build", "liboracle.so"),
            "fastmath": os.path.join(HERE, "oracle", "_build", "liboracle_fastmath.so")}
    tmp = os.path.join(HERE, "gpurun_out", "fastmath")
    os.makedirs(tmp, exist_ok=True)
    res = {"what": __doc__.strip().split("\n\n")[0], "spp": a.spp, "scenes": {}}
    if os.path.exists(a.out):  # keep the scenes rendered by earlier invocations
        with open(a.out) as fh:
            res["scenes"] = json.load(fh).get("scenes", {})
    for name in a.scenes:
        img = {}
        for k, lib in libs.items():
            out = os.path.join(tmp, f"{name}_{k}.npy")
            env = dict(os.environ, PUPIL_ORACLE_LIB=lib)
            subprocess.run([sys.executable, __file__, "--child", name, str(a.spp), out], check=True, env=env,
                           capture_output=True, text=True)
            img[k] = np.load(out)[:, :3].astype(np.float64)
        e, f = img["exact"], img["fastmath"]
        diff = np.abs(f - e)
        rel_px = diff.max(axis=1) / np.maximum(1e-6, np.abs(e).max(axis=1))
        rec = {"pixels": int(len(e)),
               "rel_l2": float(np.sqrt((diff ** 2).sum() / max(1e-30, (e ** 2).sum()))),
               "bit_identical_pixels": int(np.all(diff == 0, axis=1).sum()),
               "pixels_rel_err_gt_1e-3": int((rel_px > 1e-3).sum()),
               "pixels_rel_err_gt_1e-2": int((rel_px > 1e-2).sum()),
               "mean_exact": float(e.mean()), "mean_fastmath": float(f.mean())}
        res["scenes"][name] = rec
        print(name, json.dumps(rec), flush=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
