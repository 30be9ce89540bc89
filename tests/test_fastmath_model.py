"""The fast-math error model of tools/fastmath_sensitivity.py (oracle built with
PUPIL_FASTMATH_EMULATION: FMA contraction, reciprocal division, FTZ, transcendentals
displaced by CUDA's documented fast-math error -- the reference's -use_fast_math,
CMakeLists.txt:45).  Test infrastructure for the vs-OptiX sensitivity bound only: it
must build, render finite images close to the exact oracle, and not be bit-identical
to it (else it models nothing)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, numpy as np
sys.path.insert(0, os.environ["ROOT"])
import oracle
from pupiloptixlab_amd import World, scenes
p = scenes.cornell_xml(os.path.join(os.environ["OUT"], "cb.xml"), 48, 48, 4)
r = oracle.OracleScene(World().load_scene(p).desc()).render(spp=4, threads=4)
np.save(os.path.join(os.environ["OUT"], os.environ["TAG"] + ".npy"), r["accum"])
"""


def test_fastmath_emulation_oracle_is_close_but_not_identical(tmp_path):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "_build/liboracle_fastmath.so"],
                   check=True)
    for tag, lib in (("exact", "liboracle.so"), ("fast", "liboracle_fastmath.so")):
        env = dict(os.environ, ROOT=ROOT, OUT=str(tmp_path), TAG=tag,
                   PUPIL_ORACLE_LIB=os.path.join(ROOT, "oracle", "_build", lib))
        subprocess.run([sys.executable, "-c", CHILD], check=True, env=env, timeout=300)
    e, f = np.load(tmp_path / "exact.npy"), np.load(tmp_path / "fast.npy")
    assert np.isfinite(f).all()
    assert not np.array_equal(e.view(np.uint32), f.view(np.uint32))
    rel = np.sqrt(((f[:, :3] - e[:, :3]) ** 2).sum() / (e[:, :3] ** 2).sum())
    assert rel < 1e-3, rel


def test_committed_sensitivity_record_is_complete():
    path = os.path.join(ROOT, "profiles", "r03_fastmath_sensitivity.json")
    rec = json.load(open(path))
    assert {"config4_field_1m_1080p", "config2_cornell_7_materials_1024", "material_test", "mis",
            "cornellbox"} <= set(rec["scenes"])
    for s in rec["scenes"].values():
        assert 0 <= s["rel_l2"] < 1 and s["pixels"] > 0
