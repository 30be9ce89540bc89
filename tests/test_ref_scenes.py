"""The reference's own scene files (data/static/*.xml), as committed numeric fixtures
(tests/golden/ref_scenes, made by tests/golden/make_ref_scenes.py from this repo's
XML loader).  CPU: fixtures round-trip and the oracle renders them; when the
reference tree is mounted, a fixture and a fresh load of its XML render the same
pixels.  GPU: the engine renders every scene bit-identically to the oracle."""
import glob
import os

import numpy as np
import pytest

import oracle
from pupiloptixlab_amd import World, scene_io

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_scenes")
SCENES = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(GOLD, "*.npz")))
REF_XML = "/root/reference/data/static"

# film sizes for the parity renders (the reference's aspect ratios, a quarter of the width)
SMALL = {"cornellbox": (128, 128), "default": (180, 180), "denoised_scene": (180, 180),
         "material_test": (320, 180), "mis": (320, 180), "restir_test": (320, 180)}


def test_all_reference_scenes_present():
    assert set(SCENES) == set(SMALL)


@pytest.mark.parametrize("name", SCENES)
def test_fixture_round_trip_and_oracle(name, tmp_path):
    sc = scene_io.LoadedScene(os.path.join(GOLD, name + ".npz"))
    again = str(tmp_path / "again.npz")
    scene_io.save_desc(sc.desc, again)
    a, b = np.load(os.path.join(GOLD, name + ".npz")), np.load(again)
    assert sorted(a.files) == sorted(b.files)
    for k in a.files:
        if k in ("header",) or k.startswith(("shape", "mat", "area", "env")) and a[k].dtype == np.uint8:
            continue  # struct bytes carry pointer values
        assert np.array_equal(a[k], b[k]), k
    d = sc.resized(*SMALL[name])
    r = oracle.OracleScene(d).render(spp=1, pixels=np.arange(0, d.width * d.height, 97, dtype=np.uint32))
    assert np.isfinite(r["accum"]).all()
    assert r["accum"][:, :3].max() > 0


@pytest.mark.skipif(not os.path.isdir(REF_XML), reason="reference tree not mounted")
@pytest.mark.parametrize("name", SCENES)
def test_fixture_matches_fresh_xml_load(name):
    fix = scene_io.LoadedScene(os.path.join(GOLD, name + ".npz")).resized(*SMALL[name])
    w = World().load_scene(os.path.join(REF_XML, name + ".xml"))
    xml = scene_io.LoadedScene.__new__(scene_io.LoadedScene)
    xml.desc = w.desc()
    xml_small = scene_io.LoadedScene.resized(xml, *SMALL[name])
    px = np.arange(0, fix.width * fix.height, 13, dtype=np.uint32)
    ra = oracle.OracleScene(fix).render(spp=2, pixels=px)["accum"]
    rb = oracle.OracleScene(xml_small).render(spp=2, pixels=px)["accum"]
    assert np.array_equal(ra.view(np.uint32), rb.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("accel", ["flat", "two_level"])
@pytest.mark.parametrize("name", SCENES)
def test_reference_scene_gpu_parity(name, accel, monkeypatch):
    """The engine renders each reference scene (its own film aspect, depth, emitters,
    materials) bit-identically to the oracle: 4 spp at a quarter of the width."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_ACCEL", accel)
    sc = scene_io.LoadedScene(os.path.join(GOLD, name + ".npz"))
    d = sc.resized(*SMALL[name])
    pt = PTPass(device=0)
    pt.set_scene(d)
    pt.render(4)
    torch.cuda.synchronize()
    gpu = pt.buffers.get("pt accum buffer").cpu().numpy().reshape(-1, 4)
    albedo = pt.buffers.get("albedo").cpu().numpy().reshape(-1, 3)
    pt.close_engine()
    ref = oracle.OracleScene(d).render(spp=4)
    exact = int(np.all(gpu.view(np.uint32) == ref["accum"].view(np.uint32), axis=1).sum())
    print(f"{name}-{accel}: {exact}/{len(gpu)} pixels bit-exact")
    assert exact == len(gpu)
    assert np.array_equal(albedo, ref["albedo"])
