"""GPU parity tests: the HIP engine (through the C ABI) against the CPU oracle.

Bar: the engine reproduces the oracle bit for bit on identical RNG seeds
(both compute every float in the reference's order with the same
deterministic libm); the SURVEY.md §8(d) acceptance metric, relative image
L2 < 1e-4, is asserted as well and the exact-match count is reported.
"""
import os

import numpy as np
import pytest

import oracle
from pupiloptixlab_amd import World, scenes
from pupiloptixlab_amd import world as world_mod
from pupiloptixlab_amd import abi

pytestmark = pytest.mark.gpu

TMP = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "test_scenes")


def rel_l2(a, b):
    a, b = np.asarray(a)[..., :3], np.asarray(b)[..., :3]
    return float(np.sqrt(((a - b) ** 2).sum() / max(1e-30, (b ** 2).sum())))


def render_gpu(desc, spp, seed=0, cnt=0, max_depth=0, accumulate=True, tile=(32, 0, 1), prev=None, stats=True):
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    pt = PTPass(device=0)
    pt.set_scene(desc)
    if tile[2] > 1:
        pt.set_tiling(*tile)
    if max_depth:
        pt.max_depth = max_depth
    pt.accumulate = accumulate
    pt.dirty = False
    pt.random_seed, pt.sample_cnt = seed, cnt
    if prev is not None:
        pt.buffers.get("pt accum buffer").copy_(torch.from_numpy(prev))
    pt.render(spp, collect_stats=stats)
    torch.cuda.synchronize()
    out = {k: pt.buffers.get(k).cpu().numpy() for k in ("pt accum buffer", "final result", "albedo", "normal", "test")}
    out["stats"] = pt.stats()
    pt.close_engine()
    return out


def compare(gpu, ref, name):
    g, r = gpu["pt accum buffer"], ref["accum"]
    exact = int(np.all(g == r, axis=1).sum())
    err = rel_l2(g, r)
    print(f"{name}: rel_L2 {err:.3e}, bit-exact pixels {exact}/{len(r)}, "
          f"pixels rel>1e-3: {int((np.abs(g - r).max(axis=1) > 1e-3 * np.maximum(1e-6, np.abs(r).max(axis=1))).sum())}")
    assert np.isfinite(g).all()
    assert err < 1e-4, f"{name}: relative L2 {err}"
    return exact


def test_detmath_bit_exact():
    lib = abi.load_library()
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-12.6, 12.6, 50000), rng.uniform(-1, 1, 50000),
                        np.array([0.0, -0.0, 1.0, -1.0, 0.5, np.pi, 1e-8, 2 * np.pi])]).astype(np.float32)
    y = np.concatenate([rng.uniform(-5, 5, len(x) - 4), np.array([0.0, -1.0, 1.0, 0.0])]).astype(np.float32)
    out = np.zeros((len(x), 6), np.float32)
    f = abi.f32p
    abi.check(lib.pupil_debug_math(0, len(x), x.ctypes.data_as(f), y.ctypes.data_as(f), out.ctypes.data_as(f)))
    ref = oracle.math_probe(x, y)
    mism = (out.view(np.uint32) != ref.view(np.uint32)) & ~(np.isnan(out) & np.isnan(ref))
    assert not mism.any(), f"{mism.sum(axis=0)} mismatches per function (sin cos acos atan2 sqrt rcp)"


def _cornell(res, depth=4):
    return World().load_scene(scenes.cornell_xml(os.path.join(TMP, f"cb{res}.xml"), res, res, depth))


@pytest.mark.parametrize("refill", ["1", "16", "64"])
def test_primary_hits_match_oracle(refill, monkeypatch):
    monkeypatch.setenv("PUPIL_REFILL", refill)
    w = _cornell(96)
    desc = w.desc()
    o = oracle.OracleScene(desc)
    rays = np.array([o.camera_ray(p, 3) for p in range(96 * 96)], np.float32)
    # plus random rays from inside the box
    rng = np.random.default_rng(1)
    org = rng.uniform([-0.9, 0.1, -0.9], [0.9, 1.9, 0.9], (5000, 3))
    dirs = rng.normal(size=(5000, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    rays = np.concatenate([rays, np.concatenate([org, dirs], 1).astype(np.float32)])
    ref = o.closest(rays)
    import ctypes as C
    from pupiloptixlab_amd.pt_pass import PTPass

    pt = PTPass(device=0)
    pt.set_scene(desc)
    r8 = np.concatenate([rays, np.full((len(rays), 1), 0.001, np.float32), np.full((len(rays), 1), 1e16, np.float32)],
                        1)
    r8 = np.ascontiguousarray(r8, np.float32)
    out = np.zeros((len(rays), 4), np.float32)
    abi.check(pt._lib.pupil_pt_trace_rays(pt._pt, len(rays), r8.ctypes.data_as(abi.f32p),
                                          out.ctypes.data_as(abi.f32p), 0))
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), \
        f"{(out.view(np.uint32) != ref.view(np.uint32)).any(axis=1).sum()} rays differ"
    # shadow (any-hit) queries agree with closest-hit occupancy
    abi.check(pt._lib.pupil_pt_trace_rays(pt._pt, len(rays), r8.ctypes.data_as(abi.f32p),
                                          out.ctypes.data_as(abi.f32p), 1))
    assert np.array_equal(out[:, 0] > 0, ref[:, 0] > 0)
    pt.close_engine()


def test_cornell_parity_config1():
    """Config 1 geometry (cornellbox.xml), 128^2, 4 spp, max depth 4."""
    w = _cornell(128)
    desc = w.desc()
    gpu = render_gpu(desc, 4)
    ref = oracle.OracleScene(desc).render(spp=4)
    exact = compare(gpu, ref, "cornell128x4")
    assert exact == 128 * 128
    for k, rk in (("albedo", "albedo"), ("normal", "normal")):
        assert np.array_equal(gpu[k], ref[rk]), k
    assert np.array_equal(gpu["test"].reshape(-1), ref["test"])
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"], s["shadow_rays_reference"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"], rs["shadow_rays_reference"])


def test_config1_cornellbox_named_size():
    """BASELINE config 1 exactly as named: the reference's own cornellbox.xml (committed
    numeric fixture), 256x256, 1 spp, max depth 4, seed 0 (`main.cu:36-194`).  Every pixel,
    the AOVs and the ray counts are bit-identical to the oracle."""
    from pupiloptixlab_amd import scene_io

    gold = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_scenes", "cornellbox.npz")
    d = scene_io.LoadedScene(gold).resized(256, 256)
    assert d.max_depth == 4
    gpu = render_gpu(d, 1)
    ref = oracle.OracleScene(d).render(spp=1)
    exact = compare(gpu, ref, "config1-cornellbox256x1")
    assert exact == 256 * 256
    assert np.array_equal(gpu["pt accum buffer"].view(np.uint32), ref["accum"].view(np.uint32))
    assert np.array_equal(gpu["albedo"], ref["albedo"]) and np.array_equal(gpu["normal"], ref["normal"])
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"], s["shadow_rays_reference"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"], rs["shadow_rays_reference"])
    # the reference traces a shadow ray on every loop iteration past RR (main.cu:119-123)
    assert rs["shadow_rays"] <= rs["shadow_rays_reference"] <= rs["primary_rays"] * (d.max_depth - 1)


@pytest.mark.parametrize("accel", ["flat", "two_level"])
def test_materials_parity_config2(accel, monkeypatch):
    """Config 2 (all seven BSDFs, spheres + boxes) at 192^2, 8 spp, depth 6; one flattened
    BVH4, or a TLAS over the mesh and sphere instances."""
    monkeypatch.setenv("PUPIL_ACCEL", accel)
    p = scenes.cornell_materials_xml(os.path.join(TMP, "cbmat.xml"), 192, 192, 6)
    desc = World().load_scene(p).desc()
    gpu = render_gpu(desc, 8)
    assert gpu["stats"]["two_level"] == (accel == "two_level")
    ref = oracle.OracleScene(desc).render(spp=8)
    assert compare(gpu, ref, f"materials192x8-{accel}") == 192 * 192


@pytest.mark.parametrize("refill", ["1", "16", "64"])
def test_sphere_field_parity(refill, monkeypatch):
    monkeypatch.setenv("PUPIL_REFILL", refill)
    w = scenes.sphere_field(27, 240, 136, 4, seed=3)
    desc = w.desc()
    gpu = render_gpu(desc, 2)
    ref = oracle.OracleScene(desc).render(spp=2)
    compare(gpu, ref, f"field27-refill{refill}")


@pytest.mark.parametrize("node_min", ["1", "8", "64"])
def test_stage_schedules_parity(node_min, monkeypatch):
    """The mixed extension + shadow launch with the node phase left at 1, 8 (default) or 64
    active lanes: lanes switch between node and leaf phases at other points, hits do not change."""
    monkeypatch.setenv("PUPIL_NODE_MIN", node_min)
    monkeypatch.setenv("PUPIL_FRAME_PATHS", "0")  # the stage launches, not the one-launch frame
    desc = scenes.sphere_field(27, 200, 120, 5, seed=4).desc()
    gpu = render_gpu(desc, 3)
    ref = oracle.OracleScene(desc).render(spp=3)
    exact = compare(gpu, ref, f"schedule-node_min{node_min}")
    assert exact == 200 * 120
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"])


def test_deep_paths_parity():
    """max_depth 70 > 63: the flags byte carries no bounce tag and is cleared every bounce."""
    w = _cornell(48, depth=70)
    desc = w.desc()
    gpu = render_gpu(desc, 2)
    ref = oracle.OracleScene(desc).render(spp=2)
    assert compare(gpu, ref, "cornell48-depth70") == 48 * 48
    s, rs = gpu["stats"], ref["stats"]
    assert (s["extension_rays"], s["shadow_rays"]) == (rs["extension_rays"], rs["shadow_rays"])


# (PUPIL_REFILL, PUPIL_NODE_MIN) of the persistent BVH4 kernel: refill thresholds from one idle lane to a
# whole wave, node-phase exits from one lane to the whole wave
TRAVERSALS = [("1", "8"), ("16", "8"), ("16", "1"), ("24", "64"), ("64", "8")]


def _set_traversal(monkeypatch, refill, node_min):
    monkeypatch.setenv("PUPIL_REFILL", refill)
    monkeypatch.setenv("PUPIL_NODE_MIN", node_min)


def _trace(desc, rays, any_hit=0, tmin=0.001, tmax=1e16):
    from pupiloptixlab_amd.pt_pass import PTPass

    r8 = np.ascontiguousarray(np.concatenate([rays, np.full((len(rays), 1), tmin, np.float32),
                                              np.full((len(rays), 1), tmax, np.float32)], 1), np.float32)
    pt = PTPass(device=0)
    pt.set_scene(desc)
    out = np.zeros((len(rays), 4), np.float32)
    abi.check(pt._lib.pupil_pt_trace_rays(pt._pt, len(rays), r8.ctypes.data_as(abi.f32p),
                                          out.ctypes.data_as(abi.f32p), any_hit))
    pt.close_engine()
    return out


def test_field_hits_random_rays_all_traversals(monkeypatch):
    """Closest hits of 200k random rays in a 54k-triangle field: every traversal kernel and the oracle agree."""
    w = scenes.sphere_field(27, 64, 36, 4, seed=9)
    desc = w.desc()
    rng = np.random.default_rng(11)
    org = rng.uniform([-7.5, 0.1, -9.5], [7.5, 13.9, 13.5], (200000, 3))
    d = rng.normal(size=(200000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([org, d], 1).astype(np.float32)
    ref = oracle.OracleScene(desc).closest(rays)
    for refill, node_min in TRAVERSALS:
        _set_traversal(monkeypatch, refill, node_min)
        out = _trace(desc, rays)
        bad = (out.view(np.uint32) != ref.view(np.uint32)).any(axis=1)
        assert not bad.any(), f"refill {refill} node_min {node_min}: {bad.sum()} rays differ"
        occ = _trace(desc, rays, any_hit=1)
        assert np.array_equal(occ[:, 0] > 0, ref[:, 0] > 0), f"refill {refill} node_min {node_min}: any-hit differs"


@pytest.mark.parametrize("accel", ["flat", "two_level"])
def test_instanced_hits_random_rays(accel, monkeypatch):
    """Closest and any hits of 100k random rays among 12 instances of one BLAS under rotations,
    non-uniform scales and translations: the two-level traversal (object-space BLAS boxes,
    world-space triangle tests) equals the flattened BVH and the oracle bit for bit."""
    monkeypatch.setenv("PUPIL_ACCEL", accel)
    w = scenes.instanced_field(num_instances=12, width=32, height=18, max_depth=4, seed=3, spheres_per_blas=10,
                               scale_range=(0.4, 2.5))
    desc = w.desc()
    rng = np.random.default_rng(13)
    n = 100000
    org = rng.uniform([-12, 0.1, -12], [12, 14, 12], (n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([org, d], 1).astype(np.float32)
    ref = oracle.OracleScene(desc).closest(rays)
    assert (ref[:, 0] > 0).mean() > 0.3
    out = _trace(desc, rays)
    bad = (out.view(np.uint32) != ref.view(np.uint32)).any(axis=1)
    assert not bad.any(), f"{accel}: {bad.sum()} rays differ"
    occ = _trace(desc, rays, any_hit=1)
    assert np.array_equal(occ[:, 0] > 0, ref[:, 0] > 0)


def _quad_stack(n, spacing=0.01):
    """n parallel unit quads stacked along z: every ray along z crosses all of them, so the
    traversal stack grows past the 16-entry LDS ring and spills to HBM."""
    w = World()
    z = np.arange(n, dtype=np.float32) * spacing
    pos = np.zeros((n, 4, 3), np.float32)
    pos[:, :, 0] = [-1, 1, 1, -1]
    pos[:, :, 1] = [-1, -1, 1, 1]
    pos[:, :, 2] = z[:, None]
    idx = (np.arange(n, dtype=np.uint32)[:, None] * 4 + np.array([0, 1, 2, 0, 2, 3], np.uint32)).reshape(-1, 3)
    s = w.add_mesh(pos.reshape(-1, 3), idx)
    m = w.add_material(world_mod.diffuse((0.5, 0.5, 0.5)))
    w.add_instance(s, m)
    w.set_film(16, 16, 2)
    w.set_sensor(40.0, world_mod.look_at_mitsuba((0, 0, -3), (0, 0, 0), (0, 1, 0)))
    return w


@pytest.mark.parametrize("accel", ["flat", "two_level"])
def test_deep_stack_spills_match_oracle(accel, monkeypatch):
    monkeypatch.setenv("PUPIL_ACCEL", accel)
    w = _quad_stack(6000)
    desc = w.desc()
    rng = np.random.default_rng(5)
    n = 20000
    org = np.concatenate([rng.uniform(-0.9, 0.9, (n, 2)), np.full((n, 1), -1.0)], 1)
    d = np.concatenate([rng.uniform(-0.02, 0.02, (n, 2)), np.ones((n, 1))], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # half the rays start inside the stack and go backwards (farthest-first order)
    org[n // 2:, 2] = 70.0
    d[n // 2:, 2] *= -1
    rays = np.concatenate([org, d], 1).astype(np.float32)
    ref = oracle.OracleScene(desc).closest(rays)
    assert (ref[:, 0] > 0).mean() > 0.9
    for refill, node_min in TRAVERSALS if accel == "flat" else [("24", "8")]:
        _set_traversal(monkeypatch, refill, node_min)
        out = _trace(desc, rays)
        bad = (out.view(np.uint32) != ref.view(np.uint32)).any(axis=1)
        assert not bad.any(), f"{accel} refill {refill} node_min {node_min}: {bad.sum()} rays differ"


@pytest.mark.parametrize("accel", ["flat", "two_level"])
@pytest.mark.parametrize("ntri", [1, 2, 4, 5])
def test_tiny_scenes(ntri, accel, monkeypatch):
    """The root is a leaf (<= 4 primitives): traversal terminates and hits match."""
    monkeypatch.setenv("PUPIL_ACCEL", accel)
    w = World()
    tri_pos = np.array([[-1, -1, 0], [1, -1, 0], [0, 1, 0]], np.float32)
    pos = np.concatenate([tri_pos + [0, 0, 0.1 * k] for k in range(ntri)]).astype(np.float32)
    s = w.add_mesh(pos, np.arange(3 * ntri, dtype=np.uint32).reshape(-1, 3))
    w.add_instance(s, w.add_material(world_mod.diffuse((0.5, 0.5, 0.5))))
    w.set_film(16, 16, 2)
    w.set_sensor(40.0, world_mod.look_at_mitsuba((0, 0, -3), (0, 0, 0), (0, 1, 0)))
    desc = w.desc()
    rng = np.random.default_rng(2)
    org = np.concatenate([rng.uniform(-1, 1, (500, 2)), np.full((500, 1), -2.0)], 1)
    d = np.concatenate([rng.uniform(-0.2, 0.2, (500, 2)), np.ones((500, 1))], 1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([org, d], 1).astype(np.float32)
    ref = oracle.OracleScene(desc).closest(rays)
    for refill, node_min in TRAVERSALS if accel == "flat" else [("24", "8")]:
        _set_traversal(monkeypatch, refill, node_min)
        out = _trace(desc, rays)
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), f"refill {refill} node_min {node_min}"
    gpu = render_gpu(desc, 1)
    assert np.isfinite(gpu["pt accum buffer"]).all()


def test_accumulation_equals_onrun_sequence():
    """spp=3 in one batch == three OnRun frames (pt_pass.cpp:51-56), incl. the lerp."""
    desc = _cornell(48).desc()
    batch = render_gpu(desc, 3)
    seq = None
    for f in range(3):
        seq = render_gpu(desc, 1, seed=f, cnt=f, prev=None if seq is None else seq["pt accum buffer"])
    assert np.array_equal(batch["pt accum buffer"], seq["pt accum buffer"])


def test_tile_sharding_matches_full_frame():
    desc = _cornell(80).desc()
    full = render_gpu(desc, 2)["pt accum buffer"]
    import ctypes as C

    lib = abi.load_library()
    got = np.zeros_like(full)
    seen = np.zeros(len(full), bool)
    for rank in range(3):
        part = render_gpu(desc, 2, tile=(16, rank, 3))["pt accum buffer"]
        n = C.c_uint32(0)
        lib.pupil_pt_local_pixels(80, 80, 16, rank, 3, None, C.byref(n))
        pix = np.zeros(n.value, np.uint32)
        lib.pupil_pt_local_pixels(80, 80, 16, rank, 3, pix.ctypes.data_as(abi.u32p), C.byref(n))
        got[pix] = part
        assert not seen[pix].any()
        seen[pix] = True
    assert seen.all()
    assert np.array_equal(got, full)


@pytest.mark.parametrize("case", ["cornell", "cornell_spp3_depth7", "materials", "materials_two_level", "field",
                                  "field_tiles", "field_stages", "quad_stack"])
def test_one_launch_frames_match_oracle(case, monkeypatch):
    """Renders that start no frame ahead and are small (PUPIL_FRAME_PATHS) run as ONE persistent
    launch per frame (pt_frame.hip): per-wave rounds of traversal (a bounce's shadow and
    extension rays together) and shading, no partitions.  Every pixel, AOV and ray count equals
    the oracle's: single-material and all-material shading, the two-level world structure, several
    samples per pixel, depth 7, one rank's compact tiles; "field_stages" (PUPIL_FRAME_PATHS=0) is
    the same render through the stage pipeline; "quad_stack" (6,000 stacked quads) takes
    k_frame's traversal stack past its LDS ring into the HBM overflow column and back."""
    import ctypes as C

    if case == "field_stages":
        monkeypatch.setenv("PUPIL_FRAME_PATHS", "0")
    if case == "materials_two_level":
        monkeypatch.setenv("PUPIL_ACCEL", "two_level")
    spp, tile = 1, (32, 0, 1)
    if case.startswith("cornell"):
        desc = _cornell(64, depth=7 if "depth7" in case else 4).desc()
        spp = 3 if "spp3" in case else 1
    elif case == "quad_stack":
        desc = _quad_stack(6000).desc()
        spp = 2
    elif case.startswith("materials"):
        desc = World().load_scene(scenes.cornell_materials_xml(os.path.join(TMP, "cbmat80.xml"), 80, 80, 6)).desc()
        spp = 2
    else:
        desc = scenes.sphere_field(27, 160, 96, 4, seed=5).desc()
        tile = (16, 1, 3) if case == "field_tiles" else tile
    gpu = render_gpu(desc, spp, tile=tile, stats=False)
    assert gpu["stats"]["frame_launches"] == (0 if case == "field_stages" else 1)
    pixels = None
    if tile[2] > 1:
        lib = abi.load_library()
        n = C.c_uint32(0)
        lib.pupil_pt_local_pixels(desc.width, desc.height, tile[0], tile[1], tile[2], None, C.byref(n))
        pixels = np.zeros(n.value, np.uint32)
        lib.pupil_pt_local_pixels(desc.width, desc.height, tile[0], tile[1], tile[2],
                                  pixels.ctypes.data_as(abi.u32p), C.byref(n))
    ref = oracle.OracleScene(desc).render(spp=spp, pixels=pixels)
    assert compare(gpu, ref, f"one-launch-{case}") == len(ref["accum"])
    assert np.array_equal(gpu["albedo"], ref["albedo"]) and np.array_equal(gpu["normal"], ref["normal"])
    assert np.array_equal(gpu["test"].reshape(-1), ref["test"])
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"])


def test_non_accumulating_frame_overwrites():
    desc = _cornell(32).desc()
    a = render_gpu(desc, 1, seed=5, accumulate=False)
    b = render_gpu(desc, 1, seed=5, accumulate=False, prev=np.full((32 * 32, 4), 7.0, np.float32))
    assert np.array_equal(a["pt accum buffer"], b["pt accum buffer"])


@pytest.mark.parametrize("accel", ["flat", "two_level"])
def test_instanced_rough_materials_parity(accel, monkeypatch):
    """Config 5 in miniature: instances of one BLAS under rigid transforms, rough dielectric +
    rough plastic, depth 6 (scenes.instanced_field); flattened or two-level acceleration."""
    monkeypatch.setenv("PUPIL_ACCEL", accel)
    w = scenes.instanced_field(num_instances=6, width=160, height=90, max_depth=6, seed=2, spheres_per_blas=12)
    desc = w.desc()
    gpu = render_gpu(desc, 4)
    ref = oracle.OracleScene(desc).render(spp=4)
    exact = compare(gpu, ref, f"instanced6x12-{accel}")
    assert gpu["stats"]["two_level"] == (accel == "two_level")
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"])
    assert exact == 160 * 90


@pytest.mark.parametrize("accel", ["flat", "two_level"])
def test_instance_update_equals_fresh_engine(accel, monkeypatch):
    """RenderInstanceUpdate: moving a sphere instance and the emissive light through
    World.set_instance_transform + PTPass.update_instance renders exactly what a
    freshly created engine (and the oracle) renders for the moved scene."""
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_ACCEL", accel)
    w = scenes.sphere_field(8, 96, 64, 4, seed=5, merge=False)
    desc0 = w.desc()
    n = desc0.num_instances
    pt = PTPass(device=0)
    pt.set_scene(desc0)
    pt.render(2)
    before = pt.buffers.get("pt accum buffer").cpu().numpy()
    w.set_instance_transform(3, world_mod.transform(scale=(1.7, 1.7, 1.7), rotate=((0, 1, 0), 30),
                                                    translate=(1.0, 5.0, -2.0)))
    pt.update_instance(w, 3)
    w.set_instance_transform(n - 1, world_mod.transform(scale=(2, 4, 1), rotate=((1, 0, 0), 90),
                                                        translate=(1.5, 13.5, -1.0)))
    pt.update_instance(w, n - 1)
    pt.render(2)
    import torch

    torch.cuda.synchronize()
    moved = pt.buffers.get("pt accum buffer").cpu().numpy()
    pt.close_engine()
    desc1 = w.desc()
    fresh = render_gpu(desc1, 2)["pt accum buffer"]
    assert not np.array_equal(before, moved)
    assert np.array_equal(moved, fresh)
    ref = oracle.OracleScene(desc1).render(spp=2)["accum"]
    assert np.array_equal(moved, ref)


def test_env_map_and_bitmap_textures_parity():
    """Env-map emitter (PFM, rotated, scaled) with its sampling CDF, bitmap textures
    with point and bilinear filtering and to_uv scale, checkerboard, open sky."""
    p = scenes.textured_env_xml(os.path.join(TMP, "texenv.xml"), 160, 120, 5)
    desc = World().load_scene(p).desc()
    gpu = render_gpu(desc, 4)
    ref = oracle.OracleScene(desc).render(spp=4)
    exact = compare(gpu, ref, "texenv160x4")
    assert exact == 160 * 120
    for k in ("albedo", "normal"):
        assert np.array_equal(gpu[k], ref[k])


@pytest.mark.parametrize("env_format,tex_format", [("exr", "png"), ("hdr", "jpg")])
def test_env_map_and_bitmap_file_formats_parity(env_format, tex_format):
    """The same scene with the env map as EXR / Radiance HDR and the bitmap as PNG /
    JPEG (util::BitmapTexture::Load, texture.cpp:87-174): the decoded textures are
    sampled on the GPU bit-identically to the oracle."""
    p = scenes.textured_env_xml(os.path.join(TMP, f"texenv_{env_format}", "texenv.xml"), 160, 120, 5,
                                env_format=env_format, tex_format=tex_format)
    desc = World().load_scene(p).desc()
    assert desc.env and desc.env.contents.radiance.type == abi.TEX_BITMAP
    gpu = render_gpu(desc, 4)
    ref = oracle.OracleScene(desc).render(spp=4)
    assert compare(gpu, ref, f"texenv-{env_format}-{tex_format}") == 160 * 120


def test_render_from_another_thread():
    """SURVEY §8(b) threading: PTPass::OnRun runs on a render thread other than the one that
    created the engine (system.cpp:93-106); every call sets its HIP device, so a render issued
    from a worker thread equals one issued from the creating thread."""
    import threading

    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    desc = _cornell(48).desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    pt.render(2)
    torch.cuda.synchronize()
    main = pt.buffers.get("pt accum buffer").cpu().numpy()
    out = {}

    def worker():
        pt.mark_dirty()
        pt.render(2)
        torch.cuda.synchronize()
        out["img"] = pt.buffers.get("pt accum buffer").cpu().numpy()

    t = threading.Thread(target=worker)
    t.start()
    t.join(timeout=60)
    pt.close_engine()
    assert "img" in out and np.array_equal(out["img"], main)


def test_camera_change_uploads_new_sensor():
    """CameraChange after World.set_sensor: the pass re-reads the sensor and renders
    exactly what a fresh engine on the moved camera renders (pt_pass.cpp:40-49)."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass, Events
    from pupiloptixlab_amd import world as W

    w = _cornell(64)
    pt = PTPass(device=0)
    pt.set_scene(w)
    pt.render(2)
    torch.cuda.synchronize()
    before = pt.buffers.get("pt accum buffer").cpu().numpy()
    w.set_sensor(40.0, W.look_at_mitsuba((0.3, 1.2, 3.5), (0.0, 0.9, 0.0), (0.0, 1.0, 0.0)), fov_axis="x")
    pt.events.dispatch(Events.CAMERA_CHANGE)
    pt.render(2)
    torch.cuda.synchronize()
    moved = pt.buffers.get("pt accum buffer").cpu().numpy()
    pt.close_engine()
    fresh = render_gpu(w.desc(), 2)["pt accum buffer"]
    assert not np.array_equal(before, moved)
    assert np.array_equal(moved.view(np.uint32), fresh.view(np.uint32))
    ref = oracle.OracleScene(w.desc()).render(spp=2)["accum"]
    assert np.array_equal(moved.view(np.uint32), ref.view(np.uint32))


PIPE_CASES = ["flat", "two_level", "two_level_world", "bins", "batched", "hint", "deep", "pipe3", "tiles", "group",
              "group_tiles", "group_bins", "group_hint", "group2", "group2_deep", "group_nosplit"]


@pytest.mark.parametrize("case", PIPE_CASES)
def test_pipelined_onrun_sequence(case, monkeypatch):
    """Pipelined frames (engine.hip render_pipelined): consecutive renders that continue
    each other keep up to max_depth frames in flight, and each render's launches advance
    all of them.  A sequence of OnRuns on one engine must equal the oracle after every
    render -- accumulation, "final result" and the AOVs (albedo / normal / test of the
    render's own frame, shaded renders earlier and kept in the slot scratch) -- including
    when the camera moves, an instance moves, the seed jumps or max_depth changes (the
    frames in flight are dropped), on multi-material scenes (material partition over the
    ring), two-level structures, batched renders (PUPIL_AHEAD=2 / the hint), a ring
    capped below max_depth (PUPIL_PIPE=3) and tile-sharded compact buffers.  The group
    cases batch 4 consecutive frames per ring slot (small renders: PUPIL_PIPE_GROUP_PATHS),
    so most renders only accumulate a frame an earlier render's launches completed; the
    render before the one that needs the next iteration runs its trace half, that render its
    shade half (r06 pacing; "group2": the default two frames per group, "group_nosplit":
    PUPIL_PIPE_SPLIT=0).  Camera moves, seed jumps and depth changes land between the halves."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass, Events
    from pupiloptixlab_amd import world as W

    grouped = case.startswith("group")
    if grouped:
        monkeypatch.setenv("PUPIL_PIPE_GROUP_MAX", "2" if case.startswith("group2") else "4")
        if case == "group_nosplit":
            monkeypatch.setenv("PUPIL_PIPE_SPLIT", "0")
        case = {"group": "flat", "group_tiles": "tiles", "group_bins": "bins", "group_hint": "hint", "group2": "flat",
                "group2_deep": "deep", "group_nosplit": "flat"}[case]
    if case == "two_level":
        monkeypatch.setenv("PUPIL_ACCEL", "two_level")
        monkeypatch.setenv("PUPIL_TL_MODE", "object")
    if case == "two_level_world":
        monkeypatch.setenv("PUPIL_ACCEL", "two_level")
    if case == "batched":
        monkeypatch.setenv("PUPIL_AHEAD", "2")
    if case == "pipe3":
        monkeypatch.setenv("PUPIL_PIPE", "3")
    if case == "bins":
        w = World().load_scene(scenes.cornell_materials_xml(os.path.join(TMP, "cbmat48.xml"), 48, 40, 5))
    elif case in ("two_level", "two_level_world"):
        w = scenes.instanced_field(num_instances=6, width=48, height=32, max_depth=5, seed=2, spheres_per_blas=8)
    elif case in ("flat", "tiles"):
        w = scenes.sphere_field(8, 48, 32, 4, seed=5, merge=False)
    elif case in ("deep", "pipe3"):
        w = World().load_scene(scenes.cornell_xml(os.path.join(TMP, "cb40d8.xml"), 40, 40, 8))
    else:
        w = _cornell(48)
    spp = 2 if case in ("batched", "hint") else 1  # hint: PUPIL_HINT_CONTINUE on batched renders
    # one frame per ring slot unless grouped (4 frames of this render size per slot)
    npaths = (2 * 16 * 16 if case == "tiles" else w.desc().width * w.desc().height) * spp  # tiles 1, 4 of 3 x 2
    monkeypatch.setenv("PUPIL_PIPE_GROUP_PATHS", str(4 * npaths - 1 if grouped else 1))
    if grouped and spp > 1:
        monkeypatch.setenv("PUPIL_PIPE_GROUP_ALL", "1")
    pt = PTPass(device=0)
    pt.set_scene(w)
    if case == "tiles":
        pt.set_tiling(16, 1, 3)
    depth = w.desc().max_depth
    slots = min(depth, 3) if case == "pipe3" else depth
    keys = ("pt accum buffer", "final result", "albedo", "normal", "test")

    def step(k_frames, o, seed0=0, max_depth=0):
        pt.render(spp, continues=case == "hint")
        torch.cuda.synchronize()
        got = {k: pt.buffers.get(k).cpu().numpy() for k in keys}
        px = pt.local_pixels() if case == "tiles" else None
        ref = o.render(spp=k_frames * spp, random_seed=seed0, max_depth=max_depth, pixels=px)
        for k, rk in zip(keys, ("accum", "accum", "albedo", "normal", "test")):
            assert np.array_equal(got[k].reshape(ref[rk].shape).view(np.uint32), ref[rk].view(np.uint32)), \
                (case, k, k_frames, seed0)

    o = oracle.OracleScene(w.desc())
    for k in range(1, 2 * slots + 2):  # long enough to reach one launch per render
        step(k, o)
    st = pt.stats()
    if grouped:
        assert st["pipeline_slots"] == slots and st["frames_in_flight"] >= 1, (case, st)
    else:
        assert st["pipeline_slots"] == slots and st["frames_in_flight"] == slots - 1, (case, st["pipeline_slots"],
                                                                                      st["frames_in_flight"])
    if case in ("flat", "batched", "hint", "tiles"):  # the camera moves: accumulation restarts on the new view
        w.set_sensor(40.0, W.look_at_mitsuba((0.3, 1.2, 3.5), (0.0, 0.9, 0.0), (0.0, 1.0, 0.0)), fov_axis="x")
        pt.events.dispatch(Events.CAMERA_CHANGE)
        o = oracle.OracleScene(w.desc())
        for k in range(1, slots + 2):
            step(k, o)
    if case in ("flat", "two_level", "two_level_world"):  # an instance moves: frames in flight hit the old geometry
        w.set_instance_transform(1, W.transform(scale=(1.5, 1.5, 1.5), rotate=((0, 1, 0), 30), translate=(0.5, 1.0, -0.5)))
        pt.update_instance(w, 1)
        o = oracle.OracleScene(w.desc())
        for k in range(1, slots + 2):
            step(k, o)
    # the seed jumps: the frames started for the next seeds are not used
    pt.random_seed, pt.sample_cnt = 9, 0
    step(1, o, seed0=9)
    step(2, o, seed0=9)
    # max_depth changes (the inspector): frames in flight were shaded for the old depth
    pt.max_depth = 2
    pt.random_seed, pt.sample_cnt = 0, 0
    for k in range(1, 4):
        step(k, o, max_depth=2)
    # max_depth 1: a frame is one launch, nothing to pipeline; the next render still matches
    pt.max_depth = 1
    pt.random_seed, pt.sample_cnt = 0, 0
    step(1, o, max_depth=1)
    step(2, o, max_depth=1)
    pt.close_engine()


def test_pipelined_ray_accounting():
    """rays_traced_total (device running totals of the flags partitions + the host's camera
    rays) equals the sum of the per-render ray counts over a pipelined OnRun sequence, and,
    with pipelining off (PUPIL_PIPE=1), the oracle's ray counts frame by frame."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    w = _cornell(48, depth=5)
    o = oracle.OracleScene(w.desc())
    totals = {}
    for pipe in ("0", "1"):
        os.environ["PUPIL_PIPE"] = pipe
        os.environ["PUPIL_PIPE_GROUP_PATHS"] = "1"  # one frame per slot (test_pipelined_onrun_sequence covers groups)
        try:
            pt = PTPass(device=0)
            pt.set_scene(w)
        finally:
            del os.environ["PUPIL_PIPE"]
            del os.environ["PUPIL_PIPE_GROUP_PATHS"]
        t0 = pt.stats()["rays_traced_total"]
        per = 0
        for _ in range(12):
            pt.render(1)
            torch.cuda.synchronize()
            c = pt.stats()
            per += c["primary_rays"] + c["extension_rays"] + c["shadow_rays"]
        t1 = pt.stats()["rays_traced_total"]
        assert t1 - t0 == per, (pipe, t1 - t0, per)
        totals[pipe] = (per, pt.stats()["frames_in_flight"])
        pt.close_engine()
    rs = o.render(spp=12)["stats"]
    assert totals["1"] == (rs["primary_rays"] + rs["extension_rays"] + rs["shadow_rays"], 0)
    # pipelined: the 12 completed frames plus part of the 4 frames in flight
    assert totals["0"][1] == 4 and totals["0"][0] > totals["1"][0]


def test_max_depth_above_128_renders():
    """The reference takes integrator.max_depth unclamped at SetScene (pt_pass.cpp:112-115;
    only the inspector clamps to 1..128): a scene with max_depth 150 renders exactly like
    the oracle (per-bounce flags tags alias above 63 bounces, so the flags are cleared per
    bounce, and the ray log grows with the depth)."""
    w = World().load_scene(scenes.cornell_xml(os.path.join(TMP, "cb24d150.xml"), 24, 24, 150))
    desc = w.desc()
    assert desc.max_depth == 150
    gpu = render_gpu(desc, 2)
    ref = oracle.OracleScene(desc).render(spp=2)
    assert np.array_equal(gpu["pt accum buffer"].view(np.uint32), ref["accum"].view(np.uint32))
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"])


def test_huge_max_depth_renders_and_stops_early():
    """max_depth = 2^32 - 1 (the ABI takes any depth): the host neither wraps
    its iteration arithmetic nor creates events per bounce, and it stops issuing bounces
    once every path has terminated (the list lengths are read back every 16 iterations
    above depth 64).  The image equals the oracle's render at the same depth."""
    import time

    w = World().load_scene(scenes.cornell_xml(os.path.join(TMP, "cb24dmax.xml"), 24, 24, 4))
    desc = w.desc()
    desc.max_depth = 0xFFFFFFFF
    t0 = time.perf_counter()
    gpu = render_gpu(desc, 2)
    assert time.perf_counter() - t0 < 60
    ref = oracle.OracleScene(desc).render(spp=2)
    assert np.array_equal(gpu["pt accum buffer"].view(np.uint32), ref["accum"].view(np.uint32))
    s, rs = gpu["stats"], ref["stats"]
    assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"]) == \
        (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"])


def test_coalesced_instance_updates_cost_one_refit():
    """RenderInstanceUpdate events only record the moved instances (pt_pass.cpp:216-218);
    the next render refits once for all of them: 5 events on 3 instances -> one refit,
    and the render equals a fresh engine's and the oracle's for the moved scene."""
    import torch
    from pupiloptixlab_amd.pt_pass import Events, PTPass

    w = scenes.sphere_field(8, 64, 48, 4, seed=5, merge=False)
    n = w.desc().num_instances
    pt = PTPass(device=0)
    pt.set_scene(w)
    pt.render(1)
    r0 = pt.stats()["accel_refits"]
    moves = [(2, (0.5, 1.0, 0.0)), (3, (1.0, 5.0, -2.0)), (2, (0.7, 1.2, 0.1)), (n - 1, (1.5, 13.5, -1.0)),
             (3, (1.1, 5.1, -2.2))]
    for inst, t in moves:
        w.set_instance_transform(inst, world_mod.transform(rotate=((0, 1, 0), 15), translate=t))
        pt.events.dispatch(Events.RENDER_INSTANCE_UPDATE, (w, inst))
    assert pt.stats()["accel_refits"] == r0  # nothing done until the next render
    pt.render(2)
    torch.cuda.synchronize()
    assert pt.stats()["accel_refits"] == r0 + 1
    moved = pt.buffers.get("pt accum buffer").cpu().numpy()
    pt.close_engine()
    desc1 = w.desc()
    assert np.array_equal(moved, render_gpu(desc1, 2)["pt accum buffer"])
    ref = oracle.OracleScene(desc1).render(spp=2)["accum"]
    assert np.array_equal(moved.view(np.uint32), ref.view(np.uint32))


def test_tlas_reserve_contents_do_not_move_the_node_bound(monkeypatch):
    """The slab-test bound is taken over live BVH4 nodes only: junk (huge, inf, NaN) in the
    never-written TLAS reserve of the two-level node array leaves it unchanged (ADVICE r03:
    leftover allocator contents used to loosen every ray's box test)."""
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_ACCEL", "two_level")
    w = scenes.instanced_field(num_instances=6, width=32, height=18, max_depth=4, seed=3, spheres_per_blas=10)
    pt = PTPass(device=0)
    pt.set_scene(w.desc())
    b0 = pt.stats()["node_bound"]
    assert all(np.isfinite(b0)) and max(b0) > 0
    for junk in (1e30, float("inf"), float("nan")):
        abi.check(pt._lib.pupil_debug_fill_tlas_reserve(pt._pt, junk))
        assert pt.stats()["node_bound"] == b0, junk
    pt.close_engine()


@pytest.mark.parametrize("fallback", [1, 2])
def test_world_to_object_fallback_keeps_the_blas_nodes(monkeypatch, fallback):
    """A world-mode two-level build that falls back to object mode (1: world record slots
    beyond the 28-bit leaf links, 2: world BLAS copies beyond the node limit; forced here by
    PUPIL_DEBUG_TL_FALLBACK) keeps only the per-instance TLAS slots before the BLASes (ADVICE
    r05: the braided reserve used to stay, so the node bound skipped BLAS nodes and the
    reserve fill overwrote them).  Junk written into the reserve changes nothing, and the
    render equals the oracle's."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_ACCEL", "two_level")
    monkeypatch.setenv("PUPIL_TL_MODE", "world")
    monkeypatch.setenv("PUPIL_DEBUG_TL_FALLBACK", str(fallback))
    w = scenes.instanced_field(num_instances=6, width=32, height=18, max_depth=4, seed=3, spheres_per_blas=10)
    desc = w.desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    b0 = pt.stats()["node_bound"]
    abi.check(pt._lib.pupil_debug_fill_tlas_reserve(pt._pt, 1e30))
    assert pt.stats()["node_bound"] == b0
    pt.render(2)
    torch.cuda.synchronize()
    img = pt.buffers.get("pt accum buffer").cpu().numpy()
    pt.close_engine()
    ref = oracle.OracleScene(desc).render(spp=2)["accum"]
    assert np.array_equal(img.view(np.uint32), ref.reshape(img.shape).view(np.uint32))


def test_moving_camera_cadence_starts_no_frames_ahead():
    """The OnRun cadence with a camera change before every OnRun (interactive use): no
    render continues the previous one, so none starts frames ahead (they would be
    discarded) and every traced ray belongs to a displayed frame; once the camera stops,
    continued OnRuns pipeline again.  Every frame equals the oracle's."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    w = _cornell(48, depth=5)
    desc = w.desc()
    c2w0 = np.array(list(desc.camera_to_world), np.float32)
    pt = PTPass(device=0)
    pt.set_scene(desc)
    lib = pt._lib
    for k in range(4):
        c2w = c2w0.copy()
        c2w[3] += 0.01 * k
        abi.check(lib.pupil_pt_set_camera(pt._pt, desc.sample_to_camera, c2w.ctypes.data_as(abi.f32p)))
        pt.dirty = False
        pt.random_seed = pt.sample_cnt = 0
        t0 = pt.stats()["rays_traced_total"]
        pt.render(1)
        torch.cuda.synchronize()
        c = pt.stats()
        assert c["frames_in_flight"] == 0, k
        assert c["rays_traced_total"] - t0 == c["primary_rays"] + c["extension_rays"] + c["shadow_rays"]
        one_frame_ring = c["ring_bytes"]
        if k == 0:
            ring0 = one_frame_ring
        assert one_frame_ring == ring0, k  # no render speculated: the ring holds one frame
        d = World().load_scene(scenes.cornell_xml(os.path.join(TMP, "cb48d5.xml"), 48, 48, 5)).desc()
        d.camera_to_world[:] = [float(x) for x in c2w]
        ref = oracle.OracleScene(d).render(spp=1)["accum"]
        got = pt.buffers.get("pt accum buffer").cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
    # ... and that footprint (path state, queues, AOV scratch) is exactly the one of an engine
    # that never pipelines (PUPIL_AHEAD=0, read at create)
    os.environ["PUPIL_AHEAD"] = "0"
    try:
        pt0 = PTPass(device=0)
        pt0.set_scene(desc)
        pt0.render(1)
        torch.cuda.synchronize()
        assert pt0.stats()["ring_bytes"] == ring0
        pt0.close_engine()
    finally:
        del os.environ["PUPIL_AHEAD"]
    for _ in range(3):  # the camera stops: the OnRuns continue each other and pipeline
        pt.render(1)
    torch.cuda.synchronize()
    c = pt.stats()
    assert c["frames_in_flight"] > 0
    assert c["ring_bytes"] > ring0  # the first speculating render allocated the ring
    pt.close_engine()


def test_render_orders_with_torch_default_stream():
    """A render enqueued on torch's default stream (handle NULL) runs on that stream: a
    read on the same stream right after it, with no device synchronisation, sees the
    finished frame (r02: NULL used to select the engine's own non-blocking stream, and
    the multi-rank gather could copy a frame still being rendered)."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    w = _cornell(96)
    pt = PTPass(device=0)
    pt.set_scene(w)
    assert torch.cuda.current_stream().cuda_stream == 0
    frames = []
    for _ in range(3):
        pt.render(4, continues=True)
        frames.append(pt.buffers.get("pt accum buffer").cpu().numpy())  # ordered on the same stream
    pt.close_engine()
    o = oracle.OracleScene(w.desc())
    for k, got in enumerate(frames):
        ref = o.render(spp=4 * (k + 1))["accum"]
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), f"frame {k}"


@pytest.mark.parametrize("accel", ["flat", "two_level"])
def test_skewed_scene_stays_within_stack_capacity(accel, monkeypatch):
    """A geometric chain of triangles (size and spacing x1.15 per triangle) makes the
    nearest-neighbour PLOC build a caterpillar far deeper than the traversal stacks
    hold; create() detects the depth and rebuilds with the Morton-bounded Karras
    LBVH, so every traversal variant still returns the oracle's hits."""
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_ACCEL", accel)
    n = 300
    a = 1.15 ** np.arange(n)
    pos = np.zeros((n, 3, 3), np.float32)
    pos[:, 0] = np.stack([a, np.zeros(n), np.zeros(n)], 1)
    pos[:, 1] = np.stack([a + 0.5 * a, np.zeros(n), np.zeros(n)], 1)
    pos[:, 2] = np.stack([a, 0.5 * a, 0.25 * a], 1)
    w = World()
    s = w.add_mesh(pos.reshape(-1, 3), np.arange(3 * n, dtype=np.uint32).reshape(-1, 3))
    w.add_instance(s, w.add_material(world_mod.diffuse((0.5, 0.5, 0.5))))
    w.set_film(16, 16, 2)
    w.set_sensor(40.0, world_mod.look_at_mitsuba((0, 0, -3), (0, 0, 0), (0, 1, 0)))
    desc = w.desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    depth = pt.stats()["bvh_depth"]
    pt.close_engine()
    assert 0 < depth and 3 * depth + 2 <= 176, depth  # kRing + kStackOvf entries, 3 per level
    rng = np.random.default_rng(9)
    m = 20000
    tgt = pos[rng.integers(0, n, m)].mean(axis=1) + rng.normal(0, 0.05, (m, 3)) * a[rng.integers(0, n, m)][:, None]
    org = rng.uniform(-2, 2, (m, 3)) + np.array([0, 0, -5.0])
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([org, d], 1).astype(np.float32)
    ref = oracle.OracleScene(desc).closest(rays)
    assert (ref[:, 0] > 0).sum() > 1000
    for refill, node_min in TRAVERSALS if accel == "flat" else [("24", "8")]:
        _set_traversal(monkeypatch, refill, node_min)
        out = _trace(desc, rays)
        bad = (out.view(np.uint32) != ref.view(np.uint32)).any(axis=1)
        assert not bad.any(), f"{accel} refill {refill} node_min {node_min}: {bad.sum()} rays differ"


def _emissive_field(spheres=24, w=96, h=64, groups=2):
    return scenes.sphere_field(spheres, w, h, 4, seed=5, slices=12, stacks=8, emissive_groups=groups)


@pytest.mark.parametrize("mode", ["guide", "binary"])
def test_emitter_pick_equals_the_reference_linear_scan(mode, monkeypatch):
    """SelectOneEmiiter (render/emitter.h:110-135) is a linear scan over the sequentially
    accumulated select_probability; the device's guide table (and the binary search it
    narrows) must return exactly that index for every p, including p equal to a CDF
    entry, its float neighbours and the guide's bucket boundaries."""
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_EMITTER_SELECT", mode)
    desc = _emissive_field().desc()
    n = desc.num_area_emitters
    assert n > 500
    prob = np.array([desc.area_emitters[i].select_probability for i in range(n)], np.float32)
    cdf = np.zeros(n, np.float32)
    s = np.float32(0.0)
    for i in range(n):  # fl(sum_p + p_i), in order
        cdf[i] = s + prob[i]
        s = cdf[i]
    rng = np.random.default_rng(3)
    m = 1 << int(np.ceil(np.log2(n)))
    p = np.concatenate([(rng.integers(0, 1 << 24, 200000) / float(1 << 24)).astype(np.float32), cdf,
                        np.nextafter(cdf, np.float32(0)), np.nextafter(cdf, np.float32(2)),
                        (np.arange(m + 1) / m).astype(np.float32),
                        np.nextafter((np.arange(1, m + 1) / m).astype(np.float32), np.float32(0)),
                        np.float32([0.0, (2 ** 24 - 1) / 2 ** 24])])
    p = p[(p >= 0) & (p < 1)].astype(np.float32)
    ref = np.searchsorted(cdf, p, side="left").astype(np.int64)  # first i with p <= cdf[i]
    ref = np.where(ref >= n, n - 1, ref)  # no env: the last area emitter (emitter_cb)
    pt = PTPass(device=0)
    pt.set_scene(desc)
    out = np.zeros(len(p), np.int32)
    abi.check(pt._lib.pupil_debug_select_emitter(pt._pt, len(p), np.ascontiguousarray(p).ctypes.data_as(abi.f32p),
                                                 out.ctypes.data_as(abi.C.POINTER(abi.C.c_int32))))
    pt.close_engine()
    assert np.array_equal(out, ref), f"{(out != ref).sum()} picks differ"


def test_emissive_mesh_render_parity():
    """An emissive-mesh scene (two sphere groups emit, one emitter per triangle): NEE
    selection, area sampling and MIS render bit-identically to the oracle."""
    desc = _emissive_field().desc()
    gpu = render_gpu(desc, 2)
    ref = oracle.OracleScene(desc).render(spp=2)
    assert compare(gpu, ref, "emissive-mesh") == desc.width * desc.height


@pytest.mark.parametrize("accel,update", [("flat", "refit"), ("flat", "rebuild"), ("two_level", "refit"),
                                          ("two_level", "rebuild")])
def test_builtin_sphere_update_refit_equals_fresh_engine(accel, update, monkeypatch):
    """RenderInstanceUpdate on a built-in sphere and a mesh, with the refit (default:
    records rewritten, boxes refitted bottom up, topology kept -- the reference refits
    its IAS, ias_manager.cpp:116-151) and with a full rebuild: both render exactly what
    a fresh engine renders for the moved scene."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    monkeypatch.setenv("PUPIL_ACCEL", accel)
    monkeypatch.setenv("PUPIL_FLAT_UPDATE" if accel == "flat" else "PUPIL_TL_UPDATE", update)
    w = scenes.sphere_field(6, 80, 60, 4, seed=7, merge=False)
    sph = w.add_builtin("sphere")
    s_inst = w.add_instance(sph, w.add_material(world_mod.rough_plastic(alpha=0.3)),
                            world_mod.transform(scale=(0.8, 0.8, 0.8), translate=(-1.0, 2.0, 0.5)))
    desc0 = w.desc()
    pt = PTPass(device=0)
    pt.set_scene(desc0)
    pt.render(1)
    w.set_instance_transform(s_inst, world_mod.transform(scale=(1.3, 0.6, 1.0), translate=(2.0, 3.0, -1.5)))
    pt.update_instance(w, s_inst)
    w.set_instance_transform(2, world_mod.transform(scale=(1.2, 1.2, 1.2), translate=(-2.0, 6.0, 1.0)))
    pt.update_instance(w, 2)
    pt.render(2)
    torch.cuda.synchronize()
    moved = pt.buffers.get("pt accum buffer").cpu().numpy()
    pt.close_engine()
    fresh = render_gpu(w.desc(), 2)["pt accum buffer"]
    assert np.array_equal(moved.view(np.uint32), fresh.view(np.uint32))


def test_cpu_oracle_on_the_engine_bvh4_arrays():
    """SURVEY §8(d) CPU baseline: the oracle traverses the GPU's own BVH4 arrays
    (pupil_pt_export_bvh4) and renders the same frame bit for bit; closest hits of
    random rays agree with the oracle's own BVH."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    desc = scenes.sphere_field(27, 160, 90, 4, seed=4).desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    pt.dirty = False
    pt.render(2)
    torch.cuda.synchronize()
    gpu = pt.buffers.get("pt accum buffer").cpu().numpy()
    nodes, recs, root = pt.export_bvh4()
    pt.close_engine()
    # record slots: every primitive exactly once, holes between leaves (pt_scene.h kRecF4)
    ids = np.ascontiguousarray(recs).view(np.uint32).reshape(len(recs), -1)[:, 3]
    live = ids != 0xFFFFFFFF
    n_prims = oracle.OracleScene(desc).num_prims
    assert len(nodes) > 1 and root == 0 and len(recs) >= n_prims
    assert np.array_equal(np.sort(ids[live] & 0x7FFFFFFF), np.arange(n_prims, dtype=np.uint32))
    own = oracle.OracleScene(desc)
    q4 = oracle.OracleScene(desc)
    q4.use_bvh4(nodes, recs, root)
    ref = q4.render(spp=2)
    assert np.array_equal(gpu.view(np.uint32), ref["accum"].view(np.uint32))
    rng = np.random.default_rng(5)
    org = rng.uniform([-7.5, 0.1, -9.5], [7.5, 13.9, 13.5], (20000, 3))
    d = rng.normal(size=(20000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([org, d], 1).astype(np.float32)
    assert np.array_equal(q4.closest(rays).view(np.uint32), own.closest(rays).view(np.uint32))


@pytest.mark.parametrize("leaf_size", [1, 2, 3])
def test_record_slots_put_every_leaf_on_one_line(leaf_size):
    """Record slots (pt_scene.h kRecF4): every leaf link names an even slot (a 128-B line),
    a leaf of c primitives owns 2 ceil(c/2) slots, no slot belongs to two leaves, every
    primitive sits in exactly one leaf slot and no leaf names a hole; the frame stays equal
    to the oracle's at each leaf size.  Runs in a subprocess (PUPIL_LEAF_SIZE is read once)."""
    import subprocess
    import sys
    code = f"""
import numpy as np, torch, oracle
from pupiloptixlab_amd import scenes
from pupiloptixlab_amd.pt_pass import PTPass
desc = scenes.sphere_field(9, 64, 48, 3, seed=7).desc()
pt = PTPass(device=0); pt.set_scene(desc); pt.dirty = False
pt.render(1); torch.cuda.synchronize()
gpu = pt.buffers.get("pt accum buffer").cpu().numpy()
nodes, recs, root = pt.export_bvh4(); pt.close_engine()
links = np.ascontiguousarray(nodes).view(np.int32).reshape(len(nodes), 16)[:, 4:8].ravel()
leaves = [int(l) for l in links if l < 0] + ([root] if root < 0 else [])
ids = np.ascontiguousarray(recs).view(np.uint32).reshape(len(recs), 12)[:, 3]
owner = np.full(len(recs), -1)
for l in leaves:
    v = (~l) & 0xFFFFFFFF
    first, count = v >> 3, (v & 7) + 1
    assert first % 2 == 0 and count <= {leaf_size}
    span = (count + 1) & ~1
    assert (owner[first:first + span] < 0).all()
    owner[first:first + span] = l
    assert (ids[first:first + count] != 0xFFFFFFFF).all()
    assert (ids[first + count:first + span] == 0xFFFFFFFF).all()
n = oracle.OracleScene(desc).num_prims
assert np.array_equal(np.sort(ids[ids != 0xFFFFFFFF] & 0x7FFFFFFF), np.arange(n, dtype=np.uint32))
ref = oracle.OracleScene(desc).render(spp=1)
assert np.array_equal(gpu.view(np.uint32), ref["accum"].view(np.uint32))
print("ok", len(recs), n)
"""
    env = dict(os.environ, PUPIL_LEAF_SIZE=str(leaf_size), PUPIL_ACCEL="flat")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_consecutive_launches_on_one_engine():
    """The persistent kernels reset their own dequeue heads and exit counters (the
    last wave out, pt_kernels.hip trace4_body): eight renders on ONE engine with
    changing seeds, depths and tilings, then ray queries of awkward sizes, each equal
    to the oracle -- a dropped or repeated work item would change a pixel or a count."""
    import torch
    from pupiloptixlab_amd.pt_pass import PTPass

    desc = scenes.sphere_field(27, 96, 64, 4, seed=6).desc()
    o = oracle.OracleScene(desc)
    pt = PTPass(device=0)
    pt.set_scene(desc)
    n = 96 * 64
    for k, (depth, spp, tile) in enumerate([(4, 2, None), (1, 1, None), (2, 3, (16, 1, 3)), (6, 1, None),
                                            (3, 2, (8, 0, 2)), (4, 1, (8, 1, 2)), (5, 2, None), (4, 1, None)]):
        pt.set_tiling(*(tile or (32, 0, 1)))
        pt.max_depth = depth
        pt.dirty = False
        pt.random_seed, pt.sample_cnt = 10 + k, 0
        pt.render(spp, collect_stats=True)
        torch.cuda.synchronize()
        got = pt.buffers.get("pt accum buffer").cpu().numpy()
        pix = pt.local_pixels() if tile else np.arange(n, dtype=np.uint32)
        ref = o.render(spp=spp, random_seed=10 + k, max_depth=depth, pixels=pix)
        assert np.array_equal(got.view(np.uint32), ref["accum"].view(np.uint32)), f"render {k}"
        s, rs = pt.stats(), ref["stats"]
        assert (s["primary_rays"], s["extension_rays"], s["shadow_rays"]) == \
            (rs["primary_rays"], rs["extension_rays"], rs["shadow_rays"]), f"render {k}"
    rng = np.random.default_rng(3)
    for m in (1, 63, 64, 65, 4097, 300001):
        org = rng.uniform([-7.5, 0.1, -9.5], [7.5, 13.9, 13.5], (m, 3))
        d = rng.normal(size=(m, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays = np.concatenate([org, d], 1).astype(np.float32)
        r8 = np.ascontiguousarray(np.concatenate([rays, np.full((m, 1), 0.001, np.float32),
                                                  np.full((m, 1), 1e16, np.float32)], 1), np.float32)
        out = np.zeros((m, 4), np.float32)
        abi.check(pt._lib.pupil_pt_trace_rays(pt._pt, m, r8.ctypes.data_as(abi.f32p), out.ctypes.data_as(abi.f32p), 0))
        assert np.array_equal(out.view(np.uint32), o.closest(rays).view(np.uint32)), f"{m} rays"
    pt.close_engine()


@pytest.mark.parametrize("mode", ["bins", "list"])
def test_shade_list_modes_parity(mode, monkeypatch):
    """Shading over the material-bin partition, or over the traced list with per-path
    bins (the default for single-material scenes), forced on a scene with all seven BSDFs."""
    monkeypatch.setenv("PUPIL_SHADE_LIST", mode)
    monkeypatch.setenv("PUPIL_FRAME_PATHS", "0")  # shade modes of the stage pipeline
    p = scenes.cornell_materials_xml(os.path.join(TMP, "cbmat96.xml"), 96, 96, 6)
    desc = World().load_scene(p).desc()
    gpu = render_gpu(desc, 4)
    ref = oracle.OracleScene(desc).render(spp=4)
    assert compare(gpu, ref, f"shade-{mode}") == 96 * 96
    assert np.array_equal(gpu["albedo"], ref["albedo"]) and np.array_equal(gpu["normal"], ref["normal"])
    s, rs = gpu["stats"], ref["stats"]
    assert (s["extension_rays"], s["shadow_rays"], s["shadow_rays_reference"]) == \
        (rs["extension_rays"], rs["shadow_rays"], rs["shadow_rays_reference"])


@pytest.mark.parametrize("family", ["bvh4", "bvh4_refill1", "two_level_world", "two_level_object"])
def test_persistent_queue_accounting(family, monkeypatch):
    """Every persistent traversal family hands out each listed ray exactly once: per
    launch, the items the XCD dequeue heads handed out = the lanes activated with them =
    the lanes retired = the list length, summed over a counter render (primary extend +
    mixed launches) and over closest-hit and any-hit ray queries.  (A round-2 experiment
    with a spilled 6-wave BVH8 kernel, since removed, once left whole 64-ray batches
    untraced; this is the check that would catch it in any family.)"""
    from pupiloptixlab_amd.pt_pass import PTPass

    if family == "bvh4_refill1":
        monkeypatch.setenv("PUPIL_REFILL", "1")
    if family.startswith("two_level"):
        monkeypatch.setenv("PUPIL_ACCEL", "two_level")
        monkeypatch.setenv("PUPIL_TL_MODE", "object" if family == "two_level_object" else "world")
    w = scenes.sphere_field(27, 64, 36, 4, seed=9)
    desc = w.desc()
    pt = PTPass(device=0)
    pt.set_scene(desc)
    pt.render(4, collect_stats=1)
    c = pt.stats()
    rays = c["primary_rays"] + c["extension_rays"] + c["shadow_rays"]
    assert (c["queue_handed"], c["queue_activated"], c["queue_retired"], c["queue_listed"]) == (rays,) * 4, c
    rng = np.random.default_rng(11)
    n = 200000
    org = rng.uniform([-7.5, 0.1, -9.5], [7.5, 13.9, 13.5], (n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r8 = np.ascontiguousarray(np.concatenate([org, d, np.full((n, 1), 0.001), np.full((n, 1), 1e16)], 1), np.float32)
    ref = oracle.OracleScene(desc).closest(r8[:, :6])
    monkeypatch.setenv("PUPIL_TRACE_RAYS_STATS", "1")
    for any_hit in (0, 1):
        out = np.full((n, 4), -7.0, np.float32)  # a t no record carries (-1 = miss, >0 = hit)
        abi.check(pt._lib.pupil_pt_trace_rays(pt._pt, n, r8.ctypes.data_as(abi.f32p), out.ctypes.data_as(abi.f32p),
                                              any_hit))
        c = pt.stats()
        assert (c["queue_handed"], c["queue_activated"], c["queue_retired"], c["queue_listed"]) == (n,) * 4, \
            (any_hit, c["queue_handed"], c["queue_activated"], c["queue_retired"], c["queue_listed"])
        assert (out[:, 0] != -7.0).all()  # every ray's record written
        assert np.array_equal(out[:, 0] > 0, ref[:, 0] > 0)
    pt.close_engine()
