"""The oracle's closest hit against an independent float64 ray-triangle restatement.

The reference's closest hit is OptiX's built-in triangle test over its GAS / IAS
(main.cu:77-82,158-163: optixTrace with tmin 0.001, then optixGetTriangleBarycentrics in
__closesthit__default, main.cu:216-230); no hit values ship with it.  Here
the oracle's watertight float32 test (on its own BVH) must report, for random rays into a
soup of random triangles, the same hit / miss, the same primitive and -- within float32
rounding -- the same distance and barycentrics (the weights of vertices 1 and 2, OptiX's
convention) as a float64 Moller-Trumbore over every triangle.  Rays whose answer is
numerically ambiguous (a barycentric or the t-gap between the two nearest hits within
1e-5 of the decision) are skipped.  Test infrastructure only; CPU.
"""
import numpy as np

import oracle
from pupiloptixlab_amd import World
from pupiloptixlab_amd import world as W


def mt_all(o, d, v0, v1, v2, tmin=0.001):
    """float64 Moller-Trumbore of one ray against every triangle: t (inf = miss), u, v."""
    e1, e2 = v1 - v0, v2 - v0
    p = np.cross(d, e2)
    det = np.einsum("ij,ij->i", e1, p)
    ok = np.abs(det) > 1e-14
    inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
    s = o - v0
    u = np.einsum("ij,ij->i", s, p) * inv
    q = np.cross(s, e1)
    v = (q @ d) * inv
    t = np.einsum("ij,ij->i", e2, q) * inv
    hit = ok & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > tmin)
    return np.where(hit, t, np.inf), u, v


def test_oracle_closest_hit_matches_float64_restatement():
    rng = np.random.default_rng(7)
    n_tri = 400
    centers = rng.uniform(-4, 4, (n_tri, 1, 3))
    tris = centers + rng.normal(scale=0.6, size=(n_tri, 3, 3))
    wd = World()
    wd.set_film(8, 8, 4)
    mesh = wd.add_mesh(tris.reshape(-1, 3).astype(np.float32), np.arange(3 * n_tri, dtype=np.uint32).reshape(-1, 3))
    wd.add_instance(mesh, wd.add_material(W.diffuse(0.5)))
    wd.set_sensor(40.0, W.look_at_mitsuba((0, 0, 12), (0, 0, 0), (0, 1, 0)))
    orc = oracle.OracleScene(wd.desc())
    v = tris.astype(np.float32).astype(np.float64)
    v0, v1, v2 = v[:, 0], v[:, 1], v[:, 2]

    n = 3000
    org = rng.uniform(-6, 6, (n, 3))
    tgt = rng.uniform(-4, 4, (n, 3))
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([org, d], 1).astype(np.float32)
    got = orc.closest(rays)
    o64, d64 = rays[:, :3].astype(np.float64), rays[:, 3:].astype(np.float64)

    checked = hits = 0
    for i in range(n):
        t, u, w = mt_all(o64[i], d64[i], v0, v1, v2)
        order = np.argsort(t)
        k = order[0]
        t_best = t[k]
        # ambiguous: the nearest two hits too close, or an edge decision within 1e-5
        if np.isfinite(t[order[1]]) and t[order[1]] - t_best < 1e-5 * max(1.0, t_best):
            continue
        e1, e2 = v1 - v0, v2 - v0
        p = np.cross(d64[i], e2)
        det = np.einsum("ij,ij->i", e1, p)
        s = o64[i] - v0
        uu = np.einsum("ij,ij->i", s, p) / det
        vv = (np.cross(s, e1) @ d64[i]) / det
        margin = np.minimum(np.minimum(np.abs(uu), np.abs(vv)), np.abs(1 - uu - vv))
        if (margin < 1e-5).any():
            continue
        checked += 1
        if not np.isfinite(t_best):
            assert got[i, 0] < 0, (i, got[i])
            continue
        hits += 1
        assert got[i, 0] > 0, (i, t_best)
        assert int(got[i, 3].view(np.uint32)) == k, (i, int(got[i, 3].view(np.uint32)), k)
        assert np.isclose(got[i, 0], t_best, rtol=3e-5, atol=1e-6), (i, got[i, 0], t_best)
        assert np.isclose(got[i, 1], u[k], atol=1e-4) and np.isclose(got[i, 2], w[k], atol=1e-4), (i, got[i], u[k], w[k])
    assert checked > 2500 and hits > 1000, (checked, hits)
