"""Area-emitter sampling of the oracle pinned by geometry (render/emitter/area.h:17-34,
sphere.h:14-31, optix/util.h UniformSampleTriangle / UniformSampleSphere).

The reference ships no sampled values.  Two independent checks, in float64:
  * per sample, the direction, distance and pdf the oracle returns equal a restatement of
    SampleDirect (the sampled point from the published warps, pdf = d^2 / (cos_l * area));
  * over a stratified grid of (xi0, xi1), the estimator mean(1 / pdf) over the valid samples
    converges to the solid angle the emitter subtends -- the closed form of Van Oosterom &
    Strackee (1983) for a triangle, 2 pi (1 - sqrt(1 - (r / d)^2)) for a sphere -- which holds
    only if the warp is area-uniform and the pdf is its exact density in solid angle.
Test infrastructure only; CPU.
"""
import numpy as np
import pytest

import oracle
from pupiloptixlab_amd import World
from pupiloptixlab_amd import world as W

RADIANCE = (40.0, 38.0, 34.0)
P = np.array([0.3, 0.0, 0.2])
N = np.array([0.0, 1.0, 0.0])


@pytest.fixture(scope="module")
def setup():
    wd = World()
    wd.set_film(8, 8, 4)
    rect = wd.add_builtin("rectangle")
    sph = wd.add_builtin("sphere")
    m = wd.add_material(W.twosided(W.diffuse((0.0, 0.0, 0.0))))
    # a 2 x 1.2 light at y = 3 facing down (two triangle emitters), a radius-0.5 sphere light
    rect_xf = W.transform(scale=(1.0, 0.6, 1), rotate=((1, 0, 0), 90), translate=(0.4, 3.0, -0.3))
    wd.add_instance(rect, m, rect_xf, emitter_radiance=RADIANCE)
    wd.add_instance(sph, m, W.transform(scale=(0.5, 0.5, 0.5), translate=(2.0, 1.5, 0.5)), emitter_radiance=RADIANCE)
    wd.set_sensor(40.0, W.look_at_mitsuba((0, 1, 8), (0, 1, 0), (0, 1, 0)))
    desc = wd.desc()
    return oracle.OracleScene(desc), desc


def tri_solid_angle(a, b, c):
    """Van Oosterom & Strackee: solid angle of triangle (a, b, c) seen from the origin."""
    la, lb, lc = np.linalg.norm(a), np.linalg.norm(b), np.linalg.norm(c)
    num = abs(np.dot(a, np.cross(b, c)))
    den = la * lb * lc + np.dot(a, b) * lc + np.dot(a, c) * lb + np.dot(b, c) * la
    return 2.0 * np.arctan2(num, den)


def _grid(n):
    g = (np.arange(n) + 0.5) / n
    return np.stack(np.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2).astype(np.float32)


def test_triangle_emitters_sample_and_solid_angle(setup):
    orc, desc = setup
    ems = desc.area_emitters
    for k in range(2):
        e = ems[k]
        v = np.array([[e.pos[i][j] for j in range(3)] for i in range(3)], np.float64)
        nv = np.array([[e.nrm[i][j] for j in range(3)] for i in range(3)], np.float64)
        area = float(e.area)
        inv_pdf = []
        for xi in _grid(160):
            out = orc.emitter_sample(k, P, N, xi)
            wi, pdf, dist, rad = out[:3], float(out[3]), float(out[4]), out[5:8]
            assert np.allclose(rad, RADIANCE)
            # area.h:17-34 restated: UniformSampleTriangle (util.h:33-36), the interpolated normal
            s = np.sqrt(np.float64(xi[0]))
            t = np.array([1.0 - s, s * (1.0 - xi[1]), xi[1] * s])
            pos = t @ v
            nrm = t @ nv
            nrm /= np.linalg.norm(nrm)
            w = (pos - P) / np.linalg.norm(pos - P)
            assert np.allclose(wi, w, atol=2e-6)
            lnol = np.dot(nrm, -w)
            if np.dot(N, w) > 0 and lnol > 0:
                d = np.linalg.norm(pos - P)
                assert np.isclose(dist, d, rtol=1e-5)
                assert np.isclose(pdf, d * d / (lnol * area), rtol=1e-4)
                inv_pdf.append(1.0 / pdf)
            else:
                assert pdf == 0.0
                inv_pdf.append(0.0)
        omega = tri_solid_angle(v[0] - P, v[1] - P, v[2] - P)
        assert np.isclose(np.mean(inv_pdf) * 1.0, omega, rtol=2e-3), (k, np.mean(inv_pdf), omega)


def test_sphere_emitter_solid_angle(setup):
    orc, desc = setup
    e = desc.area_emitters[2]
    c, r = np.array([2.0, 1.5, 0.5]), 0.5
    inv_pdf = []
    for xi in _grid(300):
        out = orc.emitter_sample(2, P, N, xi)
        pdf = float(out[3])
        inv_pdf.append(1.0 / pdf if pdf > 0 else 0.0)
    # the sphere lies wholly above the shading point's horizon: every cap direction is valid
    d = np.linalg.norm(c - P)
    omega = 2.0 * np.pi * (1.0 - np.sqrt(1.0 - (r / d) ** 2))
    # uniform points on the whole sphere, only the facing half contributes: mean(1/pdf) = omega
    assert np.isclose(np.mean(inv_pdf), omega, rtol=3e-3), (np.mean(inv_pdf), omega)
    assert float(e.area) == pytest.approx(4.0 * np.pi * r * r, rel=1e-5)
