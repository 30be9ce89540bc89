"""A second, independent restatement of the reference's BSDF evaluation pins the oracle's.

The reference ships no BSDF values to test against, so the oracle's seven
BSDFs are checked here against a float64 numpy restatement written separately from the
reference's formulas -- GetBsdf / GetPdf of render/material/bsdf/*.h, ggx.h (visible-area
sampling pdf), fresnel.h and the plastic precomputation of optix_material.cpp -- at random
direction pairs on both hemispheres.  The oracle computes in float32 in the reference's
operation order; the tolerance covers float32 rounding of chains of ~60 operations, away
from grazing angles and the refraction singularity (sqrt_denom ~ 0) where the relative
error of any float32 evaluation grows without bound.  Test infrastructure only; CPU.
"""
import numpy as np
import pytest

import oracle
from pupiloptixlab_amd import World
from pupiloptixlab_amd import world as W

INV_PI = 1.0 / np.pi

# the probe scene's materials, in instance order (same parameters as test_oracle_kat.py)
ALPHA = 0.35
ETA = 1.5
RC_ETA, RC_K = np.array([0.2, 0.92, 1.1]), np.array([3.9, 2.45, 2.14])
PLASTIC_DIFFUSE = 0.647814


@pytest.fixture(scope="module")
def scene():
    wd = World()
    wd.set_film(8, 8, 4)
    sph = wd.add_builtin("sphere")
    mats = [W.diffuse(0.7), W.plastic(PLASTIC_DIFFUSE, 1.0, ETA, 1.0), W.rough_conductor(ALPHA, tuple(RC_ETA), tuple(RC_K)),
            W.rough_plastic(ALPHA, PLASTIC_DIFFUSE, 1.0, ETA, 1.0), W.rough_dielectric(ALPHA, ETA, 1.0),
            W.rough_plastic(ALPHA, PLASTIC_DIFFUSE, 1.0, ETA, 1.0, nonlinear=True)]
    for m in mats:
        wd.add_instance(sph, wd.add_material(m))
    wd.set_sensor(40.0, W.look_at_mitsuba((0, 0, 5), (0, 0, 0), (0, 1, 0)))
    return oracle.OracleScene(wd.desc())


# ---- ggx.h (isotropic, GGX_Sample_Visible_Area), float64
def lam(w, a):  # ggx.h:10-14
    v2 = w * w
    return (-1.0 + np.sqrt(1.0 + (v2[0] + v2[1]) * a * a / v2[2])) / 2.0


def g1(w, a):  # ggx.h:16-18
    return 1.0 / (1.0 + lam(w, a))


def ggx_d(wh, a):  # ggx.h:24-29
    v2 = wh * wh
    t = (v2[0] + v2[1]) / (a * a) + v2[2]
    return 1.0 / (np.pi * a * a * t * t)


def ggx_pdf(wo, wh, a):  # ggx.h:31-36, visible-area branch
    return ggx_d(wh, a) * g1(wo, a) * np.dot(wo, wh) / abs(wo[2])


def norm(v):
    return v / np.linalg.norm(v)


# ---- fresnel.h, float64
def fr_dielectric(eta, cos_i):  # fresnel.h:7-25
    scale = 1.0 / eta if cos_i > 0 else eta
    ct2 = 1.0 - (1.0 - cos_i * cos_i) * scale * scale
    if ct2 <= 0.0:
        return 1.0
    ci, ct = abs(cos_i), np.sqrt(ct2)
    rs = (ci - eta * ct) / (ci + eta * ct)
    rp = (eta * ci - ct) / (eta * ci + ct)
    return 0.5 * (rs * rs + rp * rp)


def fr_conductor(eta, k, cos_i):  # fresnel.h:31-49, per channel
    c2 = cos_i * cos_i
    s2 = 1.0 - c2
    t1 = eta * eta - k * k - s2
    a2pb2 = np.sqrt(np.maximum(0.0, t1 * t1 + 4.0 * k * k * eta * eta))
    a = np.sqrt(np.maximum(0.0, 0.5 * (a2pb2 + t1)))
    term1, term2 = a2pb2 + c2, 2.0 * a * cos_i
    rs2 = (term1 - term2) / (term1 + term2)
    term3, term4 = a2pb2 * c2 + s2 * s2, term2 * s2
    rp2 = rs2 * (term3 - term4) / (term3 + term4)
    return 0.5 * (rp2 + rs2)


def diffuse_reflectance(eta):  # fresnel.h:58-84 (eta >= 1 branch and the Egan-Hilgeman fit below 1)
    if eta < 1:
        return -1.4399 * eta * eta + 0.7099 * eta + 0.6681 + 0.0636 / eta
    i = 1.0 / eta
    return 0.919317 - 3.4793 * i + 6.75335 * i ** 2 - 7.80989 * i ** 3 + 4.98554 * i ** 4 - 1.36881 * i ** 5


def plastic_params(diffuse, specular=1.0):  # optix_material.cpp:87-102 (GetLuminance, optix/util.h:161-163)
    lum = lambda c: 0.2126 * c + 0.7152 * c + 0.0722 * c  # grey textures
    ssw = lum(specular) / (lum(specular) + lum(diffuse))
    return ssw, diffuse_reflectance(1.0 / ETA)


# ---- the BSDFs' GetBsdf / GetPdf, float64; return (f rgb, pdf)
def eval_diffuse(wo, wi, refl=0.7):  # bsdf/diffuse.h:14-27
    if wi[2] > 0 and wo[2] > 0:
        return np.full(3, refl * INV_PI), INV_PI * wi[2]
    return np.zeros(3), 0.0


def eval_plastic(wo, wi):  # bsdf/plastic.h:32-51
    if wi[2] <= 0 or wo[2] <= 0:
        return np.zeros(3), 0.0
    ssw, int_fdr = plastic_params(PLASTIC_DIFFUSE)
    fo, fi = fr_dielectric(ETA, wo[2]), fr_dielectric(ETA, wi[2])
    diff = PLASTIC_DIFFUSE / (1.0 - int_fdr)
    f = diff * (1 - fi) * (1 - fo) * (INV_PI * wi[2]) / (ETA * ETA * wi[2])
    sp = fo * ssw / (fo * ssw + (1 - fo) * (1 - ssw))
    return np.full(3, f), INV_PI * wi[2] * (1 - sp)


def eval_rough_conductor(wo, wi):  # bsdf/rough_conductor.h:21-38
    if wi[2] <= 0 or wo[2] <= 0:
        return np.zeros(3), 0.0
    wh = norm(wi + wo)
    f = ggx_d(wh, ALPHA) * fr_conductor(RC_ETA, RC_K, np.dot(wo, wh)) * g1(wi, ALPHA) * g1(wo, ALPHA) / (4 * wi[2] * wo[2])
    return f, ggx_pdf(wo, wh, ALPHA) / (4 * np.dot(wo, wh))


def eval_rough_plastic(wo, wi, nonlinear=False):  # bsdf/rough_plastic.h:31-63
    if wi[2] <= 0 or wo[2] <= 0:
        return np.zeros(3), 0.0
    ssw, int_fdr = plastic_params(PLASTIC_DIFFUSE)
    fo = fr_dielectric(ETA, wo[2])
    wh = norm(wi + wo)
    f = fr_dielectric(ETA, np.dot(wh, wo)) * ggx_d(wh, ALPHA) * g1(wi, ALPHA) * g1(wo, ALPHA) / (4 * wo[2] * wi[2])
    fi = fr_dielectric(ETA, wi[2])
    diff = PLASTIC_DIFFUSE / (1.0 - (PLASTIC_DIFFUSE * int_fdr if nonlinear else int_fdr))
    f += diff * (1 - fi) * (1 - fo) * INV_PI / (ETA * ETA)
    sp = fo * ssw / (fo * ssw + (1 - fo) * (1 - ssw))
    pdf = sp * ggx_pdf(wo, wh, ALPHA) / (4 * np.dot(wi, wh)) + (1 - sp) * INV_PI * wi[2]
    return np.full(3, f), pdf


def eval_rough_dielectric(wo, wi):  # bsdf/rough_dielectric.h:21-71
    reflect = wo[2] * wi[2] > 0
    e = ETA if wo[2] > 0 else 1.0 / ETA
    wh = norm(wo + wi) if reflect else norm(wo + wi * e)
    wh = wh * (1.0 if wh[2] > 0 else -1.0)
    F = fr_dielectric(ETA, np.dot(wo, wh))
    G = g1(wi, ALPHA) * g1(wo, ALPHA)
    D = ggx_d(wh, ALPHA)
    if reflect:
        f = F * G * D / (4 * abs(wi[2]) * abs(wo[2]))
        dwh = 1.0 / (4 * np.dot(wi, norm(wo + wi)))
    else:
        sd = np.dot(wo, wh) + e * np.dot(wi, wh)
        f = abs((1 - F) * D * G * np.dot(wi, wh) * np.dot(wo, wh) / (sd * sd * wi[2] * wo[2]))
        whp = norm(wo + wi * e)  # GetPdf recomputes the half vector before the flip
        sdp = np.dot(wo, whp) + e * np.dot(wi, whp)
        dwh = e * e * np.dot(wi, whp) / (sdp * sdp)
    wo_up = wo * (1.0 if wo[2] > 0 else -1.0)
    pdf = abs(ggx_pdf(wo_up, wh, ALPHA) * (F if reflect else 1 - F) * dwh)
    return np.full(3, f), pdf


CASES = [(0, eval_diffuse, False), (1, eval_plastic, False), (2, eval_rough_conductor, False),
         (3, eval_rough_plastic, False), (4, eval_rough_dielectric, True),
         (5, lambda wo, wi: eval_rough_plastic(wo, wi, nonlinear=True), False)]


def _dirs(rng, n, both):
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    if not both:
        d[:, 2] = np.abs(d[:, 2])
    return d


@pytest.mark.parametrize("mat,ref,both", CASES, ids=["diffuse", "plastic", "rough_conductor", "rough_plastic",
                                                     "rough_dielectric", "rough_plastic_nonlinear"])
def test_oracle_bsdf_eval_matches_float64_restatement(scene, mat, ref, both):
    rng = np.random.default_rng(11 + mat)
    wos, wis = _dirs(rng, 600, both), _dirs(rng, 600, both)
    checked = 0
    for wo, wi in zip(wos, wis):
        wo32, wi32 = wo.astype(np.float32), wi.astype(np.float32)
        wo64, wi64 = wo32.astype(np.float64), wi32.astype(np.float64)  # the oracle's inputs, exactly
        if min(abs(wo64[2]), abs(wi64[2])) < 0.08:
            continue  # grazing: float32 relative error unbounded
        if both and wo64[2] * wi64[2] < 0:
            e = ETA if wo64[2] > 0 else 1.0 / ETA
            wh = norm(wo64 + wi64 * e)
            if abs(np.dot(wo64, wh) + e * np.dot(wi64, wh)) < 0.1 or np.linalg.norm(wo64 + wi64 * e) < 0.1:
                continue  # the refraction singularity
        elif np.linalg.norm(wo64 + wi64) < 0.1:
            continue  # wh undefined (back-scatter)
        out = scene.bsdf(mat, wo32, wi32, 0)
        f, pdf = out[8:11].astype(np.float64), float(out[11])
        rf, rpdf = ref(wo64, wi64)
        assert np.allclose(f, rf, rtol=3e-4, atol=1e-7), (mat, wo64, wi64, f, rf)
        assert np.isclose(pdf, rpdf, rtol=3e-4, atol=1e-7), (mat, wo64, wi64, pdf, rpdf)
        checked += 1
    assert checked > 150
