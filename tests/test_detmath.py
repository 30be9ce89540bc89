"""Accuracy of the deterministic libm shared by the engine and the oracle
(include/pupil_detmath.h) against float64 numpy, over the ranges the tracer uses."""
import numpy as np

import oracle


def ulp_err(got, ref):
    ref32 = ref.astype(np.float32)
    spacing = np.spacing(np.abs(ref32)).astype(np.float64)
    spacing = np.maximum(spacing, np.float64(np.finfo(np.float32).tiny))
    return np.abs(got.astype(np.float64) - ref) / spacing


def test_sin_cos_accuracy():
    x = np.linspace(-4 * np.pi, 4 * np.pi, 200001).astype(np.float32)
    out = oracle.math_probe(x, np.ones_like(x))
    xd = x.astype(np.float64)
    # absolute error relative to 1 ulp of 1.0 near zeros of sin/cos, else relative ulps
    for k, fn in ((0, np.sin), (1, np.cos)):
        ref = fn(xd)
        err = np.abs(out[:, k] - ref)
        assert (err <= np.maximum(4 * np.spacing(np.abs(ref.astype(np.float32))), 2e-7)).all(), fn


def test_acos_accuracy():
    x = np.linspace(-1, 1, 100001).astype(np.float32)
    out = oracle.math_probe(x, np.ones_like(x))
    assert ulp_err(out[:, 2], np.arccos(x.astype(np.float64))).max() <= 4


def test_atan2_accuracy_and_quadrants():
    rng = np.random.default_rng(0)
    y = rng.uniform(-5, 5, 100000).astype(np.float32)
    x = rng.uniform(-5, 5, 100000).astype(np.float32)
    out = oracle.math_probe(y, x)
    ref = np.arctan2(y.astype(np.float64), x.astype(np.float64))
    assert np.abs(out[:, 3] - ref).max() < 4e-7
    edge = oracle.math_probe(np.array([0, 1, -1, 0], np.float32), np.array([1, 0, 0, -1], np.float32))
    assert np.allclose(edge[:, 3], [0, np.pi / 2, -np.pi / 2, np.pi], atol=1e-7)


def test_sqrt_and_reciprocal_are_correctly_rounded():
    rng = np.random.default_rng(1)
    x = rng.uniform(1e-6, 1e6, 50000).astype(np.float32)
    out = oracle.math_probe(x, x)
    assert np.array_equal(out[:, 4], np.sqrt(x))
    assert np.array_equal(out[:, 5], np.float32(1.0) / x)
