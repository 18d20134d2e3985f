"""Accuracy of the deterministic fp32 math (ark_fmath.h) against double-precision
numpy, and bitwise identity of the product's host build with the oracle's."""
import numpy as np
import pytest

from arkoserenderer_amd import abi
import oracle_lib as O

ULP = 2.0 ** -23


def ulps(got, ref):
    ref = np.asarray(ref, np.float64)
    scale = np.maximum(np.abs(ref), np.finfo(np.float32).tiny)
    return np.abs(got.astype(np.float64) - ref) / (scale * ULP)


def test_sin_cos():
    x = np.concatenate([np.linspace(-7, 7, 200_001), np.random.default_rng(0).uniform(0, 2000, 200_000)]).astype(np.float32)
    s, c = O.fmath(0, x), O.fmath(1, x)
    xs = x.astype(np.float64)
    # absolute error (what matters near the zeros of sin/cos), in units of 2^-24
    assert np.max(np.abs(s - np.sin(xs))) < 4 * 2 ** -24
    assert np.max(np.abs(c - np.cos(xs))) < 4 * 2 ** -24


def test_acos_atan2():
    x = np.linspace(-1, 1, 400_001).astype(np.float32)
    a = O.fmath(2, x)
    assert np.max(np.abs(a - np.arccos(x.astype(np.float64)))) < 4 * 2 ** -23
    rng = np.random.default_rng(1)
    yv = rng.normal(size=200_000).astype(np.float32)
    xv = rng.normal(size=200_000).astype(np.float32)
    t = O.fmath(3, yv, xv)
    assert np.max(np.abs(t - np.arctan2(yv.astype(np.float64), xv.astype(np.float64)))) < 4 * 2 ** -22


def test_log2_exp2_pow():
    rng = np.random.default_rng(2)
    x = np.exp(rng.uniform(-80, 80, 200_000)).astype(np.float32)
    assert np.max(np.abs(O.fmath(4, x) - np.log2(x.astype(np.float64)))) < 2e-6 * np.max(np.abs(np.log2(x.astype(np.float64)))) + 1e-6
    z = rng.uniform(-120, 120, 200_000).astype(np.float32)
    assert np.max(ulps(O.fmath(5, z), np.exp2(z.astype(np.float64)))) < 4
    # pow: gamma encode (1/5), decode (2.5), smoothing (0.25), Schlick (5), sharpness (50)
    b = rng.uniform(0, 1, 200_000).astype(np.float32)
    for e, tol in [(0.2, 64), (2.5, 96), (0.25, 64), (5.0, 8), (50.0, 64)]:
        got = O.fmath(6, b, np.full_like(b, e))
        ref = b.astype(np.float64) ** e
        m = ref > 1e-30
        assert np.max(ulps(got[m], ref[m])) < tol, e
    # special cases (GLSL: pow(0, y>0) = 0, pow(x, 0) = 1)
    assert O.fmath(6, np.array([0.0], np.float32), np.array([50.0], np.float32))[0] == 0.0
    assert O.fmath(6, np.array([0.3], np.float32), np.array([0.0], np.float32))[0] == 1.0


def test_pow_square_root_exponents():
    """pow(x, 1/4) = sqrt(sqrt(x)), pow(x, 1/2) = sqrt(x), pow(x, n + 1/2) = powi(x, n) * sqrt(x),
    each IEEE fp32 operation correctly rounded (numpy float32 arithmetic is)."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(0, 1, 50_000), rng.uniform(0, 50, 50_000), [0.0, 1.0, np.inf]]).astype(np.float32)
    x2 = x * x
    cases = [(0.25, np.sqrt(np.sqrt(x))), (0.5, np.sqrt(x)), (1.5, x * np.sqrt(x)), (2.5, x2 * np.sqrt(x)),
             (5.5, (x * (x2 * x2)) * np.sqrt(x))]  # powi_(x, 5) = x * (x^2)^2 in binary-exponentiation order
    for y, ref in cases:
        got = O.fmath(6, x, np.full_like(x, y))
        assert np.array_equal(got.view(np.uint32), ref.astype(np.float32).view(np.uint32)), y
    assert np.isnan(O.fmath(6, np.float32([-1.0]), np.float32([2.5]))[0])


@pytest.mark.parametrize("op", [0, 1, 2, 3, 4, 5, 6])
def test_product_host_build_equals_oracle(op):
    """libark_ddgi's host compile of ark_fmath.h == the oracle's, bit for bit."""
    lib = abi.load_library()
    rng = np.random.default_rng(10 + op)
    x = rng.uniform(-3, 3, 100_000).astype(np.float32)
    if op in (4, 6):
        x = np.abs(x)
    if op == 2:
        x = np.clip(x / 3, -1, 1).astype(np.float32)
    y = rng.uniform(0.1, 60, 100_000).astype(np.float32)
    out = np.empty_like(x)
    assert lib.ark_ddgi_debug_fmath_host(op, x.ctypes.data, y.ctypes.data, out.ctypes.data, x.size) == 0
    ref = O.fmath(op, x, y)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)) or np.all((out == ref) | (np.isnan(out) & np.isnan(ref)))


def test_powf_pos_equals_powf_on_domain():
    lib = abi.load_library()
    rng = np.random.default_rng(4)
    x = np.concatenate([rng.uniform(0, 1, 200_000), np.exp(rng.uniform(-100, 0, 50_000)),
                        rng.uniform(0.9999, 1.0000002, 20_000)]).astype(np.float32)
    x = x[x > 0]
    y = rng.uniform(0.01, 64, x.size).astype(np.float32)
    y[np.floor(y) == y] += 0.25
    y[(np.floor(y) + 0.5 == y) | (y == 0.25)] += 0.125  # square-root exponents are outside powf_pos_'s domain
    out = np.empty_like(x)
    assert lib.ark_ddgi_debug_fmath_host(8, x.ctypes.data, y.ctypes.data, out.ctypes.data, x.size) == 0
    assert np.array_equal(out.view(np.uint32), O.fmath(6, x, y).view(np.uint32))
