"""Device side of the deterministic math (ark_fmath.h) and the fp16 store
conversion, bit for bit against the host side (the oracle's arithmetic)."""
import ctypes as C

import numpy as np
import pytest

from arkoserenderer_amd import abi
import oracle_lib as O

pytestmark = pytest.mark.gpu


def _inputs(op, n=200_000, seed=1):
    rng = np.random.default_rng(seed)
    if op in (0, 1):
        x = np.concatenate([rng.uniform(-7, 7, n // 2), rng.uniform(0, 2000, n // 2)])
    elif op == 2:
        x = rng.uniform(-1, 1, n)
    elif op == 3:
        x = rng.normal(size=n)
    elif op == 4:
        x = np.exp(rng.uniform(-80, 80, n))
    elif op == 5:
        x = rng.uniform(-160, 130, n)
    elif op == 6:
        x = rng.uniform(0, 1, n)
        x[: n // 4] = rng.uniform(0, 2, n // 4)
    else:
        x = rng.normal(scale=100, size=n)
    y = rng.normal(size=n) if op == 3 else (rng.uniform(0.1, 60, n) if op == 6 else np.zeros(n))
    if op == 6:
        y[: n // 3] = rng.integers(1, 65, n // 3)  # integral exponents (powi_ path)
        y[n // 3: n // 2] = rng.choice(np.float32([0.25, 0.5, 1.5, 2.5, 16.5]), n // 2 - n // 3)  # square-root exponents
    return x.astype(np.float32), y.astype(np.float32)


@pytest.mark.parametrize("op", [0, 1, 2, 3, 4, 5, 6])
def test_device_fmath_matches_host(op):
    lib = abi.load_library()
    x, y = _inputs(op)
    dev = np.empty_like(x)
    assert lib.ark_ddgi_debug_fmath(0, op, x.ctypes.data, y.ctypes.data, dev.ctypes.data, x.size) == 0
    host = O.fmath(op, x, y)
    same = (dev.view(np.uint32) == host.view(np.uint32)) | (np.isnan(dev) & np.isnan(host))
    assert same.all(), f"op {op}: {np.count_nonzero(~same)} differ, e.g. x={x[~same][:3]} dev={dev[~same][:3]} host={host[~same][:3]}"


def test_device_powf_pos_matches_powf():
    """The branch-free pow of the visibility loop == powf_ (host) on its domain."""
    lib = abi.load_library()
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.uniform(0, 1, 300_000), np.exp(rng.uniform(-100, 0, 100_000)),
                        rng.uniform(0.9999, 1.0000002, 50_000)]).astype(np.float32)
    x = x[x > 0]
    y = rng.uniform(0.01, 64, x.size).astype(np.float32)
    y[np.floor(y) == y] += 0.25  # integral exponents take powi_, not powf_pos_
    dev = np.empty_like(x)
    assert lib.ark_ddgi_debug_fmath(0, 8, x.ctypes.data, y.ctypes.data, dev.ctypes.data, x.size) == 0
    host = O.fmath(6, x, y)
    assert np.array_equal(dev.view(np.uint32), host.view(np.uint32))


def test_device_fp16_rne_ties():
    """fp32 -> fp16 on the device vs the oracle's RNE (incl. exact ties, subnormals, overflow)."""
    lib = abi.load_library()
    rng = np.random.default_rng(3)
    h = rng.integers(0, 0x7c00, 100_000).astype(np.uint16)
    base = O.f16_to_f32(h)
    nxt = O.f16_to_f32((h + 1).astype(np.uint16))
    ties = ((base.astype(np.float64) + nxt.astype(np.float64)) / 2).astype(np.float32)
    x = np.concatenate([ties, -ties, rng.normal(scale=1000, size=50_000).astype(np.float32),
                        np.array([65519.0, 65520.0, 1e8, 6e-8, 3e-8, 2.98e-8, -0.0], np.float32)])
    dev = np.empty_like(x)
    assert lib.ark_ddgi_debug_fmath(0, 7, x.ctypes.data, None, dev.ctypes.data, x.size) == 0
    ref = O.f16_to_f32(O.f32_to_f16(x))
    same = (dev.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(dev) & np.isnan(ref))
    assert same.all(), f"{np.count_nonzero(~same)} differ: x={x[~same][:4]} dev={dev[~same][:4]} ref={ref[~same][:4]}"
