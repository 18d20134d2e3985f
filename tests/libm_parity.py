"""Tolerance comparison against the libm-math oracle (test infrastructure).

The bit-exact oracle (oracle/build/libddgi_oracle.so) evaluates the GLSL
transcendentals with the product's own ark_fmath.h. The -DARK_ORACLE_LIBM build
(libddgi_oracle_libm.so) uses glibc's sinf/cosf/acosf/atan2f/exp2f/powf instead at the
reference's call sites (common.glsl:126-139, probeUpdateIrradiance.comp:57,
probeUpdateVisibility.comp:46, probeSampling.glsl:40,108,149, lighting.glsl:32-35,
probeUpdateOffset.comp:93), so it shares no transcendental code with the product.

Method (frame-local): before each compared frame the libm oracle is given the HIP
path's state (both atlases and the probe offsets after the previous frame), then both
run the same frame, so each comparison measures one frame's divergence instead of
the chaos of several frames (the indirect bounce re-reads the atlases every frame).

Results differ in the last bits, and a ray direction that moves by an ulp can flip
a discontinuous outcome: a different triangle, the other face, a shadow ray that
grazes an edge, an alpha-tested texel. No output tolerance holds across such a flip
for any two implementations (a flipped surfel changes its probe's texels by up to
its cosine weight / the probe's weight sum). So the comparison is split:

  * rays: a ray is flipped when any surfel channel differs by more than FLIP_ULP fp16
    ulps or its signed distance changes sign (front <-> back face); the flipped
    fraction must stay below FLIP_FRACTION, and every other surfel within
    SURFEL_ULP ulps;
  * atlases, over the interior texels of the compared probes that have no flipped
    ray, at SURVEY §8(d)'s tolerances: irradiance (stored gamma-encoded,
    irradiance^(1/5), probeUpdateIrradiance.comp:57) L-inf < 1e-3 and >= 99.9 % of
    the texel channels within 1 fp16 ulp; visibility (mean distance, mean squared
    distance) relative error < 1e-3 on >= 99.9 % of the texel channels;
  * reported beside it, not asserted: the same statistics over every compared probe
    (flipped ones included).
"""
from __future__ import annotations

import numpy as np

import oracle_lib as O

IRR_TOL_LINF = 1e-3
ULP_FRACTION = 0.999
VIS_REL_TOL = 1e-3
FLIP_ULP = 64
FLIP_FRACTION = 1e-3
SURFEL_ULP = 8


def tile_mask(dims, probes, res: int, interior: bool = True) -> np.ndarray:
    """Atlas mask of the (res + 2)^2 tiles of `probes` (ddgi/common.glsl:36-67),
    interior texels only by default (DDGINode.cpp:262-281: 1-texel borders)."""
    X, Y, Z = dims
    t = res + 2
    m = np.zeros((Z * t, X * Y * t), bool)
    lo, hi = (1, res + 1) if interior else (0, t)
    for p in probes:
        y, rem = divmod(int(p), X * Z)
        z, x = divmod(rem, X)
        tx, ty = x + y * X, z
        m[ty * t + lo:ty * t + hi, tx * t + lo:tx * t + hi] = True
    return m


def f16_ulp_distance(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """|ordinal(a) - ordinal(b)| of fp16 bit patterns (uint16); NaN vs NaN = 0,
    NaN vs a number = 65536."""
    a = a.astype(np.int32)
    b = b.astype(np.int32)
    ka = np.where(a & 0x8000, -(a & 0x7FFF), a & 0x7FFF)
    kb = np.where(b & 0x8000, -(b & 0x7FFF), b & 0x7FFF)
    d = np.abs(ka - kb)
    na = ((a & 0x7C00) == 0x7C00) & ((a & 0x3FF) != 0)
    nb = ((b & 0x7C00) == 0x7C00) & ((b & 0x3FF) != 0)
    d = np.where(na & nb, 0, d)
    d = np.where(na ^ nb, 1 << 16, d)
    return d


def surfel_stats(a: np.ndarray, b: np.ndarray):
    """(flipped [K, R] bool, max ulp [K, R]) of two [K, R, 4] fp16 surfel arrays."""
    u = f16_ulp_distance(a, b).max(axis=-1)
    da, db = a[..., 3].astype(np.int32), b[..., 3].astype(np.int32)
    nonzero = ((da & 0x7FFF) != 0) & ((db & 0x7FFF) != 0)
    sign = (((da ^ db) & 0x8000) != 0) & nonzero
    return (u > FLIP_ULP) | sign, u


def atlas_stats(dims, probes, irr_a, irr_b, vis_a, vis_b) -> dict:
    """Statistics over the interior texels of `probes`' tiles (uint16 fp16 atlases as
    ctx.read returns them)."""
    probes = list(probes)
    mi = tile_mask(dims, probes, 8)
    mv = tile_mask(dims, probes, 16)
    ia = irr_a.reshape(mi.shape[0], mi.shape[1], 4)[mi]
    ib = irr_b.reshape(mi.shape[0], mi.shape[1], 4)[mi]
    va = vis_a.reshape(mv.shape[0], mv.shape[1], 2)[mv]
    vb = vis_b.reshape(mv.shape[0], mv.shape[1], 2)[mv]
    fa, fb = O.f16_to_f32(ia).astype(np.float64), O.f16_to_f32(ib).astype(np.float64)
    with np.errstate(invalid="ignore"):
        d = np.abs(fa - fb)
    d[np.isnan(fa) & np.isnan(fb)] = 0.0
    d[np.isinf(fa) & np.isinf(fb) & (np.sign(fa) == np.sign(fb))] = 0.0
    d[np.isnan(d)] = np.inf
    ulp_i = f16_ulp_distance(ia, ib)
    ga, gb = O.f16_to_f32(va).astype(np.float64), O.f16_to_f32(vb).astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.abs(ga - gb) / np.maximum(np.abs(gb), 1e-6)
    same = (va == vb) | (np.isnan(ga) & np.isnan(gb))
    rel[same] = 0.0
    rel[np.isnan(rel)] = np.inf
    n_i, n_v = max(1, ia.size), max(1, va.size)
    return {
        "probes": len(probes),
        "irradiance": {
            "linf": float(d.max()) if d.size else 0.0,
            "mean_abs": float(d[np.isfinite(d)].mean()) if d.size else 0.0,
            "differing_frac": float(np.count_nonzero(ia != ib) / n_i),
            "within_1ulp_frac": float(np.count_nonzero(ulp_i <= 1) / n_i),
            "max_ulp": int(ulp_i.max()) if ulp_i.size else 0,
        },
        "visibility": {
            "rel_linf": float(rel.max()) if rel.size else 0.0,
            "rel_mean": float(rel[np.isfinite(rel)].mean()) if rel.size else 0.0,
            "within_rel_tol_frac": float(np.count_nonzero(rel < VIS_REL_TOL) / n_v),
            "differing_frac": float(np.count_nonzero(~same) / n_v),
        },
    }


def compare_window(dims, probes, surf_a, surf_b, irr_a, irr_b, vis_a, vis_b) -> dict:
    """One frame's comparison of a window: surf_* are [K, R, 4] surfels of `probes`
    (same order), the atlases whole. Returns the ray statistics, the atlas statistics
    over the probes without a flipped ray ("clean") and over all of them ("all")."""
    probes = np.asarray(probes)
    flipped, u = surfel_stats(surf_a, surf_b)
    clean = probes[~flipped.any(axis=1)]
    rays = int(flipped.size)
    return {
        "rays": rays,
        "flipped_rays": int(flipped.sum()),
        "flipped_frac": float(flipped.sum() / max(1, rays)),
        "differing_rays_frac": float(np.count_nonzero(u) / max(1, rays)),
        "max_ulp_unflipped": int(u[~flipped].max()) if (~flipped).any() else 0,
        "clean": atlas_stats(dims, clean, irr_a, irr_b, vis_a, vis_b),
        "all": atlas_stats(dims, probes, irr_a, irr_b, vis_a, vis_b),
    }


def check(stats: dict, what: str = "", surfel_ulp: int | None = SURFEL_ULP) -> None:
    """The tolerances of the module docstring. surfel_ulp None: the unflipped surfels'
    bound is reported, not asserted (the whole-grid runs: over 8.4 M rays a ray that
    stays under the flip threshold near a discontinuity can move a surfel by more)."""
    assert stats["flipped_frac"] <= FLIP_FRACTION, (what, stats)
    if surfel_ulp is not None:
        assert stats["max_ulp_unflipped"] <= surfel_ulp, (what, stats)
    c = stats["clean"]
    assert c["probes"] >= 0.9 * stats["all"]["probes"], (what, stats)
    i, v = c["irradiance"], c["visibility"]
    assert i["linf"] < IRR_TOL_LINF, (what, stats)
    assert i["within_1ulp_frac"] >= ULP_FRACTION, (what, stats)
    assert v["within_rel_tol_frac"] >= ULP_FRACTION, (what, stats)
