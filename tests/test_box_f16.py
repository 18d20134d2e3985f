"""The reduced-precision BVH8 child tests are conservative (host restatement, no GPU).

visitNode8 (ddgi_kernels.hip) tests children with fp32 slabs. Round 4 also built two
packed-fp16 forms (per-axis error bounds, and directed rounding: near planes toward
-inf, far planes toward +inf); they were measured 10x slower and removed from the
kernels in round 5, and their host restatements stay as the record that
they were conservative. ark_ddgi_debug_bvh8_trace_stats restates each form (ARK_SIM_BOX) and
counts the children that the exact test accepts and the form culls (out[8]); a
culled child could hide the closest hit, so the count must be 0. Rays: probe-like
rays of a soup, plus near-axis-parallel directions (|idir| up to 1e6) and origins
outside the scene, where the per-node fp16 scale and the range of B matter most.
"""
import ctypes as C
import os

import numpy as np
import pytest

import sys

from arkoserenderer_amd import scene as S

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "sim"))
import bvhsim  # noqa: E402  (the simulator is a tool library, not libark_ddgi.so)


def _triangles(sc):
    ws = []
    for inst in sc.instances:
        mesh = sc.meshes[inst["rt_mesh_index"]]
        idx = sc.indices[mesh["first_index"]: mesh["first_index"] + 3 * inst["triangle_count"]]
        p = sc.positions[mesh["first_vertex"] + idx.astype(np.int64)]
        M = inst["object_to_world"].reshape(3, 4)
        ws.append((p @ M[:, :3].T + M[:, 3]).reshape(-1, 9))
    return np.ascontiguousarray(np.concatenate(ws), np.float32)


def _rays(n, lo, hi, rng):
    o = rng.uniform(lo, hi, (n, 3))
    d = rng.normal(size=(n, 3))
    # a third near-axis-parallel: two components scaled down to 1e-6 .. 1e-3
    k = n // 3
    for i in range(k):
        a = i % 3
        for b in range(3):
            if b != a:
                d[i, b] *= 10.0 ** rng.uniform(-6, -3)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t = np.full((n, 1), 10000.0)
    # some rays with a short tmax (the clamp of the far distances)
    t[rng.random(n) < 0.2] = rng.uniform(0.5, 5.0)
    return np.ascontiguousarray(np.hstack([o, d, t]), np.float32)


@pytest.mark.parametrize("mode", ["kernel32", "f16s", "f16d"])
def test_box_forms_cull_no_exact_hit(mode, monkeypatch):
    lib = bvhsim.load()
    tris = _triangles(S.soup(120_000))
    lo, hi = tris.reshape(-1, 3).min(0), tris.reshape(-1, 3).max(0)
    rng = np.random.default_rng(11)
    ext = hi - lo
    rays = np.concatenate([_rays(6000, lo, hi, rng),                      # inside the soup
                           _rays(1500, lo - 2.0 * ext, hi + 2.0 * ext, rng)])  # also far outside
    monkeypatch.setenv("ARK_SIM_BOX", mode)
    out = (C.c_uint64 * 9)()
    rc = lib.ark_ddgi_debug_bvh8_trace_stats(tris.ctypes.data, tris.shape[0], rays.ctypes.data, rays.shape[0], min(8, os.cpu_count() or 8), out, None)
    assert rc == 0
    assert out[0] > 0 and out[2] > 0
    assert out[8] == 0, f"{mode}: {out[8]} children culled that the exact test accepts"


def test_box_check_has_power(monkeypatch):
    """Negative control: the fp16 form without its error bound culls exact hits, and
    the check sees it."""
    lib = bvhsim.load()
    tris = _triangles(S.soup(120_000))
    lo, hi = tris.reshape(-1, 3).min(0), tris.reshape(-1, 3).max(0)
    rays = _rays(6000, lo, hi, np.random.default_rng(11))
    monkeypatch.setenv("ARK_SIM_BOX", "f16s")
    monkeypatch.setenv("ARK_SIM_E_A", "0")
    monkeypatch.setenv("ARK_SIM_E_B", "0")
    out = (C.c_uint64 * 9)()
    assert lib.ark_ddgi_debug_bvh8_trace_stats(tris.ctypes.data, tris.shape[0], rays.ctypes.data, rays.shape[0], 4, out, None) == 0
    assert out[8] > 0


def test_presplit_references_keep_every_hit(monkeypatch):
    """Early split clipping of the BVH2 build (ARK_BVH_PRESPLIT, off by default): the
    clipped references' boxes cover their triangles, so the host traversal finds the
    same number of hits as the plain build."""
    lib = bvhsim.load()
    tris = _triangles(S.soup(60_000))
    lo, hi = tris.reshape(-1, 3).min(0), tris.reshape(-1, 3).max(0)
    rays = _rays(4000, lo, hi, np.random.default_rng(5))
    res = {}
    for ps in (None, "2,4"):
        if ps is None:
            monkeypatch.delenv("ARK_BVH_PRESPLIT", raising=False)
        else:
            monkeypatch.setenv("ARK_BVH_PRESPLIT", ps)
        out = (C.c_uint64 * 9)()
        assert lib.ark_ddgi_debug_bvh8_trace_stats(tris.ctypes.data, tris.shape[0], rays.ctypes.data, rays.shape[0], 4, out, None) == 0
        res[ps] = list(out)
    assert res["2,4"][2] == res[None][2] and res[None][2] > 0  # hits
    assert res["2,4"][8] == 0
    assert res["2,4"][7] > res[None][7]  # more triangle records: references were split
