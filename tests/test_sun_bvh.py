"""The sun's light-space BVH (k_trace_shadow<SUN>, ark_ddgi.cpp set_scene) on the host,
no GPU: built as set_scene builds it, traversed with a restatement of the kernel's
light-space node test (visitNodeSun), against brute force over every triangle with
the same Möller–Trumbore - every sun shadow ray must agree (a disagreement would be a
culled occluder: the light-space test must be conservative). Sun directions include
the reference's default (ShowcaseApp.cpp:122), axis-aligned and nearly axis-aligned
ones; origins lie on the triangles (shadow rays start at hits) and in the volume."""
import ctypes as C

import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import scene as S


def _world_triangles(sc):
    ws = []
    for inst in sc.instances:
        mesh = sc.meshes[inst["rt_mesh_index"]]
        idx = sc.indices[mesh["first_index"]: mesh["first_index"] + 3 * inst["triangle_count"]]
        p = sc.positions[mesh["first_vertex"] + idx.astype(np.int64)]
        M = inst["object_to_world"].reshape(3, 4)
        ws.append((p @ M[:, :3].T + M[:, 3]).reshape(-1, 9))
    return np.ascontiguousarray(np.concatenate(ws), np.float32)


def _origins(tris, n, rng, lo, hi):
    k = n // 2
    pick = rng.integers(0, tris.shape[0], k)
    t = tris[pick].reshape(-1, 3, 3).astype(np.float64)
    r1, r2 = rng.random(k), rng.random(k)
    sq = np.sqrt(r1)
    on = (1 - sq)[:, None] * t[:, 0] + (sq * (1 - r2))[:, None] * t[:, 1] + (sq * r2)[:, None] * t[:, 2]
    vol = lo + (hi - lo) * rng.random((n - k, 3))
    return np.ascontiguousarray(np.concatenate([on, vol]), np.float32)


def _check(tris, sun, n_rays=3000, seed=1):
    lib = abi.load_library()
    rng = np.random.default_rng(seed)
    lo, hi = tris.reshape(-1, 3).min(0), tris.reshape(-1, 3).max(0)
    o = _origins(tris, n_rays, rng, lo, hi)
    d = np.asarray(sun, np.float32)
    out = (C.c_uint64 * 8)()
    rc = lib.ark_ddgi_debug_sun_bvh_check(tris.ctypes.data, tris.shape[0], d.ctypes.data, o.ctypes.data, o.shape[0], 20000.0, out)
    res = {"rays": out[0], "occluded": out[1], "occluded_bvh": out[2], "mismatch": out[3], "visits_per_ray": out[4] / max(1, out[0]),
           "tests_per_ray": out[5] / max(1, out[0]), "nodes": out[6]}
    assert rc == 0 and res["mismatch"] == 0, res
    assert 0 < res["occluded"] < res["rays"], res
    return res


SUNS = [(0.5, -1.0, 0.2), (0.0, -1.0, 0.0), (1.0, 0.0, 0.0), (1e-4, -1.0, 3e-5), (-0.3, -0.2, 0.93), (0.577, 0.577, -0.577)]


@pytest.mark.parametrize("sun", SUNS)
def test_sun_bvh_soup(sun):
    """A 20,000-triangle strip soup (the C4 generator at 1/500 scale)."""
    tris = _world_triangles(S.soup(20_000, extent=8.0))
    r = _check(tris, sun)
    assert r["tests_per_ray"] < 0.05 * tris.shape[0]  # it culls


@pytest.mark.parametrize("sun", SUNS[:3])
def test_sun_bvh_city_block(sun):
    """Instanced boxes + ground (the C5 substitute at test size): axis-aligned faces,
    shared edges, the ground plane under every ray."""
    tris = _world_triangles(S.city_block(300, extent=30.0))
    _check(tris, sun, n_rays=2000)


def test_sun_bvh_far_from_origin():
    """The same soup translated 5,000 m away: the fp32 light coordinates are coarse
    there (ulp 5e-4 m), the box inflation must cover them."""
    tris = _world_triangles(S.soup(5_000, extent=6.0)) + np.float32(5000.0)
    _check(np.ascontiguousarray(tris, np.float32), (0.5, -1.0, 0.2), n_rays=2000)


def _choice(tris, sun):
    lib = abi.load_library()
    sd = np.asarray(sun, np.float32)
    out = (C.c_double * 4)()
    assert lib.ark_ddgi_debug_sun_choice(tris.ctypes.data, tris.shape[0], sd.ctypes.data, 2048, out) == 0
    return list(out)


def test_sun_choice_by_sampled_cost():
    """set_scene keeps the light-space BVH only where sampled sun shadow rays take fewer
    steps through it (sun_bvh_pays): the soup's scattered small triangles gain (rays
    along +w skip the slab tests' misses), the city block's walls and ground - long
    slanted boxes in light space - lose, and its sun rays stay on the world BVH."""
    soup = _world_triangles(S.soup(200_000))
    w, l, chosen, n = _choice(soup, (0.5, -1.0, 0.2))
    assert n == 2048 and chosen == 1.0 and l < 0.9 * w, (w, l)
    city = S.city_block(box_count=20_000)
    w, l, chosen, n = _choice(_world_triangles(city), city.sun[1])
    assert n == 2048 and chosen == 0.0 and l > w, (w, l)
