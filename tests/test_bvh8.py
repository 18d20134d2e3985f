"""Host-side check of the 8-wide quantized BVH that ark_ddgi_set_scene uploads
(bvh_builder.cpp): exact fp32 plane decode, conservative (outward) quantization,
every triangle in exactly one leaf. No GPU."""
import ctypes as C

import numpy as np
import pytest

from arkoserenderer_amd import abi


def check(tris, sah_optimal=None, tri_cost=0.0):
    """set_scene's build (sah_optimal None), or the _opts build for comparing collapses."""
    lib = abi.load_library()
    tris = np.ascontiguousarray(tris, dtype=np.float32).reshape(-1, 9)
    out = (C.c_uint64 * 8)()
    if sah_optimal is None:
        rc = lib.ark_ddgi_debug_bvh8_check(tris.ctypes.data, tris.shape[0], out)
    else:
        rc = lib.ark_ddgi_debug_bvh8_check_opts(tris.ctypes.data, tris.shape[0], int(sah_optimal), float(tri_cost), out)
    return rc, list(out)


def test_soup_bvh8_structure():
    rng = np.random.default_rng(7)
    n = 20000
    v0 = rng.uniform(-31, 31, (n, 3)).astype(np.float32)
    tris = np.concatenate([v0, v0 + rng.uniform(-0.3, 0.3, (n, 3)), v0 + rng.uniform(-0.3, 0.3, (n, 3))], axis=1)
    rc, out = check(tris)
    nodes, leaves, depth, violations, ntris, nodes2, internal, _ = out
    assert rc == 0 and violations == 0
    assert ntris == n
    assert internal == nodes - 1          # every node but the root is some node's internal child
    assert depth <= 12
    assert (leaves + internal) / nodes > 3  # wide nodes: several children on average


@pytest.mark.parametrize("case", ["single", "degenerate", "far", "tiny_far", "coplanar"])
def test_bvh8_edge_cases(case):
    rng = np.random.default_rng(3)
    if case == "single":
        tris = np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0]], np.float32)
    elif case == "degenerate":  # zero-area triangles and repeated points (zero-extent boxes)
        p = rng.uniform(-1, 1, (300, 3)).astype(np.float32)
        tris = np.concatenate([p, p, p], axis=1)
    elif case == "far":  # far from the origin: plane anchors need coarse grids
        v0 = rng.uniform(1e5, 1e5 + 10, (500, 3)).astype(np.float32)
        tris = np.concatenate([v0, v0 + 0.5, v0 + np.float32([0.5, 0, 0.25])], axis=1)
    elif case == "tiny_far":  # boxes far smaller than one ulp step of their position
        v0 = np.full((64, 3), 3.0e6, np.float32) + rng.integers(0, 4, (64, 3)).astype(np.float32)
        tris = np.concatenate([v0, v0, v0], axis=1)
    else:
        xy = rng.uniform(-5, 5, (2000, 2)).astype(np.float32)
        z = np.zeros((2000, 1), np.float32)
        v0 = np.concatenate([xy, z], axis=1)
        tris = np.concatenate([v0, v0 + np.float32([0.1, 0, 0]), v0 + np.float32([0, 0.1, 0])], axis=1)
    rc, out = check(tris)
    assert rc == 0 and out[3] == 0, out
    assert out[4] == tris.shape[0]



@pytest.mark.parametrize("tri_cost", [1.0, 0.3])
def test_sah_optimal_collapse(tri_cost):
    """The SAH-optimal BVH2 -> BVH8 child selection (Ylitie et al. 2017 dynamic
    programming, set_scene's choice, bvh_builder.cpp planCollapse) keeps every
    structural invariant and never costs more SAH than the greedy largest-area
    opening on the same BVH2 (it also fills nodes: fewer of them)."""
    rng = np.random.default_rng(11)
    n = 30000
    v0 = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    tris = np.concatenate([v0, v0 + rng.uniform(-0.4, 0.4, (n, 3)), v0 + rng.uniform(-0.4, 0.4, (n, 3))], axis=1)
    rc_g, g = check(tris, sah_optimal=False, tri_cost=tri_cost)
    rc_s, s = check(tris, sah_optimal=True, tri_cost=tri_cost)
    assert rc_g == 0 and rc_s == 0 and g[3] == 0 and s[3] == 0
    assert s[4] == n and s[6] == s[0] - 1
    assert s[7] <= g[7], (s[7], g[7])   # SAH cost x 1e6
    assert s[0] < g[0]                  # fuller nodes
