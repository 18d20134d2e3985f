"""The C-ABI library loads and exports every symbol the headers declare; the
ctypes mirror matches the C struct layouts. No GPU calls."""
import ctypes as C
import os
import re

import numpy as np

from arkoserenderer_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in ("ark_ddgi.h", "ark_scene.h", "ark_ddgi_debug.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(ark_[a-z0-9_]+)\s*\(", src))
    return names


def test_library_loads_and_exports_every_declared_symbol():
    lib = abi.load_library()
    decl = declared_functions()
    assert len(decl) >= 20
    missing = [n for n in sorted(decl) if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes table covers the whole declared surface
    assert decl <= set(abi.EXPORTS), sorted(decl - set(abi.EXPORTS))


def test_abi_version():
    assert abi.load_library().ark_ddgi_abi_version() == 1


def test_struct_layouts_match_c():
    lib = abi.load_library()
    n = len(abi.ABI_STRUCTS)
    out = (C.c_uint32 * n)()
    assert lib.ark_ddgi_debug_struct_sizes(out, n) == n
    for s, size in zip(abi.ABI_STRUCTS, out):
        assert C.sizeof(s) == size, (s.__name__, C.sizeof(s), size)
    # reference layouts: RTVertex 36 B scalar (RTData.h:9-13), ShaderMaterial 96 B std430 (MaterialData.h:8-33)
    assert C.sizeof(abi.ArkRTVertex) == 36
    assert C.sizeof(abi.ArkShaderMaterial) == 96
    assert C.sizeof(abi.ArkRTTriangleMesh) == 12


def test_invalid_arguments_fail_cleanly():
    lib = abi.load_library()
    h = C.c_void_p()
    assert lib.ark_ddgi_create(None, C.byref(h)) == -1
    d = abi.ArkDdgiDesc()
    d.struct_size = C.sizeof(d)  # empty grid -> no probe grid (DDGINode.cpp:39-42)
    assert lib.ark_ddgi_create(C.byref(d), C.byref(h)) == -2
    d.struct_size = 3
    assert lib.ark_ddgi_create(C.byref(d), C.byref(h)) == -1
    assert lib.ark_ddgi_update(None, None, None) == -1
    # the Z-slab exchange sequencing entry points (no device work without a context)
    assert lib.ark_ddgi_update_exchanged(None, None, None) == -1
    assert lib.ark_ddgi_exchange_begin(None, None) == -1
    assert lib.ark_ddgi_exchange_end(None, None) == -1
    assert lib.ark_ddgi_synchronize(None) == -1
    assert lib.ark_ddgi_last_error(None) == b"null context"


def test_soup_generator_deterministic():
    from arkoserenderer_amd import scene as S

    a = S.soup(16_000, extent=5.0)
    b = S.soup(16_000, extent=5.0)
    assert a.triangle_count == 16_000 and a.positions.shape == (18_000, 3)
    assert np.array_equal(a.positions, b.positions) and np.array_equal(a.indices, b.indices)
    c = S.soup(16_000, extent=5.0, seed=7)
    assert not np.array_equal(a.positions, c.positions)
    # strip normals are the CCW geometric normals of their triangles
    m = a.meshes[0]
    idx = a.indices[m["first_index"]: m["first_index"] + 3].astype(np.int64) + m["first_vertex"]
    p = a.positions[idx]
    ng = np.cross(p[1] - p[0], p[2] - p[0])
    ng /= np.linalg.norm(ng)
    assert np.allclose(ng, a.vertices["normal"][idx[0]], atol=1e-5)
    lo, hi = a.bounds()
    assert (lo > -3).all() and (hi < 8).all()
