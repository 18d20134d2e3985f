"""Known-answer tests of the CPU oracle against closed forms derived from the
reference GLSL (the reference ships no golden vectors for this path)."""
import ctypes as C

import numpy as np

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import oracle_lib as O
from parity import make_desc

M32 = 0xFFFFFFFF


def wang_hash_py(seed):  # random.glsl:40-48
    seed = ((seed ^ 61) ^ (seed >> 16)) & M32
    seed = (seed * 9) & M32
    seed = seed ^ (seed >> 4)
    seed = (seed * 0x27D4EB2D) & M32
    return seed ^ (seed >> 15)


def xorshift_py(s):  # random.glsl:25-32
    s ^= (s << 13) & M32
    s ^= s >> 17
    s ^= (s << 5) & M32
    return s


def test_wang_hash_and_xorshift():
    lib = O.load()
    for seed in [0, 1, 61, 512, 512 * 4095 + 511, 0xDEADBEEF, 0xFFFFFFFF] + list(range(1000, 1100)):
        assert lib.oracle_wang_hash(seed) == wang_hash_py(seed)
        assert lib.oracle_rand_xorshift(seed) == xorshift_py(seed)


def test_fp16_rne_matches_numpy_and_half_hpp():
    f = np.load(O.ROOT + "/tests/golden/half_rne.npz")
    x, bits = f["inputs"], f["half_bits"]
    ours = O.f32_to_f16(x)
    nan = np.isnan(x)
    # the reference's half.hpp (round_to_nearest, ties to even)
    assert np.array_equal(ours[~nan], bits[~nan])
    # numpy's float16 cast is IEEE RNE as well
    with np.errstate(over="ignore"):
        assert np.array_equal(ours[~nan], x[~nan].astype(np.float16).view(np.uint16))
    # fp16 clear value of the visibility atlas: zFar^2 = 1e8 overflows to +inf
    assert O.f32_to_f16(np.array([1e8], np.float32))[0] == 0x7C00
    assert O.f32_to_f16(np.array([np.nan], np.float32))[0] == 0x7E00


def test_spherical_fibonacci():
    lib = O.load()
    out = np.zeros(3, np.float32)
    for n in (64, 256, 512):
        for i in (0, 1, n // 3, n - 1):
            lib.oracle_fib(i, n, out.ctypes.data)
            theta = 2 * np.pi * i / 1.618034
            phi = np.arccos(2 * (i / n) - 1)
            ref = np.array([np.cos(theta) * np.sin(phi), np.sin(theta) * np.sin(phi), np.cos(phi)])
            assert np.allclose(out, ref, atol=2e-4), (n, i)


def test_rotated_fibonacci_is_a_rotation():
    lib = O.load()
    n = 128
    a = np.zeros((n, 3), np.float32)
    b = np.zeros((n, 3), np.float32)
    for i in range(n):
        lib.oracle_rotated_fib(77, i, n, 5, a[i].ctypes.data)
        lib.oracle_fib(i, n, b[i].ctypes.data)
    assert np.allclose(np.linalg.norm(a, axis=1), 1, atol=1e-5)
    # a rotation preserves all pairwise angles
    assert np.allclose(a @ a.T, b @ b.T, atol=2e-5)
    # same probe, frame 5 vs frame 5 + 512 -> same seed (frameIdx % 512, ddgi/common.glsl:17-18)
    c = np.zeros(3, np.float32)
    lib.oracle_rotated_fib(77, 3, n, 5 + 512, c.ctypes.data)
    assert np.array_equal(c, a[3])


def test_octahedral_round_trip_at_texel_centres():
    lib = O.load()
    for res in (8, 16):
        for ty in range(res):
            for tx in range(res):
                u, v = (tx + 0.5) / res * 2 - 1, (ty + 0.5) / res * 2 - 1
                d = np.zeros(3, np.float32)
                lib.oracle_oct_decode(np.float32(u), np.float32(v), d.ctypes.data)
                assert abs(np.linalg.norm(d) - 1) < 1e-6
                e = np.zeros(2, np.float32)
                lib.oracle_oct_encode(d.ctypes.data, e.ctypes.data)
                assert int((e[0] * 0.5 + 0.5) * res) == tx and int((e[1] * 0.5 + 0.5) * res) == ty


def test_atlas_texel_coordinates():
    """ddgi/common.glsl:36-67: probe i -> (x = i % X, z = (i % XZ) / X, y = i / XZ);
    tile = (x + y X, z); first texel = 1 + tile * (res + 2)."""
    lib = O.load()
    dims = np.array([4, 3, 5], np.int32)
    out = np.zeros(2, np.int32)
    for i in range(60):
        x, z, y = i % 4, (i % 20) // 4, i // 20
        for res in (8, 16):
            lib.oracle_atlas_texel(dims.ctypes.data, i, 2, 3, res, out.ctypes.data)
            assert tuple(out) == (1 + (x + y * 4) * (res + 2) + 2, 1 + z * (res + 2) + 3)


def _far_triangle_scene():
    # one tiny opaque triangle far outside the grid: every probe ray misses
    P = np.array([[500, 500, 500], [500.1, 500, 500], [500, 500.1, 500]], np.float32)
    vx = np.zeros(3, dtype=S.VERTEX_DTYPE)
    vx["normal"] = (0, 0, 1)
    inst = np.zeros(1, dtype=S.INSTANCE_DTYPE)
    inst[0]["object_to_world"] = np.eye(3, 4, dtype=np.float32).reshape(-1)
    inst[0]["triangle_count"] = 1
    inst[0]["hit_mask"] = abi.ARK_RT_HIT_MASK_OPAQUE
    return S.SceneData(positions=P, vertices=vx, indices=np.arange(3, dtype=np.uint32),
                       meshes=np.array([(0, 0, 0)], dtype=S.MESH_DTYPE),
                       materials=np.array([S.default_material()], dtype=S.MATERIAL_DTYPE), instances=inst)


def test_empty_scene_converges_to_environment():
    """All rays miss: radiance = envMultiplier * env (white) = L; irradiance texels =
    fp16(L^(1/5)) (gamma 5, probeUpdateIrradiance.comp:52-57); visibility =
    (min(zFar, 1.5 s), same^2)."""
    sc = _far_triangle_scene()
    grid = D.ProbeGrid((2, 2, 2), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=8, max_rays_per_probe=64, max_probe_updates=8)
    orc = O.Oracle(make_desc(grid, 10000.0, cfg))
    orc.set_scene(sc)
    L = 0.7
    orc.update(D.frame_params(cfg, grid, D.AppState(0), 0, light_pre_exposure=1.0, environment_brightness=L))
    sf = O.f16_to_f32(orc.read(abi.ARK_DDGI_SURFELS)).reshape(8, 64, 4)
    assert np.all(sf[..., :3] == np.float32(np.float16(L))) and np.all(sf[..., 3] == 10000.0)
    irr = O.f16_to_f32(orc.read(abi.ARK_DDGI_ATLAS_IRRADIANCE)).reshape(2 * 10, 2 * 2 * 10, 4)  # (H = Z*10, W = X*10*Y)
    interior = irr[1:9, 1:9, :3]
    expect = float(np.float16(L)) ** 0.2
    assert np.all(np.abs(interior - expect) <= 2 * 2 ** -11 * expect)
    vis = O.f16_to_f32(orc.read(abi.ARK_DDGI_ATLAS_VISIBILITY)).reshape(2 * 18, 2 * 2 * 18, 2)
    assert np.allclose(vis[1:17, 1:17, 0], 1.5, rtol=1e-3)
    # zFar^2 clear = +inf in fp16, so frame 0's mix(new, inf, 0) = new*1 + inf*0 = NaN
    # (SURVEY App. A-2): the reference's variance channel is NaN after the first update
    assert np.all(np.isnan(vis[1:17, 1:17, 1]))
    # with the saturating clear (65504) the blend is well defined: mean of d^2
    cfg2 = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=8, max_rays_per_probe=64, max_probe_updates=8,
                        clear_overflow_mode=abi.ARK_DDGI_CLEAR_OVERFLOW_MAX_FINITE)
    orc2 = O.Oracle(make_desc(grid, 10000.0, cfg2))
    orc2.set_scene(sc)
    orc2.update(D.frame_params(cfg2, grid, D.AppState(0), 0, light_pre_exposure=1.0, environment_brightness=L))
    vis2 = O.f16_to_f32(orc2.read(abi.ARK_DDGI_ATLAS_VISIBILITY)).reshape(2 * 18, 2 * 2 * 18, 2)
    assert np.allclose(vis2[1:17, 1:17, 1], 2.25, rtol=2e-3)


def _cube_scene(inward: bool, emissive: float):
    """Unit cube around the origin; faces CCW seen from inside (inward) or outside."""
    v = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], np.float32)
    quads = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    tris = []
    for q in quads:
        a, b, c, d = q
        for t in ((a, b, c), (a, c, d)):
            p = v[list(t)]
            n = np.cross(p[1] - p[0], p[2] - p[0])
            outward = np.dot(n, p.mean(0)) > 0
            if outward == inward:
                t = (t[0], t[2], t[1])
            tris.append(t)
    idx = np.array(tris, np.uint32).reshape(-1)
    vx = np.zeros(8, dtype=S.VERTEX_DTYPE)
    vx["normal"] = -v / np.linalg.norm(v, axis=1, keepdims=True) if inward else v / np.linalg.norm(v, axis=1, keepdims=True)
    m = S.default_material()
    m["color_tint"] = (0, 0, 0, 1)
    m["emissive_factor"] = (emissive, emissive, emissive)
    inst = np.zeros(1, dtype=S.INSTANCE_DTYPE)
    inst[0]["object_to_world"] = np.eye(3, 4, dtype=np.float32).reshape(-1)
    inst[0]["triangle_count"] = 12
    inst[0]["hit_mask"] = abi.ARK_RT_HIT_MASK_OPAQUE
    return S.SceneData(positions=v, vertices=vx, indices=idx, meshes=np.array([(0, 0, 0)], dtype=S.MESH_DTYPE),
                       materials=np.array([m], dtype=S.MATERIAL_DTYPE), instances=inst)


def _cube_t(dirs):
    return 1.0 / np.max(np.abs(dirs), axis=1)


def _probe_dirs(n, frame=0):
    lib = O.load()
    d = np.zeros((n, 3), np.float32)
    for i in range(n):
        lib.oracle_rotated_fib(0, i, n, frame, d[i].ctypes.data)
    return d


def test_inside_emissive_cube_front_faces():
    """Probe at the centre of a cube facing inwards with emissive 1, black albedo:
    every ray hits a front face at t = 1/max|d| (radiance = emissive exactly)."""
    sc = _cube_scene(inward=True, emissive=1.0)
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=1, max_rays_per_probe=64, max_probe_updates=1, compute_probe_offsets=False)
    orc = O.Oracle(make_desc(grid, 10000.0, cfg))
    orc.set_scene(sc)
    orc.update(D.frame_params(cfg, grid, D.AppState(0), 0))
    sf = O.f16_to_f32(orc.read(abi.ARK_DDGI_SURFELS)).reshape(64, 4)
    assert np.all(sf[:, :3] == 1.0)
    t = _cube_t(_probe_dirs(64))
    assert np.allclose(sf[:, 3], t, rtol=2e-3)


def test_inside_outward_cube_all_backfaces():
    """Faces CCW seen from outside: from the centre every hit is a backface ->
    radiance 0 and depth * 0.2 (raygen.rgen:129-134), stored negative."""
    sc = _cube_scene(inward=False, emissive=1.0)
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=1, max_rays_per_probe=64, max_probe_updates=1, compute_probe_offsets=True)
    orc = O.Oracle(make_desc(grid, 10000.0, cfg))
    orc.set_scene(sc)
    orc.update(D.frame_params(cfg, grid, D.AppState(0), 0))
    sf = O.f16_to_f32(orc.read(abi.ARK_DDGI_SURFELS)).reshape(64, 4)
    assert np.all(sf[:, :3] == 0.0)
    t = _cube_t(_probe_dirs(64))
    assert np.allclose(sf[:, 3], -0.2 * t, rtol=2e-3)
    # >= 25 % backfaces: the offset steps 0.125 towards the mean backface direction
    # (probeUpdateOffset.comp:58-65), then the exponential lerp (:80-81)
    off = orc.read(abi.ARK_DDGI_PROBE_OFFSETS)[:3]
    d = _probe_dirs(64)
    step = d.sum(0) / np.linalg.norm(d.sum(0)) * 0.125
    lerp = 2.0 ** (-10.0 / 60.0)
    assert np.allclose(off, step * (1 - lerp), rtol=1e-3, atol=1e-6)


def test_hysteresis_blend():
    """frame 1 blends new and old with hysteresis (mix(new, old, h))."""
    sc = _far_triangle_scene()
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=32, probe_updates_per_frame=1, max_rays_per_probe=32, max_probe_updates=1, compute_probe_offsets=False)
    orc = O.Oracle(make_desc(grid, 10000.0, cfg))
    orc.set_scene(sc)
    orc.update(D.frame_params(cfg, grid, D.AppState(0), 0, environment_brightness=1.0))
    a = O.f16_to_f32(orc.read(abi.ARK_DDGI_ATLAS_IRRADIANCE)).reshape(10, 10, 4)[5, 5, 0]
    orc.update(D.frame_params(cfg, grid, D.AppState(1), 0, environment_brightness=0.0))
    b = O.f16_to_f32(orc.read(abi.ARK_DDGI_ATLAS_IRRADIANCE)).reshape(10, 10, 4)[5, 5, 0]
    assert a == np.float32(np.float16(1.0)) and abs(b - 0.93 * a) < 1e-3


def test_octahedral_texel_orbits_are_exact():
    """The probe-update kernel (csrc/ddgi_update.hip) evaluates each orbit
    {t, x-mirror t', antipode -t, -t'} of tile texels from one decoded direction:
    the quadrant texel (qx, qy) has the orbit (res-1-qx, qy), (qy+h, qx+h),
    (h-1-qy, qx+h), h = res/2. Pin that the decoded directions are exact sign
    flips of each other (z = 0 texels: the antipode's z is +0 as well) and that
    the orbits partition the tile."""
    lib = O.load()

    def dec(res, tx, ty):
        d = np.zeros(3, np.float32)
        lib.oracle_oct_decode(np.float32((tx + 0.5) / res * 2 - 1), np.float32((ty + 0.5) / res * 2 - 1), d.ctypes.data)
        return d

    for res in (8, 16):
        h = res // 2
        seen = set()
        for qy in range(h):
            for qx in range(h):
                orbit = [(qx, qy), (res - 1 - qx, qy), (qy + h, qx + h), (h - 1 - qy, qx + h)]
                seen.update(orbit)
                t, tm, ta, tam = (dec(res, *o) for o in orbit)
                assert np.array_equal(tm.view(np.uint32), np.array([-t[0], t[1], t[2]], np.float32).view(np.uint32))
                want_a = np.array([-t[0], -t[1], -t[2] if t[2] != 0 else 0.0], np.float32)
                want_am = np.array([t[0], -t[1], -t[2] if t[2] != 0 else 0.0], np.float32)
                assert np.array_equal(ta.view(np.uint32), want_a.view(np.uint32))
                assert np.array_equal(tam.view(np.uint32), want_am.view(np.uint32))
        assert len(seen) == res * res
