"""Per-frame scene inputs through the C-ABI (VERDICT r04 "do this" #1).

The reference re-uploads its lights every frame with the camera's current
pre-exposure (GpuScene.cpp:790-858) and updates + rebuilds the TLAS from the
instances' current transforms (:872-1009). ark_ddgi_set_lights / _set_instances carry
both into a context between updates; the oracle is fed the same inputs
(oracle_set_lights / oracle_set_instances). Bar: bit-exact surfels, atlases and
offsets every frame, also with frames in flight (no host sync between an update and
the next frame's set_lights).
"""
import os

import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import oracle_lib as O
import scenes
from parity import RESOURCES, diff_report

pytestmark = pytest.mark.gpu

GRID = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))


def _cfg(R=128, K=144):
    return D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=K, compute_probe_offsets=True,
                        max_rays_per_probe=R, max_probe_updates=144)


def _compare(ctx, orc, frame, what):
    for k, w in RESOURCES.items():
        r = diff_report(k, ctx.read(w), orc.read(w))
        assert r["mismatch"] == 0, f"frame {frame} ({what}): {r}"


def _sun_mode(value):
    """ArkDdgiDesc.sun_bvh of a test's contexts: "1" the light-space BVH whenever there is
    a sun, "0" the world BVHs."""
    return abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE if value == "1" else abi.ARK_DDGI_SUN_BVH_WORLD


def _scaled_lights(sc, pre, spots=None):
    spots = sc.spots if spots is None else spots
    sun = None if sc.sun is None else (tuple(np.float32(c) * np.float32(pre) for c in sc.sun[0]), sc.sun[1])
    out = [S.SpotLight(tuple(np.float32(c) * np.float32(pre) for c in s.color), s.direction, s.right, s.up, s.position,
                       s.outer_cone_half_angle, s.ies_profile_index) for s in spots]
    return sun, out


def _rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float32)


@pytest.mark.parametrize("sun_bvh,sync", [("1", True), ("0", True), ("1", False)])
def test_lights_per_frame_exposure_spots_sun(sun_bvh, sync):
    """Frame 1: camera exposure 1 -> 1.7 (every light colour and the ambient term
    re-pre-exposed); frame 2: a spot moves and turns; frame 3: the sun rotates (the
    light-space sun BVH no longer serves it: the world BVHs do, while a new one is
    built in the background); frame 4: the sun back (whichever light-space BVH is
    installed by then, or the world BVHs), one spot removed; frame 5: three spots (the shadow-ray
    list grows); frame 6: no sun. Bit-exact against the oracle after every frame, or
    (sync = False) with all seven frames and their light changes queued back to back
    and the atlases compared at the end."""
    sc = scenes.features_scene()
    cfg = _cfg()
    cfg.sun_bvh = _sun_mode(sun_bvh)
    ctx = D.DDGIContext(GRID, 100.0, cfg)
    ctx.set_scene(sc)
    stats = ctx.bvh_stats()
    if sun_bvh == "1":
        assert stats.sun_node_count > 0
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    sun0 = sc.sun
    turned = tuple(float(x) for x in (np.array([-0.5, -0.8, 0.3]) / np.linalg.norm([-0.5, -0.8, 0.3])))
    moved_spot = S.SpotLight((30.0, 25.0, 20.0), (0.28, -0.96, 0.0), (0.96, 0.28, 0.0), (0.0, 0.0, 1.0), (0.4, 2.7, -0.5), 0.7, 2)
    extra = S.SpotLight((5.0, 5.0, 9.0), (0.0, -0.6, -0.8), (1.0, 0.0, 0.0), (0.0, 0.8, -0.6), (0.5, 2.0, 1.5), 0.5, -1)
    plan = [
        (1.0, sun0, sc.spots),
        (1.7, sun0, sc.spots),
        (1.7, sun0, [moved_spot, sc.spots[1]]),
        (1.7, (sun0[0], turned), [moved_spot, sc.spots[1]]),
        (1.2, sun0, [moved_spot]),
        (1.2, sun0, [moved_spot, sc.spots[1], extra]),
        (1.2, None, [moved_spot, sc.spots[1], extra]),
    ]
    idx = 0
    for f, (pre, sun, spots) in enumerate(plan):
        base = S.SceneData(**{**sc.__dict__, "sun": sun})
        lsun, lspots = _scaled_lights(base, pre, spots)
        if f > 0:
            ctx.set_lights(lsun, lspots)
        orc.set_lights(lsun, lspots)
        p = D.frame_params(cfg, GRID, D.AppState(f), idx, light_pre_exposure=pre, ambient_illuminance=0.05,
                           environment_brightness=0.5)
        ctx.update(p)
        orc.update(p)
        if sync or f == len(plan) - 1:
            ctx.synchronize()
            _compare(ctx, orc, f, f"exposure {pre}, sun {'on' if sun else 'off'}, {len(spots)} spots")
        idx = (idx + p.probe_updates) % GRID.probe_count()
    ctx.close()


def test_set_lights_rejects_bad_input():
    sc = scenes.features_scene()
    ctx = D.DDGIContext(GRID, 100.0, _cfg(32, 144))
    with pytest.raises(abi.ArkDdgiError):
        ctx.set_lights(sc.sun, [sc.spots[0]] * (abi.ARK_DDGI_MAX_SPOT_LIGHTS + 1))  # no scene yet
    ctx.set_scene(sc)
    with pytest.raises(abi.ArkDdgiError):
        ctx.set_lights(sc.sun, [sc.spots[0]] * (abi.ARK_DDGI_MAX_SPOT_LIGHTS + 1))
    ctx.set_lights(sc.sun, [sc.spots[0]] * abi.ARK_DDGI_MAX_SPOT_LIGHTS)
    ctx.close()


@pytest.mark.parametrize("sun_bvh", ["1", "0"])
def test_instances_per_frame_refit(sun_bvh):
    """Frames 1-3 move instances between updates: the box turns and slides, the
    mirrored box loses its mirroring (facing flips), the masked quads move up, the
    whole room shifts; the refitted BVH gives the oracle's hits bit for bit (the oracle
    rebuilds its own BVH from the same transforms)."""
    sc = scenes.features_scene()
    cfg = _cfg()
    cfg.sun_bvh = _sun_mode(sun_bvh)
    ctx = D.DDGIContext(GRID, 100.0, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    inst0 = sc.instances.copy()

    def moved(f):
        inst = inst0.copy()
        M = inst["object_to_world"].reshape(-1, 3, 4).copy()
        if f >= 1:  # box (instance 3): turn about y and slide
            M[3, :, :3] = _rot_y(0.35 * f) @ M[3, :, :3]
            M[3, :, 3] += np.float32(0.15 * f)
        if f >= 2:  # mirrored box (instance 4) loses its mirroring; masked quads (1) rise
            M[4, :, :3] = np.diag([1.0, 1.2, 1.0]).astype(np.float32)
            M[1, 1, 3] += np.float32(0.3)
        if f >= 3:  # the room (0) and the translucent quad (2) shift
            M[0, :, 3] += np.array([0.05, -0.02, 0.1], np.float32)
            M[2, :, :3] = _rot_y(0.5) @ M[2, :, :3]
        inst["object_to_world"] = M.reshape(len(inst), 12)
        return inst

    idx = 0
    for f in range(4):
        if f > 0:
            inst = moved(f)
            ctx.set_instances(inst)
            orc.set_instances(inst)
            # the light-space BVH is refitted with the world BVHs (not dropped)
            assert (ctx.bvh_stats().sun_node_count > 0) == (sun_bvh == "1")
            assert ctx.bvh_stats().refit_ms > 0
        p = D.frame_params(cfg, GRID, D.AppState(f), idx, light_pre_exposure=1.0, ambient_illuminance=0.05,
                           environment_brightness=0.5)
        ctx.update(p)
        orc.update(p)
        ctx.synchronize()
        _compare(ctx, orc, f, "instances moved" if f else "initial")
        idx = (idx + p.probe_updates) % GRID.probe_count()
    # a changed topology is refused and leaves the context as it was
    bad = moved(3)
    bad["triangle_count"][0] -= 1
    with pytest.raises(abi.ArkDdgiError):
        ctx.set_instances(bad)
    p = D.frame_params(cfg, GRID, D.AppState(4), idx, light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
    ctx.update(p)
    orc.update(p)
    ctx.synchronize()
    _compare(ctx, orc, 4, "after a refused set_instances")
    ctx.close()


def test_soup_lights_and_instances_every_frame():
    """A C4-like soup (64 k triangles in 16 scene-spanning instances, light-space sun
    BVH forced): every frame a new exposure, a turned sun and all instances moved,
    window K < N with offsets, 4 frames. Bit-exact against the oracle."""
    sc = S.soup(64_000, extent=7.0)
    grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=300, compute_probe_offsets=True,
                       max_rays_per_probe=128, max_probe_updates=512)
    cfg.sun_bvh = _sun_mode("1")
    ctx = D.DDGIContext(grid, 10000.0, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    inst0 = sc.instances.copy()
    idx = 0
    for f in range(4):
        pre = 1.0 + 0.25 * f
        d = np.array([0.5 + 0.2 * f, -1.0, 0.2 - 0.1 * f], np.float32)
        sun = (tuple(np.float32(3.0) * np.float32(pre) for _ in range(3)), tuple(float(x) for x in d / np.linalg.norm(d)))
        ctx.set_lights(sun, [])
        orc.set_lights(sun, [])
        if f > 0:
            inst = inst0.copy()
            M = inst["object_to_world"].reshape(-1, 3, 4).copy()
            for i in range(len(inst)):
                M[i, :, 3] += np.array([0.03 * f * ((i % 3) - 1), 0.02 * f, -0.01 * f * (i % 2)], np.float32)
            inst["object_to_world"] = M.reshape(len(inst), 12)
            ctx.set_instances(inst)
            orc.set_instances(inst)
        p = D.frame_params(cfg, grid, D.AppState(f), idx, light_pre_exposure=pre, environment_brightness=1.0)
        ctx.update(p)
        orc.update(p)
        ctx.synchronize()
        _compare(ctx, orc, f, f"soup frame {f}")
        idx = (idx + p.probe_updates) % grid.probe_count()
    ctx.close()


def test_shared_scene_refit_reaches_every_context():
    """Two Z-slab contexts share one scene (ark_ddgi_share_scene); a refit through one
    of them is seen by the other's next update (its kernel view re-derived, the dropped
    light-space sun BVH never dereferenced)."""
    sc = scenes.features_scene()
    cfg = _cfg(64, 144)
    cfg.sun_bvh = _sun_mode("1")
    a = D.DDGIContext(GRID, 100.0, cfg, shard_rank=0, shard_count=2)
    b = D.DDGIContext(GRID, 100.0, cfg, shard_rank=1, shard_count=2)
    a.set_scene(sc)
    b.share_scene(a)
    ref = D.DDGIContext(GRID, 100.0, cfg)
    ref.set_scene(sc)
    inst = sc.instances.copy()
    M = inst["object_to_world"].reshape(-1, 3, 4).copy()
    M[3, :, 3] += np.float32(0.4)
    inst["object_to_world"] = M.reshape(len(inst), 12)
    # b derived its kernel view (with the light-space sun BVH) at share_scene; the refit
    # through a drops that BVH; b's first update must see the refitted scene
    a.set_instances(inst)
    ref.set_instances(inst)
    p0 = D.frame_params(cfg, GRID, D.AppState(0), 0, light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
    for c in (b, ref):
        c.update(p0)
        c.synchronize()
    # slab 1's surfels are the unsharded context's slab-1 probes (compacted slots)
    half = GRID.grid_dimensions[2] // 2
    probes = [i for i in range(GRID.probe_count()) if (i % (6 * 6)) // 6 >= half]
    R = cfg.rays_per_probe
    sb = b.read(abi.ARK_DDGI_SURFELS).reshape(cfg.max_probe_updates, cfg.max_rays_per_probe, 4)
    sr = ref.read(abi.ARK_DDGI_SURFELS).reshape(cfg.max_probe_updates, cfg.max_rays_per_probe, 4)
    assert np.array_equal(sb[: len(probes), :R], sr[probes, :R])
    for c in (a, b, ref):
        c.close()


@pytest.mark.parametrize("cause", ["direction", "refit"])
def test_sun_bvh_rebuilt_in_background(cause):
    """The light-space sun BVH follows the sun: after a sun-direction change (or a refit,
    whose records it no longer holds) the sun's shadow rays traverse the world BVHs
    while a host thread builds a new light-space BVH from the device's triangle records;
    the next update after it is done installs it (ArkDdgiBvhStats.sun_rebuilds). Every
    frame bit-exact against the oracle, before, during and after the rebuild."""
    import time

    sc = S.soup(64_000, extent=7.0)
    grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=512)
    cfg.sun_bvh = _sun_mode("1")
    ctx = D.DDGIContext(grid, 10000.0, cfg)
    ctx.set_scene(sc)
    assert ctx.bvh_stats().sun_node_count > 0
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    exposure = dict(light_pre_exposure=1.0, environment_brightness=1.0)
    try:
        f, installed_at = 0, None
        t0 = time.time()
        while installed_at is None or f < installed_at + 2:
            if f == 1:
                if cause == "direction":
                    d = np.array([0.3, -1.0, -0.4], np.float32)
                    sun = (sc.sun[0], tuple(float(x) for x in d / np.linalg.norm(d)))
                    ctx.set_lights(sun, ())
                    orc.set_lights(sun, ())
                else:
                    inst = sc.instances.copy()
                    inst["object_to_world"][3, 3] += 0.25
                    ctx.set_instances(inst)
                    orc.set_instances(inst)
                    assert ctx.bvh_stats().sun_node_count > 0  # refitted with the world BVHs, then rebuilt
            p = D.frame_params(cfg, grid, D.AppState(f), 0, **exposure)
            ctx.update(p)
            orc.update(p)
            ctx.synchronize()
            _compare(ctx, orc, f, f"sun BVH rebuild after a {cause}")
            st = ctx.bvh_stats()
            if installed_at is None and st.sun_rebuilds > 0:
                installed_at = f
                assert st.sun_node_count > 0 and st.max_depth >= st.sun_max_depth
            f += 1
            assert time.time() - t0 < 90, "no light-space BVH rebuilt within 90 s"
            if installed_at is None:
                time.sleep(0.05)
        assert installed_at is not None and installed_at >= 1
    finally:
        ctx.close()
        orc.close()


def test_close_during_sun_bvh_rebuild():
    """A context closed while its scene's light-space BVH is being rebuilt in the
    background: the scene's destructor joins the thread before it frees the triangle
    records the thread reads (no crash, no hang); a context sharing the scene keeps it
    and installs the rebuild at its next update."""
    import time

    sc = S.soup(256_000, extent=9.0)
    grid = D.ProbeGrid((6, 6, 6), (1.5, 1.5, 1.5), (0.5, 0.5, 0.5))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=216, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=216)
    cfg.sun_bvh = _sun_mode("1")
    a = D.DDGIContext(grid, 10000.0, cfg)
    b = D.DDGIContext(grid, 10000.0, cfg)
    a.set_scene(sc)
    b.share_scene(a)
    d = np.array([0.2, -1.0, 0.5], np.float32)
    sun = (sc.sun[0], tuple(float(x) for x in d / np.linalg.norm(d)))
    a.set_lights(sun, ())  # starts the rebuild on the shared scene
    b.set_lights(sun, ())
    a.close()
    p = D.frame_params(cfg, grid, D.AppState(0), 0, light_pre_exposure=1.0, environment_brightness=1.0)
    t0 = time.time()
    while b.bvh_stats().sun_rebuilds == 0:
        assert time.time() - t0 < 90, "the shared scene's rebuild was never installed"
        b.update(p)
        b.synchronize()
        time.sleep(0.05)
    assert b.bvh_stats().sun_node_count > 0
    b.close()
    # and a context closed with its rebuild still running, nothing sharing it
    cfg.sun_bvh = _sun_mode("1")
    c = D.DDGIContext(grid, 10000.0, cfg)
    c.set_scene(sc)
    c.set_lights(sun, ())
    c.set_lights(sun, ())  # the second request for the same sun starts the rebuild
    c.close()


def test_continuous_motion_installs_rebuilds():
    """VERDICT r05 "do this" #3: an instance moves every frame, its refit enqueued on the
    update's stream (ark_ddgi_set_instances_async: no host wait). Refits loosen the
    BVHs; host threads rebuild the world BVHs and the light-space sun BVH from device
    snapshots of the refitted records, and updates install them while the motion goes
    on - refitted forward over the frames that came in meanwhile. Every frame bit-exact
    against the oracle (fed the same transforms), before, across and after the
    installs; both rebuilds are installed at least once."""
    import time

    import torch

    sc = S.soup(64_000, extent=7.0)
    grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=200, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=200, sun_bvh=abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE)
    ctx = D.DDGIContext(grid, 10000.0, cfg)
    ctx.set_scene(sc)
    assert ctx.bvh_stats().sun_node_count > 0
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    stream = torch.cuda.Stream()
    exposure = dict(light_pre_exposure=1.0, environment_brightness=1.0)
    inst0 = sc.instances.copy()
    first, f, t0 = 0, 0, time.time()
    try:
        while True:
            inst = inst0.copy()
            M = inst["object_to_world"].reshape(-1, 3, 4).copy()
            M[f % len(inst), :, 3] += np.float32(0.02 * (f + 1))  # one instance a frame, each further each time
            M[1, :, :3] = _rot_y(0.05 * f) @ M[1, :, :3]
            inst["object_to_world"] = M.reshape(len(inst), 12)
            ctx.set_instances_async(inst, stream.cuda_stream)
            orc.set_instances(inst)
            p = D.frame_params(cfg, grid, D.AppState(f), first, **exposure)
            ctx.update(p, stream.cuda_stream)
            orc.update(p)
            ctx.synchronize()
            _compare(ctx, orc, f, "continuous motion")
            st = ctx.bvh_stats()
            first = (first + p.probe_updates) % grid.probe_count()
            f += 1
            if st.bvh_rebuilds >= 2 and st.sun_rebuilds >= 1:
                break
            assert time.time() - t0 < 120, (f"rebuilds not installed within 120 s (world {st.bvh_rebuilds}, failed {st.bvh_rebuild_failures}; "
                                                 f"sun {st.sun_rebuilds}, failed {st.sun_rebuild_failures})")
        assert st.refit_version == f and st.sun_node_count > 0
        print(f"continuous motion: {f} frames, world rebuilds {st.bvh_rebuilds} ({st.bvh_rebuild_ms:.1f} ms), sun rebuilds {st.sun_rebuilds}")
    finally:
        ctx.close()
        orc.close()


def test_partial_refits_equal_full_refit():
    """Refits reach only the nodes with a moved instance below them (node instance masks,
    the back copy brought from its own transforms): after a sequence of moves - one
    instance, then another, one back, a mirrored one, and a pause - the geometry the
    kernels read (world and light-space BVH nodes and records) is byte-identical to a
    context that refits every node once to the final transforms (no background rebuilds:
    the topology stays)."""
    sc = S.soup(64_000, extent=7.0)
    grid = D.ProbeGrid((4, 4, 4), (2.0, 2.0, 2.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=32, probe_updates_per_frame=64, max_rays_per_probe=32, max_probe_updates=64,
                       sun_bvh=abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE, background_rebuild=False)
    a = D.DDGIContext(grid, 10000.0, cfg)
    a.set_scene(sc)
    inst = sc.instances.copy()
    M = inst["object_to_world"].reshape(-1, 3, 4)
    p = D.frame_params(cfg, grid, D.AppState(0), 0, light_pre_exposure=1.0, environment_brightness=1.0)
    moves = [(3, 0.1), (5, -0.2), (3, -0.1), (7, 0.05), (None, 0.0), (5, 0.3), (9, 0.0)]
    for f, (i, dx) in enumerate(moves):
        if i == 9:
            M[i, :, 0] *= -1.0  # mirrored
        elif i is not None:
            M[i, 1, 3] += np.float32(dx)
        inst["object_to_world"] = M.reshape(-1, 12)
        a.set_instances(inst)
        a.update(p)
    a.synchronize()
    b = D.DDGIContext(grid, 10000.0, cfg)
    b.set_scene(sc)
    b.set_instances(inst)
    b.synchronize()
    da, db = a.scene_digest(), b.scene_digest()
    assert da[2] != 0, "no light-space sun BVH"
    assert da == db, (da, db)
    a.close()
    b.close()


def test_motion_frames_in_flight_unsynchronized():
    """Refits overlapping the frames in flight (the double-buffered geometry of
    ark_ddgi_set_instances_async): 48 frames, each moving instances and updating on one
    stream with no host wait in between - frame n's refit writes the back copy while
    frame n - 1 still traces and shades the front one, and background rebuilds install
    on the way - then the atlases and offsets against the oracle fed the same sequence.
    Any frame that read a half-refitted copy, or a refit that overwrote geometry a frame
    still read, shows in the final atlases (each frame blends into them)."""
    import torch

    sc = S.soup(64_000, extent=7.0)
    grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=300, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=300, sun_bvh=abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE)
    ctx = D.DDGIContext(grid, 10000.0, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    stream = torch.cuda.Stream()
    exposure = dict(light_pre_exposure=1.0, environment_brightness=1.0)
    inst0 = sc.instances.copy()
    first = 0
    try:
        for f in range(48):
            inst = inst0.copy()
            M = inst["object_to_world"].reshape(-1, 3, 4).copy()
            M[f % len(inst), :, 3] += np.float32(0.05 * ((f % 5) + 1))
            M[2, :, :3] = _rot_y(0.03 * f) @ M[2, :, :3]
            inst["object_to_world"] = M.reshape(len(inst), 12)
            ctx.set_instances_async(inst, stream.cuda_stream)
            orc.set_instances(inst)
            p = D.frame_params(cfg, grid, D.AppState(f), first, **exposure)
            ctx.update(p, stream.cuda_stream)
            orc.update(p)
            first = (first + p.probe_updates) % grid.probe_count()
        stream.synchronize()
        ctx.synchronize()
        _compare(ctx, orc, 47, "48 frames in flight with a refit each")
        st = ctx.bvh_stats()
        assert st.refit_version == 48
        print(f"frames in flight: world rebuilds {st.bvh_rebuilds}, sun rebuilds {st.sun_rebuilds}")
    finally:
        ctx.close()
        orc.close()


def _install_sun_on_a(a, b, sc, grid, cfg, exposure, sun):
    """Two contexts share a scene; A asks twice for a new sun (a stable request starts
    the background rebuild) and updates until it installs the light-space BVH; B has
    not seen the new version yet."""
    import time

    a.set_lights(sun, ())
    a.set_lights(sun, ())
    t0, f = time.time(), 0
    while a.bvh_stats().sun_rebuilds == 0:
        assert time.time() - t0 < 90, "no light-space BVH installed within 90 s"
        a.update(D.frame_params(cfg, grid, D.AppState(f), 0, **exposure))
        a.synchronize()
        f += 1
        time.sleep(0.02)
    return f


def test_shared_scene_set_lights_after_other_context_installs():
    """B shares A's scene; A installs a (possibly deeper) light-space
    sun BVH; B then calls set_lights - which re-derives its scene view and must size its
    traversal spill for the new depth - and updates. B's frames stay bit-exact against
    an oracle fed the same lights."""
    sc = S.soup(96_000, extent=7.0)
    grid = D.ProbeGrid((6, 6, 6), (1.2, 1.2, 1.2), (0.5, 0.5, 0.5))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=216, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=216, sun_bvh=abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE)
    exposure = dict(light_pre_exposure=1.0, environment_brightness=1.0)
    a = D.DDGIContext(grid, 10000.0, cfg)
    b = D.DDGIContext(grid, 10000.0, cfg)
    a.set_scene(sc)
    b.share_scene(a)
    orc = O.Oracle(b.desc)
    orc.set_scene(sc)
    try:
        for f in range(2):
            p = D.frame_params(cfg, grid, D.AppState(f), 0, **exposure)
            b.update(p)
            orc.update(p)
        b.synchronize()
        _compare(b, orc, 1, "before the install")
        d = np.array([-0.6, -1.0, 0.3], np.float32)
        sun = (sc.sun[0], tuple(float(x) for x in d / np.linalg.norm(d)))
        _install_sun_on_a(a, b, sc, grid, cfg, exposure, sun)
        b.set_lights(sun, ())
        orc.set_lights(sun, ())
        assert b.bvh_stats().max_depth >= b.bvh_stats().sun_max_depth
        for f in range(2, 4):
            p = D.frame_params(cfg, grid, D.AppState(f), 0, **exposure)
            b.update(p)
            orc.update(p)
            b.synchronize()
            _compare(b, orc, f, "B after A installed a sun BVH")
    finally:
        a.close()
        b.close()
        orc.close()


def test_shared_scene_reflections_after_other_context_installs():
    """B shares A's scene; A installs a light-space sun BVH; B's next
    operation is rt_reflections, which must size (and only then point into) its spill
    area for the scene's new depth. B's reflections equal the oracle's bit for bit."""
    import torch

    import reflection_inputs as RI

    sc = scenes.features_scene()
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=144, max_rays_per_probe=64, max_probe_updates=144,
                       sun_bvh=abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE)
    exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
    a = D.DDGIContext(GRID, 100.0, cfg)
    b = D.DDGIContext(GRID, 100.0, cfg)
    a.set_scene(sc)
    b.share_scene(a)
    orc = O.Oracle(b.desc)
    orc.set_scene(sc)
    try:
        d = np.array([0.4, -1.0, -0.5], np.float32)
        sun = (sc.sun[0], tuple(float(x) for x in d / np.linalg.norm(d)))
        for ctx in (b,):
            ctx.set_lights(sun, list(sc.spots))
        orc.set_lights(sun, list(sc.spots))
        for f in range(2):
            p = D.frame_params(cfg, GRID, D.AppState(f), 0, **exposure)
            b.update(p)
            orc.update(p)
        b.synchronize()
        a.set_lights(sun, list(sc.spots))
        a.set_lights(sun, list(sc.spots))
        import time

        t0, f = time.time(), 0
        while a.bvh_stats().sun_rebuilds == 0:
            assert time.time() - t0 < 90, "no light-space BVH installed within 90 s"
            a.update(D.frame_params(cfg, GRID, D.AppState(f), 0, **exposure))
            a.synchronize()
            f += 1
            time.sleep(0.02)
        W, H = 64, 48
        cam = RI.camera(W, H)
        g, _ = RI.gbuffer(W, H, cam, seed=3)
        kw = dict(environment_multiplier=0.5, ambient_amount=0.05)
        want_rad, want_dir = orc.rt_reflections(W, H, cam, g, **kw)
        dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in g.items()}
        rad = torch.zeros((H, W, 4), dtype=torch.int16, device="cuda")
        dirs = torch.zeros((H, W, 4), dtype=torch.int16, device="cuda")
        D.RTReflectionsNode().execute(b, cam, {k: dev[k] for k in ("depth", "material", "normal_velocity")}, dev["blue_noise"], rad, dirs, **kw)
        assert np.array_equal(rad.cpu().numpy().view(np.uint16), want_rad)
        assert np.array_equal(dirs.cpu().numpy().view(np.uint16), want_dir)
    finally:
        a.close()
        b.close()
        orc.close()
