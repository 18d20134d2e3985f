"""Stream semantics of the C-ABI (include/ark_ddgi.h, "Streams"): operations of one
context run in call order whatever streams they are given, and NULL is the null
stream. Frames are queued on one torch side stream and a consumer on another with no
host synchronisation in between; the consumer shares the traversal spill area (RT
reflections) or reads the atlases (probe debug), so a missing cross-stream order
shows up as a mismatch against the oracle."""
import numpy as np
import pytest
import torch

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
import oracle_lib as O
import reflection_inputs as RI
import scenes

pytestmark = pytest.mark.gpu


def _setup(frames, z_far=100.0):
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=144, max_rays_per_probe=64, max_probe_updates=144)
    ctx = D.DDGIContext(grid, z_far, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    params = [D.frame_params(cfg, grid, D.AppState(f), 0, light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
              for f in range(frames)]
    for p in params:
        orc.update(p)
    return ctx, orc, params


@pytest.mark.parametrize("update_on", ["side", "null"])
def test_reflections_after_update_on_another_stream(update_on):
    ctx, orc, params = _setup(3)
    W, H = 96, 64
    cam = RI.camera(W, H)
    g, _ = RI.gbuffer(W, H, cam, seed=3)
    kw = dict(environment_multiplier=0.5, ambient_amount=0.05)
    want_rad, want_dir = orc.rt_reflections(W, H, cam, g, **kw)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in g.items()}
    torch.cuda.synchronize()
    s_upd, s_refl = torch.cuda.Stream(), torch.cuda.Stream()
    rad = torch.zeros((H, W, 4), dtype=torch.int16, device="cuda")
    dirs = torch.zeros((H, W, 4), dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    for p in params:  # queued back to back, no host sync
        ctx.update(p, s_upd.cuda_stream if update_on == "side" else None)
    node = D.RTReflectionsNode()
    node.execute(ctx, cam, {k: dev[k] for k in ("depth", "material", "normal_velocity")}, dev["blue_noise"], rad, dirs,
                 stream=s_refl.cuda_stream, **kw)
    s_refl.synchronize()  # only the consumer's stream: the C-ABI ordered it after the updates
    got_rad, got_dir = rad.cpu().numpy().view(np.uint16), dirs.cpu().numpy().view(np.uint16)
    assert np.array_equal(got_rad, want_rad) and np.array_equal(got_dir, want_dir)
    # the next update, on the null stream, is ordered after the reflections (same spill area)
    p3 = D.frame_params(ctx.config, ctx.grid, D.AppState(3), 0, light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
    ctx.update(p3, None)
    ctx.synchronize()
    orc.update(p3)
    for which in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY, abi.ARK_DDGI_SURFELS):
        assert np.array_equal(ctx.read(which), orc.read(which))
    ctx.close()
    orc.close()


def test_probe_debug_on_torch_default_stream_after_side_stream_update():
    """The consumer on torch's default (null) stream right after frames queued on a
    side stream; torch zero-fills the output on the null stream first."""
    ctx, orc, params = _setup(2)
    s_upd = torch.cuda.Stream()
    for p in params:
        ctx.update(p, s_upd.cuda_stream)
    rng = np.random.default_rng(1)
    probes = rng.integers(0, 144, 4096).astype(np.uint32)
    dirs = rng.normal(size=(4096, 3)).astype(np.float32)
    want = orc.probe_debug(abi.ARK_PROBE_DEBUG_IRRADIANCE, 0.01, probes, dirs)
    node = D.DDGIProbeDebug()
    node.debug_visualisation = abi.ARK_PROBE_DEBUG_IRRADIANCE
    out = torch.zeros((4096, 4), dtype=torch.int16, device="cuda")
    node.execute(ctx, torch.from_numpy(probes.view(np.int32)).cuda(), torch.from_numpy(dirs).cuda(), out)
    got = out.cpu().numpy().view(np.uint16)  # torch's default stream: ordered after the launch
    assert np.array_equal(got, want)
    ctx.close()
    orc.close()
