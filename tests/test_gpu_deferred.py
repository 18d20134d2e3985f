"""Deferred probe update (ark_ddgi_set_deferred_update): frame n's probe update on the
context's update stream beside frame n+1's traversal, frames queued back to back with
no host sync. Bit-exact against the oracle's serial frames, with probe offsets on (the
traversal then waits for the pending update) and off (it does not), a rolling window
that wraps, sub-windows, and consumers reading the atlases straight after a deferred
update."""
import numpy as np
import pytest
import torch

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import oracle_lib as O
import scenes
from parity import run_pair

pytestmark = pytest.mark.gpu


def _exact(reps):
    for f, rep in enumerate(reps):
        for r in rep:
            assert r["mismatch"] == 0, f"frame {f}: {r}"


def test_deferred_cornell_all_probes_offsets_off():
    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=512)
    reps = run_pair(sc, grid, cfg, 5, ex["z_far"], dict(light_pre_exposure=ex["light_pre_exposure"],
                                                         environment_brightness=ex["environment_brightness"]),
                    check_each_frame=False, deferred=True)
    _exact(reps)


@pytest.mark.parametrize("offsets", [True, False])
def test_deferred_features_window(offsets):
    """Lights, masked and translucent geometry; K = 100 of 144 so the windows wrap and
    the two slot tables hold different windows."""
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=100, compute_probe_offsets=offsets,
                       max_rays_per_probe=128, max_probe_updates=144)
    reps = run_pair(sc, grid, cfg, 5, 100.0, dict(light_pre_exposure=1.0, ambient_illuminance=0.05,
                                                  environment_brightness=0.5),
                    check_each_frame=False, deferred=True)
    _exact(reps)


def test_deferred_with_subwindows(monkeypatch):
    monkeypatch.setenv("ARK_SUBWINDOWS", "2")
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=144, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=144)
    reps = run_pair(sc, grid, cfg, 4, 100.0, dict(light_pre_exposure=1.0, environment_brightness=0.5),
                    check_each_frame=False, deferred=True)
    _exact(reps)


def test_consumer_after_deferred_update():
    """The probe debug node reads the atlases right after a deferred update, on torch's
    stream: the context joins the pending update first."""
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=144, max_rays_per_probe=64, max_probe_updates=144)
    ctx = D.DDGIContext(grid, 100.0, cfg)
    ctx.set_scene(sc)
    ctx.set_deferred_update(True)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    for f in range(3):
        p = D.frame_params(cfg, grid, D.AppState(f), 0, environment_brightness=0.5)
        ctx.update(p)
        orc.update(p)
    sphere = D.DDGIProbeDebug.sphere_samples(8, 8)
    probes = np.repeat(np.arange(grid.probe_count(), dtype=np.uint32), len(sphere))
    dirs = np.tile(sphere, (grid.probe_count(), 1))
    dirs[np.all(dirs == 0, axis=1)] = (0, 1, 0)
    node = D.DDGIProbeDebug()
    node.debug_visualisation = abi.ARK_PROBE_DEBUG_IRRADIANCE
    # an explicit (non-null) stream: no host sync in the node, the C entry's join
    # orders the launch after the pending update
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        out = torch.zeros((len(probes), 4), dtype=torch.int16, device="cuda")
        node.execute(ctx, torch.from_numpy(probes.astype(np.int32)).cuda(), torch.from_numpy(dirs).cuda(), out,
                     stream=side.cuda_stream)
    side.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    want = orc.probe_debug(abi.ARK_PROBE_DEBUG_IRRADIANCE, 0.01, probes, dirs)
    assert np.array_equal(got, want)
    assert np.count_nonzero(got[:, :3]) > 0
    ctx.close()
    orc.close()
