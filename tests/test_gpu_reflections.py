"""RT reflections raygen (rt-reflections/raygen.rgen:54-166 with
WITH_DDGI) through ark_ddgi_rt_reflections against the CPU oracle, bit for bit: the
features scene (sun + 2 IES spots with shadow rays, masked and translucent geometry,
mirrored instance, textures), atlases after two DDGI frames, a synthetic G-buffer
with sky, untraced rough and traced pixels."""
import numpy as np
import pytest
import torch

from arkoserenderer_amd import ddgi as D
import oracle_lib as O
import reflection_inputs as RI
import scenes

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("roughness,size,z_far", [(None, (96, 64), 100.0), (0, (96, 64), 100.0), (None, (97, 61), 10000.0)])
def test_reflections_features_scene(roughness, size, z_far):
    """(97, 61): partial 8 x 8 tiles on both edges. z_far 100: a miss passes the
    raygen's hitT <= 10000 test with hitT = zFar + 1 (miss.rmiss:12), ray length 101;
    z_far 10000 (the camera default): misses keep 10000."""
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=144, max_rays_per_probe=64, max_probe_updates=144)
    ctx = D.DDGIContext(grid, z_far, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(sc)
    for f in range(2):
        p = D.frame_params(cfg, grid, D.AppState(f), 0, light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
        ctx.update(p)
        orc.update(p)
    ctx.synchronize()
    W, H = size
    cam = RI.camera(W, H)
    g, _ = RI.gbuffer(W, H, cam, seed=11, roughness=roughness)
    kw = dict(environment_multiplier=0.5, ambient_amount=0.05)
    want_rad, want_dir = orc.rt_reflections(W, H, cam, g, **kw)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in g.items()}
    rad = torch.zeros((H, W, 4), dtype=torch.int16, device="cuda")
    dirs = torch.zeros((H, W, 4), dtype=torch.int16, device="cuda")
    node = D.RTReflectionsNode()
    node.execute(ctx, cam, {k: dev[k] for k in ("depth", "material", "normal_velocity")}, dev["blue_noise"], rad, dirs, **kw)
    got_rad, got_dir = rad.cpu().numpy().view(np.uint16), dirs.cpu().numpy().view(np.uint16)
    for name, got, want in (("radiance", got_rad, want_rad), ("direction", got_dir, want_dir)):
        bad = np.argwhere(np.any(got != want, axis=-1))
        assert bad.size == 0, f"{name}: {len(bad)} pixels differ, first {bad[:4].tolist()}: got {got[tuple(bad[0])].view(np.float16)} want {want[tuple(bad[0])].view(np.float16)}"
    traced = np.any(want_dir != 0, axis=-1)
    assert traced.sum() > W * H // 2
    rl = want_rad.view(np.float16)[..., 3].astype(np.float32)[traced]
    miss_t = min(z_far + 1.0, 10000.0)
    assert (rl < miss_t).any() and (rl == np.float32(np.float16(miss_t))).any()  # both hits and misses
    rough = (g["material"][..., 0] / 255.0 >= 0.6) & (g["depth"] < 1.0 - 1e-6)
    assert ((g["material"][..., 0] == 160) & rough).any() and (got_rad[rough] == 0).all() and (got_dir[rough] == 0).all()
    ctx.close()
    orc.close()
