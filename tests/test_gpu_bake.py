"""GPU parity of the AO / bent-normal bake: the HIP
path (ark_ddgi_bake_ao through the C-ABI) against the CPU oracle, bit for bit:
triangle-index image, fp16 barycentrics and the R8 / RGBA8 output."""
import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import bake_scenes as B
import oracle_lib as O
from parity import make_desc

pytestmark = pytest.mark.gpu


def _pair(scene):
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=1, probe_updates_per_frame=1, max_rays_per_probe=1, max_probe_updates=1)
    ctx = D.DDGIContext(grid, 100.0, cfg)
    ctx.set_scene(scene)
    orc = O.Oracle(make_desc(grid, 100.0, cfg))
    orc.set_scene(scene)
    return ctx, orc


def _check(ctx, orc, inst, W, H, samples, bent):
    ctx.bake_ao(inst, W, H, samples, bent)
    g = [ctx.bake_read(w) for w in (abi.ARK_BAKE_TRIANGLE_INDEX, abi.ARK_BAKE_BARYCENTRICS, abi.ARK_BAKE_OUTPUT)]
    o = orc.bake_ao(inst, W, H, samples, bent)
    for name, a, b in zip(("triangle index", "barycentrics", "output"), g, o):
        assert a.shape == b.shape, name
        n = int(np.count_nonzero(a != b))
        assert n == 0, f"{name}: {n} of {a.size} differ"
    return g


@pytest.mark.parametrize("bent", [False, True])
def test_helmet_bake_bit_exact(bent):
    """DamagedHelmet (C1 mesh) at 128x128, 16 samples per texel."""
    ctx, orc = _pair(S.damaged_helmet())
    tri, _, out = _check(ctx, orc, 0, 128, 128, 16, bent)
    cov = tri > 0
    assert cov.mean() > 0.3
    if not bent:
        assert 0 < (out[cov] < 255).mean() < 1  # some occlusion, not all
    ctx.close()


def test_quad_kats_on_gpu():
    """Closed forms on the device: open quad -> AO 255; boxed quad -> AO 0, bent (128,128,128,255)."""
    ctx, orc = _pair(B.quad_scene())
    _, _, ao = _check(ctx, orc, 0, 32, 32, 16, False)
    assert (ao == 255).all()
    ctx.close()
    ctx, orc = _pair(B.quad_scene(with_box=True))
    _, _, ao = _check(ctx, orc, 0, 16, 16, 8, False)
    assert (ao == 0).all()
    _, _, bn = _check(ctx, orc, 0, 16, 16, 8, True)
    assert (bn[..., :3] == 128).all()
    ctx.close()


def test_partial_lid_and_rebake_sizes():
    """A lid over part of the quad: mixed AO, then a rebake at another extent
    reuses the context (results depend only on the desc)."""
    ctx, orc = _pair(B.quad_scene(lid=True))
    _, _, ao = _check(ctx, orc, 0, 24, 24, 32, False)
    assert 0 < (ao < 255).mean() <= 1
    _check(ctx, orc, 0, 40, 12, 8, True)
    ctx.close()
