"""CPU oracle of the AO / bent-normal bake against
closed forms of bakeAmbientOcclusion.rgen:33-118 and the parameterization rules
(DESIGN.md §AO bake). The reference ships no golden vectors for this path; its
rasterizer is the Vulkan driver's (parity unpinned there)."""
import numpy as np

from arkoserenderer_amd import scene as S
from arkoserenderer_amd import ddgi as D
import bake_scenes as B
import oracle_lib as O
from parity import make_desc


def _oracle(scene):
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=1, probe_updates_per_frame=1, max_rays_per_probe=1, max_probe_updates=1)
    o = O.Oracle(make_desc(grid, 100.0, cfg))
    o.set_scene(scene)
    return o


def test_quad_parameterization_covers_every_texel_once():
    o = _oracle(B.quad_scene())
    for W, H in ((16, 16), (37, 23)):
        tri, bary, _ = o.bake_ao(0, W, H, 1, False)
        assert (tri > 0).all()
        # the diagonal texels go to exactly one of the two triangles (tie rule)
        n1, n2 = int((tri == 1).sum()), int((tri == 2).sum())
        assert n1 + n2 == W * H and n1 > 0 and n2 > 0
        b = O.f16_to_f32(bary)
        assert np.allclose(b[..., :3].sum(-1), 1.0, atol=2e-3)
        assert (bary[..., 3] == 0x3C00).all()
        # position from barycentrics = texel centre (the quad maps (x, y) = (u, v))
        ys, xs = np.mgrid[0:H, 0:W]
        verts = np.array([(0, 0), (1, 0), (1, 1), (0, 1)], np.float64)
        tri_v = {1: verts[[0, 1, 2]], 2: verts[[0, 2, 3]]}
        for t in (1, 2):
            m = tri == t
            p = np.einsum("nk,kc->nc", b[m][:, :3].astype(np.float64), tri_v[t])
            assert np.allclose(p[:, 0], (xs[m] + 0.5) / W, atol=2e-3)
            assert np.allclose(p[:, 1], (ys[m] + 0.5) / H, atol=2e-3)


def test_open_quad_is_unoccluded():
    """No occluder: every cosine ray escapes -> AO byte 255; the mean bent normal
    is E[cos-weighted dir] = (0, 0, 2/3) -> encoded (0.5, 0.5, 5/6), cone 1."""
    o = _oracle(B.quad_scene())
    _, _, ao = o.bake_ao(0, 16, 16, 32, False)
    assert (ao == 255).all()
    _, _, bn = o.bake_ao(0, 16, 16, 64, True)
    enc = bn.reshape(-1, 4).astype(np.float64) / 255.0
    assert (bn[..., 3] == 255).all()
    assert abs(enc[:, 0].mean() - 0.5) < 0.01 and abs(enc[:, 1].mean() - 0.5) < 0.01
    assert abs(enc[:, 2].mean() - (0.5 + 1.0 / 3.0)) < 0.01


def test_closed_box_is_fully_occluded():
    o = _oracle(B.quad_scene(with_box=True))
    _, _, ao = o.bake_ao(0, 8, 8, 16, False)
    assert (ao == 0).all()
    _, _, bn = o.bake_ao(0, 8, 8, 16, True)
    assert (bn[..., :3] == 128).all() and (bn[..., 3] == 255).all()


def test_uncovered_texels_and_determinism():
    """Helmet at 96x96: uncovered texels keep the rgen's early-out values; a rerun is
    bit-identical; AO is neither trivially 0 nor 1 on a real mesh."""
    o = _oracle(S.damaged_helmet())
    tri, bary, ao = o.bake_ao(0, 96, 96, 8, False, threads=8)
    cov = tri > 0
    assert 0.3 < cov.mean() < 0.99
    assert (ao[~cov] == 0).all() and (bary[~cov] == 0).all()
    assert 0 < (ao[cov] < 255).mean() < 1
    tri2, bary2, ao2 = o.bake_ao(0, 96, 96, 8, False, threads=3)
    assert np.array_equal(tri, tri2) and np.array_equal(bary, bary2) and np.array_equal(ao, ao2)
    _, _, bn = o.bake_ao(0, 96, 96, 8, True)
    assert (bn[~cov[..., 0] if cov.ndim == 3 else ~cov] == np.array([128, 128, 128, 255], np.uint8)).all()
