"""The windowed Z-slab exchange on the GPU (ark_ddgi_window_exchange_info /
ark_ddgi_pack_window / ark_ddgi_unpack_window, ddgi_exchange.hip; VERDICT r05 "do
this" #2). P slab contexts on one GPU share one scene; every frame each updates the
window probes of its slab (a rolling window of K < N probes, DDGINode.cpp:138-140,
wrapping around the grid), packs the tiles it wrote into its region of one receive
buffer (the all-gather's layout), and unpacks the other regions into the other slabs'
tiles. Checked every frame:

  * every slab context's atlases equal an unsharded context's, WHOLE atlas, bit for
    bit (the windowed exchange alone keeps them whole: only K probes per frame move);
  * the info fields and every rank's packet bytes equal the host restatement
    (tests/window_packets.py) applied to the unsharded atlases.

Config C4 at P = 8 and the reference's K = 2,048 (DDGINode.h:31), and a small scene at
P = 4 with a ragged window that wraps."""
import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import scenes
import window_packets as WP

pytestmark = pytest.mark.gpu

ATLASES = (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY)


def _windowed(scene, dims, spacing, origin, R, z_far, exposure, P, K, frames, check_packets):
    import torch

    X, Y, Z = dims
    grid = D.ProbeGrid(dims, spacing, origin)
    N = grid.probe_count()
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=K, max_rays_per_probe=R, max_probe_updates=K, compute_probe_offsets=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    full = D.DDGIContext(grid, z_far, cfg)
    full.set_scene(scene)
    slabs = [D.DDGIContext(grid, z_far, cfg, 0, r, P) for r in range(P)]
    for c in slabs:
        c.share_scene(full)
    recv = torch.empty(P * min(K, N // P) * abi.ARK_DDGI_WINDOW_PACKET_BYTES, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    first = 0
    for frame in range(frames):
        p = D.frame_params(cfg, grid, D.AppState(frame), first, **exposure)
        for c in slabs:
            c.update(p, stream)
        full.update(p, stream)
        infos = [c.window_exchange_info() for c in slabs]
        n = int(infos[0].bytes_per_rank)
        for r, (c, w) in enumerate(zip(slabs, infos)):
            want = WP.info(dims, P, r, first, K)
            got = (w.full_bands, w.probes_per_rank, w.my_probes, w.first_probe, w.probe_updates, w.bytes_per_rank)
            assert got == (want.full_bands, want.probes_per_rank, want.my_probes, want.first_probe, want.probe_updates, want.bytes_per_rank), (frame, r, got)
            assert w.full_bands == 0 and w.bytes_per_rank == n and n > 0
            c.pack_window(recv.data_ptr() + r * n, n, stream)
        for c in slabs:
            c.unpack_window(recv.data_ptr(), P * n, stream)
        torch.cuda.synchronize(dev)
        want = {w: full.read(w) for w in ATLASES}
        for r, c in enumerate(slabs):
            for w in ATLASES:
                got = c.read(w)
                assert np.array_equal(got, want[w]), f"frame {frame} slab {r}: {int(np.count_nonzero(got != want[w]))} atlas values of {w} differ"
        if check_packets:
            irr = want[ATLASES[0]].reshape(Z * 10, X * Y * 40)
            vis = want[ATLASES[1]].reshape(Z * 18, X * Y * 36)
            host = recv[:P * n].cpu().numpy()
            for r in range(P):
                assert np.array_equal(host[r * n:r * n + infos[r].my_probes * WP.PACKET_BYTES],
                                      WP.pack(irr, vis, dims, P, r, first, K)[:infos[r].my_probes * WP.PACKET_BYTES]), f"frame {frame} rank {r} packets"
        first = (first + K) % N
    for c in slabs + [full]:
        c.close()


def test_window_exchange_small_wrapping():
    """features scene (sun + spots), 6 x 4 x 8 probes as 4 slabs of 2 layers, K = 45:
    ragged slab shares, and the window wraps in frame 4."""
    _windowed(scenes.features_scene(), (6, 4, 8), (0.7, 0.7, 0.35), (-1.75, 0.25, -1.4), 64, 100.0,
              dict(light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5), 4, 45, 5, True)


def test_window_exchange_c4_k2048_eight_slabs():
    """C4 (10 M triangles, 32^3 probes x 256 rays) as 8 Z-slabs at the reference's K =
    2,048: 256 probes x 2,096 B per rank instead of an 8.6-MB band, 3 frames."""
    _windowed(S.soup(10_000_000), (32, 32, 32), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), 256, 10000.0,
              dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0), 8, 2048, 3, True)
