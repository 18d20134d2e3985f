"""Z-slab sharding over 2 and 4 ranks with the gloo backend on CPU, for real: each
rank runs a SHARDED oracle (desc shard_rank / shard_count: it traces, shades and
updates only the window probes of its own slab, at compacted slots, as
k_probe_slots does), then collective.WindowExchange (the code bench.py runs over
RCCL) hands every rank the other slabs' tiles: the in-place all-gather of the atlas
row bands when the window covers the grid (K = N), else the windowed exchange - each
rank's packets of the tiles its update wrote (tests/window_packets.py, the layout of
ark_ddgi_pack_window), all-gathered, unpacked into the other slabs' tiles. They are
written back into its oracle before the next frame - the next frame's indirect
bounce samples them at arbitrary hit points (raygen.rgen:127 ->
probeSampling.glsl:64-163). After every frame each rank's gathered atlases, and
its own probes' offsets, must equal an unsharded oracle's bit for bit; the full
grid, ragged windows and windows that wrap are run, and the windowed exchange must
move fewer bytes than the bands."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, window, frames, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S
    from arkoserenderer_amd.collective import SlabExchange, WindowExchange, torch_all_gather
    import oracle_lib as O
    from parity import make_desc
    import window_packets as WP

    class _OracleWindow:
        """WindowExchange's source over a sharded oracle's atlases (window_packets.py)."""

        def __init__(self, irr, vis, dims, P, r, first, K):
            self.irr, self.vis, self.args = irr.copy(), vis.copy(), (dims, P, r, first, K)

        def window_exchange_info(self):
            return WP.info(*self.args)

        def pack_window(self, t):
            t.copy_(torch.from_numpy(WP.pack(self.irr, self.vis, *self.args)))

        def unpack_window(self, t):
            WP.unpack(self.irr, self.vis, t.numpy(), *self.args)

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((4, 4, 8), (0.5, 0.5, 0.25), (-0.75, 0.25, -0.9))
    N = grid.probe_count()
    X, Y, Z = grid.grid_dimensions
    cfg = D.DDGIConfig(rays_per_probe=32, probe_updates_per_frame=window, compute_probe_offsets=True,
                       max_rays_per_probe=32, max_probe_updates=N)
    exposure = dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    mine_orc = O.Oracle(make_desc(grid, ex["z_far"], cfg, shard_rank=rank, shard_count=world))
    full_orc = O.Oracle(make_desc(grid, ex["z_far"], cfg))
    mine_orc.set_scene(sc, 2)
    full_orc.set_scene(sc, 2)
    z = (np.arange(N) % (X * Z)) // X
    owned = (z >= rank * (Z // world)) & (z < (rank + 1) * (Z // world))
    report = []
    first = 0
    for f in range(frames):
        p = D.frame_params(cfg, grid, D.AppState(f), first, **exposure)
        mine_orc.update(p, 2)
        full_orc.update(p, 2)
        first = (first + p.probe_updates) % N
        irr = mine_orc.read(abi.ARK_DDGI_ATLAS_IRRADIANCE).reshape(Z * 10, X * Y * 10 * 4)
        vis = mine_orc.read(abi.ARK_DDGI_ATLAS_VISIBILITY).reshape(Z * 18, X * Y * 18 * 2)
        for w, a in ((abi.ARK_DDGI_ATLAS_IRRADIANCE, irr), (abi.ARK_DDGI_ATLAS_VISIBILITY, vis)):
            # negative control: before the exchange the other slabs' tiles are stale
            report.append((f, "stale", int(np.count_nonzero(a.ravel() != full_orc.read(w).ravel()))))
        src = _OracleWindow(irr, vis, (X, Y, Z), world, rank, p.first_probe_index, p.probe_updates)

        def band():
            bufs = []
            for a in (src.irr, src.vis):
                t = torch.from_numpy(a.reshape(-1).view(np.uint8))  # shares memory with the atlas copy
                slab = t.numel() // world  # a Z-slab is a contiguous texel-row band
                bufs.append((t, rank * slab, slab))
            SlabExchange(bufs, rank, world).exchange()

        wx = WindowExchange(src, band, torch_all_gather(), rank, world, N // world, "cpu")
        wx.exchange()
        report.append((f, "bytes_per_rank", wx.last_bytes_per_rank if p.probe_updates < N else -1))
        for w, a in ((abi.ARK_DDGI_ATLAS_IRRADIANCE, src.irr), (abi.ARK_DDGI_ATLAS_VISIBILITY, src.vis)):
            gathered = a.reshape(-1)
            mine_orc.write(w, gathered)  # the next frame reads the other slabs' tiles
            want = full_orc.read(w).reshape(-1)
            report.append((f, w, int(np.count_nonzero(gathered != want))))
        off_m = mine_orc.read(abi.ARK_DDGI_PROBE_OFFSETS).reshape(N, 4)[owned]
        off_f = full_orc.read(abi.ARK_DDGI_PROBE_OFFSETS).reshape(N, 4)[owned]
        report.append((f, "offsets", int(np.count_nonzero(off_m.view(np.uint32) != off_f.view(np.uint32)))))
        report.append((f, "moved", int(np.count_nonzero(off_f))))
    mine_orc.close()
    full_orc.close()
    result_q.put((rank, report))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,window,frames", [(2, 128, 3), (4, 128, 3), (2, 45, 4), (4, 45, 4), (4, 100, 3)])
def test_zslab_sharded_oracles_two_and_four_ranks_gloo(world, window, frames):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, window, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == list(range(world))
    for rank, report in res.items():
        for f, what, n in report:
            if what in ("moved", "stale"):
                continue
            if what == "bytes_per_rank":
                # windows (K < N): fewer bytes than a band (N / P probes x 2,096 B)
                assert n == -1 or 0 < n < 128 // world * 2096, (rank, f, n)
                continue
            assert n == 0, (rank, f, what, n)
    # the offsets moved somewhere (the comparison is not of zeros), and each rank's own
    # update left the other slabs' tiles stale until the exchange
    assert any(n > 0 for rep in res.values() for f, what, n in rep if what == "moved")
    assert all(any(n > 0 for f, what, n in rep if what == "stale") for rep in res.values())
