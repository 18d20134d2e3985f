"""Z-slab sharding over 2 ranks with the gloo backend on CPU: each rank updates
only its slab (here: the oracle's full update with the other band discarded),
then SlabExchange's in-place all-gather must rebuild exactly the unsharded
atlases. Exercises the same exchange code bench.py runs over RCCL."""
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


def _worker(rank, world, port, result_q):
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
    from arkoserenderer_amd.collective import SlabExchange
    import oracle_lib as O
    from parity import make_desc

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((4, 4, 4), (0.5, 0.5, 0.5), (-0.75, 0.25, -0.75))
    cfg = D.DDGIConfig(rays_per_probe=32, probe_updates_per_frame=64, max_rays_per_probe=32, max_probe_updates=64)
    orc = O.Oracle(make_desc(grid, ex["z_far"], cfg))
    orc.set_scene(sc, 2)
    X, Y, Z = grid.grid_dimensions
    ok = True
    for f in range(3):
        p = D.frame_params(cfg, grid, D.AppState(f), 0, light_pre_exposure=ex["light_pre_exposure"],
                           environment_brightness=ex["environment_brightness"])
        orc.update(p, 2)
        full = {w: orc.read(w).copy() for w in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY)}
        bufs = []
        tensors = {}
        for w, tile in ((abi.ARK_DDGI_ATLAS_IRRADIANCE, 10), (abi.ARK_DDGI_ATLAS_VISIBILITY, 18)):
            a = full[w].view(np.uint8).copy()
            total = a.size
            slab = total // world
            # this rank only "computed" its own band: scramble the rest
            mine = a[rank * slab:(rank + 1) * slab].copy()
            a[:] = 0xAB
            a[rank * slab:(rank + 1) * slab] = mine
            t = torch.from_numpy(a)
            tensors[w] = t
            # a Z-slab is a contiguous row band: rows [z0*tile, z1*tile) of the atlas
            assert slab == (Z // world) * tile * (X * tile * Y) * (8 if tile == 10 else 4)
            bufs.append((t, rank * slab, slab))
        SlabExchange(bufs, rank, world).exchange()
        for w, t in tensors.items():
            ok &= np.array_equal(t.numpy(), full[w].view(np.uint8))
    result_q.put((rank, bool(ok)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_zslab_allgather_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}
