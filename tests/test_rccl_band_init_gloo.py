"""RcclBandExchange's setup reaches one outcome on every rank: when
librccl cannot be loaded on a NON-root rank, no rank may enter ncclCommInitRank
(it blocks until every rank joins); all ranks must raise together, so that bench.py
falls back to SlabExchange everywhere. 2 gloo ranks on CPU; rank 1's _rccl fails."""
import os
import socket

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


def _worker(rank, world, port, failing_rank, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import arkoserenderer_amd.collective as Cl

    def broken():
        raise OSError("librccl.so: cannot open shared object file (test)")

    if rank == failing_rank:
        Cl._rccl = broken
    full = torch.zeros(world * 64, dtype=torch.uint8)
    try:
        Cl.RcclBandExchange([(full, rank * 64, 64)], rank, world)
        q.put((rank, "constructed"))
    except RuntimeError as e:
        q.put((rank, "raised: " + str(e)))
    dist.destroy_process_group()


@pytest.mark.parametrize("failing_rank", [1, 0])
def test_rccl_band_exchange_load_failure_raises_on_every_rank(failing_rank):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, failing_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    alive = [p.pid for p in procs if p.is_alive()]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not alive, "a rank hung in RcclBandExchange setup"
    res = dict(q.get(timeout=5) for _ in range(world))
    assert all(v.startswith("raised: RcclBandExchange: librccl or the ncclUniqueId unavailable") for v in res.values()), res
