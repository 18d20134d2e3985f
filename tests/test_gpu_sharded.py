"""Z-slab sharding on the GPU (one box, one GPU): two contexts each own half the
grid; after every update the slab bands are exchanged; both must equal the
unsharded oracle bit for bit. Plus: the RCCL-facing torch view of the atlases
and a 1-rank RCCL all-gather through SlabExchange."""
import ctypes as C
import os

import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import oracle_lib as O
from parity import diff_report, make_desc

pytestmark = pytest.mark.gpu


def _exchange_host(ctxs):
    """Emulates the in-place all-gather with host copies of each owner's band."""
    world = len(ctxs)
    for which in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY):
        atl = [c.read(which).view(np.uint8) for c in ctxs]
        slab = atl[0].size // world
        full = np.concatenate([atl[r][r * slab:(r + 1) * slab] for r in range(world)])
        for c in ctxs:
            c.write(which, full)


@pytest.mark.parametrize("window", [512, 150])
def test_two_slabs_equal_unsharded(window):
    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=window, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=512)
    exposure = dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    ctxs = [D.DDGIContext(grid, ex["z_far"], cfg, 0, r, 2) for r in range(2)]
    for c in ctxs:
        c.set_scene(sc)
    orc = O.Oracle(make_desc(grid, ex["z_far"], cfg))
    orc.set_scene(sc)
    idx = 0
    N = grid.probe_count()
    for f in range(4):
        p = D.frame_params(cfg, grid, D.AppState(f), idx, **exposure)
        for c in ctxs:
            c.update(p)
        for c in ctxs:
            c.synchronize()
        _exchange_host(ctxs)
        orc.update(p)
        idx = (idx + p.probe_updates) % N
        for which in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY):
            o = orc.read(which)
            for c in ctxs:
                r = diff_report("atlas", c.read(which), o)
                assert r["mismatch"] == 0, (f, which, r)
        # offsets: each probe's offset lives on the rank owning its z (owner-only)
        o_off = orc.read(abi.ARK_DDGI_PROBE_OFFSETS).reshape(N, 4)
        z = (np.arange(N) % (8 * 8)) // 8
        for r, c in enumerate(ctxs):
            mine = (z >= 4 * r) & (z < 4 * (r + 1))
            assert np.array_equal(c.read(abi.ARK_DDGI_PROBE_OFFSETS).reshape(N, 4)[mine], o_off[mine])


def test_device_bytes_view_and_one_rank_rccl_allgather():
    import torch
    import torch.distributed as dist

    from arkoserenderer_amd.collective import SlabExchange, device_bytes

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((4, 4, 4), (0.5, 0.5, 0.5), (-0.75, 0.25, -0.75))
    cfg = D.DDGIConfig(rays_per_probe=32, probe_updates_per_frame=64, max_rays_per_probe=32, max_probe_updates=64)
    ctx = D.DDGIContext(grid, ex["z_far"], cfg)
    ctx.set_scene(sc)
    ctx.update(D.frame_params(cfg, grid, D.AppState(0), 0, light_pre_exposure=ex["light_pre_exposure"],
                              environment_brightness=ex["environment_brightness"]))
    ctx.synchronize()
    v = ctx.device_views()
    dev = torch.device("cuda", 0)
    t = device_bytes(v.irradiance_atlas, v.irradiance_bytes, dev)
    assert np.array_equal(t.cpu().numpy(), ctx.read(abi.ARK_DDGI_ATLAS_IRRADIANCE).view(np.uint8))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        before = ctx.read(abi.ARK_DDGI_ATLAS_VISIBILITY).copy()
        SlabExchange.from_views(v, 0, 1, dev).exchange()
        torch.cuda.synchronize()
        assert np.array_equal(ctx.read(abi.ARK_DDGI_ATLAS_VISIBILITY), before)
    finally:
        dist.destroy_process_group()


def test_golden_fixtures_on_gpu():
    """The HIP path reproduces the committed oracle fixtures (no oracle at run time)."""
    import hashlib
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_golden as G
    from parity import RESOURCES

    for name in G.GOLDEN_SCENES:
        f = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{name}.npz"))
        want = dict(zip(f["keys"].tolist(), f["values"].tolist()))
        sc, grid, cfg, frames, zfar, exposure = G.scene_spec(name)
        ctx = D.DDGIContext(grid, zfar, cfg)
        ctx.set_scene(sc)
        idx = 0
        for fr in range(frames):
            p = D.frame_params(cfg, grid, D.AppState(fr), idx, **exposure)
            ctx.update(p)
            ctx.synchronize()
            idx = (idx + p.probe_updates) % grid.probe_count()
            for k, w in RESOURCES.items():
                assert hashlib.sha256(ctx.read(w).tobytes()).hexdigest() == want[f"{k}_{fr}"], (name, fr, k)
        ctx.close()


@pytest.mark.parametrize("device_seq", [False, True], ids=["events", "device_seq"])
def test_overlapped_update_two_slabs_one_gpu(device_seq):
    """ark_ddgi_update_overlapped on two Z-slab contexts sharing one GPU, each on its
    own stream, with the band exchange as device copies on a third stream ordered
    only by the events (the RCCL schedule of OverlappedSlabExchange): after several
    frames enqueued without host synchronisation the atlases equal the oracle's.
    device_seq: the same through ark_ddgi_update_exchanged / ark_ddgi_exchange_begin /
    ark_ddgi_exchange_end (device-side sequence words instead of events)."""
    import torch

    from arkoserenderer_amd.collective import device_bytes

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=300, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=512)
    exposure = dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    ctxs = [D.DDGIContext(grid, ex["z_far"], cfg, 0, r, 2) for r in range(2)]
    for c in ctxs:
        c.set_scene(sc)
    dev = torch.device("cuda", 0)
    views = [c.device_views() for c in ctxs]
    atlases = []
    for v in views:
        atlases.append([(device_bytes(v.irradiance_atlas, v.irradiance_bytes, dev), int(v.irradiance_slab_offset), int(v.irradiance_slab_bytes)),
                        (device_bytes(v.visibility_atlas, v.visibility_bytes, dev), int(v.visibility_slab_offset), int(v.visibility_slab_bytes))])
    streams = [torch.cuda.Stream(dev) for _ in ctxs]
    comm = torch.cuda.Stream(dev)
    done = [torch.cuda.Event() for _ in ctxs]
    gathered = torch.cuda.Event()
    for e in done + [gathered]:
        e.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize(dev)
    orc = O.Oracle(make_desc(grid, ex["z_far"], cfg))
    orc.set_scene(sc)
    idx, N = 0, grid.probe_count()
    for f in range(5):
        p = D.frame_params(cfg, grid, D.AppState(f), idx, **exposure)
        for c, s, e in zip(ctxs, streams, done):
            if device_seq:
                c.update_exchanged(p, s.cuda_stream)
            else:
                c.update_overlapped(p, s.cuda_stream, gathered.cuda_event if f > 0 else None, e.cuda_event)
        with torch.cuda.stream(comm):
            for c, e in zip(ctxs, done):
                if device_seq:
                    c.exchange_begin(comm.cuda_stream)
                else:
                    comm.wait_event(e)
            for k in range(2):  # each owner's band into the other context
                for r in range(2):
                    full, off, n = atlases[r][k]
                    other = atlases[1 - r][k][0]
                    other[off:off + n].copy_(full[off:off + n])
            if device_seq:
                for c in ctxs:
                    c.exchange_end(comm.cuda_stream)
            gathered.record(comm)
        orc.update(p)
        idx = (idx + p.probe_updates) % N
    torch.cuda.synchronize(dev)
    for which in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY):
        o = orc.read(which)
        for c in ctxs:
            r = diff_report("atlas", c.read(which), o)
            assert r["mismatch"] == 0, (which, r)


@pytest.mark.parametrize("mode,port", [("torch_pg_events", 29541), ("torch_pg_seq", 29542), ("rccl_seq", 29543),
                                       ("window_full", 29544), ("window_k100", 29545)])
def test_bench_frame_loop_over_one_rank_rccl(mode, port):
    """bench.py's N > 1 frame loop as it runs on every rank: DDGINode.execute_overlapped
    driven by OverlappedSlabExchange (torch events, a side stream, the in-place RCCL
    all-gather of SlabExchange), here over a 1-rank communicator, several frames
    enqueued without host synchronisation: the atlases and offsets equal a plain
    node's (the exchange of one rank moves nothing, so only the event plumbing and
    stream order are under test). torch_pg_seq: device-side sequence words instead
    of events; rccl_seq: also the bench's direct RCCL group (RcclBandExchange);
    window_full / window_k100: bench.py's composition exactly - WindowExchange over the
    RCCL group, the whole grid (row bands) and a 100-probe window (packets)."""
    import torch
    import torch.distributed as dist

    from arkoserenderer_amd.collective import OverlappedSlabExchange, RcclBandExchange, SlabExchange, WindowExchange, WindowSource

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    K = 100 if mode == "window_k100" else 512
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=K, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=512)
    exposure = dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    plain, ranked = D.DDGINode(cfg), D.DDGINode(cfg)
    assert plain.construct(sc, grid, ex["z_far"], device=0, **exposure)
    assert ranked.construct(sc, grid, ex["z_far"], device=0, shard_rank=0, shard_count=1, **exposure)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    band = None
    try:
        Ex = RcclBandExchange if mode in ("rccl_seq", "window_full", "window_k100") else SlabExchange
        band = Ex.from_views(ranked.ctx.device_views(), 0, 1, dev)
        exchange = band.exchange
        if mode.startswith("window"):
            exchange = WindowExchange(WindowSource(ranked.ctx), band.exchange, band.all_gather, 0, 1, min(K, 512), dev).exchange
        exch = OverlappedSlabExchange(ranked, exchange, dev, device_seq=mode != "torch_pg_events")
        sptr = torch.cuda.current_stream(dev).cuda_stream
        for f in range(6):
            plain.execute(D.AppState(f), sptr)
            exch.step(D.AppState(f), sptr)
        torch.cuda.synchronize(dev)
        for which in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY, abi.ARK_DDGI_PROBE_OFFSETS):
            a, b = plain.ctx.read(which), ranked.ctx.read(which)
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), which
    finally:
        if isinstance(band, RcclBandExchange):
            band.close()
        dist.destroy_process_group()
        plain.ctx.close()
        ranked.ctx.close()


def _stalled_exchange_run(timeout_s, on_failure, port):
    """bench.py's N > 1 frame loop over a 1-rank RCCL communicator whose first
    all-gather queues behind a bounded ~1.5 s kernel on the exchange stream
    (torch.cuda._sleep): frame 2's step must wait for frame 0's all-gather."""
    import torch
    import torch.distributed as dist

    from arkoserenderer_amd.collective import ExchangeWatchdog, OverlappedSlabExchange, SlabExchange

    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((4, 4, 4), (0.5, 0.5, 0.5), (-0.75, 0.25, -0.75))
    cfg = D.DDGIConfig(rays_per_probe=32, probe_updates_per_frame=64, max_rays_per_probe=32, max_probe_updates=64)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    node = D.DDGINode(cfg)
    assert node.construct(sc, grid, ex["z_far"], device=0, shard_rank=0, shard_count=1,
                          light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    gather = SlabExchange.from_views(node.ctx.device_views(), 0, 1, dev).exchange
    calls = []

    def exchange():
        if not calls:
            torch.cuda._sleep(int(3.5e9))  # bounded: ends by itself after ~1.5 s
        calls.append(1)
        gather()

    wd = ExchangeWatchdog(timeout_s=timeout_s, on_failure=on_failure)
    exch = OverlappedSlabExchange(node, exchange, dev, wd)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    results = [exch.step(D.AppState(f), sptr) for f in range(OverlappedSlabExchange.RING + 1)]
    return node, exch, results


def test_python_exchange_watchdog_fires_at_deadline():
    """collective.ExchangeWatchdog (SURVEY §5 failure detection): with the exchange
    stream stalled and a 0.2 s deadline, frame RING's step does not enqueue anything and
    reports the timeout to the failure handler; a generous deadline lets the same
    stall pass."""
    import torch
    import torch.distributed as dist

    fired = []
    node, exch, res = _stalled_exchange_run(0.2, fired.append, 29547)
    try:
        assert all(r is not None for r in res[:-1]) and res[-1] is None
        assert len(fired) == 1 and "slab exchange frame n-3: not complete after" in fired[0], fired
    finally:
        torch.cuda.synchronize()  # the stall kernel finishes by itself
        dist.destroy_process_group()
        node.ctx.close()
    fired = []
    node, exch, res = _stalled_exchange_run(30.0, fired.append, 29548)
    try:
        assert all(r is not None for r in res) and not fired
        assert exch.drain()
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()
        node.ctx.close()


def test_python_exchange_watchdog_exits_process(tmp_path):
    """The default failure path in its own process: the process group is aborted, an
    Error is logged and the process ends with exit code 14 (the handler lets the
    bounded stall kernel finish first)."""
    import subprocess
    import sys

    tests = os.path.dirname(os.path.abspath(__file__))
    script = tmp_path / "wd.py"
    script.write_text(
        "import sys, torch\n"
        f"sys.path.insert(0, {os.path.dirname(tests)!r}); sys.path.insert(0, {tests!r})\n"
        "import test_gpu_sharded as T\n"
        "box = {}\n"
        "def fail(why):\n"
        "    torch.cuda.synchronize()\n"
        "    box['exch'].watchdog.abort_and_exit(why)\n"
        "class Lazy:\n"
        "    def __call__(self, why): fail(why)\n"
        "import arkoserenderer_amd.collective as Cl\n"
        "orig = Cl.OverlappedSlabExchange.__init__\n"
        "def init(self, *a, **k):\n"
        "    orig(self, *a, **k); box['exch'] = self\n"
        "Cl.OverlappedSlabExchange.__init__ = init\n"
        "T._stalled_exchange_run(0.2, Lazy(), 29549)\n"
        "print('not reached')\n")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 14, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "not reached" not in r.stdout
    assert "[Error] Z-slab exchange failed, exiting: slab exchange frame n-3: not complete after" in r.stderr
