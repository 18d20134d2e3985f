"""Per-rank cost of an S-way Z-slab run, measured on ONE GPU: a context that owns
slab 0 of S runs the C4 workload; prints its ms/step next to the unsharded one. A
proxy for strong-scaling headroom; the driver measures real N-GPU runs.

    python tools/shard_proxy.py [--shards 2 4 8] [--steps 10] [--all-ranks] [--exchange] [--window K]

--all-ranks measures every slab of each S (the strong-scaling step is the slowest
rank's), not only slab 0. --exchange adds an exchange stand-in: the frame loop of
bench.py's ranks (collective.OverlappedSlabExchange: the next frame's traversal goes
ahead, its shading waits for the exchange) with a device copy of the (S-1)/S of both
atlases a rank receives per step (60 MB at S = 8) on the side stream in place of the
RCCL all-gather, so the copy's HBM traffic and CU time contend with the traversal as
RCCL's copy kernels would (the xGMI transfer time itself is not modelled).
--window K: the reference's rolling window (K probes per frame, DDGINode.cpp:138-140)
instead of the whole grid; with --exchange the windowed exchange runs for real on the
rank (collective.WindowExchange: ark_ddgi_pack_window, a device copy standing in for the
all-gather of the other ranks' packets, ark_ddgi_unpack_window). Each line reports the
bytes a rank receives per frame.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--triangles", type=int, default=10_000_000)
    ap.add_argument("--all-ranks", action="store_true")
    ap.add_argument("--exchange", action="store_true", help="exchange stand-in (device copy of the received bands)")
    ap.add_argument("--window", type=int, default=0, help="probes per frame (0 = the whole grid)")
    ap.add_argument("--no-sun", action="store_true", help="no light: no shadow rays (a bound on what a fused shadow phase could save)")
    args = ap.parse_args()
    import torch

    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    scene = S.soup(args.triangles)
    G, R = 32, 256
    grid = D.ProbeGrid((G, G, G), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    out = {}
    for s, rank in [(s, r) for s in args.shards for r in (range(s) if args.all_ranks else [0])]:
        K = args.window or G ** 3
        cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=K, max_rays_per_probe=R, max_probe_updates=K,
                           compute_probe_offsets=True)
        node = D.DDGINode(cfg)
        assert node.construct(scene, grid, 10000.0, device=0, shard_rank=rank, shard_count=s,
                              light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
        if args.no_sun:
            node.ctx.set_lights(None, ())
        sptr = torch.cuda.current_stream(dev).cuda_stream
        run = node.execute
        received = 0
        if args.exchange and s > 1:
            from arkoserenderer_amd.collective import OverlappedSlabExchange, WindowExchange, WindowSource, device_bytes

            v = node.ctx.device_views()
            bands = []
            for ptr, total, off, n in ((v.irradiance_atlas, v.irradiance_bytes, v.irradiance_slab_offset, v.irradiance_slab_bytes),
                                       (v.visibility_atlas, v.visibility_bytes, v.visibility_slab_offset, v.visibility_slab_bytes)):
                atlas = device_bytes(ptr, total, dev)
                bands.append((atlas, atlas.clone(), int(off), int(n)))  # the clone stands for the other ranks' bands

            def band():
                for atlas, other, off, n in bands:  # everything but this rank's own band
                    if off > 0:
                        atlas[:off].copy_(other[:off])
                    if off + n < atlas.numel():
                        atlas[off + n:].copy_(other[off + n:])

            def gather(out, mine):  # the other ranks' packets (a device copy stands in for the all-gather)
                n = mine.numel()
                if rank > 0:
                    out[:rank * n].copy_(others[:rank * n])
                if rank + 1 < s:
                    out[(rank + 1) * n:s * n].copy_(others[:(s - rank - 1) * n])

            wx = WindowExchange(WindowSource(node.ctx), band, gather, rank, s, min(K, G ** 3 // s), dev)
            wx.recv.zero_()
            others = wx.recv.clone()
            loop = OverlappedSlabExchange(node, wx.exchange, dev)
            run = loop.step
            received = (s - 1) * (sum(b[3] for b in bands)) if K == G ** 3 else None
        for f in range(3):
            run(D.AppState(f), sptr)
        torch.cuda.synchronize(dev)
        node.ctx.set_timing(True)
        node.execute(D.AppState(3), sptr)
        kt = node.ctx.last_timings()
        node.ctx.set_timing(False)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for f in range(args.steps):
            run(D.AppState(4 + f), sptr)
        t_host = time.perf_counter() - t0  # enqueue time: the host keeps ahead of the GPU when this is below ms_per_step
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        if args.exchange and s > 1 and K < G ** 3:
            received = (s - 1) * wx.last_bytes_per_rank
        rec = {"ms_per_step": round(ms, 4), "host_enqueue_ms_per_step": round(t_host / args.steps * 1e3, 4), "kernels_ms": [round(x, 4) for x in kt],
               "exchange_stand_in": bool(args.exchange and s > 1), "window": K, "mrays_per_s_rank": round(K * R / s / ms / 1e3, 1),
               "received_bytes_per_frame": received}
        print(json.dumps({"shards": s, "rank": rank, **rec}), flush=True)
        if s not in out or rec["ms_per_step"] > out[s]["ms_per_step"]:
            out[s] = dict(rec, slowest_rank=rank)
        node.ctx.close()
        del node
    base = out.get(1, {}).get("ms_per_step")
    if base:
        print(json.dumps({"slowest_rank_ms": {s: v["ms_per_step"] for s, v in out.items()},
                          "speedup_without_exchange": {s: round(base / v["ms_per_step"], 2) for s, v in out.items()}}))


if __name__ == "__main__":
    main()
