"""Overlap headroom on ONE GPU: the C4 window split into S Z-slab contexts whose
updates run (a) one after the other on one stream, (b) concurrently on S streams.
(b) faster than (a) means kernels of different chunks fill each other's tails /
share CUs - the case for a chunk-pipelined update.

    python tools/overlap_proxy.py [--chunks 2 4] [--steps 10]
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
    ap.add_argument("--chunks", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--triangles", type=int, default=10_000_000)
    args = ap.parse_args()
    import torch

    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    scene = S.soup(args.triangles)
    G, R = 32, 256
    grid = D.ProbeGrid((G, G, G), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    for s in args.chunks:
        nodes = []
        for r in range(s):
            cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=G ** 3, max_rays_per_probe=R, max_probe_updates=G ** 3,
                               compute_probe_offsets=True)
            node = D.DDGINode(cfg)
            assert node.construct(scene, grid, 10000.0, device=0, shard_rank=r, shard_count=s,
                                  light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
            nodes.append(node)
        streams = [torch.cuda.Stream(dev) for _ in range(s)]
        main_s = torch.cuda.current_stream(dev).cuda_stream
        frame = 0
        for _ in range(3):
            for n in nodes:
                n.execute(D.AppState(frame), main_s)
            frame += 1
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            for n in nodes:
                n.execute(D.AppState(frame), main_s)
            frame += 1
        torch.cuda.synchronize(dev)
        serial = (time.perf_counter() - t0) / args.steps * 1e3
        t0 = time.perf_counter()
        for _ in range(args.steps):
            for n, st in zip(nodes, streams):
                n.execute(D.AppState(frame), st.cuda_stream)
            frame += 1
        torch.cuda.synchronize(dev)
        conc = (time.perf_counter() - t0) / args.steps * 1e3
        print(json.dumps({"chunks": s, "serial_ms": round(serial, 4), "concurrent_ms": round(conc, 4)}), flush=True)
        for n in nodes:
            n.ctx.close()
        del nodes


if __name__ == "__main__":
    main()
