"""Per-frame time of the reference's rolling windows (K = 4096 and 2048 probes x 256
rays, DDGINode.h:23,31) on the C4 workload, frames in flight, over many frames and
several repeats (bench.py's reference_windows times 20 frames once). For A/B runs of
library builds (ARK_DDGI_LIB) on one box.

    python tools/window_proxy.py [--frames 200] [--repeats 3]
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
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--windows", type=int, nargs="+", default=[4096, 2048])
    ap.add_argument("--no-sun", action="store_true", help="no light (ark_ddgi_set_lights): no shadow rays - the frame without any shadow work, a bound on what a fused shadow phase could save")
    args = ap.parse_args()
    import torch

    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    scene = S.soup(10_000_000)
    G, R = 32, 256
    grid = D.ProbeGrid((G, G, G), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=max(args.windows), max_rays_per_probe=R,
                       max_probe_updates=max(args.windows), compute_probe_offsets=True)
    node = D.DDGINode(cfg)
    assert node.construct(scene, grid, 10000.0, device=0, light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
    if args.no_sun:
        node.ctx.set_lights(None, ())
    sptr = torch.cuda.current_stream(dev).cuda_stream
    frame = 0
    out = {}
    for K in args.windows:
        node.config.probe_updates_per_frame = K
        for _ in range(8):
            node.execute(D.AppState(frame), sptr)
            frame += 1
        ms = []
        for _ in range(args.repeats):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.frames):
                node.execute(D.AppState(frame), sptr)
                frame += 1
            torch.cuda.synchronize(dev)
            ms.append(round((time.perf_counter() - t0) / args.frames * 1e3, 4))
        out[f"K{K}"] = {"ms_per_frame": ms, "mrays_per_s": round(K * R / min(ms) / 1e3, 1)}
        print(json.dumps({"K": K, "ms_per_frame": ms}), flush=True)
    print(json.dumps(out))
    node.ctx.close()


if __name__ == "__main__":
    main()
