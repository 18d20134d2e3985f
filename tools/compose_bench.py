"""The lighting-compose consumer (ark_ddgi_lighting_compose) alone,
for counter passes: a 32^3-probe context (the C4 grid; atlases of C4's size) over a
small strip soup, two updates, then `reps` compose launches at 1920x1080 with every
flag on over a seeded synthetic G-buffer (tests/compose_inputs.py), timed with HIP
events on the stream it runs on. Prints one JSON line: ms per launch, the plane bytes
(G-buffer in + RGBA16F out) and their rate.

    python tools/compose_bench.py [--reps 50] [--size 1920x1080]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--size", default="1920x1080")
    args = ap.parse_args()
    import torch

    import compose_inputs as CI
    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    torch.cuda.set_device(0)
    grid = D.ProbeGrid((32, 32, 32), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=32768, max_rays_per_probe=64, max_probe_updates=32768)
    ctx = D.DDGIContext(grid, 10000.0, cfg)
    ctx.set_scene(S.soup(200_000, extent=31.0))
    for f in range(2):
        ctx.update(D.frame_params(cfg, grid, D.AppState(f), 0, light_pre_exposure=1.0, environment_brightness=1.0))
    ctx.synchronize()
    W, H = (int(v) for v in args.size.split("x"))
    g = CI.gbuffer(W, H, seed=5)
    dev = {k: torch.from_numpy(v).cuda() for k, v in g.items()}
    out = torch.empty((H, W, 4), dtype=torch.int16, device="cuda")
    cam = CI.camera(W, H, eye=(16.0, 16.0, -6.0), target=(16.0, 14.0, 16.0))
    planes = {k: t.data_ptr() for k, t in dev.items()}
    side = torch.cuda.Stream()
    for _ in range(3):
        ctx.lighting_compose(W, H, abi.ARK_COMPOSE_DEFAULT_FLAGS, cam, planes, out.data_ptr(), side.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(side)
    for _ in range(args.reps):
        ctx.lighting_compose(W, H, abi.ARK_COMPOSE_DEFAULT_FLAGS, cam, planes, out.data_ptr(), side.cuda_stream)
    e1.record(side)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    plane_bytes = sum(v.nbytes for v in g.values()) + W * H * 8
    print(json.dumps({"size": args.size, "ms": round(ms, 4), "plane_bytes": plane_bytes, "gb_per_s": round(plane_bytes / ms / 1e6, 1),
                      "frac": round(plane_bytes / ms / 1e6 / 8000.0, 4), "out_sha": __import__("hashlib").sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]}))
    ctx.close()


if __name__ == "__main__":
    main()
