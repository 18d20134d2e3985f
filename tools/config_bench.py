"""Throughput of the DDGI update on the other BASELINE configs at N = 1 (the
bench.py line is C4, the metric's config). C5: the synthetic city block standing in
for Bistro (48x16x48 probes x 512 rays, sun + 4 IES spots); C3: a 262,267-triangle
strip soup standing in for Sponza (24x12x24 x 256, sun + 3 spots). Prints one JSON
line per config.

    python tools/config_bench.py [--config c5 c3] [--steps 5] [--warmup 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(cfg_name):
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S
    if cfg_name == "c5":
        sc = S.city_block()
        grid = D.ProbeGrid((48, 16, 48), (5.0, 2.5, 5.0), (2.5, 0.5, 2.5))
        R, zf = 512, 1000.0
    else:
        sc = S.sponza_substitute()
        grid = D.ProbeGrid(*S.sponza_substitute_grid())
        R, zf = 256, 10000.0
    return sc, grid, R, zf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", nargs="+", default=["c5", "c3"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import torch
    from arkoserenderer_amd import ddgi as D

    torch.cuda.set_device(0)
    for name in args.config:
        sc, grid, R, zf = build(name)
        N = grid.probe_count()
        cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N,
                           compute_probe_offsets=True)
        node = D.DDGINode(cfg)
        t = time.time()
        node.construct(sc, grid, zf, light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0)
        setup = time.time() - t
        app = D.AppState(0)
        for _ in range(args.warmup):
            node.execute(app)
            app = D.AppState(app.frame_index + 1)
        node.ctx.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            node.execute(app)
            app = D.AppState(app.frame_index + 1)
        node.ctx.synchronize()
        ms = (time.perf_counter() - t) * 1e3 / args.steps
        node.ctx.set_timing(True)
        node.execute(app)
        node.ctx.synchronize()
        tm = node.ctx.last_timings()
        node.ctx.set_timing(False)
        node.ctx.set_counting(True)
        node.execute(app)
        node.ctx.synchronize()
        c = node.ctx.counters()
        node.ctx.set_counting(False)
        rays = N * R
        print(json.dumps({"config": name, "triangles": sc.triangle_count, "grid": list(grid.grid_dimensions), "rays_per_probe": R,
                          "spot_lights": len(sc.spots), "mrays_per_s": round(rays / ms / 1e3, 1), "ms_per_step": round(ms, 3),
                          "stage_ms": {"trace": round(tm[1], 3), "shade": round(tm[2], 3), "shadow": round(tm[4], 3), "update": round(tm[3], 3)},
                          "shadow_rays_per_ray": round(c.shadow_rays / rays, 3), "nodes_per_ray": round(c.primary_node_visits / rays, 2),
                          "setup_s": round(setup, 1)}), flush=True)
        node.ctx.close()


if __name__ == "__main__":
    main()
