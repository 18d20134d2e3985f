"""Interleaved A/B of the sun's shadow-ray structure (VERDICT r05 "do this" #6): the
world BVHs (ArkDdgiDesc.sun_bvh WORLD) against the light-space BVH (LIGHT_SPACE) on the
C4 workload, in ONE process on one box, arms alternated `reps` times:

  * C4 whole grid (K = N), ms per step over `steps` steps (frames in flight);
  * the reference's window K = 2,048 (DDGINode.h:31), ms per frame over `frames` frames;
  * the 8 Z-slabs of P = 8 (slab contexts sharing the arm's scene), each rank's whole
    slab window, ms per step; the slowest rank is the strong-scaling step;
  * per arm once, the HIP-event shadow phase of a serial C4 update.

    python tools/sun_ab.py [--reps 5] [--steps 10] [--frames 100]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--frames", type=int, default=100)
    ap.add_argument("--slab-steps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    scene = S.soup(10_000_000)
    G, R = 32, 256
    N = G ** 3
    grid = D.ProbeGrid((G, G, G), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    arms = {}
    for name, mode in (("world", abi.ARK_DDGI_SUN_BVH_WORLD), ("light", abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE)):
        cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N, compute_probe_offsets=True, sun_bvh=mode)
        node = D.DDGINode(cfg)
        assert node.construct(scene, grid, 10000.0, device=0, **exposure)
        slabs = []
        for r in range(8):
            sc_cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N, compute_probe_offsets=True, sun_bvh=mode)
            sn = D.DDGINode(sc_cfg)
            sn.ctx = D.DDGIContext(grid, 10000.0, sc_cfg, 0, r, 8)
            sn.ctx.share_scene(node.ctx)
            sn.grid = grid
            sn.exposure = dict(node.exposure) if hasattr(node, "exposure") else None
            slabs.append(sn)
        st = node.ctx.bvh_stats()
        arms[name] = {"node": node, "slabs": slabs, "frame": 0, "sun_nodes": int(st.sun_node_count),
                      "c4": [], "k2048": [], "slab_slowest": [], "slab_all": []}
        print(json.dumps({"arm": name, "sun_node_count": int(st.sun_node_count), "build_ms": round(st.build_ms, 1)}), flush=True)

    def run(node, arm, n, K):
        node.config.probe_updates_per_frame = K
        for _ in range(3):
            node.execute(D.AppState(arm["frame"]), sptr)
            arm["frame"] += 1
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(n):
            node.execute(D.AppState(arm["frame"]), sptr)
            arm["frame"] += 1
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / n * 1e3

    for rep in range(args.reps):
        for name, arm in arms.items():
            node = arm["node"]
            arm["c4"].append(round(run(node, arm, args.steps, N), 4))
            arm["k2048"].append(round(run(node, arm, args.frames, 2048), 4))
            per = []
            for sn in arm["slabs"]:
                per.append(round(run(sn, arm, args.slab_steps, N), 4))
            arm["slab_all"].append(per)
            arm["slab_slowest"].append(max(per))
            print(json.dumps({"rep": rep, "arm": name, "c4_ms": arm["c4"][-1], "k2048_ms": arm["k2048"][-1], "slab_slowest_ms": arm["slab_slowest"][-1]}), flush=True)
    out = {}
    for name, arm in arms.items():
        node = arm["node"]
        node.config.probe_updates_per_frame = N
        node.ctx.set_timing(True)
        kt = []
        for _ in range(3):
            node.execute(D.AppState(arm["frame"]), sptr)
            arm["frame"] += 1
            kt.append(node.ctx.last_timings())
        node.ctx.set_timing(False)
        med = lambda v: round(statistics.median(v), 4)  # noqa: E731
        out[name] = {"sun_node_count": arm["sun_nodes"], "c4_ms": arm["c4"], "c4_median": med(arm["c4"]), "c4_mrays_per_s": round(N * R / med(arm["c4"]) / 1e3, 1),
                     "k2048_ms": arm["k2048"], "k2048_median": med(arm["k2048"]), "k2048_mrays_per_s": round(2048 * R / med(arm["k2048"]) / 1e3, 1),
                     "slab_slowest_ms": arm["slab_slowest"], "slab_slowest_median": med(arm["slab_slowest"]),
                     "serial_shadow_ms": round(sum(k[4] for k in kt) / len(kt), 4), "serial_update_ms": round(sum(k[0] for k in kt) / len(kt), 4)}
    w, l = out["world"], out["light"]
    out["light_vs_world"] = {k: round(w[k] / l[k], 4) for k in ("c4_median", "k2048_median", "slab_slowest_median")}
    out["spread"] = {name: {k: round((max(out[name][k]) - min(out[name][k])) / statistics.median(out[name][k]), 4) for k in ("c4_ms", "k2048_ms", "slab_slowest_ms")}
                     for name in ("world", "light")}
    print(json.dumps(out), flush=True)
    for arm in arms.values():
        for sn in arm["slabs"]:
            sn.ctx.close()
        arm["node"].ctx.close()


if __name__ == "__main__":
    main()
