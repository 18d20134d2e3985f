"""Background-rebuild progress under continuous motion (the loop of
tests/test_gpu_scene_update.py::test_continuous_motion_installs_rebuilds without the
oracle): one instance moves every frame through ark_ddgi_set_instances_async; every
`every` frames one JSON line of the BVH stats (rebuilds, failures, built versions).

    python tools/motion_diag.py [--seconds 30] [--every 25] [--tris 64000] [--sleep 0.03]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--every", type=int, default=25)
    ap.add_argument("--tris", type=int, default=64_000)
    ap.add_argument("--sleep", type=float, default=0.0, help="host seconds per frame (the test's oracle work)")
    args = ap.parse_args()
    import torch

    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    sc = S.soup(args.tris, extent=7.0)
    grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=200, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=200, sun_bvh=abi.ARK_DDGI_SUN_BVH_LIGHT_SPACE)
    ctx = D.DDGIContext(grid, 10000.0, cfg)
    ctx.set_scene(sc)
    stream = torch.cuda.Stream()
    inst0 = sc.instances.copy()
    first, f, t0 = 0, 0, time.time()
    keys = ("refit_version", "bvh_rebuilds", "bvh_built_refit_version", "bvh_rebuild_failures", "bvh_rebuild_ms",
            "sun_rebuilds", "sun_built_refit_version", "sun_rebuild_failures", "sun_build_ms", "sun_node_count")
    while time.time() - t0 < args.seconds:
        inst = inst0.copy()
        M = inst["object_to_world"].reshape(-1, 3, 4).copy()
        M[f % len(inst), :, 3] += np.float32(0.02 * (f + 1))
        c, s_ = np.cos(0.05 * f), np.sin(0.05 * f)
        M[1, :, :3] = np.array([[c, 0, s_], [0, 1, 0], [-s_, 0, c]], np.float32) @ M[1, :, :3]
        inst["object_to_world"] = M.reshape(len(inst), 12)
        ctx.set_instances_async(inst, stream.cuda_stream)
        p = D.frame_params(cfg, grid, D.AppState(f), first, light_pre_exposure=1.0, environment_brightness=1.0)
        ctx.update(p, stream.cuda_stream)
        ctx.synchronize()
        if args.sleep:
            time.sleep(args.sleep)
        first = (first + p.probe_updates) % grid.probe_count()
        f += 1
        if f % args.every == 0:
            st = ctx.bvh_stats()
            print(json.dumps({"frame": f, "t": round(time.time() - t0, 2), **{k: round(float(getattr(st, k)), 2) for k in keys}}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
