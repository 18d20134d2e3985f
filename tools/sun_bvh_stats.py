"""Shadow rays of the sun in world space vs light space (host simulation, no GPU):
node visits and triangle tests per shadow ray of the C4 soup (or a scaled one)
through ark_ddgi_debug_bvh8_trace_stats, for
  world: the world-space BVH8 (what k_trace_shadow traverses), rays P + t L;
  light: a BVH8 built over the triangles in the sun's frame (u, v, w = L, double
         precision), rays P' + t (0, 0, 1) (axis-aligned: the slab test of x and y
         degenerates to an interval check), with SAH face weights ARK_BVH_AREA_W.
Rays: random points on random triangles, on the side facing the sun (what
k_shadow_gen emits for lit front hits). Closest-hit statistics (the simulator's
order), a proxy for the any-hit cost.

    python tools/sun_bvh_stats.py [--triangles N] [--rays R] [--weights "1,1,1" "1,0.1,0.1" ...]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools", "sim"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def sun_frame(sun_dir):
    """L = -normalize(sun_dir) in fp32 as the kernels evaluate it, and an orthonormal
    frame (u, v, w = L / |L|) in double."""
    v = np.asarray(sun_dir, np.float32)
    dd = np.float32(v[0] * v[0]) + np.float32(v[1] * v[1])
    dd = np.float32(dd + np.float32(v[2] * v[2]))
    s = np.float32(np.float32(1.0) / np.sqrt(dd, dtype=np.float32))
    L = -(v * s).astype(np.float32)
    w = L.astype(np.float64) / np.linalg.norm(L.astype(np.float64))
    h = np.array([1.0, 0.0, 0.0]) if abs(w[0]) < 0.9 else np.array([0.0, 1.0, 0.0])
    u = np.cross(h, w)
    u /= np.linalg.norm(u)
    vv = np.cross(w, u)
    return L, np.stack([u, vv, w])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--triangles", type=int, default=10_000_000)
    ap.add_argument("--rays", type=int, default=65536)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--weights", nargs="+", default=["1,1,1", "1,0.25,0.25", "1,0.1,0.1", "1,0.02,0.02"])
    ap.add_argument("--scene", choices=["soup", "city", "sponza"], default="soup", help="soup (--triangles), the C5 city block or the C3 substitute")
    ap.add_argument("--any-hit", action="store_true", help="shadow-ray statistics: tmin 0.025, first hit ends the ray (ARK_SIM_ANYHIT)")
    args = ap.parse_args()
    from arkoserenderer_amd import abi
    from arkoserenderer_amd import scene as S
    from bvh_stats import world_triangles

    sc = {"soup": lambda: S.soup(args.triangles), "city": S.city_block, "sponza": S.sponza_substitute}[args.scene]()
    tris = world_triangles(sc)
    L, F = sun_frame(sc.sun[1] if sc.sun is not None else (0.5, -1.0, 0.2))
    if args.any_hit:
        os.environ["ARK_SIM_ANYHIT"] = "1"
    rng = np.random.default_rng(3)
    pick = rng.integers(0, tris.shape[0], args.rays)
    t = tris[pick].reshape(-1, 3, 3).astype(np.float64)
    r1, r2 = rng.random(args.rays), rng.random(args.rays)
    sq = np.sqrt(r1)
    P = (1 - sq)[:, None] * t[:, 0] + (sq * (1 - r2))[:, None] * t[:, 1] + (sq * r2)[:, None] * t[:, 2]
    rays_w = np.zeros((args.rays, 7), np.float32)
    rays_w[:, 0:3] = P
    rays_w[:, 3:6] = L
    rays_w[:, 6] = 20000.0
    tris_l = (tris.reshape(-1, 3).astype(np.float64) @ F.T).reshape(-1, 9).astype(np.float32)
    rays_l = np.zeros((args.rays, 7), np.float32)
    rays_l[:, 0:3] = P @ F.T
    rays_l[:, 3:6] = (0.0, 0.0, 1.0)
    rays_l[:, 6] = 20000.0
    lib = abi.load_library()
    import bvhsim  # tools/sim: the simulator library

    sim = bvhsim.load()
    res = {}
    for name, tr, ry, ws in [("world", tris, rays_w, ["1,1,1"])] + [("light", tris_l, rays_l, args.weights)]:
        for w in ws:
            os.environ["ARK_BVH_AREA_W"] = w
            out = (C.c_uint64 * 9)()
            t0 = time.time()
            sim.ark_ddgi_debug_bvh8_trace_stats(tr.ctypes.data, tr.shape[0], ry.ctypes.data, ry.shape[0], args.threads, out, None)
            n = ry.shape[0]
            key = f"{name} {w}"
            res[key] = {"nodes_per_ray": round(out[0] / n, 3), "tris_per_ray": round(out[1] / n, 3), "hit_frac": round(out[2] / n, 4),
                        "bvh8_nodes": out[3], "max_steps": out[5], "depth": out[6], "s": round(time.time() - t0, 1)}
            print(key, json.dumps(res[key]), flush=True)


if __name__ == "__main__":
    main()
