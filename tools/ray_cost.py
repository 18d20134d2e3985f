"""Where the traversal's launch tail comes from: per-ray traversal iterations
(ARK_DDGI_DEBUG_RAY_STEPS of a counting update) of the C4 workload, two frames of
the whole grid (K = N, the same probes with new ray rotations), and the per-probe
sums. Prints the distribution (mean / percentiles / max), hits vs misses, the share
of all iterations in the longest rays, how stable a probe's cost is from one frame
to the next (rank correlation), and where the costly probes are.

    python tools/ray_cost.py [--triangles N] [--grid G] [--rays R] [--json OUT]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def spearman(a, b):
    ra = np.argsort(np.argsort(a)).astype(np.float64)
    rb = np.argsort(np.argsort(b)).astype(np.float64)
    return float(np.corrcoef(ra, rb)[0, 1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--triangles", type=int, default=10_000_000)
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--rays", type=int, default=256)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch

    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    torch.cuda.set_device(0)
    G, R = args.grid, args.rays
    N = G ** 3
    grid = D.ProbeGrid((G, G, G), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N, compute_probe_offsets=True)
    node = D.DDGINode(cfg)
    assert node.construct(S.soup(args.triangles), grid, 10000.0, light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
    ctx = node.ctx
    ctx.set_counting(True)
    frames = []
    for f in range(2):
        node.execute(D.AppState(f))
        ctx.synchronize()
        steps = ctx.read(abi.ARK_DDGI_DEBUG_RAY_STEPS)[: N * R].reshape(N, R).astype(np.float64)
        hits = ctx.read(abi.ARK_DDGI_DEBUG_HITS).view(np.float32).reshape(-1, 4)[: N * R, 0].reshape(N, R)
        frames.append((steps, np.isinf(hits), np.abs(hits)))
    out = {}
    for f, (st, miss, dist) in enumerate(frames):
        flat = st.ravel()
        srt = np.sort(flat)[::-1]
        tot = flat.sum()
        out[f"frame{f}"] = {
            "mean": round(float(flat.mean()), 2),
            "p50": float(np.percentile(flat, 50)), "p90": float(np.percentile(flat, 90)), "p99": float(np.percentile(flat, 99)),
            "p999": float(np.percentile(flat, 99.9)), "max": float(flat.max()),
            "share_of_iterations_top1pct_rays": round(float(srt[: len(srt) // 100].sum() / tot), 4),
            "miss_frac": round(float(miss.mean()), 4),
            "mean_hit": round(float(st[~miss].mean()), 2), "mean_miss": round(float(st[miss].mean()), 2) if miss.any() else None,
            "p99_hit": float(np.percentile(st[~miss], 99)), "p99_miss": float(np.percentile(st[miss], 99)) if miss.any() else None,
        }
    p0, p1 = frames[0][0].sum(1), frames[1][0].sum(1)
    # a cost proxy k_probe_offsets could compute from the hit records it reads anyway:
    # the summed hit distance, misses (and long hits) capped
    caps = {}
    for cap in (2.0, 4.0, 8.0, 32.0):
        proxy0 = np.minimum(frames[0][2], cap).sum(1)
        caps[str(cap)] = {"rank_corr_with_steps_same_frame": round(spearman(proxy0, p0), 4),
                          "rank_corr_with_steps_next_frame": round(spearman(proxy0, p1), 4)}
    # per ray: how well distance predicts the ray's iterations
    d0 = np.minimum(frames[0][2], 64.0).ravel()
    ray_corr = round(spearman(d0[::7], frames[0][0].ravel()[::7]), 4)
    m0, m1 = frames[0][0].max(1), frames[1][0].max(1)
    idx = np.arange(N)
    x, z, y = idx % G, (idx % (G * G)) // G, idx // (G * G)
    edge = (np.minimum.reduce([x, y, z, G - 1 - x, G - 1 - y, G - 1 - z]) == 0)
    out["per_probe"] = {
        "sum_cv": round(float(p0.std() / p0.mean()), 4),
        "sum_rank_corr_frame0_frame1": round(spearman(p0, p1), 4),
        "max_rank_corr_frame0_frame1": round(spearman(m0, m1), 4),
        "edge_probe_mean_sum_over_interior": round(float(p0[edge].mean() / p0[~edge].mean()), 3),
        "top1pct_probes_frac_edge": round(float(edge[np.argsort(p0)[::-1][: N // 100]].mean()), 3),
        "per_probe_max_p50_p99": [float(np.percentile(m0, 50)), float(np.percentile(m0, 99))],
        "distance_proxy": caps,
        "ray_rank_corr_distance_steps": ray_corr,
    }
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
