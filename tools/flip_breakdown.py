"""What the witness oracle's flipped rays are (test infrastructure, one-off): the C5
substitute's whole grid, frame 0, the HIP path against the libm oracle; every flipped
ray (tests/libm_parity.py surfel_stats) classified by its surfel: the hit distance
moved (another surface: a geometric flip) or only the radiance (the same surface lit
differently: a light / shadow flip), and how far.

    python tools/flip_breakdown.py [--config c5|c4] [--variant libm]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--variant", default="libm")
    args = ap.parse_args()
    import libm_parity as L
    import oracle_lib as O
    from arkoserenderer_amd import abi
    from arkoserenderer_amd import ddgi as D
    from arkoserenderer_amd import scene as S

    if args.config == "c5":
        sc, grid, R, z_far = S.city_block(), D.ProbeGrid((48, 16, 48), (5.0, 2.5, 5.0), (2.5, 0.5, 2.5)), 512, 1000.0
        exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0)
    else:
        sc, grid, R, z_far = S.soup(10_000_000), D.ProbeGrid((32, 32, 32), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)), 256, 10000.0
        exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
    N = grid.probe_count()
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, compute_probe_offsets=True, max_rays_per_probe=R, max_probe_updates=N)
    ctx = D.DDGIContext(grid, z_far, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc, variant=args.variant)
    orc.set_scene(sc, threads=16)
    p = D.frame_params(cfg, grid, D.AppState(0), 0, **exposure)
    ctx.update(p)
    ctx.synchronize()
    orc.update(p, threads=16)
    shape = (N, R, 4)
    a = ctx.read(abi.ARK_DDGI_SURFELS).reshape(shape)
    b = orc.read(abi.ARK_DDGI_SURFELS).reshape(shape)
    flipped, _ = L.surfel_stats(a, b)
    idx = np.argwhere(flipped)
    fa = a[flipped].view(np.float16).astype(np.float32)
    fb = b[flipped].view(np.float16).astype(np.float32)
    da, db = fa[:, 3], fb[:, 3]
    dist_ulp = L.f16_ulp_distance(a[flipped][:, 3], b[flipped][:, 3])
    geometric = (dist_ulp > L.FLIP_ULP) | (np.sign(da) != np.sign(db))
    dc = np.abs(fa[:, :3] - fb[:, :3]).max(axis=1)
    out = {"config": args.config, "variant": args.variant, "rays": int(N * R), "flipped": int(len(idx)),
           "geometric": int(geometric.sum()), "radiance_only": int((~geometric).sum()),
           "radiance_only_color_delta": {"median": float(np.median(dc[~geometric])) if (~geometric).any() else 0.0,
                                         "max": float(dc[~geometric].max()) if (~geometric).any() else 0.0},
           "geometric_rel_distance_delta_median": float(np.median(np.abs(da[geometric] - db[geometric]) / np.maximum(np.abs(db[geometric]), 1e-6))) if geometric.any() else 0.0,
           "probes_with_flips": int(len(np.unique(idx[:, 0]))),
           "misses_involved": int(((np.abs(da) >= z_far * 0.99) | (np.abs(db) >= z_far * 0.99)).sum())}
    print(json.dumps(out), flush=True)
    ctx.close()
    orc.close()


if __name__ == "__main__":
    main()
