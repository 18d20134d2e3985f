"""Shared GPU-vs-oracle comparison helpers (test infrastructure)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
import oracle_lib as O

RESOURCES = {
    "surfels": abi.ARK_DDGI_SURFELS,
    "irradiance": abi.ARK_DDGI_ATLAS_IRRADIANCE,
    "visibility": abi.ARK_DDGI_ATLAS_VISIBILITY,
    "offsets": abi.ARK_DDGI_PROBE_OFFSETS,
}


def make_desc(grid, z_far, cfg, device=0, shard_rank=0, shard_count=1):
    d = abi.ArkDdgiDesc()
    d.struct_size = C.sizeof(abi.ArkDdgiDesc)
    for k in range(3):
        d.grid_dims[k] = grid.grid_dimensions[k]
        d.probe_spacing[k] = grid.probe_spacing[k]
        d.offset_to_first[k] = grid.offset_to_first[k]
    d.z_far = z_far
    d.max_rays_per_probe = cfg.max_rays_per_probe
    d.max_probe_updates = cfg.max_probe_updates
    d.device = device
    d.clear_overflow_mode = cfg.clear_overflow_mode
    d.shard_rank = shard_rank
    d.shard_count = shard_count
    return d


def diff_report(name, g, o):
    """Bitwise comparison of two fp16 (uint16) or fp32 arrays; NaN == NaN."""
    if g.dtype == np.uint16:
        gf, of = O.f16_to_f32(g), O.f16_to_f32(o)
    else:
        gf, of = g, o
    both_nan = np.isnan(gf) & np.isnan(of)
    neq = (g != o) & ~both_nan
    n = int(np.count_nonzero(neq))
    with np.errstate(invalid="ignore"):
        d = np.abs(gf.astype(np.float64) - of.astype(np.float64))
    d[both_nan] = 0
    d[np.isinf(gf) & np.isinf(of) & (np.sign(gf) == np.sign(of))] = 0
    linf = float(np.nanmax(d)) if d.size else 0.0
    return {"name": name, "mismatch": n, "total": int(g.size), "linf": linf}


def run_pair(scene, grid, cfg, frames, z_far=10000.0, exposure=None, threads=8, check_each_frame=True):
    """Runs `frames` updates through the HIP path and the oracle; returns the
    per-frame diff reports (every frame, or the last one only: frames are then
    queued back to back without a host sync between them)."""
    exposure = exposure or {}
    ctx = D.DDGIContext(grid, z_far, cfg)
    ctx.set_scene(scene)
    orc = O.Oracle(ctx.desc)
    orc.set_scene(scene, threads)
    node_idx = 0
    reports = []
    for f in range(frames):
        p = D.frame_params(cfg, grid, D.AppState(f), node_idx, **exposure)
        ctx.update(p)
        if check_each_frame or f == frames - 1:
            ctx.synchronize()
        orc.update(p, threads)
        node_idx = (node_idx + p.probe_updates) % grid.probe_count()
        if check_each_frame or f == frames - 1:
            rep = []
            for k, w in RESOURCES.items():
                g, o = ctx.read(w), orc.read(w)
                r = diff_report(k, g, o)
                r["nonzero"] = int(np.count_nonzero(o))
                rep.append(r)
            reports.append(rep)
    ctx.close()
    orc.close()
    return reports
