"""The HIP path against the libm-math oracle (VERDICT r03 "do this" #1).

The bit-exact parity suite compares the HIP kernels with an oracle that compiles the
product's own ark_fmath.h, so every sin/cos/acos/atan/pow/exp2 on the path is
witnessed by the same code on both sides. Here the witness is the -DARK_ORACLE_LIBM
build of the oracle (glibc sinf/cosf/acosf/atan2f/exp2f/powf; oracle/Makefile) at the
reference's call sites: common.glsl:126-139 (Fibonacci, Rodrigues),
probeUpdateIrradiance.comp:57 (pow 1/5), probeUpdateVisibility.comp:46 (pow cos 50),
probeSampling.glsl:40,108,149, lighting.glsl:32-35 (IES atan/acos),
probeUpdateOffset.comp:93 (exp2). Frame-local, at SURVEY §8(d)'s tolerances, with the
flipped-ray accounting of tests/libm_parity.py. Each case prints its statistics
(pytest -s; DESIGN.md §4 quotes them).

VERDICT r05 "do this" #5: the same cases against the -DARK_ORACLE_NOCONTRACT oracle
(every product and sum rounded separately, as SPIR-V NoContraction would give, where
the default oracle fuses as the kernels do: dotFma, the probe update's accumulations,
the cross and dot products of intersectTri) and against both freedoms at once
(-DARK_ORACLE_LIBM -DARK_ORACLE_NOCONTRACT, the "witness" build).
"""
import json

import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import libm_parity as L
import oracle_lib as O
import scenes
from test_gpu_fullsize import _windows

pytestmark = pytest.mark.gpu

ST = (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY, abi.ARK_DDGI_PROBE_OFFSETS)


VARIANTS = ["libm", "nocontract", "witness"]


def _report(name, frame, st):
    """The full statistics, then one line with the clean-probe and all-probe atlas
    figures side by side (the all-probe ones include the probes with a
    flipped ray, where no tolerance is asserted)."""
    print(f"LIBM {name} frame {frame}: " + json.dumps(st), flush=True)
    # name: "<case>[<variant>]"
    c, a = st["clean"], st["all"]
    print(f"LIBM-SUMMARY {name} frame {frame}: flipped {st['flipped_rays']}/{st['rays']} rays; "
          f"irradiance L-inf clean {c['irradiance']['linf']:.3g} / all {a['irradiance']['linf']:.3g}, "
          f"within 1 ulp clean {c['irradiance']['within_1ulp_frac']:.5f} / all {a['irradiance']['within_1ulp_frac']:.5f}; "
          f"visibility within 1e-3 clean {c['visibility']['within_rel_tol_frac']:.5f} / all {a['visibility']['within_rel_tol_frac']:.5f} "
          f"(probes clean {c['probes']} / all {a['probes']})", flush=True)


def _whole_grid(name, sc, grid, cfg, frames, z_far, exposure, variant="libm", surfel_ulp=L.SURFEL_ULP):
    """Every frame: the libm oracle starts from the HIP context's state, both run the
    frame, the whole window is compared."""
    ctx = D.DDGIContext(grid, z_far, cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc, variant=variant)
    orc.set_scene(sc, threads=16)
    N, R = grid.probe_count(), cfg.rays_per_probe
    first, flipped = 0, 0
    name = f"{name}[{variant}]"
    for f in range(frames):
        for w in ST:
            orc.write(w, ctx.read(w))
        p = D.frame_params(cfg, grid, D.AppState(f), first, **exposure)
        ctx.update(p)
        ctx.synchronize()
        orc.update(p, threads=16)
        K = p.probe_updates
        shape = (cfg.max_probe_updates, cfg.max_rays_per_probe, 4)
        sg = ctx.read(abi.ARK_DDGI_SURFELS).reshape(shape)[:K, :R]
        so = orc.read(abi.ARK_DDGI_SURFELS).reshape(shape)[:K, :R]
        st = L.compare_window(grid.grid_dimensions, (first + np.arange(K)) % N, sg, so,
                              ctx.read(ST[0]), orc.read(ST[0]), ctx.read(ST[1]), orc.read(ST[1]))
        _report(name, f, st)
        L.check(st, f"{name} frame {f}", surfel_ulp)
        flipped += st["flipped_rays"]
        first = (first + K) % N
    ctx.close()
    orc.close()
    return flipped


@pytest.mark.parametrize("variant", VARIANTS)
def test_cornell_c2_vs_libm_oracle(variant):
    """C2: Cornell 8^3 x 64, the level's exposure, offsets off, 4 frames."""
    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=512)
    _whole_grid("C2", sc, grid, cfg, 4, ex["z_far"], dict(light_pre_exposure=ex["light_pre_exposure"],
                                                           environment_brightness=ex["environment_brightness"]), variant)


# Drift bounds of the free-running C2 run (not SURVEY §8(d)'s one-frame tolerances,
# which the frame-local cases above assert): measured 8-frame figures are quoted in
# DESIGN.md §4; these only catch a divergence that grows without bound.
DRIFT_IRR_LINF = 0.05
DRIFT_WITHIN_1ULP = 0.9


def test_cornell_c2_free_running_drift():
    """C2, 8 frames, the libm oracle NOT re-seeded: both start from a
    reset history and each runs from its own state, so a last-bit difference of one
    frame is carried into the next frames through the indirect bounce (the surfels'
    irradiance lookups read the previous frame's atlases, probeSampling.glsl:64-163).
    Prints the drift per frame against SURVEY §8(d)'s tolerances (all probes)."""
    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=512)
    exposure = dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    ctx = D.DDGIContext(grid, ex["z_far"], cfg)
    ctx.set_scene(sc)
    orc = O.Oracle(ctx.desc, libm=True)
    orc.set_scene(sc, threads=16)
    N, R = grid.probe_count(), cfg.rays_per_probe
    rows = []
    try:
        for f in range(8):
            p = D.frame_params(cfg, grid, D.AppState(f), 0, **exposure)
            ctx.update(p)
            ctx.synchronize()
            orc.update(p, threads=16)
            shape = (cfg.max_probe_updates, cfg.max_rays_per_probe, 4)
            sg = ctx.read(abi.ARK_DDGI_SURFELS).reshape(shape)[:N, :R]
            so = orc.read(abi.ARK_DDGI_SURFELS).reshape(shape)[:N, :R]
            st = L.compare_window(grid.grid_dimensions, np.arange(N), sg, so, ctx.read(ST[0]), orc.read(ST[0]), ctx.read(ST[1]), orc.read(ST[1]))
            _report("C2-free", f, st)
            a = st["all"]
            rows.append((f, st["flipped_rays"], a["irradiance"]["linf"], a["irradiance"]["within_1ulp_frac"], a["visibility"]["within_rel_tol_frac"]))
    finally:
        ctx.close()
        orc.close()
    print("LIBM-DRIFT C2 (frame, flipped rays, irradiance L-inf, within 1 ulp, visibility within 1e-3; all probes; "
          f"one-frame tolerances L-inf < {L.IRR_TOL_LINF}, >= {L.ULP_FRACTION}): " + json.dumps(rows), flush=True)
    for f, _, linf, ulp, _ in rows:
        assert np.isfinite(linf) and linf < DRIFT_IRR_LINF, rows
        assert ulp >= DRIFT_WITHIN_1ULP, rows


@pytest.mark.parametrize("variant", VARIANTS)
def test_features_scene_vs_libm_oracle(variant):
    """Masked alpha test, translucent shadow-only geometry, mirrored instance,
    textures, sun + 2 IES spots (atan/acos LUT lookups), HDR environment, offsets on
    (exp2), 4 frames."""
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=144, compute_probe_offsets=True,
                       max_rays_per_probe=128, max_probe_updates=144)
    _whole_grid("features", sc, grid, cfg, 4, 100.0, dict(light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5), variant)


def _windows_full_size(name, scene, dims, spacing, origin, R, z_far, exposure, windows, variant="libm"):
    """The HIP path on the whole grid (K = N, as bench.py); the libm oracle on windows
    of 32 probes over every Z-slab: frame 0 from a reset oracle, frame 1 from the HIP
    path's frame-0 atlases and offsets (test_gpu_fullsize.py's method)."""
    grid = D.ProbeGrid(dims, spacing, origin)
    N = grid.probe_count()
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, max_rays_per_probe=R, max_probe_updates=N, compute_probe_offsets=True)
    ctx = D.DDGIContext(grid, z_far, cfg)
    ctx.set_scene(scene)
    ocfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=32, max_rays_per_probe=R, max_probe_updates=32, compute_probe_offsets=True)
    orc = O.Oracle(D.desc_for(grid, z_far, ocfg), variant=variant)
    orc.set_scene(scene, threads=16)
    start = None
    name = f"{name}[{variant}]"
    for frame in range(2):
        p = D.frame_params(cfg, grid, D.AppState(frame), 0, **exposure)
        ctx.update(p)
        ctx.synchronize()
        g = {w: ctx.read(w) for w in (abi.ARK_DDGI_SURFELS,) + ST}
        sg_all, so_all, probes_all = [], [], []
        for first, k in windows:
            if frame == 0:
                orc.reset_history()
            else:
                for w in ST:
                    orc.write(w, start[w])
            ocfg.probe_updates_per_frame = k
            orc.update(D.frame_params(ocfg, grid, D.AppState(frame), first, **exposure), threads=16)
            probes = np.arange(first, first + k)
            sg_all.append(g[abi.ARK_DDGI_SURFELS].reshape(N, R, 4)[probes])
            so_all.append(orc.read(abi.ARK_DDGI_SURFELS).reshape(32, R, 4)[:k])
            # the window's tiles of the oracle's atlases into a copy of the HIP ones
            for w, res, ch in ((ST[0], 8, 4), (ST[1], 16, 2)):
                m = L.tile_mask(dims, probes, res, interior=False)
                key = ("o", w)
                if key not in g:
                    g[key] = g[w].copy()
                g[key].reshape(m.shape[0], m.shape[1], ch)[m] = orc.read(w).reshape(m.shape[0], m.shape[1], ch)[m]
            probes_all.append(probes)
        st = L.compare_window(dims, np.concatenate(probes_all), np.concatenate(sg_all), np.concatenate(so_all),
                              g[ST[0]], g[("o", ST[0])], g[ST[1]], g[("o", ST[1])])
        _report(name, frame, st)
        L.check(st, f"{name} frame {frame}")
        start = g
    ctx.close()
    orc.close()


@pytest.mark.parametrize("variant", VARIANTS)
def test_c4_full_size_vs_libm_oracle(variant):
    """C4 as bench.py runs it: 10 M triangles, 32^3 x 256, sun, offsets on; 8 windows
    of 32 probes (one x row per Z-slab of 4), frames 0 and 1."""
    dims = (32, 32, 32)
    _windows_full_size("C4", S.soup(10_000_000), dims, (1.0, 1.0, 1.0), (0.0, 0.0, 0.0), 256, 10000.0,
                       dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0), _windows(dims, 8), variant)


@pytest.mark.parametrize("config", ["c4", "c5"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_whole_grid_vs_libm_oracle(variant, config):
    """C4 (the whole 32^3 x 256 window, 8.4 M rays a frame) and the C5 substitute (48x16x48
    x 512, sun + 4 IES spots, 18.9 M rays) on EVERY probe, frames 0 and 1, against each
    witness oracle: the subsets above, all probes. About a minute of oracle work per
    case: runs with ARK_SLOW_TESTS=1."""
    import os

    if os.environ.get("ARK_SLOW_TESTS") != "1":
        pytest.skip("whole grids against the witnesses: ARK_SLOW_TESTS=1")
    if config == "c4":
        sc, grid, R, z_far = S.soup(10_000_000), D.ProbeGrid((32, 32, 32), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)), 256, 10000.0
        exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)
    else:
        sc, grid, R, z_far = S.city_block(), D.ProbeGrid((48, 16, 48), (5.0, 2.5, 5.0), (2.5, 0.5, 2.5)), 512, 1000.0
        exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0)
    N = grid.probe_count()
    cfg = D.DDGIConfig(rays_per_probe=R, probe_updates_per_frame=N, compute_probe_offsets=True, max_rays_per_probe=R, max_probe_updates=N)
    # SURVEY §8(d)'s atlas tolerances and the flip fraction asserted; the largest
    # unflipped surfel difference reported (11 fp16 ulp once at C4, nocontract frame 1:
    # profiles/r06_za_c4_whole_grid_witness.log), not held to the windows' 8
    _whole_grid(f"{config.upper()}-whole", sc, grid, cfg, 2, z_far, exposure, variant, surfel_ulp=None)


@pytest.mark.parametrize("variant", VARIANTS)
def test_c5_substitute_full_size_vs_libm_oracle(variant):
    """C5 substitute: the instanced city block (~3 M triangles), 48x16x48 x 512, sun +
    4 IES spot lights (the IES LUT's atan/acos on every lit spot sample); 8 windows of
    32 probes over every Z-slab, frames 0 and 1."""
    dims = (48, 16, 48)
    _windows_full_size("C5", S.city_block(), dims, (5.0, 2.5, 5.0), (2.5, 0.5, 2.5), 512, 1000.0,
                       dict(light_pre_exposure=1.0, ambient_illuminance=0.02, environment_brightness=1.0), _windows(dims, 8), variant)
