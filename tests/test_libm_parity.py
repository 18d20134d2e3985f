"""The independent-math witness on the CPU: the bit-exact oracle
(ark_fmath.h, the product's transcendentals; the HIP path equals it bit for bit, see
tests/test_gpu_parity.py) against the -DARK_ORACLE_LIBM oracle (glibc
sinf/cosf/acosf/atan2f/exp2f/powf at the reference's call sites), frame-local, at
SURVEY §8(d)'s tolerances as libm_parity.py states them. The GPU-side counterpart is
tests/test_gpu_libm_parity.py (HIP path vs the libm oracle directly)."""
import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S
import libm_parity as L
import oracle_lib as O
import scenes

ST = (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY, abi.ARK_DDGI_PROBE_OFFSETS)


def _frame_local(sc, grid, cfg, frames, z_far, exposure, variant="libm"):
    d = D.desc_for(grid, z_far, cfg)
    a, b = O.Oracle(d), O.Oracle(d, variant=variant)
    a.set_scene(sc)
    b.set_scene(sc)
    N, R = grid.probe_count(), cfg.rays_per_probe
    first, out = 0, []
    for f in range(frames):
        for w in ST:
            b.write(w, a.read(w))
        p = D.frame_params(cfg, grid, D.AppState(f), first, **exposure)
        a.update(p)
        b.update(p)
        K = p.probe_updates
        shape = (cfg.max_probe_updates, cfg.max_rays_per_probe, 4)
        sa = a.read(abi.ARK_DDGI_SURFELS).reshape(shape)[:K, :R]
        sb = b.read(abi.ARK_DDGI_SURFELS).reshape(shape)[:K, :R]
        st = L.compare_window(grid.grid_dimensions, (first + np.arange(K)) % N, sa, sb,
                              a.read(ST[0]), b.read(ST[0]), a.read(ST[1]), b.read(ST[1]))
        L.check(st, f"frame {f}")
        out.append(st)
        first = (first + K) % N
    a.close()
    b.close()
    return out


def test_libm_oracle_is_a_separate_build():
    """The two builds differ exactly in the transcendentals: ark_fmath.h's sin/cos
    match glibc's to a few ulp, not bit for bit on every input."""
    assert O.load(False).oracle_math_is_libm() == 0 and O.load(True).oracle_math_is_libm() == 1
    x = np.linspace(-2000.0, 2000.0, 100_001, dtype=np.float32)
    ours = O.fmath(0, x)
    assert np.max(np.abs(ours.astype(np.float64) - np.sin(x.astype(np.float64)))) < 1e-6


def test_nocontract_oracle_is_a_separate_build():
    """-DARK_ORACLE_NOCONTRACT: no fused multiply-add; the witness build
    has both freedoms."""
    assert O.load(variant="nocontract").oracle_math_is_nocontract() == 1
    assert O.load(variant="nocontract").oracle_math_is_libm() == 0
    w = O.load(variant="witness")
    assert w.oracle_math_is_nocontract() == 1 and w.oracle_math_is_libm() == 1
    assert O.load().oracle_math_is_nocontract() == 0


@pytest.mark.parametrize("variant", ["libm", "nocontract", "witness"])
def test_cornell_c2_libm_witness(variant):
    """C2 (Cornell 8^3 x 64, the level's exposure, offsets off), 4 frames, within
    SURVEY §8(d) (_frame_local checks); glibc math alone: no flipped ray, every
    surfel within 1 ulp, every atlas texel within 1 ulp."""
    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False,
                       max_rays_per_probe=64, max_probe_updates=512)
    st = _frame_local(sc, grid, cfg, 4, ex["z_far"], dict(light_pre_exposure=ex["light_pre_exposure"],
                                                           environment_brightness=ex["environment_brightness"]), variant)
    print(f"WITNESS C2[{variant}] (flipped rays, irradiance L-inf all, max ulp all, visibility within 1e-3 all) per frame: "
          + str([(s["flipped_rays"], round(s["all"]["irradiance"]["linf"], 6), s["all"]["irradiance"]["max_ulp"],
                  round(s["all"]["visibility"]["within_rel_tol_frac"], 5)) for s in st]))
    if variant == "libm":
        assert all(s["flipped_rays"] == 0 and s["all"]["irradiance"]["max_ulp"] <= 1 for s in st)


@pytest.mark.parametrize("variant", ["libm", "nocontract", "witness"])
def test_features_scene_libm_witness(variant):
    """The features scene (masked alpha test, translucent shadow-only geometry, a
    mirrored instance, textures, sun + 2 IES spots, HDR environment, offsets on),
    4 frames: a few flipped rays per frame, the rest within SURVEY §8(d)."""
    sc = scenes.features_scene()
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=144, compute_probe_offsets=True,
                       max_rays_per_probe=128, max_probe_updates=144)
    st = _frame_local(sc, grid, cfg, 4, 100.0, dict(light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5), variant)
    print(f"WITNESS features[{variant}] (flipped rays, irradiance L-inf all, within 1 ulp all, visibility within 1e-3 all) per frame: "
          + str([(s["flipped_rays"], round(s["all"]["irradiance"]["linf"], 6), round(s["all"]["irradiance"]["within_1ulp_frac"], 5),
                  round(s["all"]["visibility"]["within_rel_tol_frac"], 5)) for s in st]))
    if variant != "nocontract":  # the flips come from the transcendentals (glibc vs ark_fmath.h)
        assert sum(s["flipped_rays"] for s in st) > 0  # the edge cases exist in this scene
