"""GPU parity on the edge cases of the oracle's closed-form scenes: every ray a miss
(environment only), a single probe inside a front-facing emissive cube, every hit a
backface (outward cube), the maximum 512 rays per probe, a one-probe window with
offsets on, and a ragged window wrapping around the grid end."""
import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from parity import run_pair
import test_oracle_kat as K

pytestmark = pytest.mark.gpu


def _exact(reps):
    for f, rep in enumerate(reps):
        for r in rep:
            assert r["mismatch"] == 0, f"frame {f}: {r}"


def test_all_rays_miss():
    grid = D.ProbeGrid((2, 2, 2), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=8, max_rays_per_probe=64, max_probe_updates=8)
    _exact(run_pair(K._far_triangle_scene(), grid, cfg, 3, 10000.0, dict(light_pre_exposure=1.0, environment_brightness=0.7)))


@pytest.mark.parametrize("inward", [True, False])
def test_single_probe_in_cube(inward):
    """inward: all front hits of an emissive cube; outward: all backfaces (colour 0,
    distance x 0.2, the offset rule's backface branch)."""
    grid = D.ProbeGrid((1, 1, 1), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
    cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=1, max_rays_per_probe=128, max_probe_updates=1,
                       compute_probe_offsets=True)
    _exact(run_pair(K._cube_scene(inward=inward, emissive=1.0), grid, cfg, 3, 100.0, dict(light_pre_exposure=1.0)))


def test_max_rays_per_probe():
    """R = 512 (ARK_DDGI_MAX_RAYS_PER_PROBE): 8 waves of rays per probe, the update's
    LDS staging at its largest."""
    grid = D.ProbeGrid((3, 2, 3), (0.6, 0.6, 0.6), (-0.6, 0.4, -0.6))
    cfg = D.DDGIConfig(rays_per_probe=512, probe_updates_per_frame=18, max_rays_per_probe=512, max_probe_updates=18,
                       compute_probe_offsets=True)
    _exact(run_pair(K._cube_scene(inward=True, emissive=0.5), grid, cfg, 2, 100.0, dict(light_pre_exposure=1.0)))


def test_wrapping_ragged_window():
    """K = 7 of N = 18 probes, R = 37: windows wrap around the grid end (first + K > N)
    and neither K nor R is a multiple of anything the kernels tile by."""
    grid = D.ProbeGrid((3, 2, 3), (0.6, 0.6, 0.6), (-0.6, 0.4, -0.6))
    cfg = D.DDGIConfig(rays_per_probe=37, probe_updates_per_frame=7, max_rays_per_probe=40, max_probe_updates=8,
                       compute_probe_offsets=True)
    _exact(run_pair(K._cube_scene(inward=True, emissive=0.5), grid, cfg, 5, 100.0, dict(light_pre_exposure=1.0)))
