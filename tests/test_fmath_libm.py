"""ark_fmath.h against an independent libm: the probe-ray directions of a whole C4
frame (32^3 probes x 256 rays = 8.4 M rays, ddgi/common.glsl:12-25 with
common.glsl:121-142 and random.glsl:40-74) computed with the shared transcendental
code that both the HIP kernels and the CPU oracle use, and with glibc's
sinf/cosf/acosf/sqrtf, plus a double-precision evaluation of the same formula from
the same fp32 arguments. The oracle compiles ark_fmath.h too, so without this test
the code would be the only witness for itself (tests/test_fmath.py bounds each
function against float64 numpy; this bounds what the path actually consumes).

Recorded in DESIGN.md §4: max component distance 48 ulp of 1/8 (7.2e-7 absolute),
max angle 6.8e-7 rad between the two fp32 direction sets, and both within 1.3e-6
rad of the double-precision directions."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CXX = shutil.which("g++")


@pytest.mark.skipif(CXX is None, reason="g++ not available")
@pytest.mark.parametrize("dims,rays,frame", [((32, 32, 32), 256, 0), ((48, 16, 48), 512, 1), ((8, 8, 8), 64, 3)])
def test_ray_directions_fmath_vs_glibc(tmp_path, dims, rays, frame):
    exe = str(tmp_path / "fmath_vs_libm")
    src = os.path.join(ROOT, "tests", "cpp", "fmath_vs_libm.cpp")
    r = subprocess.run([CXX, "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "arkoserenderer_amd", "csrc"), src, "-o", exe, "-lm"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe, *map(str, dims), str(rays), str(frame)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    j = json.loads(r.stdout)
    assert j["rays"] == dims[0] * dims[1] * dims[2] * rays
    # fp32 directions of unit length: a few ulp of 1.0 apart (2^-23 = 1.19e-7)
    assert j["max_abs"] <= 1.0e-6, j
    assert j["max_angle_rad"] <= 1.0e-6, j
    assert j["max_component_ulp"] <= 64, j
    assert j["mean_component_ulp"] <= 2.0, j
    # neither is systematically worse than glibc against the exact directions
    assert j["max_angle_fmath_vs_exact_rad"] <= 2.0e-6, j
    assert j["max_angle_fmath_vs_exact_rad"] <= 1.25 * j["max_angle_libm_vs_exact_rad"], j
