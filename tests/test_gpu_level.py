"""GPU parity of scenes loaded by the reference's rules:
Sponza.arklvl's DamagedHelmet object with its decoded textures (sRGB albedo and
emissive, metallic-roughness data map), sun and three IES spot lights from the
level, exposure from the level camera; texture wrap modes (mirrored repeat, per-axis
wraps) on the features scene. Bar: bit-exact against the CPU oracle. The JPEG
texels come from PIL's decoder, so they are not pinned to the reference's image
loader; the loading rules are (tests/test_level.py)."""
import os

import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import level as LV
import scenes
from parity import run_pair

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _assert_exact(reports):
    for f, rep in enumerate(reports):
        for r in rep:
            assert r["mismatch"] == 0, f"frame {f}: {r}"
            if r["name"] != "offsets":
                assert r["nonzero"] > 0, f"frame {f}: oracle output {r['name']} is all zero"


def test_sponza_level_textured_helmet():
    lv = LV.load_level(os.path.join(HERE, "assets", "levels", "Sponza.arklvl"), allow_missing_meshes=True)
    assert len(lv.scene.textures) == 5 + 3 and len(lv.scene.spots) == 3 and lv.scene.sun is not None
    # a probe cage around the helmet (at y = 4.5, scale 1.2) instead of the level's auto grid
    grid = D.ProbeGrid((5, 4, 5), (0.6, 0.6, 0.6), (-1.2, 3.6, -1.2))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=100, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=100)
    reps = run_pair(lv.scene, grid, cfg, 2, lv.z_far, lv.exposure())
    _assert_exact(reps)


@pytest.mark.parametrize("wrap", [abi.ARK_WRAP_MIRRORED_REPEAT, abi.ARK_WRAP_CLAMP_TO_EDGE,
                                  abi.ark_wrap_axes(abi.ARK_WRAP_MIRRORED_REPEAT, abi.ARK_WRAP_CLAMP_TO_EDGE),
                                  abi.ark_wrap_axes(abi.ARK_WRAP_REPEAT, abi.ARK_WRAP_MIRRORED_REPEAT)])
def test_features_scene_wrap_modes(wrap):
    sc = scenes.features_scene(room_wrap=wrap)
    grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=144, compute_probe_offsets=True,
                       max_rays_per_probe=64, max_probe_updates=144)
    reps = run_pair(sc, grid, cfg, 2, 100.0, dict(light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5))
    _assert_exact(reps)
