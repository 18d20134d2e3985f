"""Generates the committed golden fixtures in tests/golden/.

* half_rne.npz   — fp32 inputs and their fp16 bits from the reference's own
                   deps/half/half.hpp (oracle/_ref/half_kat, built by
                   oracle/Makefile.ref from /root/reference); pins the oracle's
                   fp16 store rounding.
* <scene>.npz    — oracle outputs (sha256 per frame and resource, plus the last
                   irradiance atlas) for the parity scenes; the CPU suite re-derives
                   them from the oracle, the GPU suite checks the HIP path against them.

Run from the repo root:  python tests/golden/make_golden.py
"""
import hashlib
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from arkoserenderer_amd import abi  # noqa: E402
from arkoserenderer_amd import ddgi as D  # noqa: E402
from arkoserenderer_amd import scene as S  # noqa: E402
import oracle_lib as O  # noqa: E402
from parity import RESOURCES, make_desc  # noqa: E402
import scenes  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def half_inputs():
    rng = np.random.default_rng(1234)
    h = np.arange(0, 0x7c00, dtype=np.uint32).astype(np.uint16)
    base = O.f16_to_f32(h[:-1])
    nxt = O.f16_to_f32(h[1:])
    ties = ((base.astype(np.float64) + nxt.astype(np.float64)) / 2).astype(np.float32)
    edge = np.array([0.0, -0.0, 65504.0, 65519.99, 65520.0, 1e8, 1e-8, 5.96e-8, 2.98e-8, 2.9802322e-08,
                     6.1035156e-05, 6.1e-05, np.inf, -np.inf, 10000.0, 1e4 * 1e4], np.float32)
    return np.concatenate([ties, -ties, rng.normal(scale=3, size=20000).astype(np.float32),
                           (rng.standard_cauchy(20000) * 100).astype(np.float32), edge]).astype(np.float32)


def make_half():
    exe = os.path.join(ROOT, "oracle", "_ref", "half_kat")
    if not os.path.exists(exe):
        subprocess.run(["make", "-f", "Makefile.ref"], cwd=os.path.join(ROOT, "oracle"), check=True)
    x = half_inputs()
    r = subprocess.run([exe], input=x.tobytes(), capture_output=True, check=True)
    bits = np.frombuffer(r.stdout, dtype=np.uint16)
    np.savez_compressed(os.path.join(OUT, "half_rne.npz"), inputs=x, half_bits=bits)
    print("half_rne.npz", x.size)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


SCENES = {}


def scene_spec(name):
    if name == "cornell_c2":
        sc, ex = S.cornell_box()
        grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
        cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=512, compute_probe_offsets=False,
                           max_rays_per_probe=64, max_probe_updates=512)
        return sc, grid, cfg, 4, ex["z_far"], dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    if name == "cornell_window_offsets":
        sc, ex = S.cornell_box()
        grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
        cfg = D.DDGIConfig(rays_per_probe=96, probe_updates_per_frame=200, compute_probe_offsets=True,
                           max_rays_per_probe=128, max_probe_updates=256)
        return sc, grid, cfg, 6, ex["z_far"], dict(light_pre_exposure=ex["light_pre_exposure"], environment_brightness=ex["environment_brightness"])
    if name == "features":
        sc = scenes.features_scene()
        grid = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))
        cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=144, compute_probe_offsets=True,
                           max_rays_per_probe=128, max_probe_updates=144)
        return sc, grid, cfg, 3, 100.0, dict(light_pre_exposure=1.0, ambient_illuminance=0.05, environment_brightness=0.5)
    if name == "soup_small":
        sc = S.soup(64_000, extent=7.0)
        grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
        cfg = D.DDGIConfig(rays_per_probe=128, probe_updates_per_frame=512, compute_probe_offsets=True,
                           max_rays_per_probe=128, max_probe_updates=512)
        return sc, grid, cfg, 2, 10000.0, dict(light_pre_exposure=1.0, environment_brightness=1.0)
    raise KeyError(name)


GOLDEN_SCENES = ["cornell_c2", "cornell_window_offsets", "features", "soup_small"]


def oracle_run(name, threads=8):
    sc, grid, cfg, frames, zfar, ex = scene_spec(name)
    orc = O.Oracle(make_desc(grid, zfar, cfg))
    orc.set_scene(sc, threads)
    idx = 0
    hashes = {}
    last = None
    for f in range(frames):
        p = D.frame_params(cfg, grid, D.AppState(f), idx, **ex)
        orc.update(p, threads)
        idx = (idx + p.probe_updates) % grid.probe_count()
        for k, w in RESOURCES.items():
            hashes[f"{k}_{f}"] = sha(orc.read(w))
        last = orc.read(abi.ARK_DDGI_ATLAS_IRRADIANCE)
    orc.close()
    return hashes, last


def make_scene(name):
    hashes, last = oracle_run(name)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), keys=np.array(list(hashes.keys())),
                        values=np.array(list(hashes.values())), last_irradiance=last)
    print(name, len(hashes))


if __name__ == "__main__":
    make_half()
    for n in GOLDEN_SCENES:
        make_scene(n)
