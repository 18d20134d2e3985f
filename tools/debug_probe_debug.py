"""Dumps the rows where ark_ddgi_probe_debug and the oracle disagree on random atlases
(tests/test_gpu_probe_debug.py::test_probe_debug_random_atlases), with the atlas
round trip checked first. Diagnostic only."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from arkoserenderer_amd import abi  # noqa: E402
from arkoserenderer_amd import ddgi as D  # noqa: E402
import oracle_lib as O  # noqa: E402

grid = D.ProbeGrid((5, 3, 4), (0.5, 0.6, 0.7), (-1.0, 0.0, -1.0))
cfg = D.DDGIConfig(rays_per_probe=16, probe_updates_per_frame=60, max_rays_per_probe=16, max_probe_updates=60)
ctx = D.DDGIContext(grid, 50.0, cfg)
orc = O.Oracle(ctx.desc)
rng = np.random.default_rng(3)
irr = np.asarray(rng.uniform(0, 1.2, ctx.size(abi.ARK_DDGI_ATLAS_IRRADIANCE) // 2), np.float32).astype(np.float16).view(np.uint16)
vis = np.asarray(rng.uniform(-0.5, 3.0, ctx.size(abi.ARK_DDGI_ATLAS_VISIBILITY) // 2), np.float32).astype(np.float16).view(np.uint16)
for side in (ctx, orc):
    side.write(abi.ARK_DDGI_ATLAS_IRRADIANCE, irr)
    side.write(abi.ARK_DDGI_ATLAS_VISIBILITY, vis)
for side, name in ((ctx, "gpu"), (orc, "oracle")):
    for which, ref in ((abi.ARK_DDGI_ATLAS_IRRADIANCE, irr), (abi.ARK_DDGI_ATLAS_VISIBILITY, vis)):
        back = side.read(which).reshape(-1).view(np.uint16)
        print(name, which, "round trip equal:", np.array_equal(back, ref), back.size, ref.size)
n = 5000
probes = rng.integers(0, grid.probe_count(), n).astype(np.uint32)
dirs = rng.normal(size=(n, 3)).astype(np.float32)
for mode in (1, 2, 3):
    node = D.DDGIProbeDebug()
    node.debug_visualisation, node.distance_scale = mode, 0.1
    out = torch.zeros((n, 4), dtype=torch.int16, device="cuda")
    node.execute(ctx, torch.from_numpy(probes.astype(np.int32)).cuda(), torch.from_numpy(dirs).cuda(), out)
    ctx.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    want = orc.probe_debug(mode, 0.1, probes, dirs)
    bad = np.nonzero(np.any(got != want, axis=1))[0]
    print(f"mode {mode}: {bad.size} rows differ")
    for i in bad[:12]:
        print("  row", i, "probe", probes[i], "dir", dirs[i], "got", got[i].view(np.float16), "want", want[i].view(np.float16))
