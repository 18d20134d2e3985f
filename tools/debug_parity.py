"""Debug helper: prints the GPU-vs-oracle mismatches of one scene/frame."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: F401,E402

from arkoserenderer_amd import abi  # noqa: E402
from arkoserenderer_amd import ddgi as D  # noqa: E402
from arkoserenderer_amd import scene as S  # noqa: E402
import oracle_lib as O  # noqa: E402

sc = S.soup(64_000, extent=7.0)
grid = D.ProbeGrid((8, 8, 8), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
cfg = D.DDGIConfig(rays_per_probe=256, probe_updates_per_frame=512, compute_probe_offsets=False, max_rays_per_probe=256, max_probe_updates=512)
ctx = D.DDGIContext(grid, 10000.0, cfg)
ctx.set_scene(sc)
orc = O.Oracle(ctx.desc)
orc.set_scene(sc)
p = D.frame_params(cfg, grid, D.AppState(0), 0)
ctx.update(p)
ctx.synchronize()
orc.update(p)
g = ctx.read(abi.ARK_DDGI_SURFELS).reshape(512, 256, 4)
o = orc.read(abi.ARK_DDGI_SURFELS).reshape(512, 256, 4)
gf, of = O.f16_to_f32(g), O.f16_to_f32(o)
bad = np.argwhere((g != o).any(-1))
print("mismatching rays:", len(bad))
for slot, s in bad[:20]:
    print(slot, s, "gpu", gf[slot, s], "orc", of[slot, s])

# brute force the mismatching rays in float32 with the exact Möller–Trumbore sequence
hits = ctx.read(abi.ARK_DDGI_DEBUG_HITS).view(np.float32).reshape(512, 256, 4)
P = sc.positions
tri_idx = sc.indices.reshape(-1, 3).astype(np.int64)
# soup: one mesh per material, identity transforms; build world triangles in instance order
W = []
for inst in sc.instances:
    m = sc.meshes[inst["rt_mesh_index"]]
    idx = sc.indices[m["first_index"]: m["first_index"] + 3 * inst["triangle_count"]].reshape(-1, 3).astype(np.int64) + m["first_vertex"]
    W.append(P[idx])
W = np.concatenate(W).astype(np.float32)
v0, e1, e2 = W[:, 0], (W[:, 1] - W[:, 0]).astype(np.float32), (W[:, 2] - W[:, 0]).astype(np.float32)
f32 = np.float32


def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1], a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2], a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1)


def dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


for slot, s in bad[:4]:
    pidx = slot  # window first = 0
    X, Y, Z = 8, 8, 8
    y = pidx // (X * Z); x = (pidx % (X * Z)) % X; z = (pidx % (X * Z)) // X
    o = np.array([x, y, z], np.float32)
    dvec = np.zeros(3, np.float32)
    O.load().oracle_rotated_fib(pidx, s, 256, 0, dvec.ctypes.data)
    d = dvec[None, :]
    pv = cross(d, e2); det = dot(e1, pv)
    with np.errstate(all="ignore"):
        inv = f32(1) / det
        sv = (o[None, :] - v0).astype(np.float32)
        u = dot(sv, pv) * inv
        q = cross(sv, e1)
        v = dot(d, q) * inv
        t = dot(e2, q) * inv
        ok = (det != 0) & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= f32(1e-4)) & (t <= f32(10000))
    ts = np.where(ok, t, np.inf)
    order = np.argsort(ts)[:3]
    print("ray", slot, s, "gpu hit", hits[slot, s], "brute nearest", [(int(i), float(ts[i]), float(det[i])) for i in order])
