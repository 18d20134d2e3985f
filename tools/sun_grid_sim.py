"""Host simulation of a light-space uniform grid for the sun's shadow rays (an alternative
to the light-space BVH8): the soup scaled to T triangles at C4's density, every
triangle listed in the cells of its (u, v) bounding box, each cell's list sorted by the
triangle's highest w; a shadow ray from a point on a sun-facing triangle walks its cell's
list from the top until a triangle covers the point above it (occluded) or the next
triangle lies wholly below it (lit). Prints the entries tested per ray.

    python tools/sun_grid_sim.py <triangles> <cell size> [rays]
"""
import sys, time, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from arkoserenderer_amd import scene as S
T = int(sys.argv[1]); cell = float(sys.argv[2]); N = int(sys.argv[3]) if len(sys.argv) > 3 else 20000
ext = 31.0 * (T / 10_000_000) ** (1 / 3)
t0 = time.time()
sc = S.soup(T, extent=ext)
P = np.asarray(sc.positions, np.float64); I = np.asarray(sc.indices, np.int64).reshape(-1, 3)
m = sc.meshes[0]; P = P[int(m['first_vertex']):] if 'first_vertex' in m.dtype.names else P
tri = P[I]  # (T,3,3)
sd = np.array(sc.sun[1], np.float64); w = -sd / np.linalg.norm(sd)
a = np.array([1.0, 0, 0]) if abs(w[0]) < 0.9 else np.array([0, 1.0, 0])
u = np.cross(a, w); u /= np.linalg.norm(u); v = np.cross(w, u)
L = tri @ np.stack([u, v, w], 1)  # (T,3,3) light coords
umin, umax = L[:, :, 0].min(1), L[:, :, 0].max(1); vmin, vmax = L[:, :, 1].min(1), L[:, :, 1].max(1); wmax = L[:, :, 2].max(1)
U0, V0 = umin.min(), vmin.min()
nu = int(np.ceil((umax.max() - U0) / cell)) + 1; nv = int(np.ceil((vmax.max() - V0) / cell)) + 1
cu0 = ((umin - U0) / cell).astype(np.int64); cu1 = ((umax - U0) / cell).astype(np.int64)
cv0 = ((vmin - V0) / cell).astype(np.int64); cv1 = ((vmax - V0) / cell).astype(np.int64)
nc = (cu1 - cu0 + 1) * (cv1 - cv0 + 1)
tid = np.repeat(np.arange(len(tri)), nc)
k = np.arange(nc.sum()) - np.repeat(np.cumsum(nc) - nc, nc)
wu = np.repeat(cu1 - cu0 + 1, nc)
cid = (np.repeat(cv0, nc) + k // wu) * nu + np.repeat(cu0, nc) + k % wu
order = np.lexsort((-wmax[tid], cid))
cid, tid = cid[order], tid[order]
start = np.searchsorted(cid, np.arange(nu * nv + 1))
print(f"T={len(tri)} ext={ext:.1f} grid {nu}x{nv} cell {cell} refs {len(tid)} ({len(tid)/len(tri):.1f}/tri, {len(tid)/(nu*nv):.1f}/cell) build {time.time()-t0:.1f}s")
# shadow origins: random points on sun-facing triangles
rng = np.random.default_rng(1)
n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
facing = np.nonzero(n @ w > 0)[0]
pick = rng.choice(facing, N)
r1, r2 = rng.random(N), rng.random(N); s = np.sqrt(r1)
b0, b1, b2 = 1 - s, s * (1 - r2), s * r2
O = L[pick, 0] * b0[:, None] + L[pick, 1] * b1[:, None] + L[pick, 2] * b2[:, None]
tmin = 1e-3
tests = np.zeros(N, np.int64); occl = np.zeros(N, bool); above = np.zeros(N, np.int64)
for i in range(N):
    c = int((O[i, 1] - V0) // cell) * nu + int((O[i, 0] - U0) // cell)
    e = tid[start[c]:start[c + 1]]
    Le = L[e]
    # 2D point in triangle + w at point
    p = O[i]
    d0 = Le[:, 0, :2] - p[:2]; d1 = Le[:, 1, :2] - p[:2]; d2 = Le[:, 2, :2] - p[:2]
    c0 = d0[:, 0] * d1[:, 1] - d0[:, 1] * d1[:, 0]; c1 = d1[:, 0] * d2[:, 1] - d1[:, 1] * d2[:, 0]; c2 = d2[:, 0] * d0[:, 1] - d2[:, 1] * d0[:, 0]
    inside = ((c0 >= 0) & (c1 >= 0) & (c2 >= 0)) | ((c0 <= 0) & (c1 <= 0) & (c2 <= 0))
    A = c0 + c1 + c2; A[A == 0] = 1
    wp = (c1 * Le[:, 0, 2] + c2 * Le[:, 1, 2] + c0 * Le[:, 2, 2]) / A
    hit = inside & (wp > p[2] + tmin) & (e != pick[i])
    stop_low = wmax[e] < p[2] + tmin
    above[i] = int((~stop_low).sum())
    cand = np.nonzero(hit | stop_low)[0]
    if len(cand):
        j = cand[0]; tests[i] = j + 1; occl[i] = hit[j]
    else:
        tests[i] = len(e)
print(f"occluded {occl.mean():.3f}; entries tested mean {tests.mean():.2f} p50 {np.median(tests):.0f} p90 {np.percentile(tests,90):.0f} p99 {np.percentile(tests,99):.0f}; entries above origin mean {above.mean():.1f}")
wv = tests[: N // 64 * 64].reshape(-1, 64)
print(f"wave max (64 rays) mean {wv.max(1).mean():.1f}; lane util {wv.mean()/wv.max(1).mean():.2f}; unoccluded rays' tests mean {tests[~occl].mean() if (~occl).any() else 0:.1f}")
