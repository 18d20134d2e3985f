"""Experiment: per-wave timeline of k_trace / k_trace_shadow at C4 (needs the
ARK tail instrumentation build). Prints when waves find the ray pool exhausted and
when they end, relative to the kernel's first wave start (100 MHz clock)."""
import ctypes as C
import sys
import numpy as np
from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S

K = int(sys.argv[1]) if len(sys.argv) > 1 else 0
scene = S.soup(10_000_000)
grid = D.ProbeGrid((32, 32, 32), (1.0, 1.0, 1.0), (0.0, 0.0, 0.0))
N = grid.probe_count()
K = K or N
cfg = D.DDGIConfig(rays_per_probe=256, probe_updates_per_frame=K, max_rays_per_probe=256, max_probe_updates=N, compute_probe_offsets=True)
ctx = D.DDGIContext(grid, 10000.0, cfg)
ctx.set_scene(scene)
for frame in range(4):
    ctx.update(D.frame_params(cfg, grid, D.AppState(frame), 0, light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0))
ctx.synchronize()
lib = C.CDLL(abi.library_path())
buf = np.zeros((2, 32768, 6), np.uint64)
assert lib.ark_debug_tail(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
for k, name in enumerate(("k_trace", "k_trace_shadow")):
    r = buf[k]
    r = r[r[:, 2] > 0].astype(np.int64)
    t0 = r[:, 0].min()
    st, ex, en = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0, (r[:, 2] - t0) / 100.0  # us
    ex = np.where(r[:, 1] > 0, ex, en)
    span = en.max()
    print(f"{name}: waves {len(r)}  span {span:.1f} us  start max {st.max():.1f}")
    print(f"  first exhaust {ex.min():.1f}  median exhaust {np.median(ex):.1f}  last exhaust {ex.max():.1f}")
    print(f"  end pct 10/50/90/99/100: " + " ".join(f"{np.percentile(en, q):.1f}" for q in (10, 50, 90, 99, 100)))
    print(f"  iters/wave mean {r[:, 3].mean():.0f}  after exhaust mean {r[:, 4].mean():.0f} max {r[:, 4].max()}  max ray steps {r[:, 5].max()}  p99 wave-max steps {np.percentile(r[:, 5], 99):.0f}")
    # active waves over time
    ts = np.linspace(0, span, 21)
    alive = [(np.sum((st <= t) & (en > t))) for t in ts]
    print("  alive: " + " ".join(str(a) for a in alive))
ctx.close()
