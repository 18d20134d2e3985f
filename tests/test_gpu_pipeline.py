"""Frames in flight (ark_ddgi.h, ark_ddgi_update): a rolling window's slot table and
primary traversal overlap the previous frame's shadow rays, shading and update. The
dependence rule must leave every result equal to the serial run (ARK_DDGI_FLAG_SERIAL_FRAMES):
disjoint windows with probes moving, windows that intersect (they pipeline too: the
offsets of update n run on the traversal stream before update n+1's slot table, so
the next traversal reads them in order), an offsets write through ark_ddgi_write
between two updates, and one through the device views on the update stream flagged
with ark_ddgi_mark_external_write (the next traversal must see either)."""

import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
import scenes

pytestmark = pytest.mark.gpu
EXPOSURE = dict(light_pre_exposure=0.5, ambient_illuminance=0.1, environment_brightness=0.8)
GRID = D.ProbeGrid((6, 4, 6), (0.7, 0.7, 0.7), (-1.75, 0.25, -1.75))  # 144 probes
WHICH = (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY, abi.ARK_DDGI_PROBE_OFFSETS, abi.ARK_DDGI_SURFELS)


def _node(sc, K, pipelined):
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=K, max_rays_per_probe=64, max_probe_updates=K,
                       compute_probe_offsets=True, serial_frames=not pipelined)
    n = D.DDGINode(cfg)
    assert n.construct(sc, GRID, 100.0, **EXPOSURE)
    return n


def _run(n, frames, poke=None):
    out = []
    for f in range(frames):
        if poke is not None and f == poke:
            n.ctx.synchronize()
            off = n.ctx.read(abi.ARK_DDGI_PROBE_OFFSETS).copy()
            off[..., :3] += np.float32(0.03)  # every probe moves: the next window sees it
            n.ctx.write(abi.ARK_DDGI_PROBE_OFFSETS, off)
        n.execute(D.AppState(f))
        if f in (2, frames - 1):
            n.ctx.synchronize()
            out.append({w: n.ctx.read(w).copy() for w in WHICH})
    n.ctx.close()
    return out


@pytest.mark.parametrize("K", [48, 36, 100])
def test_pipelined_equals_serial(K):
    """K = 48 / 36: consecutive windows are disjoint; K = 100: they intersect while
    probes move. All pipeline (no serial fallback exists or is needed: the offsets run
    in order on the traversal stream)."""
    sc = scenes.features_scene()
    a = _run(_node(sc, K, True), 8)
    b = _run(_node(sc, K, False), 8)
    for fa, fb in zip(a, b):
        for w in WHICH:
            assert np.array_equal(fa[w], fb[w]), (K, w)


def test_offsets_write_between_updates():
    sc = scenes.features_scene()
    a = _run(_node(sc, 48, True), 7, poke=4)
    b = _run(_node(sc, 48, False), 7, poke=4)
    for fa, fb in zip(a, b):
        for w in WHICH:
            assert np.array_equal(fa[w], fb[w]), w


def test_device_view_offsets_write_marked_external():
    """A torch kernel writes every probe's offset through ark_ddgi_get_device_views on
    the stream of the next update, then ark_ddgi_mark_external_write: the pipelined
    node (whose traversal would otherwise start on the internal stream before the
    write) equals the serial one bit for bit."""
    import torch

    from arkoserenderer_amd.collective import device_bytes

    sc = scenes.features_scene()
    dev = torch.device("cuda", 0)
    outs = []
    for pipelined in (True, False):
        n = _node(sc, 48, pipelined)
        v = n.ctx.device_views()
        off = device_bytes(v.probe_offsets, v.probe_offsets_bytes, dev).view(torch.float32).view(-1, 4)
        stream = torch.cuda.Stream(dev)
        out = []
        for f in range(7):
            if f == 4:
                with torch.cuda.stream(stream):
                    off[:, :3] += 0.03
                n.ctx.mark_external_write()
            n.execute(D.AppState(f), stream.cuda_stream)
        torch.cuda.synchronize(dev)
        out = {w: n.ctx.read(w).copy() for w in WHICH}
        n.ctx.close()
        outs.append(out)
    for w in WHICH:
        assert np.array_equal(outs[0][w], outs[1][w]), w
