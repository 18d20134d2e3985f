"""Fail-closed frame sequencing (VERDICT r03 "do this" #3).

A pipelined update hands its frame between streams with one-wave sequence-word
kernels (k_seq_signal / k_seq_wait, ddgi_kernels.hip). A wait that gives up must not
let the kernels after it compute without their inputs: the path kernels check the
context's timed-out word at entry and leave their outputs untouched, the next
context call reports ARK_DDGI_E_DEVICE and switches the context to events, and the
frames after it are bit-exact again.

What a dropped frame leaves behind (ark_ddgi_set_sequencing's contract):
its traversal and probe offsets run on the traversal stream before the wait that
gives up, so with offsets on its offsets are applied and the rolling window moves past
it; its surfels and both atlases are untouched. The offsets case pins exactly that:
the reference runs the dropped frame in full and then restores the atlases it had
before it.

The stall: the Z-slab exchange's stream (ark_ddgi_exchange_begin / _end) runs a
bounded ~1.5 s kernel (torch.cuda._sleep) before exchange_end, so the next
update's shading wait (bounded at 100 ms here) gives up. The exchange stream is a
high-priority stream: HIP keeps its hardware queues apart from the normal-priority
ones (a stream sharing the update stream's queue would run the signal before the
wait in queue order, and nothing would time out).
"""
import numpy as np
import pytest

from arkoserenderer_amd import abi
from arkoserenderer_amd import ddgi as D
from arkoserenderer_amd import scene as S

pytestmark = pytest.mark.gpu

READ = (abi.ARK_DDGI_SURFELS, abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY, abi.ARK_DDGI_PROBE_OFFSETS)


def _setup(offsets=False):
    sc, ex = S.cornell_box()
    grid = D.ProbeGrid((8, 8, 8), (0.257, 0.257, 0.257), (-0.9, 0.1, -0.9))
    K = 200 if offsets else 512  # offsets: a rolling window K < N, as the node advances it
    cfg = D.DDGIConfig(rays_per_probe=64, probe_updates_per_frame=K, max_rays_per_probe=64, max_probe_updates=512,
                       compute_probe_offsets=offsets)
    params = [D.frame_params(cfg, grid, D.AppState(f), (f * K) % 512, light_pre_exposure=ex["light_pre_exposure"],
                             environment_brightness=ex["environment_brightness"]) for f in range(5)]
    ctx = D.DDGIContext(grid, ex["z_far"], cfg, device=0)
    ctx.set_scene(sc)
    ref = D.DDGIContext(grid, ex["z_far"], cfg, device=0)
    ref.set_scene(sc)
    return ctx, ref, params


@pytest.mark.parametrize("observer,offsets", [("update", False), ("synchronize", False), ("update", True)])
def test_seq_wait_timeout_fails_closed(observer, offsets):
    import torch

    ctx, ref, params = _setup(offsets)
    try:
        ctx.set_sequencing(True, 100)
        assert ctx.sequencing() == {"device_sequence_words": True, "timeout_ms": 100, "timeouts": 0}
        s = torch.cuda.current_stream().cuda_stream
        x = torch.cuda.Stream(priority=-1)

        def frame(f, stall=False):
            ctx.update_exchanged(params[f], s)
            ctx.exchange_begin(x.cuda_stream)
            if stall:
                with torch.cuda.stream(x):
                    torch.cuda._sleep(int(3.5e9))  # bounded: ends by itself after ~1.5 s
            ctx.exchange_end(x.cuda_stream)

        frame(0)
        frame(1, stall=True)
        # frame 2's shading waits for exchange 1, which ends after the sleep: the wait
        # gives up after 100 ms and frame 2's shading and atlas update skip
        ctx.update_exchanged(params[2], s)
        torch.cuda.synchronize()  # the sleep ends by itself
        assert ctx.sequencing()["timeouts"] == 0
        with pytest.raises(abi.ArkDdgiError) as ei:
            if observer == "update":
                ctx.update_exchanged(params[3], s)
            else:
                ctx.synchronize()
        assert ei.value.status == -5  # ARK_DDGI_E_DEVICE
        assert "gave up after 100 ms" in str(ei.value) and "events" in str(ei.value)
        seq = ctx.sequencing()
        assert seq["device_sequence_words"] is False and seq["timeouts"] == 1
        # the context runs again, now with events
        ctx.exchange_begin(x.cuda_stream)
        ctx.exchange_end(x.cuda_stream)
        frame(3)
        frame(4)
        ctx.synchronize()
        # frame 2 dropped: the reference runs frames 0, 1, 3, 4 - with offsets, frame 2
        # too, followed by a restore of the atlases frame 1 left (its offsets stay)
        for f in (0, 1):
            ref.update(params[f])
        if offsets:
            ref.synchronize()
            keep = {w: ref.read(w) for w in (abi.ARK_DDGI_ATLAS_IRRADIANCE, abi.ARK_DDGI_ATLAS_VISIBILITY)}
            ref.update(params[2])
            ref.synchronize()
            for w, a in keep.items():
                ref.write(w, a)
        for f in (3, 4):
            ref.update(params[f])
        ref.synchronize()
        for which in READ:
            a, b = ctx.read(which), ref.read(which)
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), which
    finally:
        torch.cuda.synchronize()
        ctx.close()
        ref.close()


def test_seq_wait_no_timeout_runs_every_frame():
    """Negative control: the same stall under the default 10-s bound - the wait just
    waits, no error, and all five frames are applied (bit-exact against a serial
    context that runs all five)."""
    import torch

    ctx, ref, params = _setup()
    try:
        assert ctx.sequencing()["timeout_ms"] == 10000
        s = torch.cuda.current_stream().cuda_stream
        x = torch.cuda.Stream(priority=-1)
        for f in range(5):
            ctx.update_exchanged(params[f], s)
            ctx.exchange_begin(x.cuda_stream)
            if f == 1:
                with torch.cuda.stream(x):
                    torch.cuda._sleep(int(3.5e9))
            ctx.exchange_end(x.cuda_stream)
        ctx.synchronize()
        assert ctx.sequencing()["timeouts"] == 0
        for f in range(5):
            ref.update(params[f])
        ref.synchronize()
        for which in READ:
            a, b = ctx.read(which), ref.read(which)
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), which
    finally:
        torch.cuda.synchronize()
        ctx.close()
        ref.close()
