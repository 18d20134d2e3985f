"""Z-slab exchange of the DDGI atlases across GPUs (RCCL over xGMI via
torch.distributed, backend "nccl" = RCCL on ROCm).

A Z-slab of the probe grid is a contiguous texel-row band of both atlases
(tile row = probe z, ddgi/common.glsl:58-61), so after every update each rank
contributes its band to an in-place all-gather of the whole atlas. The full
atlas (not a one-probe halo) is exchanged because the indirect bounce of the
next frame samples the previous frame's atlases at arbitrary hit points
(raygen.rgen:127 -> probeSampling.glsl:64-163).
"""
from __future__ import annotations


class _CudaArray:
    """Minimal __cuda_array_interface__ view of raw device bytes owned by libark_ddgi."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {
            "shape": (int(nbytes),),
            "typestr": "|u1",
            "data": (int(ptr), False),
            "version": 3,
            "strides": None,
        }


def device_bytes(ptr: int, nbytes: int, device):
    import torch

    return torch.as_tensor(_CudaArray(ptr, nbytes), device=device)


class SlabExchange:
    """In-place all-gather of the irradiance and visibility atlases of one
    DDGIContext (one Z-slab per rank). Works with any torch.distributed backend
    whose tensors live where the atlases live (nccl = RCCL on GPU; gloo on CPU
    for the multi-process tests)."""

    def __init__(self, buffers, rank: int, world: int, group=None):
        """buffers: [(full_atlas_bytes_tensor, slab_offset, slab_bytes), ...]"""
        self.rank, self.world, self.group = rank, world, group
        self.bufs = []
        for full, off, slab in buffers:
            assert slab * world == full.numel() and off == rank * slab, "Z-slab bands must tile the atlas in rank order"
            self.bufs.append((full, full[off:off + slab]))

    @classmethod
    def from_views(cls, views, rank: int, world: int, device, group=None):
        bufs = []
        for ptr, total, off, slab in (
            (views.irradiance_atlas, views.irradiance_bytes, views.irradiance_slab_offset, views.irradiance_slab_bytes),
            (views.visibility_atlas, views.visibility_bytes, views.visibility_slab_offset, views.visibility_slab_bytes),
        ):
            bufs.append((device_bytes(ptr, total, device), int(off), int(slab)))
        return cls(bufs, rank, world, group)

    def exchange(self):
        import torch.distributed as dist

        for full, mine in self.bufs:
            dist.all_gather_into_tensor(full, mine, group=self.group)


EXCHANGE_FAILURE_EXIT_CODE = 14  # as the C++ ExchangeWatchdog (SlabExchange.h)


def _rccl_async_error(group) -> int:
    """ncclCommGetAsyncError of the RCCL communicator behind a torch process group
    (ProcessGroupNCCL._comm_ptr), 0 = ncclSuccess; 0 when there is none to ask
    (gloo, or a communicator not created yet)."""
    import ctypes as C

    import torch.distributed as dist

    try:
        pg = group if group is not None else dist.distributed_c10d._get_default_group()
        backend = pg._get_backend(__import__("torch").device("cuda"))
        comm = int(backend._comm_ptr())
    except (RuntimeError, AttributeError, ValueError):
        return 0
    if not comm:
        return 0
    global _RCCL
    if _RCCL is None:
        _RCCL = C.CDLL("librccl.so")
        _RCCL.ncclCommGetAsyncError.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        _RCCL.ncclCommGetAsyncError.restype = C.c_int
    err = C.c_int(0)
    rc = _RCCL.ncclCommGetAsyncError(C.c_void_p(comm), C.byref(err))
    # ncclInProgress (7) is a non-blocking communicator still initialising: not an error
    return rc if rc != 0 else (err.value if err.value != 7 else 0)


_RCCL = None


class ExchangeWatchdog:
    """Failure detection of the Z-slab exchange (ncclCommGetAsyncError
    polling in multi-GPU mode), the Python twin of the C++ ExchangeWatchdog
    (SlabExchange.h). wait(event) polls the exchange's completion event and the
    communicator's asynchronous error until a deadline (ARK_EXCHANGE_TIMEOUT_S,
    default 120 s); on an error or at the deadline it calls on_failure(why), whose
    default aborts the process group (the communicator's pending work is cancelled and
    peers see an error), logs an Error and ends the process with exit code 14. No
    re-exec. A dead peer would otherwise hang every rank: the next frame's shading
    waits for the all-gather on the device and the host blocks at its next sync."""

    def __init__(self, timeout_s: float | None = None, group=None, on_failure=None):
        import os

        if timeout_s is None or timeout_s <= 0:
            timeout_s = float(os.environ.get("ARK_EXCHANGE_TIMEOUT_S", "0") or 0) or 120.0
        self.timeout_s, self.group = float(timeout_s), group
        self.on_failure = on_failure or self.abort_and_exit

    def wait(self, event, what: str) -> bool:
        import time

        t0 = time.monotonic()
        pause = 1e-5
        while not event.query():
            err = _rccl_async_error(self.group)
            if err:
                self.on_failure(f"{what}: communicator error {err}")
                return False
            waited = time.monotonic() - t0
            if waited > self.timeout_s:
                self.on_failure(f"{what}: not complete after {waited:.3f} s (deadline {self.timeout_s:.3f} s)")
                return False
            time.sleep(pause)
            # capped at 0.1 ms: a longer sleep overshoots the event by up to its own
            # length, and the host would then enqueue the next frame late
            pause = min(2 * pause, 1e-4)
        return True

    def abort_and_exit(self, why: str):
        import os
        import sys

        import torch.distributed as dist

        try:
            if dist.is_initialized():
                dist.distributed_c10d._abort_process_group(self.group)
        finally:
            print(f"[Error] Z-slab exchange failed, exiting: {why}", file=sys.stderr, flush=True)
            sys.stdout.flush()
            os._exit(EXCHANGE_FAILURE_EXIT_CODE)


class OverlappedSlabExchange:
    """One rank's frame loop with the atlas all-gather of frame N on a side stream,
    overlapped with frame N+1's probe-ray traversal (which reads only the scene,
    the slot table and this rank's own probe offsets). Frame N+1's shading waits
    for the all-gather (it samples the previous atlases at any probe); the
    all-gather waits for frame N's probe update (ark_ddgi_update_overlapped).

    Bounded: before frame N is enqueued, frame N-RING's all-gather must have completed
    (ExchangeWatchdog.wait on its event, polled against a deadline): the host runs at
    most RING exchanges ahead of the device, and a peer that stops answering ends the
    process at the deadline instead of hanging it. drain() waits (bounded) for the last.
    RING = 3: with 2 the host waits for frame N-2's exchange, which ends only after
    frame N-2's update, and enqueues frame N's traversal after the traversal stream
    has already gone idle (Z-slab proxy at P = 8 with an exchange stand-in, round 3)."""

    RING = 3

    def __init__(self, node, exchange, device, watchdog: ExchangeWatchdog | None = None):
        import torch

        self.node, self.exchange = node, exchange
        self.watchdog = watchdog or ExchangeWatchdog()
        self.comm = torch.cuda.Stream(device)
        self.updated = torch.cuda.Event()
        # completion of frame n's all-gather in slot n % RING
        self.gathered = [torch.cuda.Event() for _ in range(self.RING)]
        # torch creates events lazily: record once so the raw handles exist
        cur = torch.cuda.current_stream(device)
        self.updated.record(cur)
        for e in self.gathered:
            e.record(cur)
        self.frames = 0

    def step(self, app, stream_ptr: int):
        import torch

        prev = self.gathered[(self.frames - 1) % self.RING]
        wait = prev.cuda_event if self.frames > 0 else None
        slot = self.gathered[self.frames % self.RING]
        if self.frames >= self.RING and not self.watchdog.wait(slot, f"slab exchange frame n-{self.RING}"):
            return None
        p = self.node.execute_overlapped(app, stream_ptr, wait, self.updated.cuda_event)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.updated)
            self.exchange()
            slot.record(self.comm)
        self.frames += 1
        return p

    def drain(self) -> bool:
        if self.frames == 0:
            return True
        return self.watchdog.wait(self.gathered[(self.frames - 1) % self.RING], "slab exchange drain")


def slab_bands(total_bytes: int, world: int):
    """(offset, bytes) of every rank's band; used by the CPU (gloo) tests."""
    slab = total_bytes // world
    return [(r * slab, slab) for r in range(world)]
