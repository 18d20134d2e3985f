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


class RcclBandExchange:
    """The same in-place all-gather of the two atlas bands, issued straight to RCCL
    (ncclGroupStart; ncclAllGather x 2; ncclGroupEnd) on the caller's current stream,
    through a communicator of its own (ncclCommInitRank; the ncclUniqueId travels over
    the torch.distributed group). torch's ProcessGroupNCCL runs a collective on its
    internal stream behind an event wait each way; on MI355X every cross-queue wait
    costs 12-16 us of queue latency, and both bands in one group halve the launches.
    The C++ node's RcclSlabExchange (SlabExchange.cpp) issues the same group."""

    NCCL_UINT8 = 1  # ncclDataType_t

    def __init__(self, buffers, rank: int, world: int, group=None):
        import ctypes as C

        import torch
        import torch.distributed as dist

        self.rank, self.world = rank, world
        self.bufs = []
        for full, off, slab in buffers:
            assert slab * world == full.numel() and off == rank * slab, "Z-slab bands must tile the atlas in rank order"
            self.bufs.append((full.data_ptr(), full.data_ptr() + off, slab))
        # Every rank reaches the same outcome: before any rank calls ncclCommInitRank
        # (which would block until all ranks join it), the ranks agree on their local
        # status - librccl loaded everywhere, the unique id obtained on rank 0 - by a
        # MIN all-reduce, and raise together if any failed; after ncclCommInitRank they
        # agree again before any rank uses the communicator. bench.py then falls back
        # to SlabExchange on every rank.
        dev = buffers[0][0].device
        lib = uid = None
        ok = 1
        try:
            lib = _rccl()
            uid = _NcclUniqueId()
            if rank == 0:
                _nccl_check(lib.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        except (OSError, AttributeError, RuntimeError):
            ok = 0
        status = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(status, op=dist.ReduceOp.MIN, group=group)
        if int(status.item()) != 1:
            raise RuntimeError(f"RcclBandExchange: librccl or the ncclUniqueId unavailable on some rank (here: {'ok' if ok else 'failed'})")
        t = torch.tensor(list(bytes(uid.internal)), dtype=torch.uint8, device=dev)
        dist.broadcast(t, 0, group=group)
        got = [1] + t.cpu().tolist()
        self.lib = lib
        self.comm = C.c_void_p()
        rc = lib.ncclCommInitRank(C.byref(self.comm), world, _NcclUniqueId((C.c_uint8 * 128)(*got[1:])), rank)
        flag = torch.tensor([1 if rc == 0 else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if int(flag.item()) != 1:
            if rc == 0:
                self.close()
            self.comm = None
            raise RuntimeError(f"RcclBandExchange: ncclCommInitRank failed on some rank (here: ncclResult {rc})")

    from_views = classmethod(SlabExchange.from_views.__func__)

    def exchange(self):
        import ctypes as C

        import torch

        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        lib = self.lib
        _nccl_check(lib.ncclGroupStart(), "ncclGroupStart")
        for full, mine, n in self.bufs:
            _nccl_check(lib.ncclAllGather(C.c_void_p(mine), C.c_void_p(full), C.c_size_t(n), self.NCCL_UINT8, self.comm, s), "ncclAllGather")
        _nccl_check(lib.ncclGroupEnd(), "ncclGroupEnd")

    def all_gather(self, out, mine):
        """ncclAllGather of equal byte counts (mine = this rank's slot of out, in place) on
        the current stream, through this communicator (the windowed exchange's packets)."""
        import ctypes as C

        import torch

        s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        _nccl_check(self.lib.ncclAllGather(C.c_void_p(mine.data_ptr()), C.c_void_p(out.data_ptr()), C.c_size_t(mine.numel()), self.NCCL_UINT8, self.comm, s),
                    "ncclAllGather")

    def async_error(self) -> int:
        import ctypes as C

        err = C.c_int(0)
        rc = self.lib.ncclCommGetAsyncError(self.comm, C.byref(err))
        return rc if rc != 0 else (err.value if err.value != 7 else 0)

    def abort(self):
        if self.comm:
            self.lib.ncclCommAbort(self.comm)
            self.comm = None

    def close(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = None


class WindowExchange:
    """The windowed Z-slab exchange (SURVEY §8e option (a); ark_ddgi.h
    ark_ddgi_window_exchange_info): with a rolling window (K < N) every rank packs the
    tiles its update wrote (one 2,096-B packet per window probe of its slab, in slot
    order), the packets of all ranks are all-gathered (equal counts, padded to the
    largest slab share), and every rank writes the other slabs' packets into their
    tiles. A window that covers the grid (K = N) exchanges the row bands instead
    (`band`, e.g. RcclBandExchange.exchange). exchange() enqueues on the current stream,
    as OverlappedSlabExchange calls it between exchange_begin and exchange_end.

    source: window_exchange_info() / pack_window(tensor, stream) / unpack_window(tensor,
    stream) - WindowSource(DDGIContext) on the GPU; the CPU tests pass an oracle-backed
    twin. gather(out, mine): all-gather of mine (this rank's slot of out) into out."""

    def __init__(self, source, band, gather, rank: int, world: int, max_probes_per_rank: int, device):
        import torch

        from . import abi

        self.source, self.band, self.gather = source, band, gather
        self.rank, self.world = rank, world
        # every window's packets fit: at most min(K_max, N / P) probes of one slab
        self.recv = torch.empty(world * max_probes_per_rank * abi.ARK_DDGI_WINDOW_PACKET_BYTES, dtype=torch.uint8, device=device)
        self.last_bytes_per_rank = 0  # received per frame: world - 1 of these (full bands: 0)

    def exchange(self):
        info = self.source.window_exchange_info()
        if info.full_bands:
            self.last_bytes_per_rank = 0
            self.band()
            return
        n = int(info.bytes_per_rank)
        self.last_bytes_per_rank = n
        if n == 0:
            return
        if n * self.world > self.recv.numel():
            raise RuntimeError(f"WindowExchange: {n} B per rank exceeds the buffer sized at construction")
        out = self.recv[:n * self.world]
        mine = out[self.rank * n:(self.rank + 1) * n]
        self.source.pack_window(mine)
        self.gather(out, mine)
        self.source.unpack_window(out)


class WindowSource:
    """WindowExchange's view of a DDGIContext: pack / unpack on the current stream."""

    def __init__(self, ctx):
        self.ctx = ctx

    def window_exchange_info(self):
        return self.ctx.window_exchange_info()

    def pack_window(self, t):
        import torch

        self.ctx.pack_window(t.data_ptr(), t.numel(), torch.cuda.current_stream().cuda_stream)

    def unpack_window(self, t):
        import torch

        self.ctx.unpack_window(t.data_ptr(), t.numel(), torch.cuda.current_stream().cuda_stream)


def torch_all_gather(group=None):
    """WindowExchange's gather through a torch.distributed group (gloo on CPU, nccl = RCCL)."""

    def gather(out, mine):
        import torch.distributed as dist

        dist.all_gather_into_tensor(out, mine, group=group)

    return gather


def _nccl_unique_id_type():
    import ctypes as C

    class NcclUniqueId(C.Structure):  # ncclUniqueId: 128 opaque bytes, passed by value
        _fields_ = [("internal", C.c_uint8 * 128)]

    return NcclUniqueId


_NcclUniqueId = _nccl_unique_id_type()


def _rccl():
    """The librccl.so torch already loaded (dlopen by soname returns that instance)."""
    import ctypes as C

    global _RCCL
    if _RCCL is None:
        _RCCL = C.CDLL("librccl.so")
    lib = _RCCL
    if not getattr(lib, "_ark_typed", False):
        lib.ncclCommGetAsyncError.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
        lib.ncclCommGetAsyncError.restype = C.c_int
        lib.ncclGetUniqueId.argtypes = [C.POINTER(_NcclUniqueId)]
        lib.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, _NcclUniqueId, C.c_int]
        lib.ncclAllGather.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_void_p]
        lib.ncclCommAbort.argtypes = [C.c_void_p]
        lib.ncclCommDestroy.argtypes = [C.c_void_p]
        for fn in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllGather", "ncclGroupStart", "ncclGroupEnd", "ncclCommAbort", "ncclCommDestroy"):
            getattr(lib, fn).restype = C.c_int
        lib._ark_typed = True
    return lib


def _nccl_check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed: ncclResult {rc}")


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
    lib = _rccl()
    err = C.c_int(0)
    rc = lib.ncclCommGetAsyncError(C.c_void_p(comm), C.byref(err))
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

    def __init__(self, timeout_s: float | None = None, group=None, on_failure=None, rccl=None):
        import os

        if timeout_s is None or timeout_s <= 0:
            timeout_s = float(os.environ.get("ARK_EXCHANGE_TIMEOUT_S", "0") or 0) or 120.0
        self.timeout_s, self.group = float(timeout_s), group
        self.rccl = rccl  # a RcclBandExchange: its own communicator is polled and aborted too
        self.on_failure = on_failure or self.abort_and_exit

    def wait(self, event, what: str) -> bool:
        import time

        t0 = time.monotonic()
        pause = 1e-5
        while not event.query():
            err = _rccl_async_error(self.group) or (self.rccl.async_error() if self.rccl is not None else 0)
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
            if self.rccl is not None:
                self.rccl.abort()
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

    def __init__(self, node, exchange, device, watchdog: ExchangeWatchdog | None = None, device_seq: bool | None = None):
        """exchange: a callable that enqueues the all-gather on the current stream.
        device_seq (default: on): the handovers between the
        update stream and the exchange stream are the context's device-side sequence
        words (ark_ddgi_update_exchanged / ark_ddgi_exchange_begin / _end) instead of
        torch events; the events below then only bound the host."""
        import os

        import torch

        self.node, self.exchange = node, exchange
        if device_seq is None:
            device_seq = True
        self.device_seq = device_seq
        owner = getattr(exchange, "__self__", None)  # a bound RcclBandExchange.exchange: watch its communicator
        self.watchdog = watchdog or ExchangeWatchdog(rccl=owner if isinstance(owner, RcclBandExchange) else None)
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
        if self.device_seq:
            ctx = self.node.ctx
            p = self.node.execute_exchanged(app, stream_ptr)
            with torch.cuda.stream(self.comm):
                ctx.exchange_begin(self.comm.cuda_stream)
                self.exchange()
                ctx.exchange_end(self.comm.cuda_stream)
                slot.record(self.comm)
        else:
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
