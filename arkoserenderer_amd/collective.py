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


class OverlappedSlabExchange:
    """One rank's frame loop with the atlas all-gather of frame N on a side stream,
    overlapped with frame N+1's probe-ray traversal (which reads only the scene,
    the slot table and this rank's own probe offsets). Frame N+1's shading waits
    for the all-gather (it samples the previous atlases at any probe); the
    all-gather waits for frame N's probe update (ark_ddgi_update_overlapped)."""

    def __init__(self, node, exchange, device):
        import torch

        self.node, self.exchange = node, exchange
        self.comm = torch.cuda.Stream(device)
        self.updated = torch.cuda.Event()
        self.gathered = torch.cuda.Event()
        # torch creates events lazily: record once so the raw handles exist
        cur = torch.cuda.current_stream(device)
        self.updated.record(cur)
        self.gathered.record(cur)
        self.pending = False

    def step(self, app, stream_ptr: int):
        import torch

        wait = self.gathered.cuda_event if self.pending else None
        p = self.node.execute_overlapped(app, stream_ptr, wait, self.updated.cuda_event)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(self.updated)
            self.exchange()
            self.gathered.record(self.comm)
        self.pending = True
        return p


def slab_bands(total_bytes: int, world: int):
    """(offset, bytes) of every rank's band; used by the CPU (gloo) tests."""
    slab = total_bytes // world
    return [(r * slab, slab) for r in range(world)]
