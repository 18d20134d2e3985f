"""Python host for the MI355X DDGI path, mirroring the reference node's
interface (arkose/rendering/nodes/DDGINode.h/.cpp) over the C-ABI.

* ``ProbeGrid``   — arkcore/scene/ProbeGrid.h:6-15 (+ Scene::generateProbeGridFromBoundingBox,
                    arkose/scene/Scene.cpp:534-583).
* ``DDGIConfig``  — the node's private members and their defaults (DDGINode.h:25-38).
* ``DDGIContext`` — one ark_ddgi context (device resources of one node on one GPU).
* ``DDGINode``    — name() == "DDGI"; ``execute(app_state)`` is the execute lambda
                    (DDGINode.cpp:132-259): rolling window, first-frame hysteresis,
                    push-constant values. The native C++ node
                    (arkoserenderer_amd/host/rendering/nodes/DDGINode.cpp) is the
                    drop-in for the engine; this mirror drives tests and bench.py.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import abi
from .scene import SceneData


@dataclass
class ProbeGrid:
    grid_dimensions: tuple  # (x=width, y=height, z=depth)
    probe_spacing: tuple
    offset_to_first: tuple

    def probe_count(self) -> int:
        x, y, z = self.grid_dimensions
        return int(x * y * z)

    @staticmethod
    def from_bounding_box(lo, hi):
        """Scene::generateProbeGridFromBoundingBox (Scene.cpp:534-583) on the scene's
        world AABB: grown by 1 m on every side, 16 probes per axis except the largest,
        which gets 32; spacing = bounds / counts, first probe at the grown minimum
        (fp32 vec3 arithmetic). The largest axis is the reference's rule (:563-570):
        x unless y or z is strictly larger than x, then y if y > z, else z - so a
        y == z tie above x picks z, and ties with x pick x."""
        lo = np.asarray(lo, np.float32) - np.float32(1.0)
        hi = np.asarray(hi, np.float32) + np.float32(1.0)
        bounds = (hi - lo).astype(np.float32)
        largest = 0
        if bounds[1] > bounds[0] or bounds[2] > bounds[0]:
            largest = 1 if bounds[1] > bounds[2] else 2
        counts = np.array([16.0, 16.0, 16.0], np.float32)
        counts[largest] = 32.0
        spacing = (bounds / counts).astype(np.float32)
        return ProbeGrid(tuple(int(v) for v in counts), tuple(float(v) for v in spacing), tuple(float(v) for v in lo))


@dataclass
class DDGIConfig:
    rays_per_probe: int = 256            # m_raysPerProbeInt
    hysteresis_irradiance: float = 0.93  # m_hysteresisIrradiance
    hysteresis_visibility: float = 0.93  # m_hysteresisVisibility
    visibility_sharpness: float = 50.0   # m_visibilitySharpness
    probe_updates_per_frame: int = 2048  # m_probeUpdatesPerFrame
    compute_probe_offsets: bool = True   # m_computeProbeOffsets
    apply_probe_offsets: bool = True     # m_applyProbeOffsets
    use_scene_ambient: bool = True       # m_useSceneAmbient
    injected_ambient_lx: float = 100.0   # m_injectedAmbientLx
    max_rays_per_probe: int = abi.ARK_DDGI_MAX_RAYS_PER_PROBE        # DDGINode.h:22
    max_probe_updates: int = abi.ARK_DDGI_REFERENCE_MAX_PROBE_UPDATES  # DDGINode.h:23
    clear_overflow_mode: int = abi.ARK_DDGI_CLEAR_OVERFLOW_INF
    # context options beyond the reference node's (ArkDdgiDesc): the sun's shadow-ray
    # structure, serial frames (no frames in flight), host threads of the BVH builds
    sun_bvh: int = abi.ARK_DDGI_SUN_BVH_AUTO
    serial_frames: bool = False
    background_rebuild: bool = True
    build_threads: int = 0


@dataclass
class AppState:
    """arkose/rendering/AppState.h:5-29"""
    frame_index: int = 0
    delta_time: float = 1.0 / 60.0

    def is_first_frame(self) -> bool:
        return self.frame_index == 0


def _check(lib, ctx, rc, what):
    if rc != 0:
        msg = lib.ark_ddgi_last_error(ctx)
        raise abi.ArkDdgiError(rc, f"{what}: {msg.decode() if msg else ''}")


def desc_for(grid: ProbeGrid, z_far: float, config: DDGIConfig, device: int = 0, shard_rank: int = 0,
             shard_count: int = 1) -> abi.ArkDdgiDesc:
    """The ArkDdgiDesc of a context (host only; the oracle takes it too)."""
    d = abi.ArkDdgiDesc()
    d.struct_size = C.sizeof(abi.ArkDdgiDesc)
    for k in range(3):
        d.grid_dims[k] = int(grid.grid_dimensions[k])
        d.probe_spacing[k] = float(grid.probe_spacing[k])
        d.offset_to_first[k] = float(grid.offset_to_first[k])
    d.z_far = float(z_far)
    d.max_rays_per_probe = int(config.max_rays_per_probe)
    d.max_probe_updates = int(config.max_probe_updates)
    d.device = int(device)
    d.clear_overflow_mode = int(config.clear_overflow_mode)
    d.shard_rank = int(shard_rank)
    d.shard_count = int(shard_count)
    d.sun_bvh = int(config.sun_bvh)
    d.flags = (abi.ARK_DDGI_FLAG_SERIAL_FRAMES if config.serial_frames else 0) | (0 if config.background_rebuild else abi.ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD)
    d.build_threads = int(config.build_threads)
    return d


class DDGIContext:
    """Owns one ark_ddgi context (device memory of one DDGI node on one GPU)."""

    def __init__(self, grid: ProbeGrid, z_far: float, config: DDGIConfig | None = None, device: int = 0,
                 shard_rank: int = 0, shard_count: int = 1):
        self.lib = abi.load_library()
        self.grid = grid
        self.config = config or DDGIConfig()
        d = desc_for(grid, z_far, self.config, device, shard_rank, shard_count)
        self.desc = d
        h = C.c_void_p()
        rc = self.lib.ark_ddgi_create(C.byref(d), C.byref(h))
        if rc != 0:
            raise abi.ArkDdgiError(rc, "ark_ddgi_create")
        self.h = h
        self._scene = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.ark_ddgi_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def check(self, rc, what):
        _check(self.lib, self.h, rc, what)

    def set_scene(self, scene: SceneData):
        s = scene.to_abi()
        self.check(self.lib.ark_ddgi_set_scene(self.h, C.byref(s)), "ark_ddgi_set_scene")
        self._scene = scene

    def set_lights(self, sun=None, spots=()):
        """ark_ddgi_set_lights: the per-frame light set (GpuScene.cpp:790-858). sun =
        (colour, direction) with the colour pre-exposed (colour x intensity x
        lightPreExposure, :811) or None; spots = SpotLights, colours pre-exposed (:844)."""
        from .scene import lights_abi

        L, keep = lights_abi(sun, spots)
        self.check(self.lib.ark_ddgi_set_lights(self.h, C.byref(L)), "ark_ddgi_set_lights")
        del keep

    def set_instances(self, instances: np.ndarray):
        """ark_ddgi_set_instances: the per-frame TLAS instance update (GpuScene.cpp:872-1009),
        a device refit. `instances` = the scene's INSTANCE_DTYPE array with new transforms."""
        a = np.ascontiguousarray(instances)
        self.check(self.lib.ark_ddgi_set_instances(self.h, C.c_void_p(a.ctypes.data), int(a.size)), "ark_ddgi_set_instances")

    def set_instances_async(self, instances: np.ndarray, stream: int | None):
        """ark_ddgi_set_instances_async: the same refit enqueued on `stream` (no host wait)."""
        a = np.ascontiguousarray(instances)
        self.check(self.lib.ark_ddgi_set_instances_async(self.h, C.c_void_p(a.ctypes.data), int(a.size), C.c_void_p(stream) if stream else None),
                   "ark_ddgi_set_instances_async")

    def share_scene(self, src: "DDGIContext"):
        """ark_ddgi_share_scene: use src's device scene and BVH (same GPU), no copy."""
        self.check(self.lib.ark_ddgi_share_scene(self.h, src.h), "ark_ddgi_share_scene")
        self._scene = src._scene

    def mark_external_write(self):
        """ark_ddgi_mark_external_write: offsets / atlases were written through the
        device views on the next update's stream; that update then runs after it."""
        self.check(self.lib.ark_ddgi_mark_external_write(self.h), "ark_ddgi_mark_external_write")

    def update(self, params: abi.ArkDdgiFrameParams, stream: int | None = None):
        self.check(self.lib.ark_ddgi_update(self.h, C.byref(params), C.c_void_p(stream) if stream else None), "ark_ddgi_update")

    def update_overlapped(self, params: abi.ArkDdgiFrameParams, stream: int | None, shade_wait_event: int | None,
                          done_event: int | None):
        """ark_ddgi_update_overlapped: raw hipStream_t / hipEvent_t handles (ints)."""
        v = lambda x: C.c_void_p(x) if x else None  # noqa: E731
        self.check(self.lib.ark_ddgi_update_overlapped(self.h, C.byref(params), v(stream), v(shade_wait_event), v(done_event)),
                   "ark_ddgi_update_overlapped")

    def update_exchanged(self, params: abi.ArkDdgiFrameParams, stream: int | None):
        """ark_ddgi_update_exchanged: shading waits (device-side) for the last exchange_end."""
        self.check(self.lib.ark_ddgi_update_exchanged(self.h, C.byref(params), C.c_void_p(stream) if stream else None),
                   "ark_ddgi_update_exchanged")

    def exchange_begin(self, comm_stream: int | None):
        """ark_ddgi_exchange_begin: comm_stream waits (device-side) for the last update."""
        self.check(self.lib.ark_ddgi_exchange_begin(self.h, C.c_void_p(comm_stream) if comm_stream else None), "ark_ddgi_exchange_begin")

    def exchange_end(self, comm_stream: int | None):
        """ark_ddgi_exchange_end: the exchange enqueued on comm_stream so far completes the frame."""
        self.check(self.lib.ark_ddgi_exchange_end(self.h, C.c_void_p(comm_stream) if comm_stream else None), "ark_ddgi_exchange_end")

    def window_exchange_info(self) -> abi.ArkDdgiWindowExchange:
        """ark_ddgi_window_exchange_info: the packet layout of the last update's window."""
        w = abi.ArkDdgiWindowExchange()
        self.check(self.lib.ark_ddgi_window_exchange_info(self.h, C.byref(w)), "ark_ddgi_window_exchange_info")
        return w

    def pack_window(self, dst_ptr: int, nbytes: int, comm_stream: int | None):
        """ark_ddgi_pack_window: this rank's updated tiles -> dst (bytes_per_rank) on comm_stream."""
        self.check(self.lib.ark_ddgi_pack_window(self.h, C.c_void_p(dst_ptr), nbytes, C.c_void_p(comm_stream) if comm_stream else None),
                   "ark_ddgi_pack_window")

    def unpack_window(self, src_ptr: int, nbytes: int, comm_stream: int | None):
        """ark_ddgi_unpack_window: every rank's packets (world x bytes_per_rank) -> the other slabs' tiles."""
        self.check(self.lib.ark_ddgi_unpack_window(self.h, C.c_void_p(src_ptr), nbytes, C.c_void_p(comm_stream) if comm_stream else None),
                   "ark_ddgi_unpack_window")

    def synchronize(self):
        self.check(self.lib.ark_ddgi_synchronize(self.h), "ark_ddgi_synchronize")

    def set_sequencing(self, device_sequence_words: bool, timeout_ms: int = 0):
        """ark_ddgi_set_sequencing: device sequence words (True) or events between the
        context's streams, and the bound of each wait (0 = keep)."""
        self.check(self.lib.ark_ddgi_set_sequencing(self.h, int(device_sequence_words), int(timeout_ms)), "ark_ddgi_set_sequencing")

    def sequencing(self) -> dict:
        """ark_ddgi_get_sequencing: {device_sequence_words, timeout_ms, timeouts}."""
        w, t, n = C.c_int(), C.c_uint32(), C.c_uint32()
        self.check(self.lib.ark_ddgi_get_sequencing(self.h, C.byref(w), C.byref(t), C.byref(n)), "ark_ddgi_get_sequencing")
        return {"device_sequence_words": bool(w.value), "timeout_ms": int(t.value), "timeouts": int(n.value)}

    def size(self, which: int) -> int:
        n = C.c_uint64()
        self.check(self.lib.ark_ddgi_resource_size(self.h, which, C.byref(n)), "ark_ddgi_resource_size")
        return int(n.value)

    def read(self, which: int) -> np.ndarray:
        n = self.size(which)
        dt = np.float32 if which in (abi.ARK_DDGI_PROBE_OFFSETS, abi.ARK_DDGI_DEBUG_HITS) else np.uint16
        out = np.empty(n // np.dtype(dt).itemsize, dtype=dt)
        self.check(self.lib.ark_ddgi_read(self.h, which, out.ctypes.data, n), "ark_ddgi_read")
        return out

    def write(self, which: int, data: np.ndarray):
        data = np.ascontiguousarray(data)
        self.check(self.lib.ark_ddgi_write(self.h, which, data.ctypes.data, data.nbytes), "ark_ddgi_write")

    def save_state(self) -> bytes:
        """ark_ddgi_save_state: the DDGI history (atlases + offsets) as one blob."""
        n = C.c_uint64()
        self.check(self.lib.ark_ddgi_state_size(self.h, C.byref(n)), "ark_ddgi_state_size")
        buf = (C.c_uint8 * n.value)()
        self.check(self.lib.ark_ddgi_save_state(self.h, buf, n.value), "ark_ddgi_save_state")
        return bytes(buf)

    def load_state(self, blob: bytes):
        """ark_ddgi_load_state: restores a blob of a context with the same grid / zFar / shard."""
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        self.check(self.lib.ark_ddgi_load_state(self.h, buf, len(blob)), "ark_ddgi_load_state")

    def next_probe_index(self) -> int:
        """ark_ddgi_get_next_probe_index: the rolling window's next first probe."""
        v = C.c_uint32()
        self.check(self.lib.ark_ddgi_get_next_probe_index(self.h, C.byref(v)), "ark_ddgi_get_next_probe_index")
        return int(v.value)

    def device_views(self) -> abi.ArkDdgiDeviceViews:
        v = abi.ArkDdgiDeviceViews()
        self.check(self.lib.ark_ddgi_get_device_views(self.h, C.byref(v)), "ark_ddgi_get_device_views")
        return v

    def reset_history(self):
        self.check(self.lib.ark_ddgi_reset_history(self.h), "ark_ddgi_reset_history")

    def set_counting(self, on: bool):
        self.check(self.lib.ark_ddgi_set_counting(self.h, int(on)), "ark_ddgi_set_counting")

    def counters(self) -> abi.ArkDdgiCounters:
        c = abi.ArkDdgiCounters()
        self.check(self.lib.ark_ddgi_get_counters(self.h, C.byref(c)), "ark_ddgi_get_counters")
        return c

    def set_timing(self, on: bool):
        self.check(self.lib.ark_ddgi_set_timing(self.h, int(on)), "ark_ddgi_set_timing")

    def last_timings(self):
        out = (C.c_float * 5)()
        self.check(self.lib.ark_ddgi_get_last_timings(self.h, out, 5), "ark_ddgi_get_last_timings")
        return list(out)

    def bake_ao(self, instance_index: int, width: int, height: int, sample_count: int, bent_normals: bool,
                stream: int | None = None):
        """ark_ddgi_bake_ao: AO / bent-normal bake of one instance's mesh segment."""
        d = abi.ArkBakeAoDesc()
        d.struct_size = C.sizeof(abi.ArkBakeAoDesc)
        d.instance_index, d.width, d.height, d.sample_count = int(instance_index), int(width), int(height), int(sample_count)
        d.bent_normals = int(bool(bent_normals))
        self.check(self.lib.ark_ddgi_bake_ao(self.h, C.byref(d), C.c_void_p(stream) if stream else None), "ark_ddgi_bake_ao")
        self._bake = (int(width), int(height), bool(bent_normals))

    def bake_read(self, which: int) -> np.ndarray:
        w, h, bent = self._bake
        shape, dt = {abi.ARK_BAKE_TRIANGLE_INDEX: ((h, w), np.uint32), abi.ARK_BAKE_BARYCENTRICS: ((h, w, 4), np.uint16),
                     abi.ARK_BAKE_OUTPUT: ((h, w, 4 if bent else 1), np.uint8)}[which]
        out = np.empty(shape, dt)
        self.check(self.lib.ark_ddgi_bake_read(self.h, which, out.ctypes.data, out.nbytes), "ark_ddgi_bake_read")
        return out

    def lighting_compose(self, width: int, height: int, flags: int, camera: dict, planes: dict, out_ptr: int,
                         stream: int | None = None):
        """ark_ddgi_lighting_compose. `planes` maps ArkComposeDesc plane names to DEVICE
        pointers (ints; absent = NULL); `camera` holds the three column-major 4x4
        matrices (CameraState, shared/CameraState.h); `out_ptr` is the RGBA16F output."""
        d = abi.ArkComposeDesc()
        d.struct_size = C.sizeof(abi.ArkComposeDesc)
        d.width, d.height, d.flags = int(width), int(height), int(flags)
        for k in ("view_from_pixel", "view_from_world", "world_from_view"):
            m = np.ascontiguousarray(camera[k], np.float32).reshape(16)
            getattr(d, k)[:] = [float(v) for v in m]
        for name, _, _ in abi.COMPOSE_PLANES:
            ptr = planes.get(name)
            setattr(d, name, int(ptr) if ptr else None)
        d.out = int(out_ptr)
        self.check(self.lib.ark_ddgi_lighting_compose(self.h, C.byref(d), C.c_void_p(stream) if stream else None),
                   "ark_ddgi_lighting_compose")

    def rt_reflections(self, desc: abi.ArkReflectionsDesc, stream: int | None = None):
        """ark_ddgi_rt_reflections: `desc` holds device pointers (include/ark_ddgi.h)."""
        desc.struct_size = C.sizeof(abi.ArkReflectionsDesc)
        self.check(self.lib.ark_ddgi_rt_reflections(self.h, C.byref(desc), C.c_void_p(stream) if stream else None), "ark_ddgi_rt_reflections")

    def probe_debug(self, visualisation: int, distance_scale: float, count: int, probes_ptr: int, dirs_ptr: int, out_ptr: int,
                    stream: int | None = None):
        """ark_ddgi_probe_debug on device arrays (uint32 probe indices, float3 directions,
        RGBA16F out)."""
        d = abi.ArkProbeDebugDesc()
        d.struct_size = C.sizeof(abi.ArkProbeDebugDesc)
        d.visualisation, d.distance_scale, d.count = int(visualisation), float(distance_scale), int(count)
        d.probe_indices, d.directions, d.out = int(probes_ptr), int(dirs_ptr), int(out_ptr)
        self.check(self.lib.ark_ddgi_probe_debug(self.h, C.byref(d), C.c_void_p(stream) if stream else None), "ark_ddgi_probe_debug")

    def bvh_stats(self) -> abi.ArkDdgiBvhStats:
        s = abi.ArkDdgiBvhStats()
        self.check(self.lib.ark_ddgi_get_bvh_stats(self.h, C.byref(s)), "ark_ddgi_get_bvh_stats")
        return s

    def scene_digest(self) -> tuple:
        """ark_ddgi_debug_scene_digest: digests of the world BVH nodes, world records, sun
        BVH nodes, sun records the kernels read now (tests of the refit)."""
        out = (C.c_uint64 * 4)()
        self.check(self.lib.ark_ddgi_debug_scene_digest(self.h, out), "ark_ddgi_debug_scene_digest")
        return tuple(int(v) for v in out)


def frame_params(config: DDGIConfig, grid: ProbeGrid, app: AppState, first_probe_index: int,
                 light_pre_exposure: float = 1.0, ambient_illuminance: float = 0.0,
                 environment_brightness: float = 1.0) -> abi.ArkDdgiFrameParams:
    """Push-constant values of the execute lambda (DDGINode.cpp:132-259)."""
    p = abi.ArkDdgiFrameParams()
    p.struct_size = C.sizeof(abi.ArkDdgiFrameParams)
    p.frame_index = int(app.frame_index) & 0xFFFFFFFF
    p.first_probe_index = int(first_probe_index)
    p.probe_updates = min(int(config.probe_updates_per_frame), grid.probe_count())
    p.rays_per_probe = int(config.rays_per_probe)
    p.hysteresis_irradiance = 0.0 if app.is_first_frame() else config.hysteresis_irradiance
    p.hysteresis_visibility = 0.0 if app.is_first_frame() else config.hysteresis_visibility
    p.visibility_sharpness = config.visibility_sharpness
    ambient_lx = ambient_illuminance if config.use_scene_ambient else config.injected_ambient_lx
    p.ambient_amount = float(np.float32(ambient_lx) * np.float32(light_pre_exposure))
    p.environment_multiplier = float(np.float32(environment_brightness) * np.float32(light_pre_exposure))
    p.delta_time = float(app.delta_time)
    p.update_offsets = int(config.compute_probe_offsets and config.apply_probe_offsets)
    return p


class DDGINode:
    """Python mirror of DDGINode (name "DDGI") driving a DDGIContext."""

    def __init__(self, config: DDGIConfig | None = None):
        self.config = config or DDGIConfig()
        self.probe_update_idx = 0  # m_probeUpdateIdx (DDGINode.h:32)
        self.ctx: DDGIContext | None = None
        self.grid: ProbeGrid | None = None
        self.exposure = dict(light_pre_exposure=1.0, ambient_illuminance=0.0, environment_brightness=1.0)

    def name(self) -> str:
        return "DDGI"

    def construct(self, scene: SceneData, grid: ProbeGrid | None, z_far: float, device: int = 0,
                  shard_rank: int = 0, shard_count: int = 1, **exposure) -> bool:
        """DDGINode::construct (DDGINode.cpp:37-130). Returns False (no-op node)
        when there is no probe grid, like NullExecuteCallback (:39-42)."""
        if grid is None or grid.probe_count() == 0:
            return False
        self.grid = grid
        self.ctx = DDGIContext(grid, z_far, self.config, device, shard_rank, shard_count)
        self.ctx.set_scene(scene)
        self.exposure.update(exposure)
        return True

    def next_params(self, app: AppState) -> abi.ArkDdgiFrameParams:
        return frame_params(self.config, self.grid, app, self.probe_update_idx, **self.exposure)

    def execute_overlapped(self, app: AppState, stream: int | None, shade_wait_event: int | None,
                           done_event: int | None) -> abi.ArkDdgiFrameParams:
        """execute() through ark_ddgi_update_overlapped (Z-slab ranks, see collective.py)."""
        if self.ctx is None:
            return None
        p = self.next_params(app)
        self.ctx.update_overlapped(p, stream, shade_wait_event, done_event)
        self.probe_update_idx = (self.probe_update_idx + p.probe_updates) % self.grid.probe_count()
        return p

    def execute_exchanged(self, app: AppState, stream: int | None) -> abi.ArkDdgiFrameParams:
        """execute() through ark_ddgi_update_exchanged (Z-slab ranks, see collective.py)."""
        if self.ctx is None:
            return None
        p = self.next_params(app)
        self.ctx.update_exchanged(p, stream)
        self.probe_update_idx = (self.probe_update_idx + p.probe_updates) % self.grid.probe_count()
        return p

    def execute(self, app: AppState, stream: int | None = None) -> abi.ArkDdgiFrameParams:
        if self.ctx is None:
            return None
        p = self.next_params(app)
        self.ctx.update(p, stream)
        self.probe_update_idx = (self.probe_update_idx + p.probe_updates) % self.grid.probe_count()
        return p

    def save_state(self) -> bytes:
        """The node's DDGI history: atlases, offsets and the window position."""
        return self.ctx.save_state()

    def load_state(self, blob: bytes):
        """Restores save_state()'s blob and resumes the rolling window where it was."""
        self.ctx.load_state(blob)
        self.probe_update_idx = self.ctx.next_probe_index()


class BakeAmbientOcclusionNode:
    """Python mirror of BakeAmbientOcclusionNode (name "Bake ambient occlusion",
    arkose/rendering/baking/BakeAmbientOcclusionNode.{h,cpp}): bakes the mesh segment
    of one instance; the output format selects AO (R8Uint) or bent normals (RGBA8)
    (BakeAmbientOcclusionNode.cpp:20-31). The scene/BVH come from a DDGIContext."""

    R8UINT = "R8Uint"
    RGBA8 = "RGBA8"

    def __init__(self, instance_index: int, sample_count: int = 500):
        assert sample_count > 0  # BakeAmbientOcclusionNode.cpp:12
        self.instance_index = instance_index
        self.sample_count = sample_count

    def name(self) -> str:
        return "Bake ambient occlusion"

    def execute(self, ctx: DDGIContext, width: int, height: int, output_format: str, stream: int | None = None) -> np.ndarray:
        if output_format not in (self.R8UINT, self.RGBA8):
            raise ValueError("BakeAmbientOcclusionNode: unknown AO texture format - only R8Uint & RGBA8 (bent normals)")
        bent = output_format == self.RGBA8
        ctx.bake_ao(self.instance_index, width, height, self.sample_count, bent, stream)
        return ctx.bake_read(abi.ARK_BAKE_OUTPUT)



def _tensor_stream(tensor, stream: int | None) -> int:
    """Stream for a consumer node whose planes are torch tensors: the caller's, else
    torch's current stream on the tensor's device (handle 0 = the null stream), so the
    launch is ordered after torch's producers of the planes and before its readers,
    as the reference records the node into the frame's one command list. The C-ABI
    orders it after the context's earlier operations on any stream."""
    if stream:
        return stream
    import torch

    return torch.cuda.current_stream(tensor.device).cuda_stream


def _check_plane(node: str, name: str, t, h: int, w: int, channels: int | None, dtypes):
    """A device plane the kernel indexes as [h][w](channels): contiguous, that shape,
    one of `dtypes` (torch dtypes)."""
    shape = (h, w) if channels is None else (h, w, channels)
    if not t.is_cuda or not t.is_contiguous() or tuple(int(v) for v in t.shape) != shape or t.dtype not in dtypes:
        raise ValueError(f"{node}: plane {name} must be a contiguous {list(shape)} device tensor of {'/'.join(str(d) for d in dtypes)}, "
                         f"got {list(t.shape)} {t.dtype}")


class LightingComposeNode:
    """Python mirror of LightingComposeNode (name "Lighting compose",
    arkose/rendering/lighting/LightingComposeNode.{h,cpp}) for the WITH_DDGI
    configuration: the node's toggles (LightingComposeNode.h:16-25 defaults, GUI at
    LightingComposeNode.cpp:9-44) become ArkComposeDesc flags; the G-buffer planes are
    device tensors (torch) in the formats GpuScene.cpp:326-360 creates."""

    def __init__(self):
        self.include_direct_light = True
        self.include_skin_diffuse_light = True
        self.include_glossy_gi = True
        self.include_diffuse_gi = True
        self.with_baked_occlusion = True
        self.use_bent_normal_direction = True
        self.with_bent_normal_occlusion = True
        self.with_screen_space_occlusion = True
        self.include_material_color = True  # GpuScene::shouldIncludeMaterialColor

    def name(self) -> str:
        return "Lighting compose"

    def flags(self, has_screen_space_occlusion: bool) -> int:
        f = 0
        f |= abi.ARK_COMPOSE_DIRECT_LIGHT if self.include_direct_light else 0
        f |= abi.ARK_COMPOSE_SKIN_DIFFUSE_LIGHT if self.include_skin_diffuse_light else 0
        f |= abi.ARK_COMPOSE_DIFFUSE_GI if self.include_diffuse_gi else 0
        f |= abi.ARK_COMPOSE_BAKED_OCCLUSION if self.with_baked_occlusion else 0
        f |= abi.ARK_COMPOSE_USE_BENT_NORMAL if self.use_bent_normal_direction else 0
        f |= abi.ARK_COMPOSE_BENT_NORMAL_OCCLUSION if self.with_bent_normal_occlusion else 0
        # no AmbientOcclusion texture: the option is forced off (LightingComposeNode.cpp:56-60)
        f |= abi.ARK_COMPOSE_SCREEN_SPACE_OCCLUSION if (self.with_screen_space_occlusion and has_screen_space_occlusion) else 0
        f |= abi.ARK_COMPOSE_GLOSSY_GI if self.include_glossy_gi else 0
        f |= abi.ARK_COMPOSE_MATERIAL_COLOR if self.include_material_color else 0
        return f

    def execute(self, ctx: DDGIContext, camera: dict, gbuffer: dict, out, stream: int | None = None):
        """gbuffer: plane name -> contiguous device tensor [H, W(, C)] (missing = NULL,
        read as 0 like the node's black stand-ins); out: uint16/float16 device tensor
        [H, W, 4] (SceneColorWithGI, RGBA16F)."""
        h, w = int(out.shape[0]), int(out.shape[1])
        planes = {}
        for name, _, _ in abi.COMPOSE_PLANES:
            t = gbuffer.get(name)
            if t is not None:
                if not t.is_contiguous() or int(t.shape[0]) != h or int(t.shape[1]) != w:
                    raise ValueError(f"LightingComposeNode: plane {name} must be a contiguous [{h}, {w}, ...] tensor")
                planes[name] = t.data_ptr()
        s = _tensor_stream(out, stream)
        ctx.lighting_compose(w, h, self.flags("screen_space_occlusion" in gbuffer), camera, planes, out.data_ptr(), s)


class DDGIProbeDebug:
    """Python mirror of DDGIProbeDebug (name "DDGI probe debug",
    arkose/rendering/nodes/DDGIProbeDebug.{h,cpp}): the fragment stage of its probe
    spheres (probeDebug.frag) on (probe, normal) samples - `sphere_samples` gives the
    reference's 48x48 sphere vertices; rasterising them is the caller's."""

    def __init__(self):
        self.debug_visualisation = abi.ARK_PROBE_DEBUG_DISABLED  # m_debugVisualisation
        self.probe_scale = 0.1
        self.distance_scale = 0.01
        self.use_probe_offset = True

    def name(self) -> str:
        return "DDGI probe debug"

    @staticmethod
    def sphere_samples(rings: int = 48, sectors: int = 48) -> np.ndarray:
        """Unit-sphere vertex positions of createSphereRenderData (DDGIProbeDebug.cpp:75-98)."""
        r = np.arange(rings, dtype=np.float32)[:, None]
        s = np.arange(sectors, dtype=np.float32)[None, :]
        R, S = np.float32(1.0 / (rings - 1)), np.float32(1.0 / (sectors - 1))
        pi = np.float32(np.pi)
        y = np.sin(-(pi / 2) + pi * r * R) * np.ones_like(s)
        x = np.cos(2 * pi * s * S) * np.sin(pi * r * R)
        z = np.sin(2 * pi * s * S) * np.sin(pi * r * R)
        return np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)

    def execute(self, ctx: DDGIContext, probes, dirs, out, stream: int | None = None):
        """probes: uint32/int32 device tensor [n]; dirs: float32 device tensor [n, 3];
        out: 16-bit device tensor [n, 4]. A no-op when the visualisation is disabled
        (DDGIProbeDebug.cpp:53-54)."""
        if self.debug_visualisation == abi.ARK_PROBE_DEBUG_DISABLED:
            return
        s = _tensor_stream(out, stream)
        ctx.probe_debug(self.debug_visualisation, self.distance_scale, int(probes.shape[0]), probes.data_ptr(), dirs.data_ptr(),
                        out.data_ptr(), s)


def reflections_desc(width: int, height: int, camera: dict, planes: dict, no_tracing_roughness: float = 0.6,
                     environment_multiplier: float = 1.0, ambient_amount: float = 0.0) -> abi.ArkReflectionsDesc:
    """ArkReflectionsDesc from a camera dict (world_from_view, view_from_projection:
    column-major 16 floats) and a plane dict of pointers (depth, material,
    normal_velocity, blue_noise, out_radiance, out_direction; missing = NULL) plus
    noise_width / noise_height. The default threshold is RTReflectionsNode's
    (RTReflectionsNode.h:20, m_noTracingRoughnessThreshold 0.6)."""
    d = abi.ArkReflectionsDesc()
    d.struct_size = C.sizeof(abi.ArkReflectionsDesc)
    d.width, d.height = int(width), int(height)
    d.no_tracing_roughness, d.environment_multiplier, d.ambient_amount = float(no_tracing_roughness), float(environment_multiplier), float(ambient_amount)
    for k in ("world_from_view", "view_from_projection"):
        getattr(d, k)[:] = [float(v) for v in np.asarray(camera[k], np.float32).reshape(16)]
    for k in ("depth", "material", "normal_velocity", "blue_noise", "out_radiance", "out_direction"):
        v = planes.get(k)
        setattr(d, k, int(v) if v else None)
    d.noise_width, d.noise_height = int(planes.get("noise_width", 0)), int(planes.get("noise_height", 0))
    return d


class RTReflectionsNode:
    """Mirror of RTReflectionsNode's ray-tracing pass (RTReflectionsNode.cpp:60-82):
    the raygen with WITH_DDGI on torch G-buffer planes; the temporal denoiser passes
    are not on the path. Defaults are the node's members (RTReflectionsNode.h:19-20)."""

    def __init__(self):
        self.no_tracing_roughness_threshold = 0.6  # m_noTracingRoughnessThreshold (parameter2)
        self.mirror_roughness_threshold = 0.001    # m_mirrorRoughnessThreshold (parameter1): read by no code path of the raygen

    def name(self) -> str:
        return "RT reflections"

    def execute(self, ctx: DDGIContext, camera: dict, gbuffer: dict, blue_noise, out_radiance, out_direction,
                environment_multiplier: float = 1.0, ambient_amount: float = 0.0, stream: int | None = None):
        """gbuffer: depth float32 [h, w], material uint8 [h, w, 4], normal_velocity
        16-bit [h, w, 4] (missing = NULL, read as 0); blue_noise float32 [hn, wn, 2]
        (one RG layer); out_radiance / out_direction 16-bit [h, w, 4]."""
        import torch

        h, w = int(out_radiance.shape[0]), int(out_radiance.shape[1])
        half = (torch.float16, torch.int16, torch.uint16) if hasattr(torch, "uint16") else (torch.float16, torch.int16)
        node = "RTReflectionsNode"
        _check_plane(node, "out_radiance", out_radiance, h, w, 4, half)
        _check_plane(node, "out_direction", out_direction, h, w, 4, half)
        spec = {"depth": (None, (torch.float32,)), "material": (4, (torch.uint8,)), "normal_velocity": (4, half)}
        for k, t in gbuffer.items():
            if k not in spec:
                raise ValueError(f"{node}: unknown plane {k}")
            if t is not None:
                _check_plane(node, k, t, h, w, spec[k][0], spec[k][1])
        planes = {k: (t.data_ptr() if t is not None else None) for k, t in gbuffer.items()}
        planes.update(out_radiance=out_radiance.data_ptr(), out_direction=out_direction.data_ptr())
        if blue_noise is not None:
            if (not blue_noise.is_cuda or not blue_noise.is_contiguous() or blue_noise.dim() != 3 or int(blue_noise.shape[2]) != 2
                    or blue_noise.dtype != torch.float32 or blue_noise.shape[0] == 0 or blue_noise.shape[1] == 0):
                raise ValueError(f"{node}: blue_noise must be a contiguous float32 [hn, wn, 2] device tensor, "
                                 f"got {list(blue_noise.shape)} {blue_noise.dtype}")
            planes.update(blue_noise=blue_noise.data_ptr(), noise_width=int(blue_noise.shape[1]), noise_height=int(blue_noise.shape[0]))
        d = reflections_desc(w, h, camera, planes, self.no_tracing_roughness_threshold, environment_multiplier, ambient_amount)
        s = _tensor_stream(out_radiance, stream)
        ctx.rt_reflections(d, s)
