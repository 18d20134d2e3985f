"""ctypes mirror of the C-ABI in include/ark_ddgi.h, include/ark_scene.h and
include/ark_ddgi_debug.h.

This is the binding a Python host (tests, bench.py) uses; the C++ host
(arkoserenderer_amd/host) includes the header directly. Struct layouts are
checked against the library's own sizeof() in tests/test_abi.py.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ARK_DDGI_LIB") or os.path.join(_HERE, "lib", "libark_ddgi.so")  # override: tuning builds

ARK_DDGI_IRRADIANCE_RES = 8
ARK_DDGI_VISIBILITY_RES = 16
ARK_DDGI_ATLAS_PADDING = 1
ARK_DDGI_MAX_RAYS_PER_PROBE = 512
ARK_DDGI_REFERENCE_MAX_PROBE_UPDATES = 4096

ARK_RT_HIT_MASK_OPAQUE = 0x01
ARK_RT_HIT_MASK_MASKED = 0x02
ARK_RT_HIT_MASK_BLEND = 0x04

ARK_BLEND_MODE_OPAQUE = 1
ARK_BLEND_MODE_MASKED = 2
ARK_BLEND_MODE_TRANSLUCENT = 3

ARK_DDGI_OK = 0
ERRORS = {
    -1: "ARK_DDGI_E_INVALID_ARGUMENT",
    -2: "ARK_DDGI_E_NO_PROBE_GRID",
    -3: "ARK_DDGI_E_NO_SCENE",
    -4: "ARK_DDGI_E_OUT_OF_MEMORY",
    -5: "ARK_DDGI_E_DEVICE",
    -6: "ARK_DDGI_E_UNSUPPORTED",
    -7: "ARK_DDGI_E_SIZE_MISMATCH",
}

ARK_DDGI_ATLAS_IRRADIANCE = 0
ARK_DDGI_ATLAS_VISIBILITY = 1
ARK_DDGI_SURFELS = 2
ARK_DDGI_PROBE_OFFSETS = 3
ARK_DDGI_DEBUG_HITS = 100
ARK_DDGI_DEBUG_RAY_STEPS = 101

ARK_DDGI_CLEAR_OVERFLOW_INF = 0
ARK_DDGI_CLEAR_OVERFLOW_MAX_FINITE = 1
ARK_DDGI_SUN_BVH_AUTO = 0
ARK_DDGI_SUN_BVH_WORLD = 1
ARK_DDGI_SUN_BVH_LIGHT_SPACE = 2
ARK_DDGI_FLAG_SERIAL_FRAMES = 0x1
ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD = 0x2

ARK_TEX_RGBA8_UNORM = 0
ARK_TEX_RGBA8_SRGB = 1
ARK_TEX_R32F = 2
ARK_TEX_RGBA32F = 3
ARK_BRDF_DEFAULT = 0  # MaterialData.h:5-6
ARK_BRDF_SKIN = 1
ARK_WRAP_REPEAT = 0
ARK_WRAP_CLAMP_TO_EDGE = 1
ARK_WRAP_MIRRORED_REPEAT = 2
ARK_WRAP_PER_AXIS = 0x100


def ark_wrap_axes(s: int, t: int) -> int:
    """ARK_WRAP_AXES(s, t): separate wrap modes for u (s) and v (t)."""
    return ARK_WRAP_PER_AXIS | (s & 0xF) | ((t & 0xF) << 4)


class ArkDdgiDesc(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("grid_dims", C.c_int32 * 3),
        ("probe_spacing", C.c_float * 3),
        ("offset_to_first", C.c_float * 3),
        ("z_far", C.c_float),
        ("max_rays_per_probe", C.c_int32),
        ("max_probe_updates", C.c_int32),
        ("device", C.c_int32),
        ("clear_overflow_mode", C.c_int32),
        ("shard_rank", C.c_int32),
        ("shard_count", C.c_int32),
        ("sun_bvh", C.c_int32),
        ("flags", C.c_uint32),
        ("build_threads", C.c_int32),
        ("reserved", C.c_int32 * 1),
    ]


class ArkRTVertex(C.Structure):
    _fields_ = [("tex_coord", C.c_float * 2), ("normal", C.c_float * 3), ("tangent", C.c_float * 4)]


class ArkRTTriangleMesh(C.Structure):
    _fields_ = [("first_vertex", C.c_int32), ("first_index", C.c_int32), ("material_index", C.c_int32)]


class ArkShaderMaterial(C.Structure):
    _fields_ = [
        ("base_color", C.c_int32),
        ("normal_map", C.c_int32),
        ("metallic_roughness", C.c_int32),
        ("emissive", C.c_int32),
        ("occlusion", C.c_int32),
        ("bent_normal_map", C.c_int32),
        ("clearcoat", C.c_float),
        ("clearcoat_roughness", C.c_float),
        ("blend_mode", C.c_int32),
        ("mask_cutoff", C.c_float),
        ("metallic_factor", C.c_float),
        ("roughness_factor", C.c_float),
        ("emissive_factor", C.c_float * 3),
        ("brdf", C.c_int32),
        ("dielectric_reflectance", C.c_float),
        ("_unused", C.c_float * 3),
        ("color_tint", C.c_float * 4),
    ]


class ArkTexture(C.Structure):
    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("format", C.c_int32),
        ("wrap", C.c_int32),
        ("data", C.c_void_p),
    ]


class ArkRTInstance(C.Structure):
    _fields_ = [
        ("object_to_world", C.c_float * 12),
        ("rt_mesh_index", C.c_uint32),
        ("triangle_count", C.c_uint32),
        ("hit_mask", C.c_uint32),
        ("_pad", C.c_uint32),
    ]


class ArkDirectionalLight(C.Structure):
    _fields_ = [("color", C.c_float * 3), ("world_space_direction", C.c_float * 3)]


class ArkSpotLight(C.Structure):
    _fields_ = [
        ("color", C.c_float * 3),
        ("world_space_direction", C.c_float * 3),
        ("world_space_right", C.c_float * 3),
        ("world_space_up", C.c_float * 3),
        ("world_space_position", C.c_float * 3),
        ("outer_cone_half_angle", C.c_float),
        ("ies_profile_index", C.c_int32),
        ("_pad", C.c_int32),
    ]


class ArkDdgiScene(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("indices", C.c_void_p),
        ("index_count", C.c_uint64),
        ("positions", C.c_void_p),
        ("vertex_count", C.c_uint64),
        ("vertices", C.c_void_p),
        ("meshes", C.c_void_p),
        ("mesh_count", C.c_uint32),
        ("materials", C.c_void_p),
        ("material_count", C.c_uint32),
        ("textures", C.c_void_p),
        ("texture_count", C.c_uint32),
        ("instances", C.c_void_p),
        ("instance_count", C.c_uint32),
        ("has_directional_light", C.c_int32),
        ("directional_light", ArkDirectionalLight),
        ("spot_lights", C.c_void_p),
        ("spot_light_count", C.c_uint32),
        ("environment_texture", C.c_int32),
        ("reserved", C.c_int32 * 4),
    ]


ARK_DDGI_MAX_SPOT_LIGHTS = 10


class ArkDdgiLights(C.Structure):
    """include/ark_ddgi.h ArkDdgiLights: the per-frame light set (GpuScene.cpp:790-858)."""
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("has_directional_light", C.c_int32),
        ("directional_light", ArkDirectionalLight),
        ("spot_lights", C.c_void_p),
        ("spot_light_count", C.c_uint32),
        ("reserved", C.c_int32 * 4),
    ]


class ArkDdgiFrameParams(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("frame_index", C.c_uint32),
        ("first_probe_index", C.c_uint32),
        ("probe_updates", C.c_uint32),
        ("rays_per_probe", C.c_uint32),
        ("hysteresis_irradiance", C.c_float),
        ("hysteresis_visibility", C.c_float),
        ("visibility_sharpness", C.c_float),
        ("ambient_amount", C.c_float),
        ("environment_multiplier", C.c_float),
        ("delta_time", C.c_float),
        ("update_offsets", C.c_int32),
        ("reserved", C.c_int32 * 4),
    ]


class ArkDdgiCounters(C.Structure):
    _fields_ = [
        ("rays", C.c_uint64),
        ("probes", C.c_uint64),
        ("primary_node_visits", C.c_uint64),
        ("primary_tri_tests", C.c_uint64),
        ("hits", C.c_uint64),
        ("front_hits", C.c_uint64),
        ("shadow_rays", C.c_uint64),
        ("shadow_node_visits", C.c_uint64),
        ("shadow_tri_tests", C.c_uint64),
        ("primary_wave_steps", C.c_uint64),
    ]


class ArkDdgiDeviceViews(C.Structure):
    _fields_ = [
        ("irradiance_atlas", C.c_void_p),
        ("irradiance_bytes", C.c_uint64),
        ("irradiance_width", C.c_int32),
        ("irradiance_height", C.c_int32),
        ("visibility_atlas", C.c_void_p),
        ("visibility_bytes", C.c_uint64),
        ("visibility_width", C.c_int32),
        ("visibility_height", C.c_int32),
        ("probe_offsets", C.c_void_p),
        ("probe_offsets_bytes", C.c_uint64),
        ("irradiance_slab_offset", C.c_uint64),
        ("irradiance_slab_bytes", C.c_uint64),
        ("visibility_slab_offset", C.c_uint64),
        ("visibility_slab_bytes", C.c_uint64),
    ]


ARK_DDGI_WINDOW_PACKET_BYTES = 2096


class ArkDdgiWindowExchange(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("full_bands", C.c_uint32),
        ("probes_per_rank", C.c_uint32),
        ("my_probes", C.c_uint32),
        ("first_probe", C.c_uint32),
        ("probe_updates", C.c_uint32),
        ("bytes_per_rank", C.c_uint64),
    ]


class ArkDdgiBvhStats(C.Structure):
    _fields_ = [
        ("node_count", C.c_uint64),
        ("triangle_count", C.c_uint64),
        ("max_depth", C.c_uint32),
        ("max_leaf_size", C.c_uint32),
        ("sah_cost", C.c_float),
        ("build_ms", C.c_float),
        ("node_bytes", C.c_uint64),
        ("triangle_bytes", C.c_uint64),
        ("sun_node_count", C.c_uint64),
        ("sun_cost_world", C.c_float),
        ("sun_cost_light", C.c_float),
        ("sun_build_ms", C.c_float),
        ("refit_ms", C.c_float),
        ("sun_max_depth", C.c_uint32),
        ("sun_rebuilds", C.c_uint32),
        ("sun_rebuild_failures", C.c_uint32),
        ("bvh_rebuilds", C.c_uint32),
        ("bvh_rebuild_ms", C.c_float),
        ("refit_version", C.c_uint32),
        ("bvh_built_refit_version", C.c_uint32),
        ("sun_built_refit_version", C.c_uint32),
        ("bvh_rebuild_failures", C.c_uint32),
    ]


class ArkBakeAoDesc(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("instance_index", C.c_uint32),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("sample_count", C.c_uint32),
        ("bent_normals", C.c_int32),
        ("reserved", C.c_int32 * 2),
    ]


ARK_BAKE_TRIANGLE_INDEX = 0
ARK_BAKE_BARYCENTRICS = 1
ARK_BAKE_OUTPUT = 2

# lighting compose flags (lightingCompose.comp:30-41 named uniforms)
ARK_COMPOSE_DIRECT_LIGHT = 1 << 0
ARK_COMPOSE_SKIN_DIFFUSE_LIGHT = 1 << 1
ARK_COMPOSE_DIFFUSE_GI = 1 << 2
ARK_COMPOSE_BAKED_OCCLUSION = 1 << 3
ARK_COMPOSE_USE_BENT_NORMAL = 1 << 4
ARK_COMPOSE_BENT_NORMAL_OCCLUSION = 1 << 5
ARK_COMPOSE_SCREEN_SPACE_OCCLUSION = 1 << 6
ARK_COMPOSE_GLOSSY_GI = 1 << 7
ARK_COMPOSE_MATERIAL_COLOR = 1 << 8
ARK_COMPOSE_DEFAULT_FLAGS = 0x1FF


class ArkComposeDesc(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("flags", C.c_uint32),
        ("view_from_pixel", C.c_float * 16),
        ("view_from_world", C.c_float * 16),
        ("world_from_view", C.c_float * 16),
        ("depth", C.c_void_p),
        ("base_color", C.c_void_p),
        ("material", C.c_void_p),
        ("normal_velocity", C.c_void_p),
        ("bent_normal", C.c_void_p),
        ("direct_light", C.c_void_p),
        ("diffuse_irradiance", C.c_void_p),
        ("reflections", C.c_void_p),
        ("reflection_direction", C.c_void_p),
        ("screen_space_occlusion", C.c_void_p),
        ("out", C.c_void_p),
    ]


class ArkIesInfo(C.Structure):
    _fields_ = [
        ("photometric_type", C.c_int32),
        ("units_type", C.c_int32),
        ("lamp_count", C.c_int32),
        ("num_angles_v", C.c_uint32),
        ("num_angles_h", C.c_uint32),
        ("lumens_per_lamp", C.c_float),
        ("width", C.c_float),
        ("length", C.c_float),
        ("height", C.c_float),
        ("ballast_factor", C.c_float),
        ("input_watts", C.c_float),
        ("first_angle_v", C.c_float),
        ("last_angle_v", C.c_float),
        ("first_angle_h", C.c_float),
        ("last_angle_h", C.c_float),
        ("max_candela", C.c_float),
    ]


ARK_IES_OK = 0
ARK_IES_E_INVALID_ARGUMENT = -1
ARK_IES_E_IO = -2
ARK_IES_E_PARSE = -3
ARK_IES_LUT_SIZE = 256


ARK_PROBE_DEBUG_DISABLED = 0
ARK_PROBE_DEBUG_IRRADIANCE = 1
ARK_PROBE_DEBUG_DISTANCE = 2
ARK_PROBE_DEBUG_DISTANCE2 = 3


class ArkProbeDebugDesc(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("visualisation", C.c_int32),
        ("distance_scale", C.c_float),
        ("count", C.c_uint32),
        ("probe_indices", C.c_void_p),
        ("directions", C.c_void_p),
        ("out", C.c_void_p),
    ]


class ArkReflectionsDesc(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("width", C.c_uint32),
        ("height", C.c_uint32),
        ("no_tracing_roughness", C.c_float),
        ("environment_multiplier", C.c_float),
        ("ambient_amount", C.c_float),
        ("world_from_view", C.c_float * 16),
        ("view_from_projection", C.c_float * 16),
        ("depth", C.c_void_p),
        ("material", C.c_void_p),
        ("normal_velocity", C.c_void_p),
        ("blue_noise", C.c_void_p),
        ("noise_width", C.c_uint32),
        ("noise_height", C.c_uint32),
        ("out_radiance", C.c_void_p),
        ("out_direction", C.c_void_p),
    ]


# G-buffer plane name -> (dtype, channels) in ArkComposeDesc order
COMPOSE_PLANES = [
    ("depth", "float32", 1), ("base_color", "uint8", 4), ("material", "uint8", 4),
    ("normal_velocity", "float16", 4), ("bent_normal", "float16", 4), ("direct_light", "float16", 4),
    ("diffuse_irradiance", "float16", 4), ("reflections", "float16", 4), ("reflection_direction", "float16", 4),
    ("screen_space_occlusion", "float32", 1),
]


class ArkSoupParams(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("triangle_count", C.c_uint64),
        ("extent", C.c_float),
        ("step_min", C.c_float),
        ("step_max", C.c_float),
        ("width_min", C.c_float),
        ("width_max", C.c_float),
        ("seed", C.c_uint64),
        ("stream", C.c_uint64),
        ("material_count", C.c_uint32),
        ("sun_color", C.c_float * 3),
        ("sun_direction", C.c_float * 3),
        ("has_sun", C.c_int32),
    ]


ABI_STRUCTS = [
    ArkDdgiDesc, ArkRTVertex, ArkRTTriangleMesh, ArkShaderMaterial, ArkTexture, ArkRTInstance,
    ArkDirectionalLight, ArkSpotLight, ArkDdgiScene, ArkDdgiFrameParams, ArkDdgiCounters,
    ArkDdgiDeviceViews, ArkDdgiBvhStats, ArkBakeAoDesc, ArkComposeDesc, ArkProbeDebugDesc, ArkReflectionsDesc,
]

# name -> (restype, argtypes)
EXPORTS = {
    "ark_ddgi_abi_version": (C.c_int32, []),
    "ark_ddgi_create": (C.c_int, [C.POINTER(ArkDdgiDesc), C.POINTER(C.c_void_p)]),
    "ark_ddgi_destroy": (None, [C.c_void_p]),
    "ark_ddgi_last_error": (C.c_char_p, [C.c_void_p]),
    "ark_ddgi_set_scene": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiScene)]),
    "ark_ddgi_share_scene": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ark_ddgi_set_lights": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ark_ddgi_set_instances": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "ark_ddgi_set_instances_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "ark_ddgi_mark_external_write": (C.c_int, [C.c_void_p]),
    "ark_ddgi_get_next_probe_index": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint32)]),
    "ark_ddgi_update": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiFrameParams), C.c_void_p]),
    "ark_ddgi_synchronize": (C.c_int, [C.c_void_p]),
    "ark_ddgi_set_sequencing": (C.c_int, [C.c_void_p, C.c_int, C.c_uint32]),
    "ark_ddgi_get_sequencing": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "ark_ddgi_update_overlapped": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiFrameParams), C.c_void_p, C.c_void_p, C.c_void_p]),
    "ark_ddgi_update_exchanged": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiFrameParams), C.c_void_p]),
    "ark_ddgi_exchange_begin": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ark_ddgi_window_exchange_info": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiWindowExchange)]),
    "ark_ddgi_pack_window": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "ark_ddgi_unpack_window": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "ark_ddgi_exchange_end": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ark_ddgi_resource_size": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint64)]),
    "ark_ddgi_read": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64]),
    "ark_ddgi_write": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64]),
    "ark_ddgi_state_size": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "ark_ddgi_save_state": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "ark_ddgi_load_state": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "ark_ddgi_get_device_views": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiDeviceViews)]),
    "ark_ddgi_reset_history": (C.c_int, [C.c_void_p]),
    "ark_ddgi_set_counting": (C.c_int, [C.c_void_p, C.c_int]),
    "ark_ddgi_get_counters": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiCounters)]),
    "ark_ddgi_get_last_timings": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int]),
    "ark_ddgi_set_timing": (C.c_int, [C.c_void_p, C.c_int]),
    "ark_ddgi_get_bvh_stats": (C.c_int, [C.c_void_p, C.POINTER(ArkDdgiBvhStats)]),
    "ark_ddgi_bake_ao": (C.c_int, [C.c_void_p, C.POINTER(ArkBakeAoDesc), C.c_void_p]),
    "ark_ddgi_bake_read": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64]),
    "ark_ddgi_lighting_compose": (C.c_int, [C.c_void_p, C.POINTER(ArkComposeDesc), C.c_void_p]),
    "ark_ddgi_probe_debug": (C.c_int, [C.c_void_p, C.POINTER(ArkProbeDebugDesc), C.c_void_p]),
    "ark_ddgi_rt_reflections": (C.c_int, [C.c_void_p, C.POINTER(ArkReflectionsDesc), C.c_void_p]),
    # ark_ies.h
    "ark_ies_lut_from_memory": (C.c_int, [C.c_char_p, C.c_uint64, C.c_uint32, C.c_void_p, C.POINTER(ArkIesInfo)]),
    "ark_ies_lut_from_file": (C.c_int, [C.c_char_p, C.c_uint32, C.c_void_p, C.POINTER(ArkIesInfo)]),
    "ark_ies_lookup": (C.c_int, [C.c_char_p, C.c_uint64, C.c_float, C.c_float, C.POINTER(C.c_float)]),
    "ark_ies_last_error": (C.c_char_p, []),
    # ark_scene.h
    "ark_soup_default_params": (None, [C.POINTER(ArkSoupParams)]),
    "ark_soup_generate": (C.c_int, [C.POINTER(ArkSoupParams), C.POINTER(C.c_void_p)]),
    "ark_soup_scene_view": (C.POINTER(ArkDdgiScene), [C.c_void_p]),
    "ark_soup_free": (None, [C.c_void_p]),
    # ark_ddgi_debug.h
    "ark_ddgi_debug_fmath": (C.c_int, [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "ark_ddgi_debug_fmath_host": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    "ark_ddgi_debug_struct_sizes": (C.c_int, [C.POINTER(C.c_uint32), C.c_int]),
    "ark_ddgi_debug_bvh8_check": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]),
    "ark_ddgi_debug_bvh8_check_opts": (C.c_int, [C.c_void_p, C.c_uint64, C.c_int, C.c_float, C.POINTER(C.c_uint64)]),
    "ark_ddgi_debug_sun_bvh_check": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64, C.c_float, C.POINTER(C.c_uint64)]),
    "ark_ddgi_debug_sun_choice": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.POINTER(C.c_double)]),
    "ark_ddgi_debug_scene_digest": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
}

_lib = None


def library_path() -> str:
    """Path of the libark_ddgi.so this process loads (ARK_DDGI_LIB overrides)."""
    return LIB_PATH


def load_library(path: str | None = None) -> C.CDLL:
    """Loads libark_ddgi.so (built in-tree by __graft_entry__.build()). Raises if
    it is missing: there is no fallback implementation of the DDGI path."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libark_ddgi.so not found at {p}: run __graft_entry__.build() (no CPU fallback exists)")
    # torch (ROCm) ships its own libamdhip64 with the same soname: load it first so
    # the process has ONE HIP runtime. Loading ours first makes torch bind to it and
    # report "No HIP GPUs are available" once it initialises.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


class ArkDdgiError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"{ERRORS.get(status, status)}: {message}")
        self.status = status
