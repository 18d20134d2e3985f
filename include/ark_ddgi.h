/*
 * ark_ddgi.h — C-ABI of the MI355X-native DDGI probe-update path.
 *
 * This is the drop-in boundary between Arkose's C++ host (the DDGINode that
 * implements RenderPipelineNode, see arkoserenderer_amd/host/) and the HIP
 * kernels for gfx950. Plain C structs, explicit sizes, no exceptions and no
 * torch/HIP types in the signatures: a hipStream_t is passed as `void*`.
 *
 * Every entry point replaces a piece of the reference's Vulkan-RT DDGI node:
 *
 *   ark_ddgi_create      <- DDGINode::construct resource creation
 *                           (arkose/rendering/nodes/DDGINode.cpp:37-130): grid CB,
 *                           atlases + clear values (:50-55), offsets buffer (:57-60),
 *                           surfel image 4096x512 (:68).
 *   ark_ddgi_set_scene   <- the scene contract DDGINode binds at construct
 *                           (DDGINode.cpp:71-103): TLAS (GpuScene.cpp:872-1010),
 *                           SceneRTMeshDataSet (rayTracing.glsl:9-18), material set
 *                           (material.glsl:9-14), SceneLightSet (lighting.glsl:8-17),
 *                           environment map (GpuScene.cpp:1041-1048). The BVH that the
 *                           Vulkan driver builds is built here instead.
 *   ark_ddgi_share_scene <- one scene (TLAS + buffers) bound by several nodes of one
 *                           device: the Z-slab contexts of a GPU share it.
 *   ark_ddgi_set_lights  <- the per-frame light upload of GpuScene::update
 *                           (GpuScene.cpp:790-858, pre-exposure from :792).
 *   ark_ddgi_set_instances(_async) <- the per-frame TLAS instance update + build
 *                           (GpuScene.cpp:872-1009), as a device refit.
 *   ark_ddgi_update      <- the DDGINode execute lambda (DDGINode.cpp:132-259):
 *                           traceRays -> irradiance update -> visibility update ->
 *                           border copies -> probe offsets.
 *   ark_ddgi_read, ark_ddgi_write <- the published DDGISamplingSet contents
 *                           (DDGINode.cpp:62-66) and the Registry texture reuse that
 *                           carries DDGI history across rebuilds (Registry.cpp:120-150).
 *   ark_ddgi_save_state, ark_ddgi_load_state <- the DDGI history as one blob (atlases +
 *                           offsets + grid header): a checkpoint of what the reference
 *                           keeps only in its Registry textures (no reference
 *                           counterpart; SURVEY §8(b) suggested ABI).
 *
 * Profiling: ark_ddgi_update brackets its launches in roctx ranges named after the
 * reference's debug zones (DDGINode.cpp:152-247): "DDGI" > "Trace rays" (slot
 * table, traversal, shadow rays, shading) and "Update probes" (irradiance +
 * visibility + border copies + probe positions, one fused launch); rocprofv3
 * --marker-trace records them.
 *
 * Status convention: 0 = OK, negative = error (ARK_DDGI_E_*); the message of the
 * last error is available from ark_ddgi_last_error(ctx). This mirrors the
 * reference's ARKOSE_LOG(Error)+NullExecuteCallback handling (DDGINode.cpp:39-42):
 * the node maps a negative status to an Error log and a no-op.
 *
 * Threading: one context per GPU, used from one host thread.
 *
 * Streams: every asynchronous entry point takes a hipStream_t as `void*`; NULL is
 * the legacy default (null) stream, as for any HIP API, so work on it is ordered
 * against every blocking stream of the process (torch's default stream among
 * them). Operations of one context execute in the order they are called, whatever
 * streams they are given: an operation enqueued on another stream than the
 * previous one waits for it on the device (they share the traversal spill area,
 * the hit records and the atlases). Work of other producers on another stream
 * (e.g. the caller filling a G-buffer plane) is the caller's to order, as with any
 * kernel launch.
 */
#ifndef ARK_DDGI_H
#define ARK_DDGI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARK_DDGI_ABI_VERSION 1

/* DDGIData.h:4-9 */
#define ARK_DDGI_IRRADIANCE_RES 8
#define ARK_DDGI_VISIBILITY_RES 16
#define ARK_DDGI_ATLAS_PADDING 1
/* DDGINode.h:22-23 */
#define ARK_DDGI_MAX_RAYS_PER_PROBE 512
#define ARK_DDGI_REFERENCE_MAX_PROBE_UPDATES 4096

/* RTData.h:4-6 */
#define ARK_RT_HIT_MASK_OPAQUE 0x01u
#define ARK_RT_HIT_MASK_MASKED 0x02u
#define ARK_RT_HIT_MASK_BLEND 0x04u

/* ShaderBlendMode.h */
#define ARK_BLEND_MODE_OPAQUE 1
#define ARK_BLEND_MODE_MASKED 2
#define ARK_BLEND_MODE_TRANSLUCENT 3

enum {
    ARK_DDGI_OK = 0,
    ARK_DDGI_E_INVALID_ARGUMENT = -1,
    ARK_DDGI_E_NO_PROBE_GRID = -2,
    ARK_DDGI_E_NO_SCENE = -3,
    ARK_DDGI_E_OUT_OF_MEMORY = -4,
    ARK_DDGI_E_DEVICE = -5,
    ARK_DDGI_E_UNSUPPORTED = -6,
    ARK_DDGI_E_SIZE_MISMATCH = -7
};

/* Which DDGI resource an accessor refers to. */
enum {
    ARK_DDGI_ATLAS_IRRADIANCE = 0, /* RGBA16F, W_irr x H_irr texels, 8 B/texel */
    ARK_DDGI_ATLAS_VISIBILITY = 1, /* RG16F,   W_vis x H_vis texels, 4 B/texel */
    ARK_DDGI_SURFELS = 2,          /* RGBA16F, [slot][rays_per_probe] of the last update */
    ARK_DDGI_PROBE_OFFSETS = 3     /* float4 per probe (xyz used; std430 vec3 stride 16) */
};

/* How the visibility atlas clear value (zFar, zFar^2) is stored in RG16F
 * (DDGINode.cpp:53-55). zFar^2 = 1e8 overflows fp16. */
enum {
    ARK_DDGI_CLEAR_OVERFLOW_INF = 0,       /* IEEE RNE: +inf (default) */
    ARK_DDGI_CLEAR_OVERFLOW_MAX_FINITE = 1 /* saturate to 65504 */
};

/* Texture formats for the bindless material/IES/environment textures. */
enum {
    ARK_TEX_RGBA8_UNORM = 0,
    ARK_TEX_RGBA8_SRGB = 1, /* sRGB decode on fetch (baseColor/emissive/env) */
    ARK_TEX_R32F = 2,       /* IES LUT (GpuScene.cpp:1101-1124) */
    ARK_TEX_RGBA32F = 3     /* HDR environment */
};

/* Texture wrap (ImageWrapModes, GltfLoader.cpp:836-849: glTF wrapS/wrapT). A plain
 * value applies to both axes; ARK_WRAP_PER_AXIS | s | t << 4 gives each its own. */
enum {
    ARK_WRAP_REPEAT = 0,
    ARK_WRAP_CLAMP_TO_EDGE = 1,
    ARK_WRAP_MIRRORED_REPEAT = 2,
    ARK_WRAP_PER_AXIS = 0x100
};
#define ARK_WRAP_AXES(s, t) (ARK_WRAP_PER_AXIS | ((s) & 0xf) | (((t) & 0xf) << 4))

/* Grid + resource description (ProbeGrid.h:6-15, DDGIProbeGridData DDGIData.h:11-15). */
typedef struct ArkDdgiDesc {
    uint32_t struct_size;        /* sizeof(ArkDdgiDesc) */
    int32_t grid_dims[3];        /* gridDimensions x (width), y (height), z (depth) */
    float probe_spacing[3];      /* probeSpacing */
    float offset_to_first[3];    /* offsetToFirst (world position of probe (0,0,0)) */
    float z_far;                 /* camera far plane: visibility clear + miss distance */
    int32_t max_rays_per_probe;  /* surfel image height; <= 512 */
    int32_t max_probe_updates;   /* surfel image width (window capacity); reference: 4096 */
    int32_t device;              /* HIP device ordinal */
    int32_t clear_overflow_mode; /* ARK_DDGI_CLEAR_OVERFLOW_* */
    int32_t shard_rank;          /* Z-slab owned by this context (0 when unsharded) */
    int32_t shard_count;         /* number of Z-slabs (1 when unsharded); must divide grid_dims[2] */
    int32_t sun_bvh;             /* ARK_DDGI_SUN_BVH_*: the structure the sun's shadow rays traverse */
    uint32_t flags;              /* ARK_DDGI_FLAG_* */
    int32_t build_threads;       /* host threads of the BVH builds; 0 = 16 (the GPU box's per-GPU CPU share) */
    int32_t reserved[1];
} ArkDdgiDesc;

/* ArkDdgiDesc.sun_bvh. AUTO: when the scene has a sun, set_scene builds a BVH8 of all
 * triangles in the sun's light space beside the world BVHs, samples 4,096 sun shadow
 * rays through both on the host (any-hit steps per ray) and keeps it only when it is
 * cheaper; WORLD: never built; LIGHT_SPACE: built and kept whenever there is a sun.
 * Results do not depend on the choice (any-hit visibility). */
#define ARK_DDGI_SUN_BVH_AUTO 0
#define ARK_DDGI_SUN_BVH_WORLD 1
#define ARK_DDGI_SUN_BVH_LIGHT_SPACE 2
/* ArkDdgiDesc.flags. SERIAL_FRAMES: every update runs in line on the caller's stream
 * (no traversal stream, no frames in flight); results are the same. NO_BACKGROUND_REBUILD:
 * after ark_ddgi_set_instances the BVHs are only refitted, never rebuilt in the background
 * (a set_scene restores their tightness); results are the same. */
#define ARK_DDGI_FLAG_SERIAL_FRAMES 0x1u
#define ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD 0x2u

/* RTVertex, scalar layout, 36 B (RTData.h:9-13 / NonPositionVertex SceneData.h). */
typedef struct ArkRTVertex {
    float tex_coord[2];
    float normal[3];
    float tangent[4];
} ArkRTVertex;

/* RTTriangleMesh, 12 B (RTData.h:15-19). */
typedef struct ArkRTTriangleMesh {
    int32_t first_vertex;
    int32_t first_index;
    int32_t material_index;
} ArkRTTriangleMesh;

/* ShaderMaterial, std430, 96 B (MaterialData.h:8-33). Texture fields index ArkDdgiScene.textures. */
typedef struct ArkShaderMaterial {
    int32_t base_color;
    int32_t normal_map;
    int32_t metallic_roughness;
    int32_t emissive;
    int32_t occlusion;
    int32_t bent_normal_map;
    float clearcoat;
    float clearcoat_roughness;
    int32_t blend_mode; /* ARK_BLEND_MODE_* */
    float mask_cutoff;
    float metallic_factor;
    float roughness_factor;
    float emissive_factor[3];
    int32_t brdf;
    float dielectric_reflectance;
    float _unused[3];
    float color_tint[4];
} ArkShaderMaterial;

typedef struct ArkTexture {
    int32_t width;
    int32_t height;
    int32_t format; /* ARK_TEX_* */
    int32_t wrap;   /* ARK_WRAP_* */
    const void* data; /* tightly packed rows */
} ArkTexture;

/* One TLAS instance (GpuScene.cpp:901-928 / VulkanAccelerationStructureKHR.cpp:173-198):
 * object-to-world 3x4 row-major, customInstanceId = RT mesh index, hit mask
 * derived from the material blend mode, the BLAS = triangles of that mesh segment. */
typedef struct ArkRTInstance {
    float object_to_world[12];
    uint32_t rt_mesh_index;
    uint32_t triangle_count;
    uint32_t hit_mask; /* ARK_RT_HIT_MASK_* */
    uint32_t _pad;
} ArkRTInstance;

/* DirectionalLightData subset used by the closest hit (LightData.h:9-17); color is
 * pre-multiplied by intensity * lightPreExposure as GpuScene does (GpuScene.cpp:811). */
typedef struct ArkDirectionalLight {
    float color[3];
    float world_space_direction[3];
} ArkDirectionalLight;

/* SpotLightData subset (LightData.h:19-40; GpuScene.cpp:844-858). */
typedef struct ArkSpotLight {
    float color[3];
    float world_space_direction[3];
    float world_space_right[3];
    float world_space_up[3];
    float world_space_position[3];
    float outer_cone_half_angle;
    int32_t ies_profile_index; /* index into ArkDdgiScene.textures (R32F LUT) */
    int32_t _pad;
} ArkSpotLight;

typedef struct ArkDdgiScene {
    uint32_t struct_size;
    const uint32_t* indices;  uint64_t index_count;   /* global u32 index pool, local to first_vertex */
    const float* positions;   uint64_t vertex_count;  /* vec3 position pool (12 B/vertex) */
    const ArkRTVertex* vertices;                      /* non-position pool, vertex_count entries */
    const ArkRTTriangleMesh* meshes; uint32_t mesh_count;
    const ArkShaderMaterial* materials; uint32_t material_count;
    const ArkTexture* textures; uint32_t texture_count;
    const ArkRTInstance* instances; uint32_t instance_count;
    int32_t has_directional_light;
    ArkDirectionalLight directional_light;
    const ArkSpotLight* spot_lights; uint32_t spot_light_count;
    int32_t environment_texture; /* index into textures; -1 = 1x1 white sRGB (GpuScene.cpp:1041-1048) */
    int32_t reserved[4];
} ArkDdgiScene;

/* Per-frame inputs (the push constants of DDGINode.cpp:154-253). */
typedef struct ArkDdgiFrameParams {
    uint32_t struct_size;
    uint32_t frame_index;        /* parameter1 / frameIdx */
    uint32_t first_probe_index;  /* parameter3 / firstProbeIdx (window start) */
    uint32_t probe_updates;      /* K = min(updatesPerFrame, N) */
    uint32_t rays_per_probe;     /* parameter2 / raysPerProbe (R) */
    float hysteresis_irradiance; /* 0 on the first frame (DDGINode.cpp:176) */
    float hysteresis_visibility; /* 0 on the first frame (DDGINode.cpp:191) */
    float visibility_sharpness;  /* default 50 */
    float ambient_amount;        /* ambientLx * lightPreExposure */
    float environment_multiplier;/* preExposedEnvironmentBrightnessFactor */
    float delta_time;            /* AppState::deltaTime */
    int32_t update_offsets;      /* m_computeProbeOffsets && m_applyProbeOffsets */
    int32_t reserved[4];
} ArkDdgiFrameParams;

/* Work/traffic counters of the last update (counters are only collected when
 * ark_ddgi_set_counting(ctx, 1); the timed path compiles them out). */
typedef struct ArkDdgiCounters {
    uint64_t rays;                /* probe rays traced (sum K*R over this context's probes) */
    uint64_t probes;              /* probes updated */
    uint64_t primary_node_visits; /* BVH2 nodes (64 B) fetched by the probe-ray traversals */
    uint64_t primary_tri_tests;   /* triangle records (48 B) fetched by the probe-ray traversals */
    uint64_t hits;                /* probe rays with a hit (front or back face) */
    uint64_t front_hits;          /* probe rays whose hit is shaded (front face) */
    uint64_t shadow_rays;         /* shadow rays traced */
    uint64_t shadow_node_visits;  /* BVH2 nodes fetched by shadow rays */
    uint64_t shadow_tri_tests;    /* triangle records fetched by shadow rays */
    uint64_t primary_wave_steps;  /* wave iterations of the probe-ray traversal (lane utilisation = (node visits + tri tests) / (64 * this)) */
} ArkDdgiCounters;

/* Device-side views of the persistent resources, for an external collective
 * (the Z-slab all-gather) or interop. Pointers are HIP device pointers. */
typedef struct ArkDdgiDeviceViews {
    void* irradiance_atlas; uint64_t irradiance_bytes; int32_t irradiance_width, irradiance_height;
    void* visibility_atlas; uint64_t visibility_bytes; int32_t visibility_width, visibility_height;
    void* probe_offsets;    uint64_t probe_offsets_bytes;
    uint64_t irradiance_slab_offset, irradiance_slab_bytes; /* this rank's Z-slab row band */
    uint64_t visibility_slab_offset, visibility_slab_bytes;
} ArkDdgiDeviceViews;

typedef struct ArkDdgiCtx ArkDdgiCtx;

int32_t ark_ddgi_abi_version(void);

/* Allocates atlases (cleared as DDGINode.cpp:50-55), offsets (zeros, :57-60) and the
 * surfel store (max_probe_updates x max_rays_per_probe, :107). Returns
 * ARK_DDGI_E_NO_PROBE_GRID for an empty grid (DDGINode.cpp:39-42). */
int ark_ddgi_create(const ArkDdgiDesc* desc, ArkDdgiCtx** out_ctx);
void ark_ddgi_destroy(ArkDdgiCtx* ctx);
const char* ark_ddgi_last_error(const ArkDdgiCtx* ctx);

/* Copies the scene arrays to HBM and builds the BVH (host arrays are not retained).
 * On error the context is left without a scene (ARK_DDGI_E_NO_SCENE on update). */
int ark_ddgi_set_scene(ArkDdgiCtx* ctx, const ArkDdgiScene* scene);

/* Makes `ctx` use the scene of `src` (same device): the device arrays and BVH that
 * src's last set_scene built are shared, not copied, and stay alive while any context
 * uses them. For the Z-slab contexts of one GPU (the reference binds one TLAS and one
 * set of scene buffers per device, GpuScene.cpp:872-1010); a later set_scene on
 * either context gives it a scene of its own. Contexts that share a scene are driven
 * from one host thread (a refit or a sun BVH rebuild of one reaches the others). The
 * scene's last holder joins a background sun BVH rebuild still running (set_lights). */
int ark_ddgi_share_scene(ArkDdgiCtx* ctx, const ArkDdgiCtx* src);

/* The per-frame light set (GpuScene::update, GpuScene.cpp:790-858): the reference
 * re-uploads every light every frame with colour x intensity x lightPreExposure (the
 * camera's current exposure, :792, :811, :844) and its transform's forward / right / up
 * / position. Replaces this context's lights (set_scene / share_scene start it with the
 * scene's) for the updates and RT reflections called after it, without touching the
 * BVHs: the spots reach the device in stream order ahead of the next operation that
 * reads them, so frames already enqueued keep the lights they were enqueued with. At
 * most one directional light (:797) and ARK_DDGI_MAX_SPOT_LIGHTS spot lights; a spot's
 * ies_profile_index outside the scene's textures samples the 1x1 white default, as in
 * set_scene. A sun direction other than the one the scene's light-space sun BVH was
 * built for makes the sun's shadow rays traverse the world BVHs at once (identical
 * results); when set_scene chose a light-space BVH, a host thread builds one for the new
 * direction from the device's triangle records, and the first update after it is done
 * installs it (after the frames in flight; ArkDdgiBvhStats.sun_rebuilds). Host arrays
 * are not retained. */
#define ARK_DDGI_MAX_SPOT_LIGHTS 10
typedef struct ArkDdgiLights {
    uint32_t struct_size;        /* sizeof(ArkDdgiLights) */
    int32_t has_directional_light;
    ArkDirectionalLight directional_light;
    const ArkSpotLight* spot_lights; uint32_t spot_light_count;
    int32_t reserved[4];
} ArkDdgiLights;
int ark_ddgi_set_lights(ArkDdgiCtx* ctx, const ArkDdgiLights* lights);

/* The per-frame TLAS instance update (GpuScene.cpp:872-1009: instance transforms
 * re-uploaded, the TLAS updated most frames and fully rebuilt every 60). `instances`
 * is the scene's instance list with new object_to_world transforms: the same count, RT
 * meshes, triangle counts and hit masks as the last set_scene (else
 * ARK_DDGI_E_INVALID_ARGUMENT and nothing changes). The flattened world-space BVHs are
 * refitted on the device - the triangle records of every moved instance re-transformed
 * in the fp32 operation order set_scene uses, every node box recomputed bottom-up and
 * re-quantized outward - so the hits equal those of a set_scene with the same
 * instances (they never depend on the BVH's shape). The sun's light-space BVH is
 * refitted with them (its records re-transformed, its boxes of their light
 * coordinates). The refitted boxes loosen as instances move: after a refit a host
 * thread rebuilds the world BVHs (and the light-space one) from a device snapshot of
 * the refitted records, and the first update after a build is done installs it,
 * refitted forward when more refits came in meanwhile (the reference's full build every
 * 60 frames; ArkDdgiBvhStats.bvh_rebuilds / sun_rebuilds).
 * _async: enqueued on `hip_stream` behind the context's earlier operations (no host
 * wait; the next update's traversal waits for it on the device); a shared scene
 * (ark_ddgi_share_scene) first waits for the device, whose other contexts may be
 * reading it. The blocking form runs it on the context's internal stream and returns
 * when the scene is updated; ArkDdgiBvhStats.refit_ms is the call's host time. */
int ark_ddgi_set_instances_async(ArkDdgiCtx* ctx, const ArkRTInstance* instances, uint32_t count, void* hip_stream);
int ark_ddgi_set_instances(ArkDdgiCtx* ctx, const ArkRTInstance* instances, uint32_t count);

/* One DDGI update (DDGINode.cpp:132-259) enqueued on `hip_stream` (NULL = the null
 * stream). Asynchronous: call ark_ddgi_synchronize or synchronize the stream before
 * reading.
 * Frames in flight: when this update uses the same rays per probe as the previous
 * one and no other writing operation (set_scene, write, load_state, reset_history)
 * came in between, its slot table, primary-ray traversal and probe offsets run on an
 * internal stream as soon as the update before the previous one is done (and after
 * the previous update's offsets, on that stream), i.e. overlapped with the previous
 * update's shadow rays, shading and atlas update. They read only the scene, the
 * sample order and the probe offsets, which nothing in flight on `hip_stream` writes;
 * every result is the serial one. Everything else of the update (shadow rays,
 * shading, atlas update, done_event) stays on `hip_stream`, so the stream's
 * completion still means the update is complete. A caller that writes probe offsets
 * through device pointers (ark_ddgi_get_device_views) between updates calls
 * ark_ddgi_mark_external_write after enqueueing that write: the next update then runs
 * serially, after it. Instrumented updates (timing, counting) run serially. The two
 * streams hand a pipelined frame over by device-side sequence words (a one-wave
 * signal and a one-wave bounded wait per direction) instead of cross-queue events. */
int ark_ddgi_update(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* params, void* hip_stream);
/* The caller wrote context resources through device pointers (probe offsets, atlases)
 * on the stream of the next update: that update waits for the write instead of
 * starting its traversal on the internal stream (see Frames in flight above). */
int ark_ddgi_mark_external_write(ArkDdgiCtx* ctx);
/* Waits for all work of the device; ARK_DDGI_E_DEVICE if a frame-sequencing wait
 * between the context's streams gave up (see ark_ddgi_set_sequencing). */
int ark_ddgi_synchronize(ArkDdgiCtx* ctx);

/* Frame sequencing between the context's streams (no reference counterpart: the
 * reference records one command buffer per frame, VulkanBackend.cpp:1912-1935).
 * device_sequence_words = 1 (default): one-wave signal / bounded-wait kernels;
 * 0: cross-queue events. timeout_ms bounds each wait (0 keeps the current bound;
 * default 10,000 ms). A wait that gives up FAILS CLOSED: every update kernel that
 * starts after it skips (atlases, surfels and offsets are left as they were; a
 * launch already running completes), and the next ark_ddgi_update,
 * ark_ddgi_exchange_begin or ark_ddgi_synchronize drains the device (all of it: the
 * late producer may be on a caller's stream the context does not know), returns
 * ARK_DDGI_E_DEVICE and switches the context to events; the calls after it run
 * normally. The dropped frame's surfels and atlases are untouched; its primary
 * traversal and probe offsets ran on the traversal stream before the failed wait, so
 * its offsets stay applied and the rolling window has moved past it (the next
 * first_probe_index the node passes is unchanged). A Z-slab rank that gets
 * ARK_DDGI_E_DEVICE has dropped a frame the other ranks applied: a multi-rank caller
 * treats it as fatal (or gets every rank to agree before going on), else the ranks'
 * atlases diverge. ark_ddgi_get_sequencing reports the mode, the bound and the number of
 * timeouts reported so far. A context created under a counter-collecting profiler
 * (ROCPROF_COUNTER_COLLECTION set: kernels run one at a time across queues) starts
 * with events. */
int ark_ddgi_set_sequencing(ArkDdgiCtx* ctx, int device_sequence_words, uint32_t timeout_ms);
int ark_ddgi_get_sequencing(const ArkDdgiCtx* ctx, int* out_device_sequence_words, uint32_t* out_timeout_ms, uint32_t* out_timeouts);

/* ark_ddgi_update for a Z-slab rank that overlaps the atlas exchange with the next
 * frame's primary traversal: the traversal is enqueued at once, the shading work
 * (which samples the previous frame's atlases, raygen.rgen:94-106) first waits on
 * hipEvent_t shade_wait_event (e.g. recorded after the previous all-gather; NULL =
 * no wait), and hipEvent_t done_event (NULL = none) is recorded after the probe
 * update so the caller's exchange can start from it. Same work and results as
 * ark_ddgi_update (DDGINode.cpp:132-259). */
int ark_ddgi_update_overlapped(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* params, void* hip_stream, void* shade_wait_event,
                               void* done_event);

/* The same Z-slab frame loop with device-side handovers instead of events (each
 * cross-queue event wait costs 12-16 us of queue latency on MI355X):
 *   ark_ddgi_update_exchanged(ctx, params, stream)   the update; its shading first
 *       waits for the exchange ended by the last ark_ddgi_exchange_end (if any
 *       since the previous update_exchanged)
 *   ark_ddgi_exchange_begin(ctx, comm_stream)        comm_stream waits until the last
 *       update is complete (as its done_event would say)
 *   ... the caller's all-gather of the atlas bands on comm_stream ...
 *   ark_ddgi_exchange_end(ctx, comm_stream)          marks the exchange complete
 * The waits are one-wave kernels, bounded and failing closed as described at
 * ark_ddgi_set_sequencing. Same work and results as ark_ddgi_update_overlapped. */
int ark_ddgi_update_exchanged(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* params, void* hip_stream);
int ark_ddgi_exchange_begin(ArkDdgiCtx* ctx, void* comm_stream);
int ark_ddgi_exchange_end(ArkDdgiCtx* ctx, void* comm_stream);

/* Windowed exchange (SURVEY §8e option (a); DDGINode.cpp:138-140 rolling window). When
 * the last update's window does not cover the grid (K < N), a rank's update wrote only
 * the tiles of its window probes, so instead of the row bands the ranks all-gather one
 * packet per updated probe: its irradiance tile (10 x 10 RGBA16F incl. border) and its
 * visibility tile (18 x 18 RG16F), ARK_DDGI_WINDOW_PACKET_BYTES = 2,096 B. Packets are in
 * each rank's slot order (the rank of the probe among its slab's window probes), which
 * every rank derives from the window alone, so no index travels. Every rank contributes
 * bytes_per_rank (its packets, padded to the largest slab's share), in rank order.
 *   ark_ddgi_window_exchange_info(ctx, &info)        of the last update (after it)
 *   ark_ddgi_exchange_begin(ctx, comm_stream)
 *   info.full_bands ? the band all-gather (ark_ddgi_get_device_views) :
 *     ark_ddgi_pack_window(ctx, recv + rank * info.bytes_per_rank, info.bytes_per_rank, comm_stream)
 *     all-gather of bytes_per_rank per rank into recv (in place) on comm_stream
 *     ark_ddgi_unpack_window(ctx, recv, world * info.bytes_per_rank, comm_stream)
 *   ark_ddgi_exchange_end(ctx, comm_stream)
 * C4 at P = 8 and the reference's K = 2,048: 256 probes x 2,096 B = 0.54 MB per rank
 * instead of 8.6 MB of bands (a rank receives 3.8 MB instead of 60 MB). Replaces the
 * reference's single-GPU atlas writes (probeUpdateIrradiance.comp:77-78 and
 * probeUpdateVisibility.comp:61-62 store into the one shared image). */
#define ARK_DDGI_WINDOW_PACKET_BYTES 2096
typedef struct ArkDdgiWindowExchange {
    uint32_t struct_size;
    uint32_t full_bands;      /* 1: the window covered every probe (K = N): exchange the row bands */
    uint32_t probes_per_rank; /* the largest slab share of the window (packets per rank, padded) */
    uint32_t my_probes;       /* this rank's window probes */
    uint32_t first_probe;     /* the window exchanged: first probe index and count */
    uint32_t probe_updates;
    uint64_t bytes_per_rank;  /* probes_per_rank x ARK_DDGI_WINDOW_PACKET_BYTES (0 with full_bands) */
} ArkDdgiWindowExchange;
int ark_ddgi_window_exchange_info(const ArkDdgiCtx* ctx, ArkDdgiWindowExchange* out);
int ark_ddgi_pack_window(ArkDdgiCtx* ctx, void* dst, uint64_t bytes, void* comm_stream);
int ark_ddgi_unpack_window(ArkDdgiCtx* ctx, const void* src, uint64_t bytes, void* comm_stream);

/* Resource geometry and transfers (blocking, for tests / state save-load). */
int ark_ddgi_resource_size(const ArkDdgiCtx* ctx, int which, uint64_t* out_bytes);
int ark_ddgi_read(ArkDdgiCtx* ctx, int which, void* host_dst, uint64_t bytes);
int ark_ddgi_write(ArkDdgiCtx* ctx, int which, const void* host_src, uint64_t bytes);
int ark_ddgi_get_device_views(ArkDdgiCtx* ctx, ArkDdgiDeviceViews* out_views);

/* DDGI history checkpoint: irradiance + visibility atlases and probe offsets
 * behind a header (magic "ARKDDGI1", grid dims / spacing / origin, zFar, clear mode,
 * shard rank / count, the rolling window's next first probe). Blocking. load_state
 * requires a blob of a context with the same grid, zFar and shard
 * (ARK_DDGI_E_SIZE_MISMATCH / _INVALID_ARGUMENT otherwise) and leaves the context
 * unchanged on any error. */
int ark_ddgi_state_size(const ArkDdgiCtx* ctx, uint64_t* out_bytes);
int ark_ddgi_save_state(ArkDdgiCtx* ctx, void* host_dst, uint64_t bytes);
int ark_ddgi_load_state(ArkDdgiCtx* ctx, const void* host_src, uint64_t bytes);
/* The rolling window's next first probe: (first_probe_index + K) % N of the last
 * update, or the value a loaded state carried (0 for a new context). The node resumes
 * its m_probeUpdateIdx (DDGINode.h:32, advanced at DDGINode.cpp:258) from it. */
int ark_ddgi_get_next_probe_index(const ArkDdgiCtx* ctx, uint32_t* out_index);

/* Re-applies the creation-time clears (Registry created the textures anew). */
int ark_ddgi_reset_history(ArkDdgiCtx* ctx);

/* Counter collection (a separate instrumented traversal variant; off by default). */
int ark_ddgi_set_counting(ArkDdgiCtx* ctx, int enabled);
int ark_ddgi_get_counters(ArkDdgiCtx* ctx, ArkDdgiCounters* out_counters);

/* Device time of the last update's kernels, from HIP events on the update stream:
 * [0] whole update, [1] traversal (slot table + probe rays, and the shadow rays with
 * the shadow queue), [2] surface shading, [3] probe update (irradiance, visibility,
 * borders, offsets), [4] shadow rays traced in their own launch (0 with the queue).
 * Milliseconds. */
int ark_ddgi_get_last_timings(ArkDdgiCtx* ctx, float* out_ms, int count);
int ark_ddgi_set_timing(ArkDdgiCtx* ctx, int enabled);

/* BVH statistics of the last set_scene (node count, leaf triangle count, depth, SAH cost, bytes). */
typedef struct ArkDdgiBvhStats {
    uint64_t node_count;
    uint64_t triangle_count;
    uint32_t max_depth;
    uint32_t max_leaf_size;
    float sah_cost;
    float build_ms;
    uint64_t node_bytes;
    uint64_t triangle_bytes;
    /* the sun's light-space BVH8: its node count (0 = the sun's shadow rays traverse the
     * world BVHs), and the sampled any-hit steps per sun shadow ray of both structures
     * that chose it (0 when not sampled: no sun, or ARK_SUN_BVH=0) */
    uint64_t sun_node_count;
    float sun_cost_world;
    float sun_cost_light;
    float sun_build_ms;  /* host time of the light-space BVH build and its cost sampling (part of build_ms) */
    float refit_ms;      /* the last ark_ddgi_set_instances: wait + refit (0 = none since set_scene) */
    uint32_t sun_max_depth; /* depth of the light-space BVH8 (0 = none); max_depth, which sizes the
                             * traversal stacks' spill, covers it */
    uint32_t sun_rebuilds;  /* light-space BVHs rebuilt in the background and installed since
                             * set_scene (after sun-direction changes or refits; sun_build_ms is
                             * then the last rebuild's time) */
    uint32_t sun_rebuild_failures; /* background sun rebuilds that failed (not retried for the same
                                    * direction and scene version) */
    uint32_t bvh_rebuilds;  /* world BVHs rebuilt in the background after refits and installed */
    float bvh_rebuild_ms;   /* host time of the last such rebuild (0 = none) */
    uint32_t refit_version; /* refits (ark_ddgi_set_instances) since set_scene */
    uint32_t bvh_built_refit_version; /* refit_version of the records the installed world BVHs were built from */
    uint32_t sun_built_refit_version; /* the same for the installed light-space sun BVH */
    uint32_t bvh_rebuild_failures;    /* background world rebuilds that failed (the refitted BVHs stay; no more
                                       * background rebuilds of this scene) */
} ArkDdgiBvhStats;
int ark_ddgi_get_bvh_stats(ArkDdgiCtx* ctx, ArkDdgiBvhStats* out_stats);

/* ------------------------------------------------------------------------------
 * Ambient-occlusion / bent-normal bake of one mesh segment of the current scene,
 * on the same scene and BVH. Replaces the reference's
 * BakeAmbientOcclusionNode (arkose/rendering/baking/BakeAmbientOcclusionNode.cpp:15-131):
 *   1. the UV parameterization pass (bakeParameterization.vert/.frag): every texel
 *      gets the index + 1 of the triangle covering it (0 = none) and its barycentrics
 *      (RGBA16F), by a deterministic rasterizer (see DESIGN.md §AO bake);
 *   2. the ray pass (baking/ao/bakeAmbientOcclusion.rgen:33-118): `sample_count`
 *      cosine-distributed rays per covered texel from the object-space surface point,
 *      tmin 0.0005, tmax 100, any accepted hit occludes (.rahit alpha test for the
 *      masked class); output R8Uint AO (bent_normals = 0) or RGBA8 UNORM bent normal
 *      (bent_normals = 1), as BakeAmbientOcclusionNode.cpp:20-31 selects by format.
 * The mesh is the RT mesh of instance `instance_index` (its triangle_count
 * triangles), baked in object space as MeshViewerApp.cpp:845-880 sets it up. */
typedef struct ArkBakeAoDesc {
    uint32_t struct_size;
    uint32_t instance_index;
    uint32_t width, height;   /* output texture extent */
    uint32_t sample_count;    /* m_sampleCount (BakeAmbientOcclusionNode.h:21, default 500) */
    int32_t bent_normals;     /* 0: R8Uint ambient occlusion, 1: RGBA8 bent normals */
    int32_t reserved[2];
} ArkBakeAoDesc;

/* Runs both passes, enqueued on `hip_stream` (NULL = the null stream). */
int ark_ddgi_bake_ao(ArkDdgiCtx* ctx, const ArkBakeAoDesc* desc, void* hip_stream);

/* Results of the last bake (blocking): width*height texels of
 *   ARK_BAKE_TRIANGLE_INDEX  uint32 (triangle + 1, 0 = uncovered)
 *   ARK_BAKE_BARYCENTRICS    4 x fp16 (b0, b1, b2, 1)
 *   ARK_BAKE_OUTPUT          uint8 AO, or 4 x uint8 bent normal (xyz * 0.5 + 0.5, cone / (pi/2)) */
#define ARK_BAKE_TRIANGLE_INDEX 0
#define ARK_BAKE_BARYCENTRICS 1
#define ARK_BAKE_OUTPUT 2
int ark_ddgi_bake_read(ArkDdgiCtx* ctx, int which, void* host_dst, uint64_t bytes);

/* ---- DDGI consumer: lighting compose -------------------------
 * Replaces LightingComposeNode (arkose/rendering/lighting/LightingComposeNode.cpp:60-110)
 * and its compute shader lightingCompose.comp:22-135 (WITH_DDGI = 1): per pixel,
 * direct light + skin diffuse + glossy reflections + the DDGI diffuse term sampled
 * from this context's current atlases (probeSampling.glsl:64-163), written RGBA16F.
 * Flags mirror the node's named uniforms (lightingCompose.comp:30-41). */
#define ARK_COMPOSE_DIRECT_LIGHT           (1u << 0) /* includeDirectLight */
#define ARK_COMPOSE_SKIN_DIFFUSE_LIGHT     (1u << 1) /* includeSkinDiffuseLight */
#define ARK_COMPOSE_DIFFUSE_GI             (1u << 2) /* includeDiffuseGI */
#define ARK_COMPOSE_BAKED_OCCLUSION        (1u << 3) /* withBakedOcclusion */
#define ARK_COMPOSE_USE_BENT_NORMAL        (1u << 4) /* useBentNormalDirection */
#define ARK_COMPOSE_BENT_NORMAL_OCCLUSION  (1u << 5) /* withBentNormalOcclusion */
#define ARK_COMPOSE_SCREEN_SPACE_OCCLUSION (1u << 6) /* withScreenSpaceOcclusion */
#define ARK_COMPOSE_GLOSSY_GI              (1u << 7) /* includeGlossyGI */
#define ARK_COMPOSE_MATERIAL_COLOR         (1u << 8) /* withMaterialColor */
/* The node's defaults (LightingComposeNode.h:16-25, GpuScene m_includeMaterialColor):
 * all on. Screen-space occlusion is forced off when no AmbientOcclusion texture
 * exists (LightingComposeNode.cpp:56-60); here: when screen_space_occlusion is NULL. */
#define ARK_COMPOSE_DEFAULT_FLAGS 0x1ffu

/* G-buffer planes are device pointers, width x height texels row-major, in the
 * formats GpuScene.cpp:326-360 creates (RGBA16F as 4 x fp16, RGBA8 as 4 x u8 UNORM);
 * depth is the sampled non-linear depth as float. NULL inputs read as 0, like the
 * node's black stand-in textures (LightingComposeNode.cpp:62-71). Matrices are
 * CameraState's (shared/CameraState.h), column-major as GLSL mat4. */
typedef struct ArkComposeDesc {
    uint32_t struct_size;
    uint32_t width, height;          /* targetSize */
    uint32_t flags;                  /* ARK_COMPOSE_* */
    float view_from_pixel[16];
    float view_from_world[16];
    float world_from_view[16];
    const float* depth;                    /* SceneDepth */
    const uint8_t* base_color;             /* SceneBaseColor RGBA8: rgb base colour */
    const uint8_t* material;               /* SceneMaterial RGBA8: roughness, metallic, occlusion */
    const uint16_t* normal_velocity;       /* SceneNormalVelocity RGBA16F: rg = octahedral view-space normal */
    const uint16_t* bent_normal;           /* SceneBentNormal RGBA16F: rgb world bent normal, a cone */
    const uint16_t* direct_light;          /* SceneColor RGBA16F */
    const uint16_t* diffuse_irradiance;    /* SceneDiffuseIrradiance RGBA16F */
    const uint16_t* reflections;           /* DenoisedReflections RGBA16F */
    const uint16_t* reflection_direction;  /* ReflectionDirection RGBA16F (world space) */
    const float* screen_space_occlusion;   /* AmbientOcclusion .r */
    uint16_t* out;                         /* SceneColorWithGI RGBA16F */
} ArkComposeDesc;

/* Enqueues the compose on `hip_stream` (NULL = the null stream), after every
 * operation of this context called before it. */
int ark_ddgi_lighting_compose(ArkDdgiCtx* ctx, const ArkComposeDesc* desc, void* hip_stream);

/* ---- DDGI consumer: RT reflections ray generation -----------
 * Replaces the traceRays of RTReflectionsNode (RTReflectionsNode.cpp:60-82) and its
 * raygen rt-reflections/raygen.rgen:54-166 with WITH_DDGI: per pixel of the G-buffer,
 * one GGX-VNDF-sampled reflection ray (blue-noise driven) traced against the opaque
 * class, shaded by the closest-hit program (opaque.rchit:105-176: emissive + ambient +
 * sun + spots with shadow rays, on front AND back faces, hitT signed) plus the DDGI
 * diffuse term read from this context's atlases (min(metallic, 0.6), F = 0.04), or
 * the environment on a miss. Writes the reflection radiance + signed ray length and
 * the world reflection direction as RGBA16F. Depth >= 1 - 1e-6: result 0, direction
 * left as is; roughness >= no_tracing_roughness: both 0 (raygen.rgen:60-76). The
 * temporal denoiser passes after it (reproject/resolve/prefilter) are not on the path. */
typedef struct ArkReflectionsDesc {
    uint32_t struct_size;
    uint32_t width, height;              /* rt_LaunchSize */
    float no_tracing_roughness;          /* parameter2 (m_noTracingRoughnessThreshold) */
    float environment_multiplier;        /* constants.environmentMultiplier */
    float ambient_amount;                /* constants.ambientAmount (closest hit) */
    float world_from_view[16];           /* CameraState, column-major as GLSL mat4 */
    float view_from_projection[16];
    const float* depth;                  /* SceneDepth (non-linear) */
    const uint8_t* material;             /* SceneMaterial RGBA8: r roughness, g metallic */
    const uint16_t* normal_velocity;     /* SceneNormalVelocity RGBA16F: rg octahedral view-space normal */
    const float* blue_noise;             /* one layer of the blue-noise array, RG32F, noise_width x noise_height;
                                            the layer is frameIndex % layers (parameter3). Sampled at
                                            pixelCenter / size at LOD 0 with repeat: texel (x mod w, y mod h) */
    uint32_t noise_width, noise_height;
    uint16_t* out_radiance;              /* resultImage RGBA16F: radiance, signed ray length */
    uint16_t* out_direction;             /* reflectionDirectionImg RGBA16F: world direction, 0 */
} ArkReflectionsDesc;

/* Enqueues the reflection rays on `hip_stream` (NULL = the null stream), after every
 * operation of this context called before it (it shares the update's traversal
 * stack space). */
int ark_ddgi_rt_reflections(ArkDdgiCtx* ctx, const ArkReflectionsDesc* desc, void* hip_stream);

/* ---- DDGI probe debug visualisation --------------------------
 * The fragment stage of DDGIProbeDebug (DDGIProbeDebug.cpp:34-71,
 * ddgi/probeDebug.frag): for each (probe index, sphere normal) sample, the colour the
 * reference's fragment writes: irradiance pow(texel, 5), distance or distance^2 x
 * distance_scale (magenta for a negative distance), or magenta for an unknown mode.
 * The sphere rasterisation itself stays with the caller (raster is out of scope). */
#define ARK_PROBE_DEBUG_DISABLED   0 /* DDGI_PROBE_DEBUG_VISUALIZE_* (shared/DDGIData.h:17-20) */
#define ARK_PROBE_DEBUG_IRRADIANCE 1
#define ARK_PROBE_DEBUG_DISTANCE   2
#define ARK_PROBE_DEBUG_DISTANCE2  3
typedef struct ArkProbeDebugDesc {
    uint32_t struct_size;
    int32_t visualisation;          /* m_debugVisualisation */
    float distance_scale;           /* m_distanceScale (default 0.01) */
    uint32_t count;                 /* samples */
    const uint32_t* probe_indices;  /* device [count]: gl_InstanceIndex */
    const float* directions;        /* device [count][3]: vNormal */
    uint16_t* out;                  /* device [count][4] RGBA16F */
} ArkProbeDebugDesc;
int ark_ddgi_probe_debug(ArkDdgiCtx* ctx, const ArkProbeDebugDesc* desc, void* hip_stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* ARK_DDGI_H */
