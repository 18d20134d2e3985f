// ddgi_kernels.h — kernel arguments and launchers (host <-> device contract
// inside libark_ddgi; not part of the public C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ark_ddgi.h"
#include "ddgi_types.h"

namespace ark {

#ifndef ARK_STACK_LDS
#define ARK_STACK_LDS 8
#endif
#ifndef ARK_LDS_NODES
// 64 top nodes (5 KB of LDS per traversal workgroup instead of 10): the traversal itself
// is unchanged (2.29-2.35 ms serially), but with frames in flight the previous frame's
// kernels find LDS beside it: C4 step 4.06 -> 4.00 ms (128 -> 64; 32: 3.98 ms but the
// reference windows 1 % slower; stack entries 4 instead of 8 spill: +6 %), profiles/r02_m22-23.
// Round 3 added the 2 KB octant table (g_octPerm) to every traversal workgroup; 48 nodes
// bring the workgroup back to about round 2's 21 KB: C4 2,277 -> 2,312 Mrays/s in two
// 10-step A/B runs (32 / 40 / 56 nodes alike, 7 waves/SIMD at 72 VGPRs spills and loses
// 5 %), 2,224 -> 2,246 at the bench's 20 steps; windows and Z-slab proxy within noise
// (profiles/r03_q, r03_r, r03_s)
#define ARK_LDS_NODES 48
#endif
constexpr int kStackLds = ARK_STACK_LDS; // traversal stack entries (node groups, 2 words) per lane kept in LDS (power of 2)
constexpr int kTraceBlock = 256;
constexpr int kLdsNodes = ARK_LDS_NODES; // top BVH8 nodes of the opaque class cached in LDS per traversal workgroup (80 B each)
constexpr int kShadeBlock = 256;
constexpr int kUpdateProbes = 4;   // probes per probe-update workgroup
constexpr int kUpdateBlock = 320;  // 4 visibility waves (one probe each) + 1 irradiance wave (4 probes)
constexpr int kRayParts = 8;          // per-XCD ray partitions (one head counter each)
constexpr int kRayCounterStride = 32; // u32 words between partition heads (128 B: one line each)
constexpr int kShadeChunk = 1024;  // probe rays per shading block iteration (in-block compaction)
constexpr int kMaxLights = 11;     // 1 directional + 10 spot lights (GpuScene.cpp:430)
constexpr uint32_t kNoHit = 0xffffffffu;

// Probe index p as (y, z, x) of the probe order x, then z, then y (ddgi/common.glsl:53-67).
struct ProbeXZY {
    uint32_t y, z, x;
};

__host__ __device__ inline ProbeXZY probeXZY(uint32_t X, uint32_t Z, uint32_t p)
{
    const uint32_t XZ = X * Z, y = p / XZ, r = p - y * XZ, z = r / X;
    return { y, z, r - z * X };
}

// Probes with an index below q's that lie in the box x in [xa, xb), z in [za, zb)
// (every y).
__host__ __device__ inline uint32_t boxProbesBelow(ProbeXZY q, uint32_t xa, uint32_t xb, uint32_t za, uint32_t zb)
{
    const uint32_t zc = q.z < za ? za : (q.z > zb ? zb : q.z);
    const uint32_t xc = q.x < xa ? xa : (q.x > xb ? xb : q.x);
    return q.y * (xb - xa) * (zb - za) + (xb - xa) * (zc - za) + ((q.z >= za && q.z < zb) ? xc - xa : 0u);
}

// Box probes among the first s window positions (probes first, first + 1, ... mod N).
__host__ __device__ inline uint32_t windowBoxCount(uint32_t X, uint32_t Y, uint32_t Z, uint32_t first, uint32_t s, uint32_t xa, uint32_t xb, uint32_t za,
                                                   uint32_t zb)
{
    const uint32_t N = X * Y * Z;
    const uint64_t end = static_cast<uint64_t>(first) + s;
    const uint32_t below = boxProbesBelow(probeXZY(X, Z, first), xa, xb, za, zb);
    if (end <= N) return boxProbesBelow(probeXZY(X, Z, static_cast<uint32_t>(end)), xa, xb, za, zb) - below;
    return Y * (xb - xa) * (zb - za) - below + boxProbesBelow(probeXZY(X, Z, static_cast<uint32_t>(end - N)), xa, xb, za, zb);
}

// Slab probes (z rows [z0, z1) of every y sheet) among the first s window positions:
// the compacted slot of a slab probe at window position s, or the window's slab
// probe count for s = K.
__host__ __device__ inline uint32_t slabRankOf(uint32_t X, uint32_t Y, uint32_t Z, uint32_t z0, uint32_t z1, uint32_t first, uint32_t s)
{
    return windowBoxCount(X, Y, Z, first, s, 0u, X, z0, z1);
}

// Traversal-order bucket of a window probe (kRayParts = 8 blocks of the x-z plane:
// 4 along x and 2 along z of the slab [zlo, zlo + zext), or 8 along x for a one-layer
// slab) and the bucket's box.
__host__ __device__ inline uint32_t slotBucketOf(uint32_t X, uint32_t zlo, uint32_t zext, uint32_t x, uint32_t z)
{
    if (zext >= 2) return x * 4u / X + 4u * ((z - zlo) * 2u / zext < 1u ? 0u : 1u);
    return x * 8u / X;
}

__host__ __device__ inline void slotBucketBox(uint32_t X, uint32_t zlo, uint32_t zext, uint32_t b, uint32_t& xa, uint32_t& xb, uint32_t& za, uint32_t& zb)
{
    if (zext >= 2) {
        const uint32_t bx = b & 3u, zm = (zext + 1u) / 2u;
        xa = (bx * X + 3u) / 4u;
        xb = ((bx + 1u) * X + 3u) / 4u;
        za = zlo + ((b >> 2) ? zm : 0u);
        zb = zlo + ((b >> 2) ? zext : zm);
    } else {
        xa = (b * X + 7u) / 8u;
        xb = ((b + 1u) * X + 7u) / 8u;
        za = zlo;
        zb = zlo + zext;
    }
}

// Queue position of the window probe at window position s (probe p = (first + s) % N,
// inside the slab [zlo, zlo + zext)): the stable bucket sort of the window's slots by
// slotBucketOf, in closed form - the window probes of lower buckets, then those of its
// own bucket at earlier window positions.
__host__ __device__ inline uint32_t slotQueuePos(uint32_t X, uint32_t Y, uint32_t Z, uint32_t zlo, uint32_t zext, uint32_t first, uint32_t K, uint32_t s,
                                                 uint32_t p)
{
    const ProbeXZY q = probeXZY(X, Z, p);
    const uint32_t b = slotBucketOf(X, zlo, zext, q.x, q.z);
    uint32_t xa, xb, za, zb, pos = 0;
    for (uint32_t k = 0; k < b; ++k) {
        slotBucketBox(X, zlo, zext, k, xa, xb, za, zb);
        pos += windowBoxCount(X, Y, Z, first, K, xa, xb, za, zb);
    }
    slotBucketBox(X, zlo, zext, b, xa, xb, za, zb);
    return pos + windowBoxCount(X, Y, Z, first, s, xa, xb, za, zb);
}

// One shadow ray: origin + tmax, direction + owner ((probe ray << 4) | light).
struct alignas(16) ShadowRay {
    float4 origin_tmax;
    float4 dir_owner;
};

// Word offsets in the ray-counter buffer (each counter on its own 128-B line): the
// probe-ray partition heads, the shading heads, the shadow list (count + partition heads).
constexpr int kShadeHeadWord = kRayParts * kRayCounterStride;
constexpr int kShadowCountWord = 2 * kRayParts * kRayCounterStride;
constexpr int kShadowHeadWord = kShadowCountWord + kRayCounterStride; // kRayParts partition heads
// the sun's shadow-ray list (FrameArgs::sun_rays): count + partition heads
constexpr int kSunCountWord = kShadowHeadWord + kRayParts * kRayCounterStride;
constexpr int kSunHeadWord = kSunCountWord + kRayCounterStride;
constexpr int kRayCounterWords = kSunHeadWord + kRayParts * kRayCounterStride;

// Read-only scene views in HBM (SceneRTMeshDataSet + material set + SceneLightSet + TLAS).
struct SceneArgs {
    const GpuBvh8Node* nodes;
    const GpuTriangle* tris;     // = (char*)nodes + tri_byte_offset (one allocation)
    uint32_t tri_byte_offset;
    int32_t root_opaque; // -1 = no geometry of that hit-mask class
    int32_t root_masked;
    int32_t root_blend;
    uint32_t opaque_nodes; // node count of the opaque class (breadth-first from root_opaque)
    int32_t texture_count;
    const uint32_t* indices;
    const float* vertices; // RTVertex, 9 floats (36 B) each
    const ArkRTTriangleMesh* meshes;
    const ArkShaderMaterial* materials;
    const GpuInstance* instances;
    const GpuTextureInfo* tex_infos;
    const float4* texels;
    int32_t white_texture; // 1x1 white sRGB default (GpuScene.cpp:55-56)
    int32_t env_texture;
    int32_t has_sun;
    int32_t spot_count;
    float sun_color[3];
    float sun_dir[3];
    const GpuSpotLight* spots;
    // [triangle] 3 x float4: object-space vertex normals n0, n1, n2 (9 floats) and the
    // instance index; BVH triangle order. Lets k_trace find the shading normal of a
    // front hit with two dependent loads instead of five (set when lights exist).
    const float4* tri_normals; // per-triangle shading records [4]: n0 n1 n2 (9), instance, uv0 uv1 uv2
    // the sun's light-space BVH8 (ark_ddgi.cpp sunFrame): every triangle of every
    // hit-mask class, boxes in the frame (u, v, w = the shadow rays' direction), leaves
    // holding the world-space triangle records; sun_root = -1: none (the sun's shadow
    // rays then traverse the world BVHs)
    const GpuBvh8Node* sun_nodes;
    const GpuTriangle* sun_tris;
    int32_t sun_root = -1; // (a zero-initialised SceneArgs must not mean "sun BVH at node 0")
    float sun_frame[9]; // rows u, v, w

    __device__ __forceinline__ int resolveTexture(int idx) const
    {
        return (idx >= 0 && idx < texture_count) ? idx : white_texture;
    }
    // Bilinear sample of a material/environment/IES texture; the 1x1 white default
    // filters to exactly (1, 1, 1, 1) for finite coordinates, so it is not fetched.
    __device__ __forceinline__ float4 sample(int idx, float u, float v) const;
};

// Per-update arguments (push constants of DDGINode.cpp:154-253 + resources).
struct FrameArgs {
    int32_t X, Y, Z;
    int32_t Wi, Hi, Wv, Hv;
    float spacing[3];
    float origin[3];
    float z_far;
    uint32_t frame;
    uint32_t first;          // window start (firstProbeIdx)
    uint32_t window;         // K (window length over the whole grid)
    uint32_t window_probes;  // probes this context updates (K, or its Z-slab share)
    uint32_t window_rays;    // window_probes * R
    uint32_t R;
    uint32_t Rmax;
    int32_t sharded;
    int32_t slab_z0, slab_z1;
    float hysteresis_irradiance;
    float hysteresis_visibility;
    float visibility_sharpness;
    float ambient_amount;
    float environment_multiplier;
    float delta_time;
    int32_t update_offsets;
    uint16_t* irr;
    uint16_t* vis;
    float4* offsets;
    GpuProbeSlot* slots;
    float4* fib;
    const uint32_t* order;   // traversal order of the R samples (lane -> sample), see sampleTraversalOrder
    const uint32_t* slot_order; // traversal order of the window's slots (queue position -> slot), null = identity
    float4* fib_order;       // fib[order[j]] with w = order[j] (bits), j = traversal position
    GpuHit* hits;
    uint16_t* surfels;
    uint32_t* spill;
    uint32_t light_count;    // has_sun + spot lights
    uint32_t refill_min;     // trace: refill finished lanes once at least this many are idle
    uint32_t sun_refill_min; // the sun's light-space shadow traversal: the same for its lanes
    uint32_t grab_chunk;     // trace / shadow: rays a wave takes from its partition head at once (<= 64)
    uint32_t* shadow_bits;   // [window_rays] lit light bits 0-15, occluded bits 16-31 (front hits)
    ShadowRay* shadow_rays;  // k_shadow_gen's list: [window_rays * light_count] worst case
    uint32_t* shadow_count;  // = ray_counter + kShadowCountWord
    uint32_t* shadow_heads;  // = ray_counter + kShadowHeadWord (kRayParts heads, kRayCounterStride apart)
    // with a sun light-space BVH (SceneArgs::sun_root >= 0): k_shadow_gen puts the
    // sun's shadow rays in this list instead (null: every shadow ray in shadow_rays),
    // traced by k_trace_shadow<.., SUN = true>
    ShadowRay* sun_rays;
    uint32_t* sun_count;     // = ray_counter + kSunCountWord
    uint32_t* sun_heads;     // = ray_counter + kSunHeadWord
    uint32_t* ray_counter;
    unsigned long long* counters; // [0] nodes [1] tris [2] hits [3] shadow rays
    uint16_t* ray_steps;     // counting updates: traversal iterations of each probe ray (both passes) at its hit-record index
    // ray-list traversals (RT reflections): {origin, tmax}, {direction, pixel} per ray
    const float4* ray_list;
    const uint32_t* list_count;
    // fail-closed frame sequencing: the context's timed-out word (set by a k_seq_wait
    // that gave up); every kernel of the update leaves its outputs untouched once it is
    // set (frameAborted). Null = never (consumers, serial instrumented paths).
    const uint32_t* abort_word;
};

// Fail-closed frame sequencing (ark_ddgi.cpp updateImpl): true when a frame-sequencing
// wait of this context has timed out, so this launch must not compute (its inputs may
// not be ready). Read once per workgroup by thread 0 and broadcast through LDS, so the
// workgroup takes one decision (its waves share barriers further on).
__device__ __forceinline__ bool frameAborted(const uint32_t* abortWord)
{
    if (!abortWord) return false;
    __shared__ uint32_t sAbort;
    if (threadIdx.x == 0) sAbort = __hip_atomic_load(abortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return sAbort != 0u;
}

// AO / bent-normal bake of one mesh segment (ark_ddgi_bake_ao; ddgi_kernels.hip §5)
struct BakeArgs {
    uint32_t W, H, samples, tri_count;
    int32_t bent;
    uint32_t first_index, first_vertex;
    const uint32_t* indices;
    const float* positions; // vec3 pool (object space)
    const float* vertices;  // RTVertex pool (9 floats)
    uint32_t* tri_idx;      // [H][W] triangle + 1
    uint16_t* bary;         // [H][W][4] fp16
    uint8_t* out;           // [H][W] AO or [H][W][4] bent normal
    uint32_t* pixels;       // covered texels (k_bake_bary appends)
    uint32_t* counters;     // [0] covered count, [32] AO queue head
    uint32_t* spill;
};

// Per-frame scene inputs (ddgi_scene_update.hip)
// the context's spot lights as a kernel argument (ark_ddgi_set_lights)
struct LightBlock {
    GpuSpotLight spots[kMaxLights - 1];
    uint32_t count;
};
// one TLAS instance for the refit of its triangle records (ark_ddgi_set_instances)
struct alignas(16) RefitInstance {
    float m[12];           // object_to_world, 3 x 4 row-major
    int32_t first_vertex;  // its RT mesh's vertex and index offsets
    uint32_t first_index;
    uint32_t flip;         // det(object_to_world) < 0
    uint32_t dirty;        // its transform changed since the records were last written
};
// The refitted boxes' absolute inflation, from the host (enqueueRefit / refitInflations:
// the instances' transformed bounds, never less than the build's): world BVHs 1e-6
// |diagonal| (bvh8_inflation_box, as set_scene); the light-space BVH 2 x 1e-6 |light
// diagonal| + 2e-6 max |world coordinate| (build_sun_bvh)
struct RefitBoxArgs {
    double frame[9];     // light-space rows u, v, w (sun_frame); unused for the world BVHs
    float inflate;       // the inflation of this BVH's boxes
    uint32_t light;      // 1: the light-space BVH (boxes of the light coordinates)
    uint64_t dirty;      // bits (id mod 64) of the instances moved since the target copy's version; all: every node
};
hipError_t launch_store_lights(const LightBlock& b, GpuSpotLight* dst, hipStream_t s);
// one level (order[0 .. count)): masks[node] = the instance bits below it (children's masks from the deeper levels)
hipError_t launch_node_masks(const GpuBvh8Node* nodes, const GpuTriangle* tris, uint64_t* masks, const uint32_t* order, uint32_t count, hipStream_t s);
// one level: nodes order[0 .. count) whose mask meets a.dirty - their leaf slots' records of
// dirty instances re-transformed (inst), boxes [node][6] (lo, hi) of the deeper levels in, this level's out
hipError_t launch_refit_nodes(GpuBvh8Node* nodes, GpuTriangle* tris, float* boxes, const uint32_t* order, uint32_t count, const RefitBoxArgs& a,
                              const uint64_t* masks, const RefitInstance* inst, const uint32_t* indices, const float* positions, hipStream_t s);
// dst[i] = src[perm[i]] (64-B shading records), perm ~0: zeros (an installed rebuild's record order)
hipError_t launch_gather_records(float4* dst, const float4* src, const uint32_t* perm, uint64_t count, hipStream_t s);

// Windowed Z-slab exchange (ddgi_exchange.hip, ark_ddgi_pack_window / _unpack_window):
// one packet per updated probe, its irradiance tile (10 x 10 RGBA16F, border included)
// then its visibility tile (18 x 18 RG16F), in the rank's slot order (slabRankOf)
struct WindowExchangeArgs {
    uint32_t X, Y, Z, N;
    uint32_t first, K;       // the window of the update exchanged
    uint32_t Wi, Wv;         // atlas widths (texels)
    uint32_t slabDepth;      // probe layers per rank (Z / world)
    uint32_t rank, world;
    uint64_t bytesPerRank;   // the all-gather's count per rank (max window probes of a slab x packet)
    uint16_t* irr;
    uint16_t* vis;
    uint8_t* buf;            // pack: this rank's packets; unpack: all ranks' (world x bytesPerRank)
};
constexpr uint32_t kIrrTileTexels = (ARK_DDGI_IRRADIANCE_RES + 2 * ARK_DDGI_ATLAS_PADDING) * (ARK_DDGI_IRRADIANCE_RES + 2 * ARK_DDGI_ATLAS_PADDING);
constexpr uint32_t kVisTileTexels = (ARK_DDGI_VISIBILITY_RES + 2 * ARK_DDGI_ATLAS_PADDING) * (ARK_DDGI_VISIBILITY_RES + 2 * ARK_DDGI_ATLAS_PADDING);
constexpr uint32_t kWindowPacketBytes = kIrrTileTexels * 8u + kVisTileTexels * 4u; // 2,096
hipError_t launch_window_pack(const WindowExchangeArgs& a, bool unpack, hipStream_t s);

hipError_t launch_probe_slots(const FrameArgs& f, hipStream_t s);
// stage 0: parameterization raster, 1: barycentrics + work list, 2: AO rays
hipError_t launch_bake(const SceneArgs& sc, const BakeArgs& b, uint32_t blocks, int stage, hipStream_t s);
hipError_t launch_lighting_compose(const FrameArgs& f, const ArkComposeDesc& c, hipStream_t s);
// RT reflections as a ray-list pipeline: stage 0 setup (G-buffer -> ray list),
// 1 closest-hit traversal, 2 shadow-ray list, 3 shadow traversal, 4 shading
hipError_t launch_rt_reflections(const SceneArgs& sc, const FrameArgs& f, const ArkReflectionsDesc& r, uint32_t traceBlocks, uint32_t shadowBlocks,
                                 hipStream_t s);
hipError_t launch_probe_debug(const FrameArgs& f, const ArkProbeDebugDesc& d, hipStream_t s);
hipError_t launch_trace(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s);
hipError_t launch_shade(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s);
hipError_t launch_trace_shadow(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s);
hipError_t launch_shadow_gen(const SceneArgs& sc, const FrameArgs& f, hipStream_t s);
hipError_t launch_probe_update(const FrameArgs& f, hipStream_t s);
hipError_t launch_probe_offsets(const FrameArgs& f, hipStream_t s);
hipError_t launch_fill_u32(void* p, uint64_t count, uint32_t value, hipStream_t s);
// frame sequencing between two streams of one context (k_seq_signal / k_seq_wait)
hipError_t launch_seq_signal(uint32_t* word, uint32_t value, hipStream_t s);
// k_seq_wait gives up after timeoutTicks of the device wall clock (or at once when
// *timedOut is already set): it sets *timedOut (the kernels of the frame then skip,
// frameAborted) and *hostFlag (host-mapped, polled by the next context call)
hipError_t launch_seq_wait(const uint32_t* word, uint32_t value, uint32_t* timedOut, uint32_t* hostFlag, uint64_t timeoutTicks, hipStream_t s);
const void* kernel_trace_ptr(bool count);
const void* kernel_shade_ptr(bool count);
const void* kernel_trace_shadow_ptr(bool count);

} // namespace ark
