// ddgi_kernels.h — kernel arguments and launchers (host <-> device contract
// inside libark_ddgi; not part of the public C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ark_ddgi.h"
#include "ddgi_types.h"

namespace ark {

constexpr int kStackLds = 8;       // traversal stack entries (node groups, 2 words) per lane kept in LDS (power of 2)
constexpr int kTraceBlock = 256;
constexpr int kShadeBlock = 256;
constexpr int kUpdateBlock = 320;  // 4 waves visibility (16x16 texels) + 1 wave irradiance (8x8)
constexpr int kRayParts = 8;          // per-XCD ray partitions (one head counter each)
constexpr int kRayCounterStride = 32; // u32 words between partition heads (128 B: one line each)
constexpr int kShadeChunk = 1024;  // probe rays per shading block iteration (in-block compaction)
constexpr int kMaxLights = 11;     // 1 directional + 10 spot lights (GpuScene.cpp:430)
constexpr uint32_t kNoHit = 0xffffffffu;

// Read-only scene views in HBM (SceneRTMeshDataSet + material set + SceneLightSet + TLAS).
struct SceneArgs {
    const GpuBvh8Node* nodes;
    const GpuTriangle* tris;
    int32_t root_opaque; // -1 = no geometry of that hit-mask class
    int32_t root_masked;
    int32_t root_blend;
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

    __device__ __forceinline__ int resolveTexture(int idx) const
    {
        return (idx >= 0 && idx < texture_count) ? idx : white_texture;
    }
};

// Per-update arguments (push constants of DDGINode.cpp:193-292 + resources).
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
    float4* fib_order;       // fib[order[j]] with w = order[j] (bits), j = traversal position
    GpuHit* hits;
    uint16_t* surfels;
    uint32_t* spill;
    float4* shade_scratch;   // per shading block: [chunk] partial colours + [chunk][lights] light records
    uint32_t light_count;    // has_sun + spot lights
    uint32_t refill_min;     // trace: refill finished lanes once at least this many are idle
    uint32_t* ray_counter;
    unsigned long long* counters; // [0] nodes [1] tris [2] hits [3] shadow rays
};

hipError_t launch_probe_slots(const FrameArgs& f, hipStream_t s);
hipError_t launch_trace_primary(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s);
hipError_t launch_shade(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s);
size_t shade_lds_bytes(uint32_t lights);
size_t shade_scratch_bytes(uint32_t blocks, uint32_t lights);
hipError_t launch_probe_update(const FrameArgs& f, hipStream_t s);
hipError_t launch_fill_u32(void* p, uint64_t count, uint32_t value, hipStream_t s);
const void* kernel_trace_primary_ptr(bool count);
const void* kernel_shade_ptr(bool count);

} // namespace ark
