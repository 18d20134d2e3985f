// ddgi_kernels.hip — the DDGI probe-update hot path as HIP kernels for gfx950.
//
// One update (DDGINode.cpp:132-259) is these launches on one stream:
//   1. k_probe_slots    window -> slot table (probe position + offset, per-probe
//                       ray rotation), the slots' traversal order and the
//                       spherical-Fibonacci table.
//   2. k_trace          persistent traversal of all K*R probe rays: opaque pass
//                       (closest hit) then masked pass (alpha-tested any-hit),
//                       software 8-wide quantized BVH (80 B nodes) with a per-lane
//                       LDS ring stack of node groups (spilling to HBM only beyond
//                       kStackLds entries) and wave64 ballot refill of finished
//                       lanes (raygen.rgen:35-92).
//   3. k_shadow_gen     lit lights of every front hit -> shadow-ray list
//      k_trace_shadow   persistent any-hit traversal of that list (opaque.rchit:35-54).
//   4. k_shade          closest-hit shading (opaque.rchit:105-176) with the shadow
//                       bits, environment on miss (raygen.rgen:71-80), indirect from
//                       the previous frame's atlases (probeSampling.glsl:64-163)
//                       -> fp16 surfels.
//   5. k_probe_update   (ddgi_update.hip) irradiance + visibility blend,
//                       tile border copy, probe offsets.
// No MFMA: the path is traversal/gather, latency/issue bound.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/ark_ddgi.h"
#include "ddgi_device.h"
#include "ddgi_kernels.h"

namespace ark {

__device__ __forceinline__ float4 SceneArgs::sample(int idx, float u, float v) const
{
    const int r = resolveTexture(idx);
    if (r == white_texture && fabsf(u) < INFINITY && fabsf(v) < INFINITY) return make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    return dev::sampleTexture(tex_infos, texels, r, u, v);
}

namespace dev {

// ---------------------------------------------------------------------------
// 1. window -> slots
// ---------------------------------------------------------------------------
// sphericalFibonacciSample (common.glsl:121-130)
__device__ V3 sphericalFibonacciSample(uint32_t i, uint32_t n)
{
    float theta = kTwoPi * static_cast<float>(i) / kGoldenRatio;
    float phi = acosf_(2.0f * (static_cast<float>(i) / static_cast<float>(n)) - 1.0f);
    float sinPhi = sinf_(phi);
    float st, ct;
    sincosf_(theta, &st, &ct);
    return { ct * sinPhi, st * sinPhi, cosf_(phi) };
}

// Writes slot `slot` for probe `probeIdx` (ddgi/common.glsl:12-25 seed/rotation,
// :69-77 position, raygen.rgen:117-118 offset).
__device__ void writeSlot(const FrameArgs& f, uint32_t slot, uint32_t probeIdx)
{
    uint32_t tilesPerSheet = static_cast<uint32_t>(f.X * f.Z);
    uint32_t sheetProbeIdx = probeIdx % tilesPerSheet;
    int y = static_cast<int>(probeIdx / tilesPerSheet);
    int x = static_cast<int>(sheetProbeIdx % static_cast<uint32_t>(f.X));
    int z = static_cast<int>(sheetProbeIdx / static_cast<uint32_t>(f.X));
    V3 c = { static_cast<float>(x), static_cast<float>(y), static_cast<float>(z) };
    V3 pos = v3(f.origin[0], f.origin[1], f.origin[2]) + c * v3(f.spacing[0], f.spacing[1], f.spacing[2]);
    float4 off = f.offsets[probeIdx];
    pos = pos + v3(off.x, off.y, off.z);
    uint32_t st = wang_hash(512u * probeIdx + f.frame % 512u);
    // randomPointOnSphere (random.glsl:63-74)
    float theta = kTwoPi * randomFloat(st);
    float u = 2.0f * randomFloat(st) - 1.0f;
    float sr = sqrtf_(1.0f - u * u);
    float s, cth;
    sincosf_(theta, &s, &cth);
    V3 axis = { sr * cth, sr * s, u };
    float angle = kTwoPi * randomFloat(st);
    float as, ac;
    sincosf_(angle, &as, &ac);
    GpuProbeSlot ps;
    ps.pos[0] = pos.x;
    ps.pos[1] = pos.y;
    ps.pos[2] = pos.z;
    ps.probe_index = probeIdx;
    ps.axis[0] = axis.x;
    ps.axis[1] = axis.y;
    ps.axis[2] = axis.z;
    ps.angle_sin = as;
    ps.angle_cos = ac;
    ps._pad[0] = ps._pad[1] = ps._pad[2] = 0.0f;
    f.slots[slot] = ps;
}

__device__ __forceinline__ bool inSlab(const FrameArgs& f, uint32_t probeIdx)
{
    uint32_t sheetProbeIdx = probeIdx % static_cast<uint32_t>(f.X * f.Z);
    int z = static_cast<int>(sheetProbeIdx / static_cast<uint32_t>(f.X));
    return z >= f.slab_z0 && z < f.slab_z1;
}

// Unsharded: slot s <-> probe (first + s) % N (raygen.rgen:113). Sharded (Z-slab):
// the window's slab probes in window order, each slot from the closed-form count of
// slab probes before it (slabRankOf), so slots are deterministic and one thread each.
// Traversal order of the slots (f.slot_order: queue position -> slot), in the same
// pass: the probes are cut into 8 blocks of the x-z plane (4 along x, 2 along z, or
// 8 along x for a one-layer slab) and each block's slots keep their window order,
// whose slowest coordinate is y (a stable bucket sort, in closed form: slotQueuePos).
// The trace and shade queues hand the 8 per-XCD partitions out in this order, so
// partition p sweeps block p bottom to top and all XCDs work on the same few y-layers
// at any time: the chip-wide working set of BVH nodes and triangles is one slice of
// the scene (Infinity Cache sized) instead of eight. Only the order of work changes,
// never a result.
__global__ void __launch_bounds__(256) k_probe_slots(FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    const uint32_t X = static_cast<uint32_t>(f.X), Y = static_cast<uint32_t>(f.Y), Z = static_cast<uint32_t>(f.Z);
    const uint32_t N = X * Y * Z;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    // this frame's work counters (trace / shadow heads, shadow-list count): zeroed here
    // rather than by a separate fill ahead of this kernel on the traversal stream
    for (uint32_t i = tid; i < kRayCounterWords; i += gridDim.x * blockDim.x) f.ray_counter[i] = 0u;
    if (tid < f.R) {
        V3 d = sphericalFibonacciSample(tid, f.R);
        f.fib[tid] = make_float4(d.x, d.y, d.z, 0.0f);
        // traversal order: position tid traces sample order[tid] (w = sample index)
        const uint32_t sample = f.order[tid];
        V3 e = sphericalFibonacciSample(sample, f.R);
        f.fib_order[tid] = make_float4(e.x, e.y, e.z, __uint_as_float(sample));
    }
    if (tid >= f.window) return;
    const uint32_t probeIdx = (tid + f.first) % N;
    const uint32_t z0 = f.sharded ? static_cast<uint32_t>(f.slab_z0) : 0u, z1 = f.sharded ? static_cast<uint32_t>(f.slab_z1) : Z;
    if (f.sharded && !inSlab(f, probeIdx)) return;
    const uint32_t slot = f.sharded ? slabRankOf(X, Y, Z, z0, z1, f.first, tid) : tid;
    writeSlot(f, slot, probeIdx);
    if (f.slot_order)
        const_cast<uint32_t*>(f.slot_order)[slotQueuePos(X, Y, Z, z0, max(1u, z1 - z0), f.first, f.window, tid, probeIdx)] = slot;
}

// queue position -> slot (identity without an order table)
__device__ __forceinline__ uint32_t slotAt(const FrameArgs& f, uint32_t q)
{
    return f.slot_order ? f.slot_order[q] : q;
}

// ---------------------------------------------------------------------------
// BVH traversal
// ---------------------------------------------------------------------------
// Per-lane traversal stack of node groups {child_base, hits | imask << 8}: the top
// kStackLds entries live in an LDS ring (slot-major, so the 64 lanes of a wave hit
// distinct banks), deeper entries spill to a per-lane HBM area
// [entry][word][lane] that only deep descents touch.
template<int BLOCK>
struct Stack {
    uint32_t* lds;
    uint32_t* spill;
    uint32_t spillStride;
    int depth;
    __device__ __forceinline__ void push(uint32_t a, uint32_t b)
    {
        const int slot = depth & (kStackLds - 1);
        uint32_t* l = lds + slot * 2 * BLOCK;
        if (depth >= kStackLds) {
            uint32_t* sp = spill + static_cast<size_t>(depth - kStackLds) * 2 * spillStride;
            sp[0] = l[0];
            sp[spillStride] = l[BLOCK];
        }
        l[0] = a;
        l[BLOCK] = b;
        depth++;
    }
    __device__ __forceinline__ void pop(uint32_t& a, uint32_t& b)
    {
        depth--;
        const int slot = depth & (kStackLds - 1);
        uint32_t* l = lds + slot * 2 * BLOCK;
        a = l[0];
        b = l[BLOCK];
        if (depth >= kStackLds) {
            const uint32_t* sp = spill + static_cast<size_t>(depth - kStackLds) * 2 * spillStride;
            l[0] = sp[0];
            l[BLOCK] = sp[spillStride];
        }
    }
};

struct RayHit {
    float t;      // best t so far (tmax of the query)
    float u, v;
    uint32_t tri; // leaf-order triangle index, kNoHit = none
    uint32_t inst, prim;
    bool backface;
};

// Inverse ray direction for the box tests only (triangle tests use d): v_rcp_f32
// (1 ulp) instead of an IEEE divide (~10 VALU each). Every slab distance of an axis
// then carries the same relative factor 1 +- 6e-8, far inside the box test's 1e-5
// relative margin (visitNode8), so culling stays conservative; the sign, and with
// it the ray octant, is exact.
__device__ __forceinline__ V3 safeInv(V3 d)
{
    auto f = [](float x) { return __builtin_amdgcn_rcpf(fabsf_(x) < 1e-20f ? (x < 0.0f ? -1e-20f : 1e-20f) : x); };
    return { f(d.x), f(d.y), f(d.z) };
}

// Möller–Trumbore, identical op order to the oracle's intersectTri. The cross and dot
// products are fused explicitly (crossFma / dotFma: 6 and 3 VALU instead of 9 and 5;
// the ray-triangle test is the traversal step's second largest block), in the same
// places as the oracle, so results stay bit-exact under -ffp-contract=off.
__device__ __forceinline__ V3 crossFma(V3 a, V3 b)
{
    return { fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)) };
}
__device__ __forceinline__ float dotFma3(V3 a, V3 b) { return fmaf(a.x, b.x, fmaf(a.y, b.y, a.z * b.z)); }

// Branch free: in a wave some lane passes each early-out test on almost every
// step, so the early returns saved no VALU and cost an exec-mask branch each
// (~14 SALU per traversal step). The accepted set is the oracle's: u <= 1 follows
// from v >= 0 and RN(u + v) <= 1 (rounding is monotonic), and det == 0 gives
// inv = +-inf, so u or v is NaN or infinite and one of u >= 0, v >= 0, u + v <= 1
// fails, as the oracle's early return rejects it; the values of an accepted hit
// are computed exactly as the oracle computes them.
__device__ __forceinline__ bool intersectTri(V3 o, V3 d, float tmin, float tmax, const GpuTriangle& tr, float* outT, float* outU, float* outV, bool* backfaceDet)
{
    V3 v0 = { tr.t0[0], tr.t0[1], tr.t0[2] };
    V3 e1 = { tr.t0[3], tr.t1[0], tr.t1[1] };
    V3 e2 = { tr.t1[2], tr.t1[3], tr.t2[0] };
    V3 p = crossFma(d, e2);
    float det = dotFma3(e1, p);
    float inv = 1.0f / det;
    V3 s = o - v0;
    float u = dotFma3(s, p) * inv;
    V3 q = crossFma(s, e1);
    float v = dotFma3(d, q) * inv;
    float tt = dotFma3(e2, q) * inv;
    *outT = tt;
    *outU = u;
    *outV = v;
    *backfaceDet = det < 0.0f;
    return (u >= 0.0f) & (v >= 0.0f) & (u + v <= 1.0f) & (tt >= tmin) & (tt <= tmax);
}

__device__ __forceinline__ GpuTriangle loadTri(const GpuTriangle* __restrict__ tris, uint32_t i)
{
    const float4* p = reinterpret_cast<const float4*>(tris + i);
    float4 a = p[0], b = p[1], c = p[2];
    GpuTriangle t;
    t.t0[0] = a.x; t.t0[1] = a.y; t.t0[2] = a.z; t.t0[3] = a.w;
    t.t1[0] = b.x; t.t1[1] = b.y; t.t1[2] = b.z; t.t1[3] = b.w;
    t.t2[0] = c.x; t.t2[1] = c.y; t.t2[2] = c.z; t.t2[3] = c.w;
    return t;
}

// masked.rahit:16-37 — any-hit alpha test of a masked candidate.
__device__ bool alphaAccept(const SceneArgs& sc, uint32_t inst, uint32_t prim, float u, float v)
{
    const GpuInstance& gi = sc.instances[inst];
    const ArkRTTriangleMesh mesh = sc.meshes[gi.rt_mesh_index];
    const ArkShaderMaterial& mat = sc.materials[mesh.material_index];
    float bx = 1.0f - u - v, by = u, bz = v;
    float uv[2][3];
    for (int k = 0; k < 3; ++k) {
        uint32_t idx = sc.indices[static_cast<size_t>(mesh.first_index) + 3u * prim + k];
        const float* vx = sc.vertices + (static_cast<size_t>(mesh.first_vertex) + idx) * 9;
        uv[0][k] = vx[0];
        uv[1][k] = vx[1];
    }
    float uvx = uv[0][0] * bx + uv[0][1] * by + uv[0][2] * bz;
    float uvy = uv[1][0] * bx + uv[1][1] * by + uv[1][2] * bz;
    float4 c = sc.sample(mat.base_color, uvx, uvy);
    return !(c.w < mat.mask_cutoff);
}

// Ray octant (bit a: idir[a] < 0); slots are visited in increasing (slot ^ oct).
__device__ __forceinline__ uint32_t rayOctant(V3 idir)
{
    return (idir.x < 0.0f ? 1u : 0u) | (idir.y < 0.0f ? 2u : 0u) | (idir.z < 0.0f ? 4u : 0u);
}

// Node group holding only the root: one hit child (k = 0) of a virtual parent with no
// internal-children mask, so nextChild returns the group base (the root) whatever the
// ray octant - a fresh lane can fetch the root before its ray direction is known.
__device__ __forceinline__ uint32_t rootGroupBits() { return 1u; }

// Next child of a non-empty node group; removes it from the group. Group bits:
// 0-7 hit internal children in visiting order (k = slot ^ oct), 8-15 imask (slot
// order). (An "origin inside" set that went first was measured and removed in round 3;
// its bits 16-23 stayed zero and their test ran in every node step until round 5.)
__device__ __forceinline__ uint32_t nextChild(uint32_t base, uint32_t& bits, uint32_t oct)
{
    const uint32_t k = static_cast<uint32_t>(__builtin_ctz(bits & 0xffu));
    const uint32_t slot = k ^ oct;
    bits &= ~(1u << k);
    return base + static_cast<uint32_t>(__builtin_popcount((bits >> 8) & ((1u << slot) - 1u)));
}

// Tests the 8 children of one BVH8 node against [tmin, tmax]. A slab distance is
// one fma of the 8-bit plane index q:  t = q * (step * idir) + (p - o) * idir,
// where step * idir is exact (a power of two) and (p - o) * idir carries at most
// about 2 ulp of |p - o| * |idir| (idir itself within 1 ulp of 1/d, safeInv); the
// build inflates every box by 1e-6 of the
// scene diagonal on top of its own relative margin (bvh_builder.cpp), which
// covers that error, and the comparison keeps a relative margin for far boxes,
// so a box holding an exact triangle hit is never culled. The near/far plane of
// each axis is chosen by the ray octant. Scalar fp32, one slot at a time: a packed
// v_pk_fma_f32 pair issues in two slots on gfx950 and needs moves to pair its
// operands (measured 3.02 vs 2.72 ms traversal at C4 in round 1).
// Returns the hit internal children as a node group and the hit leaf children's
// triangles as a bit mask over [tBase, tBase + 24) (2 VALU: triangle rows).
// Node-visit instruction budget (tools/isa_budget.py). Dual steps of
// k_trace (travStepDual<.., GF = true>) fetch every node from global memory, with both
// sides' loads outside any branch (see travStepDual): its LDS node cache is then not
// allocated (22.3 -> 18.4 KB of LDS per workgroup); C4 step 3.66 / 3.68 -> 3.57 / 3.54
// ms, K = 4096 windows 0.606 -> 0.591 / 0.585 ms, Z-slab proxy P = 8 0.578 -> 0.570 ms
// (profiles/r03_an, r03_ao). k_trace_shadow keeps its top nodes in LDS (GF = false):
// its any-hit rays gain from them (0.704 -> 0.730 ms with global fetches).
constexpr int kShadowLdsNodes = kLdsNodes - 8; // top nodes k_trace_shadow keeps in LDS
// LDS octant permutation table of the node visit (loadNodeCache fills it; every
// kernel that visits nodes calls loadNodeCache first)
__shared__ uint8_t g_octPerm[8 * 256];

// Rejected node-test forms (measured slower, removed in round 5): packed
// fp16 child tests with error bounds or directed rounding (C4 traversal 1.95 -> 20-30
// ms from near-axis-parallel rays), origin-containing children first (+40 VALU per node
// for 0.8 % fewer visits), v_cndmask plane selects and v_max/v_min interval tests.
__device__ __forceinline__ void visitNode8(uint4 w0, uint4 w1, uint4 w2, uint4 w3, uint4 w4, V3 o, V3 idir, uint32_t oct, float tmin,
                                           float tmax, uint32_t& gBase, uint32_t& gBits, uint32_t& tBase, uint32_t& tBits)
{
    // exponent byte e: the step is 2^(e - 127) (e = 0 never occurs for a used axis:
    // the builder's steps are normal numbers); step * idir as one v_ldexp_f32
    const float ax = __builtin_amdgcn_ldexpf(idir.x, static_cast<int>(w0.w & 0xffu) - 127);
    const float ay = __builtin_amdgcn_ldexpf(idir.y, static_cast<int>((w0.w >> 8) & 0xffu) - 127);
    const float az = __builtin_amdgcn_ldexpf(idir.z, static_cast<int>((w0.w >> 16) & 0xffu) - 127);
    const float bx = (__uint_as_float(w0.x) - o.x) * idir.x;
    const float by = (__uint_as_float(w0.y) - o.y) * idir.y;
    const float bz = (__uint_as_float(w0.z) - o.z) * idir.z;
    const uint32_t imask = w0.w >> 24;
    // gfx950 issues v_bitop3_b32 and v_ashrrev_i32 in about half the cycles of a
    // v_cndmask_b32 (tools/probe/valu_table*.hip): the near/far plane words of each axis
    // are selected bitwise under the lane mask of its direction sign (all ones when the
    // component is negative - the octant bit; idir is never -0, safeInv)
    auto signMask = [](float v) { return static_cast<uint32_t>(static_cast<int32_t>(__float_as_uint(v)) >> 31); };
    auto pick = [](uint32_t m, uint32_t a, uint32_t b) {
        uint32_t r;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(m), "v"(a), "v"(b)); // m ? a : b, bitwise
        return r;
    };
    const uint32_t mx = signMask(idir.x), my = signMask(idir.y), mz = signMask(idir.z);
    const uint32_t nX0 = pick(mx, w3.z, w2.x), nX1 = pick(mx, w3.w, w2.y), fX0 = pick(mx, w2.x, w3.z), fX1 = pick(mx, w2.y, w3.w);
    const uint32_t nY0 = pick(my, w4.x, w2.z), nY1 = pick(my, w4.y, w2.w), fY0 = pick(my, w2.z, w4.x), fY1 = pick(my, w2.w, w4.y);
    const uint32_t nZ0 = pick(mz, w4.z, w3.x), nZ1 = pick(mz, w4.w, w3.y), fZ0 = pick(mz, w3.x, w4.z), fZ1 = pick(mz, w3.y, w4.w);
    // max(tn, tmin) <= f(min(tf, tmax)) with the monotone f(x) = fma(x, 1.00001, 1e-7) is
    // tn <= f(tf) && tn <= f(tmax) && tmin <= f(tf) (tmin <= f(tmax) holds for any ray
    // the traversal runs): the same accepted set as the max/min form (no NaN reaches
    // it: A, B and q are finite), three 2-cycle compares instead of two 4-cycle v_max /
    // v_min (tmin is an SGPR operand: every caller passes a wave-uniform constant)
    const float limT = fmaf(tmax, 1.00001f, 1e-7f);
    uint32_t hitSlots = 0;
    // slots 7 .. 0, each compare shifted into the mask as v_addc's carry (m = 2m + hit)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int s = 7 - k;
        const uint32_t sh = static_cast<uint32_t>(s & 3) * 8u;
        const bool hiWord = s >= 4;
        auto q = [&](uint32_t w0_, uint32_t w1_) { return static_cast<float>(((hiWord ? w1_ : w0_) >> sh) & 0xffu); };
        const float tnx = fmaf(q(nX0, nX1), ax, bx), tny = fmaf(q(nY0, nY1), ay, by), tnz = fmaf(q(nZ0, nZ1), az, bz);
        const float tfx = fmaf(q(fX0, fX1), ax, bx), tfy = fmaf(q(fY0, fY1), ay, by), tfz = fmaf(q(fZ0, fZ1), az, bz);
        const float tn = fmaxf(fmaxf(tnx, tny), tnz);
        const float lim = fmaf(fminf(fminf(tfx, tfy), tfz), 1.00001f, 1e-7f);
        uint64_t c0, c1;
        asm("v_cmp_le_f32_e64 %[c0], %[tn], %[lim]\n\t"
            "v_cmp_le_f32_e64 %[c1], %[tn], %[lt]\n\t"
            "s_and_b64 %[c0], %[c0], %[c1]\n\t"
            "v_cmp_le_f32_e64 %[c1], %[tmin], %[lim]\n\t"
            "s_and_b64 vcc, %[c0], %[c1]\n\t"
            "v_addc_co_u32_e32 %[acc], vcc, %[acc], %[acc], vcc"
            : [acc] "+v"(hitSlots), [c0] "=&s"(c0), [c1] "=&s"(c1)
            : [tn] "v"(tn), [lim] "v"(lim), [lt] "v"(limT), [tmin] "s"(tmin)
            : "vcc");
    }
    // internal children: slot bits -> visiting order bits (k = slot ^ oct), one LDS byte
    // (g_octPerm, filled by loadNodeCache) instead of three conditional swap stages
    const uint32_t m = g_octPerm[(oct << 8) | (hitSlots & imask & 0xffu)];
    // leaf children: their triangle rows (GpuBvh8Node: bit s + stride i = triangle
    // i of leaf slot s), the hit leaf slots spread over the three rows and masked
    gBase = w1.x;
    gBits = m | (imask << 8);
    tBase = w1.y;
    const uint32_t stride = w1.w & 31u, leafHits = hitSlots & (w1.w >> 8) & 0xffu;
    const uint32_t x = (leafHits << stride) | leafHits;
    tBits = ((x << stride) | x) & w1.z;
}

__device__ __forceinline__ GpuTriangle triFromWords(uint4 a, uint4 b, uint4 c)
{
    GpuTriangle t;
    t.t0[0] = __uint_as_float(a.x); t.t0[1] = __uint_as_float(a.y); t.t0[2] = __uint_as_float(a.z); t.t0[3] = __uint_as_float(a.w);
    t.t1[0] = __uint_as_float(b.x); t.t1[1] = __uint_as_float(b.y); t.t1[2] = __uint_as_float(b.z); t.t1[3] = __uint_as_float(b.w);
    t.t2[0] = __uint_as_float(c.x); t.t2[1] = __uint_as_float(c.y); t.t2[2] = __uint_as_float(c.z); t.t2[3] = __uint_as_float(c.w);
    return t;
}

// One traversal step of one lane: a pending triangle of the current leaf group is
// tested, otherwise the next child of the current node group is visited (popping
// a group when it is empty). Triangles and nodes are fetched by the same five
// 16-B loads, so a wave whose lanes mix both kinds of step waits for memory
// once per step instead of once per node plus once per triangle.
struct TravState {
    uint32_t gBase, gBits; // node group: hits (k-space) | imask << 8
    uint32_t tBase, tBits; // triangle group
};

template<int BLOCK>
__device__ __forceinline__ bool travDone(const TravState& ts, const Stack<BLOCK>& st)
{
    return ts.tBits == 0 && (ts.gBits & 0xffu) == 0 && st.depth == 0;
}

// A traversal step is split in two so that the fetch can be issued before a
// freshly refilled lane has its ray set up: travFetch picks the work item (a
// pending leaf triangle, else the next child of the current node group, popping
// a group when it is empty) and issues its five 16-B loads; travCompute tests it.
struct Fetch {
    uint4 w0, w1, w2, w3, w4;
    uint32_t i; // triangle index (triangle steps)
    bool isTri;
};

// The first kLdsNodes nodes of the opaque BVH (its top levels: nodes are laid out
// breadth first) copied into LDS once per workgroup: every ray starts there, so
// those fetches skip the vector-memory path.
struct NodeCache {
    const uint4* lds; // [count][5]
    uint32_t base;    // node index of lds[0]
    uint32_t count;
};

template<int BLOCK, int NODES = kLdsNodes>
__device__ __forceinline__ NodeCache loadNodeCache(const SceneArgs& sc, uint4* lds)
{
    NodeCache nc { lds, sc.root_opaque >= 0 ? static_cast<uint32_t>(sc.root_opaque) : 0u, 0u };
    if (sc.root_opaque >= 0) {
        nc.count = min(static_cast<uint32_t>(NODES), sc.opaque_nodes);
        const uint4* src = reinterpret_cast<const uint4*>(sc.nodes + nc.base);
        for (uint32_t i = threadIdx.x; i < nc.count * 5u; i += BLOCK) lds[i] = src[i];
    }
    // octant permutation table of visitNode8: entry (oct << 8 | m) has bit k set iff
    // bit k ^ oct of m is set
    for (uint32_t i = threadIdx.x; i < 8u * 256u; i += BLOCK) {
        const uint32_t oct = i >> 8, m = i & 0xffu;
        uint32_t r = 0;
        for (uint32_t k = 0; k < 8u; ++k) r |= ((m >> (k ^ oct)) & 1u) << k;
        g_octPerm[i] = static_cast<uint8_t>(r);
    }
    __syncthreads();
    return nc;
}

template<int BLOCK>
__device__ __forceinline__ void travFetch(const SceneArgs& sc, const NodeCache& nc, TravState& ts, Stack<BLOCK>& st, uint32_t oct, Fetch& fx)
{
    fx.isTri = ts.tBits != 0;
    const uint4* src;
    if (fx.isTri) {
        fx.i = ts.tBase + static_cast<uint32_t>(__builtin_ctz(ts.tBits));
        ts.tBits &= ts.tBits - 1u;
        src = reinterpret_cast<const uint4*>(sc.tris + fx.i);
    } else {
        if ((ts.gBits & 0xffu) == 0) st.pop(ts.gBase, ts.gBits);
        const uint32_t child = nextChild(ts.gBase, ts.gBits, oct);
        if (ts.gBits & 0xffu) st.push(ts.gBase, ts.gBits);
        src = reinterpret_cast<const uint4*>(sc.nodes + child);
    }
    const uint32_t rel = static_cast<uint32_t>(reinterpret_cast<const GpuBvh8Node*>(src) - sc.nodes) - nc.base;
    if (!fx.isTri && rel < nc.count) {
        const uint4* l = nc.lds + rel * 5u;
        fx.w0 = l[0];
        fx.w1 = l[1];
        fx.w2 = l[2];
        fx.w3 = l[3];
        fx.w4 = l[4];
        return;
    }
    fx.w0 = src[0];
    fx.w1 = src[1];
    fx.w2 = src[2];
    // five loads whatever the step: a triangle step reads 32 B of the next record
    // (the triangle array is padded), no branch around the node's last two loads
    fx.w3 = src[3];
    fx.w4 = src[4];
}

// Returns true when a triangle step produced a candidate (tt, uu, vv, backface
// with the instance's handedness applied, inst, prim) in [tmin, tmax]; node steps
// update the group state and return false.
__device__ __forceinline__ bool travCompute(const Fetch& fx, TravState& ts, V3 o, V3 d, V3 idir, uint32_t oct, float tmin, float tmax, float& tt,
                                            float& uu, float& vv, bool& backface, uint32_t& inst, uint32_t& prim, uint32_t& cNodes, uint32_t& cTris)
{
    if (fx.isTri) {
        cTris++;
        const GpuTriangle tr = triFromWords(fx.w0, fx.w1, fx.w2);
        bool bf;
        if (!intersectTri(o, d, tmin, tmax, tr, &tt, &uu, &vv, &bf)) return false;
        inst = fx.w2.y;
        prim = fx.w2.z;
        backface = bf != (fx.w2.w != 0u); // GpuTriangle t2.w: instance flips facing
        return true;
    }
    cNodes++;
    visitNode8(fx.w0, fx.w1, fx.w2, fx.w3, fx.w4, o, idir, oct, tmin, tmax, ts.gBase, ts.gBits, ts.tBase, ts.tBits);
    return false;
}

// Dual step (k_trace): one lane tests a pending leaf triangle AND visits the next
// node in the same iteration. A divergent wave runs the node and the triangle code
// every iteration anyway (28 % of the steps are triangle steps, spread over its
// lanes), so letting each lane do both roughly turns nodes + triangles iterations
// per ray into max(nodes, triangles) + a short tail. Leaf hits of a node visited
// while the lane's triangle group is still pending wait in a second group (nBase,
// nBits); the node side pauses while that one is full. The closest hit does not
// depend on the order (equal t: smaller (instance, primitive) wins). ANY (shadow
// rays): the step reports a triangle hit in [tmin, h.t] instead of recording it.
template<int BLOCK>
__device__ __forceinline__ bool travDoneDual(const TravState& ts, uint32_t nBits, const Stack<BLOCK>& st)
{
    return ts.tBits == 0 && nBits == 0 && (ts.gBits & 0xffu) == 0 && st.depth == 0;
}

template<int BLOCK, bool ANY, bool GF = false>
__device__ __forceinline__ bool travStepDual(const SceneArgs& sc, const NodeCache& nc, TravState& ts, uint32_t& nBase, uint32_t& nBits, Stack<BLOCK>& st,
                                             V3 o, V3 d, V3 idir, uint32_t oct, float tmin, RayHit& h, int pass, uint32_t& cNodes, uint32_t& cTris)
{
    bool anyHit = false;
    const bool doTri = ts.tBits != 0;
    const bool doNode = nBits == 0 && ((ts.gBits & 0xffu) != 0 || st.depth != 0);
    // fetch registers are left undefined on lanes that skip a side: zero-filling
    // them cost ~34 VALU per iteration (the compiler materialised the zeros)
    uint4 a, b, c;
    uint32_t ti = 0;
    uint4 w0, w1, w2, w3, w4;
    if constexpr (GF) {
    // Both sides' loads are issued by every lane outside any branch (a skipped side
    // reads a resident dummy record: triangle 0, the root node), triangle loads first:
    // the wait before the triangle test then covers only the triangle loads, and the
    // test runs while the node loads are in flight (the branch-local loads of the
    // other form make the compiler wait for both: vmcnt(0)). Nodes come from global
    // memory only (the LDS node cache would make these generic flat loads).
    (void)nc;
    if (doTri) {
        ti = ts.tBase + static_cast<uint32_t>(__builtin_ctz(ts.tBits));
        ts.tBits &= ts.tBits - 1u;
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(sc.tris + ti);
        a = src[0];
        b = src[1];
        c = src[2];
    }
    uint32_t child = static_cast<uint32_t>(sc.root_opaque >= 0 ? sc.root_opaque : 0);
    if (doNode) {
        if ((ts.gBits & 0xffu) == 0) st.pop(ts.gBase, ts.gBits);
        child = nextChild(ts.gBase, ts.gBits, oct);
        if (ts.gBits & 0xffu) st.push(ts.gBase, ts.gBits);
    }
    {
        const uint4* src = reinterpret_cast<const uint4*>(sc.nodes + child);
        w0 = src[0];
        w1 = src[1];
        w2 = src[2];
        w3 = src[3];
        w4 = src[4];
    }
    } else {
    if (doTri) {
        ti = ts.tBase + static_cast<uint32_t>(__builtin_ctz(ts.tBits));
        ts.tBits &= ts.tBits - 1u;
        const uint4* src = reinterpret_cast<const uint4*>(sc.tris + ti);
        a = src[0];
        b = src[1];
        c = src[2];
    }
    if (doNode) {
        if ((ts.gBits & 0xffu) == 0) st.pop(ts.gBase, ts.gBits);
        const uint32_t child = nextChild(ts.gBase, ts.gBits, oct);
        if (ts.gBits & 0xffu) st.push(ts.gBase, ts.gBits);
        const uint32_t rel = child - nc.base;
        const uint4* src = rel < nc.count ? nc.lds + rel * 5u : reinterpret_cast<const uint4*>(sc.nodes + child);
        w0 = src[0];
        w1 = src[1];
        w2 = src[2];
        w3 = src[3];
        w4 = src[4];
    }
    }
    if (doTri) {
        cTris++;
        const GpuTriangle tr = triFromWords(a, b, c);
        bool bf;
        float tt, uu, vv;
        if (intersectTri(o, d, tmin, h.t, tr, &tt, &uu, &vv, &bf)) {
            const uint32_t inst = c.y, prim = c.z;
            if (ANY) anyHit = true;
            else if (!(h.tri != kNoHit && tt == h.t && (inst > h.inst || (inst == h.inst && prim > h.prim))) &&
                !(pass == 1 && !alphaAccept(sc, inst, prim, uu, vv))) {
                h.t = tt;
                h.u = uu;
                h.v = vv;
                h.tri = ti;
                h.inst = inst;
                h.prim = prim;
                h.backface = bf != (c.w != 0u); // GpuTriangle t2.w: instance flips facing
            }
        }
    }
    if (doNode) {
        cNodes++;
        uint32_t lb, lbits;
        visitNode8(w0, w1, w2, w3, w4, o, idir, oct, tmin, h.t, ts.gBase, ts.gBits, lb, lbits);
        if (lbits) {
            if (ts.tBits == 0) {
                ts.tBase = lb;
                ts.tBits = lbits;
            } else {
                nBase = lb;
                nBits = lbits;
            }
        }
    }
    if (ts.tBits == 0 && nBits != 0) {
        ts.tBase = nBase;
        ts.tBits = nBits;
        nBits = 0;
    }
    return anyHit;
}

// ---------------------------------------------------------------------------
// 1b. The sun's shadow rays in light space (SceneArgs::sun_root, ark_ddgi.cpp sunFrame)
// ---------------------------------------------------------------------------
// Light-space coordinates (u, v, w) of a world point: three fp32 dot products (the
// BVH's box inflation covers their rounding, ark_ddgi.cpp).
__device__ __forceinline__ V3 sunCoords(const SceneArgs& sc, V3 p)
{
    const float* F = sc.sun_frame;
    return { fmaf(p.x, F[0], fmaf(p.y, F[1], p.z * F[2])), fmaf(p.x, F[3], fmaf(p.y, F[4], p.z * F[5])), fmaf(p.x, F[6], fmaf(p.y, F[7], p.z * F[8])) };
}

// Bytewise unsigned x >= y of four packed bytes, the result in bit 7 of each byte, from
// xh = x | 0x80808080 and yl = y & 0x7f7f7f7f: d = xh - yl borrows within no byte
// (each byte of xh is >= 0x80 > each of yl), so bit 7 of a byte of d says x_lo7 >= y_lo7;
// with the top bits, x >= y = (x7 & ~y7) | (~(x7 ^ y7) & d7) - one v_bitop3.
__device__ __forceinline__ uint32_t geBytes(uint32_t x, uint32_t y, uint32_t xh, uint32_t yl)
{
    const uint32_t d = xh - yl;
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xb2" : "=v"(r) : "v"(x), "v"(y), "v"(d));
    return r;
}

// Node visit of a ray along +w from light-space point pl (k_trace_shadow<SUN>). With
// the direction exactly +w the slab test of u and v degenerates to "pl's coordinate
// lies in the child's interval" and that of w to "the box reaches above pl": in the
// node's quantized grid, qlo <= floor(Q) and qhi >= ceil(Q) for Q = (pl - anchor) /
// step - no reciprocal, no per-child multiply (the world test: 8 x 19 VALU). The ray's
// tmin is not used (a box between pl and pl + tmin is visited, conservatively). The
// children are visited in slot order: the builder sorted them by their lower w bound
// (Bvh8CollapseOptions::slot_sort_axis), the order the ray meets them.
// The five conditions are tested on four children at once, bytewise within the plane
// words (geBytes), with no lane-mask compares (the per-child form: 40 SDWA v_cmp, 32
// s_and and 8 v_addc). Q is clamped to [0, 255]
// so that floor and ceil are bytes: that can only accept more children (qlo <= 0 for a
// point below the node's anchor, qhi >= 255 above its far side), never fewer, and an
// any-hit result does not depend on extra visits.
__device__ __forceinline__ void visitNodeSun(uint4 w0, uint4 w1, uint4 w2, uint4 w3, uint4 w4, V3 pl, uint32_t& gBase, uint32_t& gBits, uint32_t& tBase,
                                             uint32_t& tBits)
{
    auto quant = [](float c, uint32_t p, uint32_t ebyte) {
        return __builtin_amdgcn_fmed3f(__builtin_amdgcn_ldexpf(c - __uint_as_float(p), 127 - static_cast<int>(ebyte)), 0.0f, 255.0f);
    };
    const float qu = quant(pl.x, w0.x, w0.w & 0xffu), qv = quant(pl.y, w0.y, (w0.w >> 8) & 0xffu), qw = quant(pl.z, w0.z, (w0.w >> 16) & 0xffu);
    constexpr uint32_t kH = 0x80808080u;
    // floor (the truncating conversion: Q >= 0) and ceil of Q, in every byte (v_perm_b32
    // with selector 0: byte 0 of the second operand four times)
    auto bcast = [](float q) { return __builtin_amdgcn_perm(0u, static_cast<uint32_t>(q), 0u); };
    const uint32_t Fu = bcast(qu), Cu = bcast(ceilf(qu)), Fv = bcast(qv), Cv = bcast(ceilf(qv)), Cw = bcast(ceilf(qw));
    const uint32_t FuH = Fu | kH, FvH = Fv | kH, CuL = Cu & ~kH, CvL = Cv & ~kH, CwL = Cw & ~kH;
    // planes (GpuBvh8Node): qlo u = w2.x|y, qlo v = w2.z|w, qhi u = w3.z|w, qhi v = w4.x|y,
    // qhi w = w4.z|w (children 0-3 | 4-7, child k in byte k & 3)
    auto crossed = [&](uint32_t lu, uint32_t hu, uint32_t lv, uint32_t hv, uint32_t hw) {
        return geBytes(Fu, lu, FuH, lu & ~kH) & geBytes(hu, Cu, hu | kH, CuL) & geBytes(Fv, lv, FvH, lv & ~kH) & geBytes(hv, Cv, hv | kH, CvL) &
               geBytes(hw, Cw, hw | kH, CwL) & kH;
    };
    const uint32_t r0 = crossed(w2.x, w3.z, w2.z, w4.x, w4.z), r1 = crossed(w2.y, w3.w, w2.w, w4.y, w4.w);
    // bit 7 of byte k of r0 / r1 -> bit k / k + 4 of the slot mask: the bits of x =
    // (r0 >> 4) | r1 sit at 8k + 3 (child k) and 8k + 7 (child k + 4), and the high word
    // of x * (2^29 + 2^22 + 2^15 + 2^8) holds them at bits k and k + 4 (no two partial
    // products share a bit position, so nothing carries); its bits above 7 are cleared
    // by the 8-bit masks below
    const uint32_t hit = __umulhi((r0 >> 4) | r1, 0x20408100u);
    const uint32_t imask = w0.w >> 24;
    gBase = w1.x;
    gBits = (hit & imask) | (imask << 8);
    tBase = w1.y;
    const uint32_t stride = w1.w & 31u, leafHits = hit & (w1.w >> 8) & 0xffu;
    const uint32_t xl = (leafHits << stride) | leafHits;
    tBits = ((xl << stride) | xl) & w1.z;
}

// travStepDual for a sun shadow ray in the light-space BVH: both sides' loads issued
// by every lane (a skipped side reads the resident record 0 / the root), the
// world-space Möller–Trumbore of the leaf records (the any-hit test of the world
// BVHs, bit for bit), the light-space node test.
template<int BLOCK>
__device__ __forceinline__ bool travStepSun(const SceneArgs& sc, TravState& ts, uint32_t& nBase, uint32_t& nBits, Stack<BLOCK>& st, V3 o, V3 d, V3 pl,
                                            float tmin, float tmax, uint32_t& cNodes, uint32_t& cTris)
{
    bool anyHit = false;
    const bool doTri = ts.tBits != 0;
    const bool doNode = nBits == 0 && ((ts.gBits & 0xffu) != 0 || st.depth != 0);
    uint32_t ti = 0;
    if (doTri) {
        ti = ts.tBase + static_cast<uint32_t>(__builtin_ctz(ts.tBits));
        ts.tBits &= ts.tBits - 1u;
    }
    uint4 a, b, c;
    {
        const uint4* src = reinterpret_cast<const uint4*>(sc.sun_tris + ti);
        a = src[0];
        b = src[1];
        c = src[2];
    }
    uint32_t child = static_cast<uint32_t>(sc.sun_root);
    if (doNode) {
        if ((ts.gBits & 0xffu) == 0) st.pop(ts.gBase, ts.gBits);
        child = nextChild(ts.gBase, ts.gBits, 0u);
        if (ts.gBits & 0xffu) st.push(ts.gBase, ts.gBits);
    }
    uint4 w0, w1, w2, w3, w4;
    {
        const uint4* src = reinterpret_cast<const uint4*>(sc.sun_nodes + child);
        w0 = src[0];
        w1 = src[1];
        w2 = src[2];
        w3 = src[3];
        w4 = src[4];
    }
    if (doTri) {
        cTris++;
        const GpuTriangle tr = triFromWords(a, b, c);
        bool bf;
        float tt, uu, vv;
        anyHit = intersectTri(o, d, tmin, tmax, tr, &tt, &uu, &vv, &bf);
    }
    if (doNode) {
        cNodes++;
        uint32_t lb, lbits;
        visitNodeSun(w0, w1, w2, w3, w4, pl, ts.gBase, ts.gBits, lb, lbits);
        if (lbits) {
            if (ts.tBits == 0) {
                ts.tBase = lb;
                ts.tBits = lbits;
            } else {
                nBase = lb;
                nBits = lbits;
            }
        }
    }
    if (ts.tBits == 0 && nBits != 0) {
        ts.tBase = nBase;
        ts.tBits = nBits;
        nBits = 0;
    }
    return anyHit;
}

// opaque.rchit:118-131: world-space shading normal of a front hit. The trace
// kernel's shadow phase and the shading kernel both evaluate exactly this
// expression, so they agree on N (and on which lights need a shadow ray).
// hitShadingNormal from the triangle's shading record (a, b, c: n0 n1 n2) and its
// instance's normal matrix rows (m0, m1, m2), already read
__device__ __forceinline__ V3 shadingNormalOf(float4 a, float4 b, float4 c, float4 m0, float4 m1, float4 m2, float hu, float hv)
{
    const float bx = 1.0f - hu - hv, by = hu, bz = hv;
    // same operation sequence as k_shade (opaque.rchit:118-131)
    V3 N = normalize(v3(a.x, a.y, a.z) * bx + v3(a.w, b.x, b.y) * by + v3(b.z, b.w, c.x) * bz);
    V3 Nw = { m0.x * N.x + m0.y * N.y + m0.z * N.z, m1.x * N.x + m1.y * N.y + m1.z * N.z, m2.x * N.x + m2.y * N.y + m2.z * N.z };
    return normalize(Nw);
}

__device__ __forceinline__ V3 hitShadingNormal(const SceneArgs& sc, uint32_t tri, float hu, float hv)
{
    const float4* tn = sc.tri_normals + 4u * static_cast<size_t>(tri);
    const float4 a = tn[0], b = tn[1], c = tn[2];
    const uint32_t inst = __float_as_uint(c.y);
    const float* M = sc.instances[inst].normal_matrix;
    const float bx = 1.0f - hu - hv, by = hu, bz = hv;
    // same operation sequence as k_shade (opaque.rchit:118-131) and shadingNormalOf
    V3 N = normalize(v3(a.x, a.y, a.z) * bx + v3(a.w, b.x, b.y) * by + v3(b.z, b.w, c.x) * bz);
    V3 Nw = { M[0] * N.x + M[1] * N.y + M[2] * N.z, M[4] * N.x + M[5] * N.y + M[6] * N.z, M[8] * N.x + M[9] * N.y + M[10] * N.z };
    return normalize(Nw);
}

// opaque.rchit:56-103: lights with LdotN > 0 (bit l: sun first, then spots in order)
__device__ __forceinline__ uint32_t litLightMask(const SceneArgs& sc, V3 N)
{
    uint32_t need = 0, l = 0;
    if (sc.has_sun) {
        const V3 Ld = -normalize(v3(sc.sun_dir[0], sc.sun_dir[1], sc.sun_dir[2]));
        if (dot(Ld, N) > 0.0f) need |= 1u;
        l++;
    }
    for (int li = 0; li < sc.spot_count; ++li, ++l) {
        const V3 Ld = -normalize(v3(sc.spots[li].direction[0], sc.spots[li].direction[1], sc.spots[li].direction[2]));
        if (dot(Ld, N) > 0.0f) need |= 1u << l;
    }
    return need;
}

// Shadow ray of light l from hit point X (opaque.rchit:35-54 + :56-103): sun toward
// -sunDirection with tmax 2 zFar, spot toward its position with tmax distance - 0.001.
__device__ __forceinline__ void shadowRayOf(const SceneArgs& sc, float zFar, uint32_t l, V3 X, V3* dir, float* tmax)
{
    if (sc.has_sun && l == 0) {
        *dir = -normalize(v3(sc.sun_dir[0], sc.sun_dir[1], sc.sun_dir[2]));
        *tmax = 2.0f * zFar;
        return;
    }
    const GpuSpotLight& sl = sc.spots[l - (sc.has_sun ? 1u : 0u)];
    const V3 toLight = v3(sl.position[0], sl.position[1], sl.position[2]) - X;
    const float distanceToLight = length(toLight);
    *dir = toLight / distanceToLight;
    *tmax = distanceToLight - 0.001f;
}

// ---------------------------------------------------------------------------
// 2. traversal work distribution
// ---------------------------------------------------------------------------
// XCD-aware work split: the window's probes are cut into kRayParts contiguous
// partitions with one head counter each (ray_counter[p * kRayCounterStride]).
// A wave drains the partition of the XCD it runs on first (read from
// HW_REG_XCC_ID), then steals from the others in order. Rays of neighbouring
// probes touch the same BVH neighbourhood, so each XCD's L2 sees ~1/8 of the
// in-flight working set. Placement only affects speed: every ray is taken
// exactly once whichever wave takes it.
__device__ __forceinline__ uint32_t xccId()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & (kRayParts - 1);
}

// Same partitioned dequeue over a flat list of `total` items (shadow rays).
__device__ __forceinline__ void grabItems(uint32_t* heads, uint32_t total, uint32_t home, uint32_t& tried, uint32_t& b, uint32_t& e, uint32_t CHUNK)
{
    b = e = 0;
    for (; tried < kRayParts; ++tried) {
        const uint32_t p = (home + tried) & (kRayParts - 1);
        const uint32_t pb = static_cast<uint32_t>(static_cast<uint64_t>(total) * p / kRayParts);
        const uint32_t pe = static_cast<uint32_t>(static_cast<uint64_t>(total) * (p + 1) / kRayParts);
        if (pb >= pe) continue;
        const uint32_t off = atomicAdd(heads + p * kRayCounterStride, CHUNK);
        if (off < pe - pb) {
            b = pb + off;
            e = min(b + CHUNK, pe);
            return;
        }
    }
}

__device__ __forceinline__ uint32_t partRayBegin(const FrameArgs& f, uint32_t p)
{
    return static_cast<uint32_t>(static_cast<uint64_t>(f.window_probes) * p / kRayParts) * f.R;
}

// One lane only: next chunk of at most CHUNK consecutive rays from the head
// counters at `heads`, or b >= e when every partition is drained.
// `tried` = partitions already found empty (uniform over the caller's group).
__device__ __forceinline__ void grabRays(const FrameArgs& f, uint32_t* heads, uint32_t home, uint32_t& tried, uint32_t& b, uint32_t& e, uint32_t CHUNK)
{
    b = e = 0;
    for (; tried < kRayParts; ++tried) {
        const uint32_t p = (home + tried) & (kRayParts - 1);
        const uint32_t pb = partRayBegin(f, p), pe = partRayBegin(f, p + 1);
        if (pb >= pe) continue;
        const uint32_t off = atomicAdd(heads + p * kRayCounterStride, CHUNK);
        if (off < pe - pb) {
            b = pb + off;
            e = min(b + CHUNK, pe);
            return;
        }
    }
}

// ---------------------------------------------------------------------------
// 2b. k_trace: probe-ray traversal (persistent, per-lane wave64 ballot refill)
// ---------------------------------------------------------------------------
// Every lane owns one probe ray at a time (pass 0 opaque, 1 masked). One outer
// iteration visits one BVH8 node or one leaf triangle per active lane; lanes whose
// ray finished are refilled at the top of the next iteration from a wave-private
// pool of consecutive ray indices (ballot + mbcnt rank, one atomic per 64 rays), so
// the SIMD stays full until the global ray counter runs out.

// Ray sources of the closest-hit traversal. ProbeRays: the window's probe rays from
// the slot table (raygen.rgen:35-92: opaque pass then masked pass, tmin 1e-4, tmax
// zFar), partitions of whole probes. ListRays: a ray list of {origin, tmax},
// {direction, id} (rt-reflections/raygen.rgen:111-119: RayFlags_Opaque, cullMask
// 0x01, tmin 0.01), f.list_count entries, the hit record at the list index.
struct ProbeRays {
    static constexpr bool kMaskedPass = true;
    static constexpr float kTmin = 0.0001f;
    __device__ static void grab(const FrameArgs& f, uint32_t home, uint32_t& tried, uint32_t& b, uint32_t& e)
    {
        grabRays(f, f.ray_counter, home, tried, b, e, f.grab_chunk);
    }
    __device__ static void load(const FrameArgs& f, uint32_t r, uint32_t& ray, V3& o, V3& d, float& tmax)
    {
        const uint32_t qp = r / f.R;
        const uint32_t slot = slotAt(f, qp);
        const float4 fv = f.fib_order[r - qp * f.R]; // (direction, sample index)
        const GpuProbeSlot ps = f.slots[slot];
        ray = slot * f.R + __float_as_uint(fv.w); // hit record index
        o = { ps.pos[0], ps.pos[1], ps.pos[2] };
        d = rotate(v3(fv.x, fv.y, fv.z), v3(ps.axis[0], ps.axis[1], ps.axis[2]), ps.angle_sin, ps.angle_cos);
        tmax = f.z_far;
    }
};

struct ListRays {
    static constexpr bool kMaskedPass = false;
    static constexpr float kTmin = 0.01f;
    __device__ static void grab(const FrameArgs& f, uint32_t home, uint32_t& tried, uint32_t& b, uint32_t& e)
    {
        grabItems(f.ray_counter, *f.list_count, home, tried, b, e, f.grab_chunk);
    }
    __device__ static void load(const FrameArgs& f, uint32_t r, uint32_t& ray, V3& o, V3& d, float& tmax)
    {
        const float4 a = f.ray_list[2u * r], b = f.ray_list[2u * r + 1u];
        ray = r;
        o = { a.x, a.y, a.z };
        tmax = a.w;
        d = { b.x, b.y, b.z };
    }
};

template<bool COUNT, int WPE, class Src = ProbeRays>
__global__ void __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(WPE))) k_trace(SceneArgs sc, FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    __shared__ uint32_t ldsStack[kStackLds * 2 * kTraceBlock];
    // nodes from global memory only (GF dual steps): no LDS node cache, the octant table
    __shared__ uint4 ldsNodes[5];
    const NodeCache nc = loadNodeCache<kTraceBlock, 0>(sc, ldsNodes);
    const uint32_t gtid = blockIdx.x * kTraceBlock + threadIdx.x;
    const uint32_t nthreads = gridDim.x * kTraceBlock;
    Stack<kTraceBlock> st { ldsStack + threadIdx.x, f.spill + gtid, nthreads, 0 };
    const uint32_t lane = threadIdx.x & 63u;
    const float tmin = Src::kTmin;
    uint32_t cNodes = 0, cTris = 0, cHits = 0, cIter = 0, rSteps = 0;

    uint32_t poolNext = 0, poolEnd = 0;
    const uint32_t home = xccId();
    uint32_t tried = 0; // partitions found drained (wave-uniform)
    bool exhausted = false;
    bool active = false;
    uint32_t ray = 0;
    int pass = 0; // 0 opaque, 1 masked
    TravState ts { 0u, 0u, 0u, 0u };
    uint32_t nBase = 0, nBits = 0; // the next triangle group (dual step)
    uint32_t oct = 0;
    V3 o = { 0, 0, 0 }, d = { 0, 0, 1 }, idir = { 0, 0, 1 };
    RayHit h { 0.0f, 0.0f, 0.0f, kNoHit, 0u, 0u, false };
    float opaqueT = 0.0f; // signed t of the opaque hit, kept for the masked pass
    auto done = [&]() { return travDoneDual(ts, nBits, st); };
    // Deferred retirement: without a masked pass to continue into, a lane whose ray is
    // done only goes idle, and its hit record is written at the next refill, just
    // before the lane takes a new ray. A lane finishes a ray in nearly every step of a
    // wave (one ray per lane every ~25 steps), so the exec-masked store path would
    // otherwise run almost every step; at a refill it runs once per batch of idle
    // lanes. Lanes that finish after the ray supply is exhausted retire at once.
    bool pending = false;
    auto storeHit = [&]() {
        GpuHit out;
        if (h.tri == kNoHit) {
            out.t = __builtin_bit_cast(float, 0x7f800000u);
            out.u = out.v = 0.0f;
            out.tri = kNoHit;
        } else {
            out.t = h.backface ? -h.t : h.t;
            out.u = h.u;
            out.v = h.v;
            out.tri = h.tri;
            if (COUNT) cHits++;
        }
        f.hits[ray] = out;
        if (COUNT && f.ray_steps) f.ray_steps[ray] = static_cast<uint16_t>(min(rSteps, 65535u));
        if (COUNT) rSteps = 0;
    };

    for (;;) {
        // ---- refill finished lanes --------------------------------------------
        const uint64_t need = __ballot(!active);
        if (need != 0 && !exhausted && (static_cast<uint32_t>(__popcll(need)) >= f.refill_min || need == ~0ull)) {
            if (pending) {
                storeHit();
                pending = false;
            }
            const uint32_t n = static_cast<uint32_t>(__popcll(need));
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(need >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(need), 0u));
            const uint32_t avail = poolEnd - poolNext;
            uint32_t fb = 0, fe = 0; // fresh chunk [fb, fe)
            if (avail < n) {
                uint32_t b = 0, e = 0, t = tried;
                if (lane == 0) Src::grab(f, home, t, b, e);
                fb = __shfl(b, 0);
                fe = __shfl(e, 0);
                tried = __shfl(t, 0);
            }
            if (!active) {
                uint32_t r = kNoHit;
                if (rank < avail) r = poolNext + rank;
                else if (fb + (rank - avail) < fe) r = fb + (rank - avail);
                if (r != kNoHit) {
                    float tmax;
                    Src::load(f, r, ray, o, d, tmax);
                    idir = safeInv(d);
                    oct = rayOctant(idir);
                    active = true;
                    h = RayHit { tmax, 0.0f, 0.0f, kNoHit, 0u, 0u, false };
                    pass = 0;
                    st.depth = 0;
                    nBits = 0;
                    ts = TravState { static_cast<uint32_t>(sc.root_opaque), sc.root_opaque >= 0 ? rootGroupBits() : 0u, 0u, 0u };
                }
            }
            if (avail < n) {
                if (fb >= fe) {
                    exhausted = true;
                    poolNext = poolEnd = 0;
                } else {
                    poolNext = min(fb + (n - avail), fe);
                    poolEnd = fe;
                }
            } else {
                poolNext += n;
            }
        }
        if (__ballot(active) == 0) break;
        if (COUNT) {
            cIter++;
            rSteps += active ? 1u : 0u;
        }
        // ---- one step: a pending leaf triangle and the next node -------------------
        // (an active lane is never done here: the check after the step retires or
        // restarts it, and a step of a done lane would change nothing anyway)
        if (active) travStepDual<kTraceBlock, false, true>(sc, nc, ts, nBase, nBits, st, o, d, idir, oct, tmin, h, pass, cNodes, cTris);
        // ---- pass finished -------------------------------------------------------------
        if (active && done() && (!Src::kMaskedPass || sc.root_masked < 0) && !exhausted) {
            active = false;
            pending = true;
        } else if (active && done()) {
            bool finished = true;
            if (Src::kMaskedPass && pass == 0) {
                // opaque pass done (raygen.rgen:35-62); masked pass: RayFlags_NoOpaque,
                // cullMask 0x02, tmax = previous hit T (:64-92); a negative tmax
                // (backface) is an empty interval.
                opaqueT = (h.tri != kNoHit) ? (h.backface ? -h.t : h.t) : f.z_far;
                if (sc.root_masked >= 0 && opaqueT >= tmin) {
                    pass = 1;
                    finished = false;
                    ts = TravState { static_cast<uint32_t>(sc.root_masked), rootGroupBits(), 0u, 0u };
                    st.depth = 0;
                    // stash the opaque hit; the masked pass searches [tmin, opaqueT]
                    f.hits[ray] = GpuHit { h.tri == kNoHit ? __builtin_bit_cast(float, 0x7f800000u) : opaqueT, h.u, h.v, h.tri };
                    h = RayHit { opaqueT, 0.0f, 0.0f, kNoHit, 0u, 0u, false };
                }
            }
            if (finished) {
                GpuHit out;
                if (pass == 1 && h.tri == kNoHit) {
                    // masked pass found nothing: the opaque result (already stored) stands
                    out = f.hits[ray];
                    if (COUNT && out.tri != kNoHit) cHits++;
                    if (COUNT && f.ray_steps) f.ray_steps[ray] = static_cast<uint16_t>(min(rSteps, 65535u));
                    if (COUNT) rSteps = 0;
                } else {
                    storeHit();
                }
                active = false;
            }
        }
    }
    if (COUNT) {
        atomicAdd(&f.counters[0], static_cast<unsigned long long>(cNodes));
        atomicAdd(&f.counters[1], static_cast<unsigned long long>(cTris));
        atomicAdd(&f.counters[2], static_cast<unsigned long long>(cHits));
        if (lane == 0) atomicAdd(&f.counters[7], static_cast<unsigned long long>(cIter));
    }
}

// ---------------------------------------------------------------------------
// 3. shading helpers
// ---------------------------------------------------------------------------
// probeSampling.glsl:9-27
__device__ __forceinline__ void atlasSampleUV(const FrameArgs& f, int px, int py, int pz, V3 dir, int res, float invW, float invH, float* u, float* v)
{
    const int pad = ARK_DDGI_ATLAS_PADDING;
    int tileX = px + py * f.X, tileY = pz;
    int firstX = pad + tileX * (res + 2 * pad), firstY = pad + tileY * (res + 2 * pad);
    float ex, ey;
    octahedralEncode(dir, &ex, &ey);
    float tx = (ex * 0.5f + 0.5f) * static_cast<float>(res);
    float ty = (ey * 0.5f + 0.5f) * static_cast<float>(res);
    float ax = static_cast<float>(firstX) + tx, ay = static_cast<float>(firstY) + ty;
    *u = ax * invW;
    *v = ay * invH;
}

// Linear filter, clamp to edge, over an fp16 atlas (DDGINode.cpp:274).
template<int CH, int NOUT>
__device__ __forceinline__ void sampleAtlas(const uint16_t* __restrict__ atlas, int W, int H, float u, float v, float* out)
{
    float x = u * static_cast<float>(W) - 0.5f;
    float y = v * static_cast<float>(H) - 0.5f;
    float x0f = floorf_(x), y0f = floorf_(y);
    float fx = x - x0f, fy = y - y0f;
    int x0 = static_cast<int>(x0f), y0 = static_cast<int>(y0f);
    int xa = min(max(x0, 0), W - 1), xb = min(max(x0 + 1, 0), W - 1);
    int ya = min(max(y0, 0), H - 1), yb = min(max(y0 + 1, 0), H - 1);
    uint16_t q[4][CH];
    // one load per texel row when the two texels are adjacent (xb = xa + 1, i.e. not
    // clamped at the atlas edge): 16 B for RGBA16F, 8 B for RG16F, at the texel's
    // own (8 B / 4 B) alignment - the device handles the misaligned wide load
    // (tools/probe/unaligned_load.hip)
    auto loadRow = [&](int k, int yy) {
        const uint16_t* pa = atlas + (static_cast<size_t>(yy) * W + xa) * CH;
        const uint16_t* pb = atlas + (static_cast<size_t>(yy) * W + xb) * CH;
        if (CH == 4) {
            uint2 wa, wb;
            if (xb == xa + 1) {
                const uint4 w = *reinterpret_cast<const uint4*>(pa);
                wa = make_uint2(w.x, w.y);
                wb = make_uint2(w.z, w.w);
            } else {
                wa = *reinterpret_cast<const uint2*>(pa);
                wb = *reinterpret_cast<const uint2*>(pb);
            }
            q[k][0] = static_cast<uint16_t>(wa.x & 0xffffu);
            q[k][1] = static_cast<uint16_t>(wa.x >> 16);
            q[k][2 % CH] = static_cast<uint16_t>(wa.y & 0xffffu);
            q[k][3 % CH] = static_cast<uint16_t>(wa.y >> 16);
            q[k + 1][0] = static_cast<uint16_t>(wb.x & 0xffffu);
            q[k + 1][1] = static_cast<uint16_t>(wb.x >> 16);
            q[k + 1][2 % CH] = static_cast<uint16_t>(wb.y & 0xffffu);
            q[k + 1][3 % CH] = static_cast<uint16_t>(wb.y >> 16);
        } else {
            uint32_t wa, wb;
            if (xb == xa + 1) {
                const uint2 w = *reinterpret_cast<const uint2*>(pa);
                wa = w.x;
                wb = w.y;
            } else {
                wa = *reinterpret_cast<const uint32_t*>(pa);
                wb = *reinterpret_cast<const uint32_t*>(pb);
            }
            q[k][0] = static_cast<uint16_t>(wa & 0xffffu);
            q[k][1] = static_cast<uint16_t>(wa >> 16);
            q[k + 1][0] = static_cast<uint16_t>(wb & 0xffffu);
            q[k + 1][1] = static_cast<uint16_t>(wb >> 16);
        }
    };
    loadRow(0, ya); // q[0] = (xa, ya), q[1] = (xb, ya)
    loadRow(2, yb); // q[2] = (xa, yb), q[3] = (xb, yb)
    for (int c = 0; c < NOUT; ++c) {
        float t00 = f16_to_f32(q[0][c]), t10 = f16_to_f32(q[1][c]);
        float t01 = f16_to_f32(q[2][c]), t11 = f16_to_f32(q[3][c]);
        out[c] = lerpf(lerpf(t00, t10, fx), lerpf(t01, t11, fx), fy);
    }
}

// One bilinear tap of an fp16 atlas, split into fetch and filter so that the taps of
// several probes can be in flight at once. The two texels (xa, xb) of a row come
// from one wide load at texel m = min(xa, W - 2) (xb is xa or xa + 1, both in
// {m, m + 1}); `sel` says which half each one is. Same texels, weights and lerps as
// sampleAtlas.
template<int CH>
struct AtlasTap {
    using Row = typename std::conditional<CH == 4, uint4, uint2>::type;
    Row r0, r1; // rows ya, yb: texels (m, m + 1)
    float fx, fy;
    uint32_t sel; // bit 0: texel a is m + 1, bit 1: texel b is m + 1
};

template<int CH>
__device__ __forceinline__ AtlasTap<CH> atlasTap(const uint16_t* __restrict__ atlas, int W, int H, float u, float v)
{
    using Row = typename AtlasTap<CH>::Row;
    AtlasTap<CH> t;
    float x = u * static_cast<float>(W) - 0.5f;
    float y = v * static_cast<float>(H) - 0.5f;
    float x0f = floorf_(x), y0f = floorf_(y);
    t.fx = x - x0f;
    t.fy = y - y0f;
    int x0 = static_cast<int>(x0f), y0 = static_cast<int>(y0f);
    int xa = min(max(x0, 0), W - 1), xb = min(max(x0 + 1, 0), W - 1);
    int ya = min(max(y0, 0), H - 1), yb = min(max(y0 + 1, 0), H - 1);
    const int m = min(xa, W - 2);
    t.sel = (xa != m ? 1u : 0u) | (xb != m ? 2u : 0u);
    t.r0 = *reinterpret_cast<const Row*>(atlas + (static_cast<size_t>(ya) * W + m) * CH);
    t.r1 = *reinterpret_cast<const Row*>(atlas + (static_cast<size_t>(yb) * W + m) * CH);
    return t;
}

template<int CH, int NOUT>
__device__ __forceinline__ void atlasFilter(const AtlasTap<CH>& t, float* out)
{
    uint16_t q[4][CH];
    auto split = [&](int k, const typename AtlasTap<CH>::Row& r) {
        if constexpr (CH == 4) {
            const uint2 lo = make_uint2(r.x, r.y), hi = make_uint2(r.z, r.w);
            const uint2 wa = (t.sel & 1u) ? hi : lo, wb = (t.sel & 2u) ? hi : lo;
            q[k][0] = static_cast<uint16_t>(wa.x & 0xffffu);
            q[k][1] = static_cast<uint16_t>(wa.x >> 16);
            q[k][2] = static_cast<uint16_t>(wa.y & 0xffffu);
            q[k][3] = static_cast<uint16_t>(wa.y >> 16);
            q[k + 1][0] = static_cast<uint16_t>(wb.x & 0xffffu);
            q[k + 1][1] = static_cast<uint16_t>(wb.x >> 16);
            q[k + 1][2] = static_cast<uint16_t>(wb.y & 0xffffu);
            q[k + 1][3] = static_cast<uint16_t>(wb.y >> 16);
        } else {
            const uint32_t wa = (t.sel & 1u) ? r.y : r.x, wb = (t.sel & 2u) ? r.y : r.x;
            q[k][0] = static_cast<uint16_t>(wa & 0xffffu);
            q[k][1] = static_cast<uint16_t>(wa >> 16);
            q[k + 1][0] = static_cast<uint16_t>(wb & 0xffffu);
            q[k + 1][1] = static_cast<uint16_t>(wb >> 16);
        }
    };
    split(0, t.r0); // q[0] = (xa, ya), q[1] = (xb, ya)
    split(2, t.r1); // q[2] = (xa, yb), q[3] = (xb, yb)
    for (int c = 0; c < NOUT; ++c) {
        float t00 = f16_to_f32(q[0][c]), t10 = f16_to_f32(q[1][c]);
        float t01 = f16_to_f32(q[2][c]), t11 = f16_to_f32(q[3][c]);
        out[c] = lerpf(lerpf(t00, t10, t.fx), lerpf(t01, t11, t.fx), t.fy);
    }
}

// probeSampling.glsl:64-163. The 8 cage probes in groups of GB whose visibility and
// irradiance taps are issued together before their weights are formed; every weight
// and sum is the same IEEE sequence as the per-probe loop, and the irradiance sums run
// in probe order. GB = 1 (kGatherBatch): 2 and 4 measured no faster on C4.
constexpr int kGatherBatch = 1;
template<int GB>
__device__ V3 sampleDDGI(const FrameArgs& f, V3 P, V3 N, V3 Vw)
{
    const V3 spacing = v3(f.spacing[0], f.spacing[1], f.spacing[2]);
    const V3 origin = v3(f.origin[0], f.origin[1], f.origin[2]);
    V3 rel = (P - origin) / spacing;
    int bx = min(max(static_cast<int>(rel.x), 0), f.X - 1);
    int by = min(max(static_cast<int>(rel.y), 0), f.Y - 1);
    int bz = min(max(static_cast<int>(rel.z), 0), f.Z - 1);
    V3 baseProbePos = origin + v3(static_cast<float>(bx), static_cast<float>(by), static_cast<float>(bz)) * spacing;
    V3 sumIrradiance = splat(0.0f);
    float sumWeight = 0.0f;
    V3 al = (P - baseProbePos) / spacing;
    V3 alpha = { clampf(al.x, 0.0f, 1.0f), clampf(al.y, 0.0f, 1.0f), clampf(al.z, 0.0f, 1.0f) };
    const float invWi = 1.0f / static_cast<float>(f.Wi), invHi = 1.0f / static_cast<float>(f.Hi);
    const float invWv = 1.0f / static_cast<float>(f.Wv), invHv = 1.0f / static_cast<float>(f.Hv);
    const float minDistanceBetweenProbes = fminf_(spacing.x, fminf_(spacing.y, spacing.z));
    const V3 nN = normalize(N);
    const float tunableShadowBias = 0.3f;
    const V3 selfShadowBias = (N * 0.2f + Vw * 0.8f) * (0.75f * minDistanceBetweenProbes) * tunableShadowBias;
    const V3 biasedPosition = P + selfShadowBias;
    auto probeOf = [&](int i, int& px, int& py, int& pz) {
        px = min(max(bx + (i & 1), 0), f.X - 1);
        py = min(max(by + ((i >> 1) & 1), 0), f.Y - 1);
        pz = min(max(bz + ((i >> 2) & 1), 0), f.Z - 1);
    };
    auto probePosOf = [&](int px, int py, int pz) {
        return origin + v3(static_cast<float>(px), static_cast<float>(py), static_cast<float>(pz)) * spacing;
    };
    // --- 4 probes at a time: visibility and irradiance taps issued together, then
    // the weights, then the sums in probe order -----------------------------------
#pragma unroll
    for (int h = 0; h < 8; h += GB) {
        AtlasTap<2> vt[GB];
        AtlasTap<4> it[GB];
#pragma unroll
        for (int j = 0; j < GB; ++j) {
            int px, py, pz;
            probeOf(h + j, px, py, pz);
            const V3 directionToProbe = normalize(probePosOf(px, py, pz) - biasedPosition);
            float u, v;
            atlasSampleUV(f, px, py, pz, -directionToProbe, ARK_DDGI_VISIBILITY_RES, invWv, invHv, &u, &v);
            vt[j] = atlasTap<2>(f.vis, f.Wv, f.Hv, u, v);
            atlasSampleUV(f, px, py, pz, nN, ARK_DDGI_IRRADIANCE_RES, invWi, invHi, &u, &v);
            it[j] = atlasTap<4>(f.irr, f.Wi, f.Hi, u, v);
        }
#pragma unroll
        for (int j = 0; j < GB; ++j) {
            const int i = h + j;
            int px, py, pz;
            probeOf(i, px, py, pz);
            const int ox = i & 1, oy = (i >> 1) & 1, oz = (i >> 2) & 1;
            V3 tri = { fmaxf_(0.001f, mixf(1.0f - alpha.x, alpha.x, static_cast<float>(ox))),
                       fmaxf_(0.001f, mixf(1.0f - alpha.y, alpha.y, static_cast<float>(oy))),
                       fmaxf_(0.001f, mixf(1.0f - alpha.z, alpha.z, static_cast<float>(oz))) };
            float trilinearWeight = tri.x * tri.y * tri.z;
            float weight = 1.0f;
            const V3 probePos = probePosOf(px, py, pz);
            const V3 pointToProbe = probePos - biasedPosition;
            V3 unbiasedDirectionToProbe = normalize(probePos - P);
            const float smoothFloor = 0.02f, additionalSmoothening = 0.25f;
            weight *= smoothFloor + (1.0f - smoothFloor) * powf_(saturate(dot(unbiasedDirectionToProbe, N)), additionalSmoothening);
            {
                float vis[2];
                atlasFilter<2, 2>(vt[j], vis);
                float meanDistanceToOccluder = vis[0];
                float variance = fabsf_(vis[1] - square(vis[0]));
                float distToProbe = length(pointToProbe);
                float chebychevWeight = 1.0f;
                if (distToProbe > meanDistanceToOccluder) {
                    chebychevWeight = variance / (variance + square(distToProbe - meanDistanceToOccluder));
                    chebychevWeight = chebychevWeight * chebychevWeight * chebychevWeight;
                }
                chebychevWeight = fmaxf_(0.05f, chebychevWeight);
                weight *= chebychevWeight;
            }
            weight = fmaxf_(0.000001f, weight);
            const float crushThreshold = 0.2f;
            if (weight < crushThreshold) weight *= square(weight) * (1.0f / square(crushThreshold));
            weight *= trilinearWeight;
            float irr[3];
            atlasFilter<4, 3>(it[j], irr);
            V3 probeIrradiance = pow3(v3(irr[0], irr[1], irr[2]), 5.0f * 0.5f);
            sumIrradiance = sumIrradiance + weight * probeIrradiance;
            sumWeight += weight;
        }
    }
    V3 irradiance = sumIrradiance / sumWeight;
    irradiance = irradiance * irradiance;
    irradiance = irradiance * (0.5f * kPi);
    return irradiance;
}


// ---------------------------------------------------------------------------
// 3. shading
// ---------------------------------------------------------------------------
// k_shade takes chunks of kShadeChunk consecutive probe rays. Misses and backface
// hits are finished in a classify pass; front hits are compacted into an LDS list
// and shaded densely (material, textures, BRDF per lit light, DDGI indirect). The
// shadow rays were traced before (k_shadow_gen + k_trace_shadow), and their per-ray light bits say
// which lit lights are occluded: base (+ T or Z per lit light, in light order) +
// indirect, the IEEE sequence of the single-pass closest-hit shader
// (opaque.rchit:105-176 with traceShadowRay's shadowFactor 1 or 0).
__device__ __forceinline__ void storeSurfel(const FrameArgs& f, uint32_t ray, V3 color, float dist)
{
    const uint32_t slot = ray / f.R, sample = ray - slot * f.R;
    uint2 packed;
    packed.x = static_cast<uint32_t>(f32_to_f16(color.x)) | (static_cast<uint32_t>(f32_to_f16(color.y)) << 16);
    packed.y = static_cast<uint32_t>(f32_to_f16(color.z)) | (static_cast<uint32_t>(f32_to_f16(dist)) << 16);
    reinterpret_cast<uint2*>(f.surfels)[static_cast<size_t>(slot) * f.Rmax + sample] = packed;
}

__device__ __forceinline__ void rayOf(const FrameArgs& f, uint32_t ray, V3* origin, V3* dir)
{
    const uint32_t slot = ray / f.R, sample = ray - slot * f.R;
    const GpuProbeSlot ps = f.slots[slot];
    const float4 fb = f.fib[sample];
    *origin = { ps.pos[0], ps.pos[1], ps.pos[2] };
    *dir = rotate(v3(fb.x, fb.y, fb.z), v3(ps.axis[0], ps.axis[1], ps.axis[2]), ps.angle_sin, ps.angle_cos);
}

template<bool COUNT, int WPE>
__global__ void __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(WPE))) k_shade(SceneArgs sc, FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    // compacted front hits (ray index) from the start, misses from the end
    __shared__ uint32_t listA[kShadeChunk];
    __shared__ uint32_t counts[4];          // [0] front hits, [1] misses, [2,3] chunk
    uint32_t cFront = 0;
    // the spot lights, read once per workgroup: per front hit and lit spot they were a
    // dependent 96-B read ahead of the IES lookup (C5: k_shade 2.06 -> 1.97 ms, +1.2 %;
    // profiles/r04_s_shade_spots_lds.log)
    __shared__ GpuSpotLight spotsL[kMaxLights - 1];
    {
        const uint32_t words = static_cast<uint32_t>(sc.spot_count) * static_cast<uint32_t>(sizeof(GpuSpotLight) / 4u);
        for (uint32_t i = threadIdx.x; i < words; i += kShadeBlock)
            reinterpret_cast<uint32_t*>(spotsL)[i] = reinterpret_cast<const uint32_t*>(sc.spots)[i];
        __syncthreads();
    }

    // chunks come from the second set of per-XCD partition heads (see grabRays)
    uint32_t* heads = f.ray_counter + kRayParts * kRayCounterStride;
    const uint32_t home = xccId();
    uint32_t tried = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t b, e;
            grabRays(f, heads, home, tried, b, e, static_cast<uint32_t>(kShadeChunk));
            counts[0] = 0;
            counts[1] = 0;
            counts[2] = b;
            counts[3] = e;
        }
        __syncthreads();
        const uint32_t chunk = counts[2], chunkEnd = counts[3];
        if (chunk >= chunkEnd) break;
        // ---- A. classify: backfaces finish here; front hits and misses are listed -
        // (a miss's environment lookup - atan2, acos, a texture sample - runs densely in
        // C below: inline, the few misses of a chunk made most of its waves run it)
        for (uint32_t r = threadIdx.x; r < kShadeChunk; r += kShadeBlock) {
            if (chunk + r >= chunkEnd) break;
            const uint32_t q = (chunk + r) / f.R;
            const uint32_t ray = slotAt(f, q) * f.R + (chunk + r - q * f.R);
            const GpuHit hit = f.hits[ray];
            if (hit.tri == kNoHit) {
                const uint32_t k = atomicAdd(&counts[1], 1u);
                listA[kShadeChunk - 1u - k] = ray;
            } else if (hit.t < 0.0f) {
                // backface: colour 0, depth x 0.2 (raygen.rgen:129-134); the closest-hit
                // colour and the indirect term are overwritten, so they are not evaluated.
                storeSurfel(f, ray, splat(0.0f), hit.t * 0.2f);
            } else {
                const uint32_t k = atomicAdd(&counts[0], 1u);
                listA[k] = ray;
            }
        }
        __syncthreads();
        const uint32_t nA = counts[0];
        // ---- B. dense surface shading of front hits -----------------------------
        for (uint32_t k0 = 0; k0 < nA; k0 += kShadeBlock) {
            const uint32_t kk = k0 + threadIdx.x;
            const bool valid = kk < nA;
            const uint32_t ray = valid ? listA[kk] : 0u;
            // surface (opaque.rchit:105-131)
            V3 origin = splat(0.0f), dir = splat(0.0f), N = splat(0.0f), baseColor = splat(0.0f), base = splat(0.0f);
            float T = 0.0f, metallic = 0.0f, roughness = 0.0f, clearcoat = 0.0f, ccRough = 0.0f;
            uint32_t need = 0;
            if (valid) {
                if (COUNT) cFront++;
                const GpuHit hit = f.hits[ray];
                rayOf(f, ray, &origin, &dir);
                T = hit.t;
                // the triangle's shading record: vertex normals, instance, UVs
                const float4* rec = sc.tri_normals + 4u * static_cast<size_t>(hit.tri);
                const float4 ra = rec[0], rb = rec[1], rc = rec[2], rd = rec[3];
                const GpuInstance gi = sc.instances[__float_as_uint(rc.y)];
                const ArkShaderMaterial& mat = sc.materials[gi.material_index];
                const float bx = 1.0f - hit.u - hit.v, by = hit.u, bz = hit.v;
                // opaque.rchit:118-131 (front face: no flip)
                N = normalize(v3(ra.x, ra.y, ra.z) * bx + v3(ra.w, rb.x, rb.y) * by + v3(rb.z, rb.w, rc.x) * bz);
                const float* M = gi.normal_matrix;
                V3 Nw = { M[0] * N.x + M[1] * N.y + M[2] * N.z, M[4] * N.x + M[5] * N.y + M[6] * N.z, M[8] * N.x + M[9] * N.y + M[10] * N.z };
                N = normalize(Nw);
                const float uvx = rc.z * bx + rd.x * by + rd.z * bz;
                const float uvy = rc.w * bx + rd.y * by + rd.w * bz;
                float4 c = sc.sample(mat.base_color, uvx, uvy);
                baseColor = v3(c.x, c.y, c.z) * v3(mat.color_tint[0], mat.color_tint[1], mat.color_tint[2]);
                c = sc.sample(mat.emissive, uvx, uvy);
                const V3 emissive = v3(c.x, c.y, c.z) * v3(mat.emissive_factor[0], mat.emissive_factor[1], mat.emissive_factor[2]);
                c = sc.sample(mat.metallic_roughness, uvx, uvy);
                metallic = c.z * mat.metallic_factor;
                roughness = c.y * mat.roughness_factor;
                clearcoat = mat.clearcoat;
                ccRough = mat.clearcoat_roughness;
                const V3 ambient = f.ambient_amount * baseColor;
                base = emissive + ambient;
                // lit lights (LdotN > 0): one shadow ray each (opaque.rchit:56-103)
                uint32_t l = 0;
                if (sc.has_sun) {
                    const V3 Ld = -normalize(v3(sc.sun_dir[0], sc.sun_dir[1], sc.sun_dir[2]));
                    if (dot(Ld, N) > 0.0f) need |= 1u;
                    l++;
                }
                for (int li = 0; li < sc.spot_count; ++li, ++l) {
                    const V3 Ld = -normalize(v3(spotsL[li].direction[0], spotsL[li].direction[1], spotsL[li].direction[2]));
                    if (dot(Ld, N) > 0.0f) need |= 1u << l;
                }
            }
            if (!valid) continue;
            const uint32_t occ = need ? f.shadow_bits[ray] >> 16 : 0u;
            V3 color = base;
            const V3 V = -dir;
            const V3 hitPoint = origin + T * dir;
            uint32_t l = 0;
            if (sc.has_sun) { // opaque.rchit:56-73
                if (need & 1u) {
                    const V3 Ld = -normalize(v3(sc.sun_dir[0], sc.sun_dir[1], sc.sun_dir[2]));
                    const float LdotN = dot(Ld, N);
                    const V3 brdf = evaluateDefaultBRDF(Ld, V, N, baseColor, roughness, metallic, clearcoat, ccRough);
                    const V3 lc = v3(sc.sun_color[0], sc.sun_color[1], sc.sun_color[2]);
                    const V3 tT = brdf * LdotN * (lc * 1.0f);
                    const V3 tZ = brdf * LdotN * (lc * 0.0f);
                    color = color + ((occ >> l) & 1u ? tZ : tT);
                }
                l++;
            }
            for (int li = 0; li < sc.spot_count; ++li, ++l) { // opaque.rchit:75-103
                if (!((need >> l) & 1u)) continue;
                const GpuSpotLight sl = spotsL[li];
                V3 sdir = v3(sl.direction[0], sl.direction[1], sl.direction[2]);
                V3 Ld = -normalize(sdir);
                float LdotN = dot(Ld, N);
                {
                        V3 toLight = v3(sl.position[0], sl.position[1], sl.position[2]) - hitPoint;
                        float distanceToLight = length(toLight);
                        V3 normalizedToLight = toLight / distanceToLight;
                        float distanceAttenuation = 1.0f / square(distanceToLight);
                        // evaluateIESLookupTable (lighting.glsl:20-39)
                        V3 lrd = -normalizedToLight;
                        float iesValue = 0.0f;
                        float angleV = dot(lrd, sdir);
                        if (!(angleV <= 0.0f)) {
                            float hx = dot(lrd, v3(sl.right[0], sl.right[1], sl.right[2]));
                            float hy = dot(lrd, v3(sl.up[0], sl.up[1], sl.up[2]));
                            float angleH = atan2f_(hy, hx) + kPi;
                            float lx = acosf_(angleV) / (2.0f * sl.position[3]);
                            float ly = clampf(angleH / kTwoPi, 0.0f, 1.0f);
                            iesValue = sc.sample(sl.ies_texture, lx, ly).x;
                        }
                        V3 brdf = evaluateDefaultBRDF(Ld, V, N, baseColor, roughness, metallic, clearcoat, ccRough);
                        V3 lc = v3(sl.color[0], sl.color[1], sl.color[2]);
                        V3 tT = brdf * LdotN * (lc * 1.0f * distanceAttenuation * iesValue);
                        V3 tZ = brdf * LdotN * (lc * 0.0f * distanceAttenuation * iesValue);
                    color = color + ((occ >> l) & 1u ? tZ : tT);
                }
            }
            // raygen.rgen:125-127 + evaluateIndirectLightFromPreviousFrame (:94-106)
            const V3 Vi = -dir;
            const V3 F0 = mix3(splat(kDielectricReflectance), baseColor, metallic);
            const V3 F = F_Schlick3(fmaxf_(0.0f, dot(Vi, N)), F0);
            const V3 irradiance = sampleDDGI<kGatherBatch>(f, hitPoint, N, Vi);
            const V3 indirect = splat(1.0f - metallic) * (splat(1.0f) - F) * irradiance;
            const V3 bi = baseColor * indirect;
            storeSurfel(f, ray, color + bi, T);
        }
        // ---- C. misses (raygen.rgen:70-79) ------------------------------------------
        const uint32_t nM = counts[1];
        for (uint32_t k = threadIdx.x; k < nM; k += kShadeBlock) {
            const uint32_t ray = listA[kShadeChunk - 1u - k];
            V3 origin, dir;
            rayOf(f, ray, &origin, &dir);
            float u, v;
            sphericalUvFromDirection(dir, &u, &v);
            float4 c = sc.sample(sc.env_texture, u, v);
            storeSurfel(f, ray, f.environment_multiplier * v3(c.x, c.y, c.z), f.z_far);
        }
        __syncthreads();
    }
    if (COUNT) atomicAdd(&f.counters[6], static_cast<unsigned long long>(cFront));
}

// ---------------------------------------------------------------------------
// Intra-wave splitting of the traversal tail
// ---------------------------------------------------------------------------
// Once the ray supply has run dry, a persistent traversal wave only runs its last,
// longest rays, one dependent node fetch per iteration, while most of its lanes
// idle (C4: the shadow kernel spent 0.28 of 0.64 ms draining). So an idle lane of
// an exhausted wave takes work from a lane that is still traversing: the donor
// hands over the bottom entry of its node-group stack (the oldest deferred group,
// usually the largest subtree left) and the helper traverses that group with a
// copy of the donor's ray. Helpers can donate again; every helper reports to the
// ray's root lane, which finishes the ray only when its helper count is back to
// zero. The result does not depend on who visits which subtree: any-hit rays OR
// their occlusion, closest-hit rays keep the nearest hit with the (instance,
// primitive) tie rule, and box culling is conservative for any tmax that bounds
// the closest hit.
// Per wave LDS: a 64-entry donor table (rank -> donor lane) and, per lane, a byte
// with its outstanding helper count (bits 0-6) and a "ray resolved" flag (bit 7).
struct TailLds {
    uint8_t* table;  // [kTraceBlock]
    uint32_t* bytes; // [kTraceBlock / 4], one byte per lane
};

__device__ __forceinline__ uint32_t tailByte(const TailLds& tl, uint32_t t)
{
    return (__hip_atomic_load(tl.bytes + (t >> 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT) >> (8u * (t & 3u))) & 0xffu;
}

__device__ __forceinline__ void tailAdd(const TailLds& tl, uint32_t t, uint32_t v)
{
    __hip_atomic_fetch_add(tl.bytes + (t >> 2), v << (8u * (t & 3u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ void tailSub(const TailLds& tl, uint32_t t, uint32_t v)
{
    __hip_atomic_fetch_sub(tl.bytes + (t >> 2), v << (8u * (t & 3u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ void tailOr(const TailLds& tl, uint32_t t, uint32_t v)
{
    __hip_atomic_fetch_or(tl.bytes + (t >> 2), v << (8u * (t & 3u)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ void tailClear(const TailLds& tl, uint32_t t)
{
    __hip_atomic_fetch_and(tl.bytes + (t >> 2), ~(0xffu << (8u * (t & 3u))), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Removes the bottom entry (entry 0) of a non-empty stack and returns it; the top
// entry moves into its place (visiting order only affects speed).
template<int BLOCK>
__device__ __forceinline__ void stackTakeBottom(Stack<BLOCK>& st, uint32_t& a, uint32_t& b)
{
    // entry i is in LDS slot i % kStackLds while i >= depth - kStackLds, else at spill[i]
    if (st.depth <= kStackLds) {
        a = st.lds[0];
        b = st.lds[BLOCK];
    } else {
        a = st.spill[0];
        b = st.spill[st.spillStride];
    }
    uint32_t ta, tb;
    st.pop(ta, tb);
    if (st.depth > 0) {
        if (st.depth <= kStackLds) {
            st.lds[0] = ta;
            st.lds[BLOCK] = tb;
        } else {
            st.spill[0] = ta;
            st.spill[st.spillStride] = tb;
        }
    }
}

__device__ __forceinline__ V3 shfl3(V3 v, uint32_t src)
{
    return v3(__shfl(v.x, static_cast<int>(src)), __shfl(v.y, static_cast<int>(src)), __shfl(v.z, static_cast<int>(src)));
}

// Persistent any-hit traversal of the shadow-ray list (opaque.rchit:35-54:
// TerminateOnFirstHit | SkipClosestHit | Opaque, cullMask 0xff, tmin 0.025): the
// three hit-mask classes in turn, no alpha test, dual steps. Lanes are refilled
// from a wave-private pool like k_trace; an occluded ray sets bit 16 + light of its
// probe ray's word. `pass` of a helper lane holds (root lane + 1) << 8.
// MODE: kShadowWorld - the shadow rays through the three world BVHs; kShadowSun - the
// sun's list (FrameArgs::sun_rays) through the light-space BVH (one pass, travStepSun);
// kShadowSunWorld - both in one launch: each wave drains the sun's list, then takes
// rays from the other list, so the first list's tail overlaps the second list's work
// instead of ending a launch (C5: 1.98 ms one list, 3.27 ms two launches).
constexpr int kShadowWorld = 0, kShadowSun = 1, kShadowSunWorld = 2;

template<bool COUNT, bool SUN>
__device__ __forceinline__ void shadowPhase(const SceneArgs& sc, const FrameArgs& f, const NodeCache& nc, Stack<kTraceBlock>& st, const TailLds& tl,
                                            uint32_t& cNodes, uint32_t& cTris, uint32_t& cShadow)
{
    const uint32_t lane = threadIdx.x & 63u, wbase = threadIdx.x & ~63u;
    if (lane < 16u) tl.bytes[(wbase >> 2) + lane] = 0u; // wave-private tail bytes
    const float tmin = 0.025f;
    const uint32_t total = SUN ? *f.sun_count : *f.shadow_count;
    uint32_t* const heads = SUN ? f.sun_heads : f.shadow_heads;
    const ShadowRay* const list = SUN ? f.sun_rays : f.shadow_rays;
    const int32_t roots[3] = { SUN ? sc.sun_root : sc.root_opaque, SUN ? -1 : sc.root_masked, SUN ? -1 : sc.root_blend };

    uint32_t poolNext = 0, poolEnd = 0;
    const uint32_t home = xccId();
    uint32_t tried = 0;
    bool exhausted = false, active = false;
    uint32_t owner = 0;
    int pass = 0;
    float tmax = 0.0f;
    TravState ts { 0u, 0u, 0u, 0u };
    uint32_t nBase = 0, nBits = 0; // the next triangle group (dual step)
    uint32_t oct = 0;
    V3 o = { 0, 0, 0 }, d = { 0, 0, 1 }, idir = { 0, 0, 1 };
    auto done = [&]() { return travDoneDual(ts, nBits, st); };
    auto stop = [&]() { ts = TravState { 0u, 0u, 0u, 0u }; nBits = 0; st.depth = 0; };
    for (;;) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && !exhausted && (static_cast<uint32_t>(__popcll(need)) >= (SUN ? f.sun_refill_min : f.refill_min) || need == ~0ull)) {
            const uint32_t n = static_cast<uint32_t>(__popcll(need));
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(need >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(need), 0u));
            const uint32_t avail = poolEnd - poolNext;
            uint32_t fb = 0, fe = 0;
            if (avail < n) {
                uint32_t b = 0, e = 0, t = tried;
                if (lane == 0) grabItems(heads, total, home, t, b, e, f.grab_chunk);
                fb = __shfl(b, 0);
                fe = __shfl(e, 0);
                tried = __shfl(t, 0);
            }
            if (!active) {
                uint32_t r = kNoHit;
                if (rank < avail) r = poolNext + rank;
                else if (fb + (rank - avail) < fe) r = fb + (rank - avail);
                if (r != kNoHit) {
                    const ShadowRay sr = list[r];
                    o = v3(sr.origin_tmax.x, sr.origin_tmax.y, sr.origin_tmax.z);
                    d = v3(sr.dir_owner.x, sr.dir_owner.y, sr.dir_owner.z);
                    tmax = sr.origin_tmax.w;
                    owner = __float_as_uint(sr.dir_owner.w);
                    // SUN: idir holds the origin's light-space coordinates
                    idir = SUN ? sunCoords(sc, o) : safeInv(d);
                    oct = SUN ? 0u : rayOctant(idir);
                    stop();
                    pass = 0;
                    active = true;
                    if (tmax >= tmin) {
                        if (COUNT) cShadow++;
                        while (pass < 3 && roots[pass] < 0) ++pass;
                        if (pass < 3) ts = TravState { static_cast<uint32_t>(roots[pass]), rootGroupBits(), 0u, 0u };
                    } else {
                        pass = 3; // !(maxDistance >= tmin): not traced, not occluded
                    }
                }
            }
            if (avail < n) {
                if (fb >= fe) {
                    exhausted = true;
                    poolNext = poolEnd = 0;
                } else {
                    poolNext = min(fb + (n - avail), fe);
                    poolEnd = fe;
                }
            } else {
                poolNext += n;
            }
        }
        if (__ballot(active) == 0) break;
        if (exhausted) {
            // ---- tail: resolved rays stop, idle lanes take stack bottoms --------------
            const uint32_t root = pass >= 256 ? static_cast<uint32_t>(pass >> 8) - 1u : lane;
            if (active && (tailByte(tl, wbase + root) & 0x80u)) stop();
            const uint64_t idle = __ballot(!active);
            const bool can = active && st.depth > 0;
            const uint64_t donors = __ballot(can);
            const uint32_t m = min(static_cast<uint32_t>(__popcll(idle)), static_cast<uint32_t>(__popcll(donors)));
            if (m != 0) {
                const uint32_t dr = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(donors >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(donors), 0u));
                const uint32_t ir = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(idle >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(idle), 0u));
                uint32_t gB = 0, gBits = 0;
                if (can && dr < m) {
                    stackTakeBottom(st, gB, gBits);
                    tl.table[wbase + dr] = static_cast<uint8_t>(lane);
                    tailAdd(tl, wbase + root, 1u);
                }
                // every lane shuffles (a lane that takes nothing reads its own values)
                const bool take = !active && ir < m;
                const uint32_t src = take ? tl.table[wbase + ir] : lane;
                o = shfl3(o, src);
                d = shfl3(d, src);
                tmax = __shfl(tmax, static_cast<int>(src));
                owner = __shfl(owner, static_cast<int>(src));
                const uint32_t sroot = __shfl(root, static_cast<int>(src));
                gB = __shfl(gB, static_cast<int>(src));
                gBits = __shfl(gBits, static_cast<int>(src));
                if (take) {
                    idir = SUN ? sunCoords(sc, o) : safeInv(d);
                    oct = SUN ? 0u : rayOctant(idir);
                    pass = static_cast<int>((sroot + 1u) << 8);
                    stop();
                    ts = TravState { gB, gBits, 0u, 0u };
                    active = true;
                }
            }
        }
        if (active) {
            // (a done lane - a root waiting for its helpers - steps as a no-op)
            bool occluded;
            if constexpr (SUN) {
                occluded = travStepSun<kTraceBlock>(sc, ts, nBase, nBits, st, o, d, idir, tmin, tmax, cNodes, cTris);
            } else {
                RayHit h { tmax, 0.0f, 0.0f, kNoHit, 0u, 0u, false };
                occluded = travStepDual<kTraceBlock, true, false>(sc, nc, ts, nBase, nBits, st, o, d, idir, oct, tmin, h, 0, cNodes, cTris);
            }
            const bool helper = pass >= 256;
            const uint32_t root = helper ? static_cast<uint32_t>(pass >> 8) - 1u : lane;
            if (occluded) {
                atomicOr(&f.shadow_bits[owner >> 4], 1u << (16u + (owner & 15u)));
                if (exhausted) tailOr(tl, wbase + root, 0x80u);
                stop();
                if (!helper) pass = 3; // no further hit-mask classes
            }
            if (done()) {
                if (helper) {
                    tailSub(tl, wbase + root, 1u);
                    active = false;
                } else if (!exhausted || (tailByte(tl, wbase + lane) & 0x7fu) == 0) {
                    if (exhausted && (tailByte(tl, wbase + lane) & 0x80u)) pass = 3; // a helper found the occluder
                    ++pass;
                    while (pass < 3 && roots[pass] < 0) ++pass;
                    if (pass < 3) {
                        st.depth = 0;
                        ts = TravState { static_cast<uint32_t>(roots[pass]), rootGroupBits(), 0u, 0u };
                    } else {
                        if (exhausted) tailClear(tl, wbase + lane);
                        active = false;
                    }
                }
            }
        }
    }
}

template<bool COUNT, int WPE, int MODE = kShadowWorld>
__global__ void __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(WPE))) k_trace_shadow(SceneArgs sc, FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    __shared__ uint32_t ldsStack[kStackLds * 2 * kTraceBlock];
    // 8 cached nodes fewer than k_trace: the tail tables then fit 6 workgroups per CU
    // (the light-space traversal caches none)
    constexpr int kNodes = MODE == kShadowSun ? 1 : kShadowLdsNodes;
    __shared__ uint4 ldsNodes[kNodes * 5];
    __shared__ uint8_t ldsTable[kTraceBlock];
    __shared__ uint32_t ldsBytes[kTraceBlock / 4];
    NodeCache nc { nullptr, 0u, 0u };
    if constexpr (MODE != kShadowSun) nc = loadNodeCache<kTraceBlock, kNodes>(sc, ldsNodes);
    (void)ldsNodes;
    const TailLds tl { ldsTable, ldsBytes };
    const uint32_t gtid = blockIdx.x * kTraceBlock + threadIdx.x;
    Stack<kTraceBlock> st { ldsStack + threadIdx.x, f.spill + gtid, gridDim.x * kTraceBlock, 0 };
    uint32_t cNodes = 0, cTris = 0, cShadow = 0;
    if constexpr (MODE != kShadowWorld) shadowPhase<COUNT, true>(sc, f, nc, st, tl, cNodes, cTris, cShadow);
    if constexpr (MODE != kShadowSun) shadowPhase<COUNT, false>(sc, f, nc, st, tl, cNodes, cTris, cShadow);
    if (COUNT) {
        atomicAdd(&f.counters[4], static_cast<unsigned long long>(cNodes));
        atomicAdd(&f.counters[5], static_cast<unsigned long long>(cTris));
        atomicAdd(&f.counters[3], static_cast<unsigned long long>(cShadow));
    }
}

// Shadow-ray list: one thread per window ray in
// slot order; a front hit (raygen.rgen:121-127) stores its lit-light mask
// (opaque.rchit:56-103, LdotN > 0 with the shading normal) in shadow_bits[ray] and
// appends one shadow ray per lit light, owner = (ray << 4) | light. k_trace_shadow
// then sets the occluded bits 16 + light, and k_shade finishes every surfel
// in one pass (no per-light records, no finishing kernel).
// Block b owns the kGenSteps x 256 consecutive queue positions from b * kGenSpan:
// pass 1 stores the light masks (LDS + shadow_bits) and counts; one global atomic
// per block reserves the block's shadow rays (a per-wave atomic on the one list
// counter serialises at L2: 1.45 ms for 131K waves on C4); pass 2 writes them in
// position order (wave scans), so a shadow-kernel grab of 64 list entries holds the
// neighbouring rays of one probe. kGenSteps = 4 (16: 0.185 ms, 4: 0.163, 2: 0.215 at
// C4). Measured and removed: the list binned by light-space cell (-15 %
// shadow HBM, +34 % shadow phase) and a straight-line staged form (179 VGPRs, 0.416 ms).
constexpr uint32_t kGenSteps = 4, kGenSpan = kGenSteps * 256u;

__device__ __forceinline__ uint32_t waveInclusiveScan(uint32_t x)
{
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= static_cast<uint32_t>(off)) x += y;
    }
    return x;
}

// REFL: the reflection ray list (rt-reflections/raygen.rgen:122): queue position =
// list index, and the closest hit shades back faces too, with the normal flipped
// (opaque.rchit:121-125): N = -(shading normal), as negation commutes exactly with
// the normal matrix product and the normalisation.
template<bool REFL = false>
__global__ void __launch_bounds__(256) k_shadow_gen(SceneArgs sc, FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    __shared__ uint32_t bitsL[kGenSpan];
    __shared__ uint32_t waveOff[kGenSteps][4];
    __shared__ uint32_t blockBase, sunBlockBase;
    // the sun's rays (light 0) to their own list when the scene has a light-space BVH
    const bool splitSun = !REFL && f.sun_rays != nullptr;
    const uint32_t total = REFL ? *f.list_count : f.window_rays;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t first = blockIdx.x * kGenSpan;
    if (REFL && first >= total) return; // launched for the largest possible list
    // pass 1 in stages over the thread's kGenSteps rays, so that each stage's
    // dependent loads (slot order -> hit -> triangle normals -> instance) are in
    // flight for all of them at once (the kernel is latency bound)
    uint32_t rays[kGenSteps];
    GpuHit hits[kGenSteps];
#pragma unroll
    for (uint32_t k = 0; k < kGenSteps; ++k) {
        const uint32_t pos = first + k * 256u + threadIdx.x;
        if (REFL) {
            rays[k] = pos < total ? pos : kNoHit;
        } else {
            const uint32_t q = pos / f.R;
            rays[k] = pos < total ? slotAt(f, q) * f.R + (pos - q * f.R) : kNoHit;
        }
    }
#pragma unroll
    for (uint32_t k = 0; k < kGenSteps; ++k) {
        hits[k] = rays[k] != kNoHit ? f.hits[rays[k]] : GpuHit { 0.0f, 0.0f, 0.0f, kNoHit };
        if (!REFL && hits[k].t < 0.0f) hits[k].tri = kNoHit; // backface: no shading, no shadow ray
    }
#pragma unroll
    for (uint32_t k = 0; k < kGenSteps; ++k) {
        uint32_t bits = 0;
        if (hits[k].tri != kNoHit) {
            V3 N = hitShadingNormal(sc, hits[k].tri, hits[k].u, hits[k].v);
            if (REFL && hits[k].t < 0.0f) N = -N;
            bits = litLightMask(sc, N);
            f.shadow_bits[rays[k]] = bits;
        }
        bitsL[k * 256u + threadIdx.x] = bits;
    }
    // counts packed: world-list rays in bits 0-15, sun-list rays in bits 16-31 (a
    // block has at most kGenSpan x kMaxLights = 11,264 of either, no carry)
    auto packedCount = [&](uint32_t bits) {
        const uint32_t sun = splitSun ? (bits & 1u) : 0u;
        return static_cast<uint32_t>(__builtin_popcount(bits & ~sun)) | (sun << 16);
    };
#pragma unroll
    for (uint32_t k = 0; k < kGenSteps; ++k) {
        const uint32_t x = waveInclusiveScan(packedCount(bitsL[k * 256u + threadIdx.x]));
        if (__lane_id() == 63u) waveOff[k][wave] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t k = 0; k < kGenSteps; ++k)
            for (uint32_t w = 0; w < 4; ++w) {
                const uint32_t c = waveOff[k][w];
                waveOff[k][w] = run;
                run += c;
            }
        blockBase = (run & 0xffffu) ? atomicAdd(f.shadow_count, run & 0xffffu) : 0u;
        sunBlockBase = (run >> 16) ? atomicAdd(f.sun_count, run >> 16) : 0u;
    }
    __syncthreads();
    for (uint32_t k = 0; k < kGenSteps; ++k) {
        const uint32_t bits = bitsL[k * 256u + threadIdx.x];
        const uint32_t c = packedCount(bits);
        const uint32_t before = waveOff[k][wave] + waveInclusiveScan(c) - c;
        uint32_t sj = blockBase + (before & 0xffffu);
        uint32_t sunj = sunBlockBase + (before >> 16);
        if (bits == 0) continue;
        const uint32_t pos = first + k * 256u + threadIdx.x;
        uint32_t ray;
        V3 hitPoint;
        if (REFL) {
            ray = pos;
            const float4 a = f.ray_list[2u * pos], b = f.ray_list[2u * pos + 1u];
            const V3 origin = v3(a.x, a.y, a.z), dir = v3(b.x, b.y, b.z);
            const float t = fabsf_(f.hits[ray].t); // rt_RayHitT of a front or back face
            hitPoint = origin + t * dir;
        } else {
            const uint32_t q = pos / f.R;
            ray = slotAt(f, q) * f.R + (pos - q * f.R);
            const float t = f.hits[ray].t;
            V3 origin, dir;
            rayOf(f, ray, &origin, &dir);
            hitPoint = origin + t * dir;
        }
        for (uint32_t b = bits; b; b &= b - 1) {
            const uint32_t l = static_cast<uint32_t>(__builtin_ctz(b));
            V3 ld;
            float tmax;
            shadowRayOf(sc, f.z_far, l, hitPoint, &ld, &tmax);
            const ShadowRay sr { make_float4(hitPoint.x, hitPoint.y, hitPoint.z, tmax), make_float4(ld.x, ld.y, ld.z, __uint_as_float((ray << 4) | l)) };
            if (splitSun && l == 0u) f.sun_rays[sunj++] = sr;
            else f.shadow_rays[sj++] = sr;
        }
    }
}

// Frame sequencing between a context's two streams (ark_ddgi.cpp updateImpl): the
// producer stream ends its part of frame n with k_seq_signal (word = n, a release
// store after the kernels before it on that stream), the consumer stream starts with
// k_seq_wait (one wave polls the word with acquire loads until it reaches n). A
// cross-queue event wait costs 12-16 us of queue latency per frame, satisfied or not
// (profiles/r03_v, r03_w); this pair costs two one-wave launches. Every wait ends:
// the word is written by work enqueued earlier on the other stream, which nothing
// blocks - unless something serialises the queues (a counter-collecting profiler
// runs one kernel at a time: the wait can then be scheduled ahead of its signal).
// The wait therefore fails closed: after timeout_ticks of the wall clock (or at once
// when an earlier wait of the context already gave up) it sets *timed_out, which
// every kernel of the path checks at entry (frameAborted: the frame's remaining
// launches leave their outputs untouched), and the host-mapped *host_flag, which the
// context's next call polls (ark_ddgi.cpp checkSequencing: ARK_DDGI_E_DEVICE, then
// event sequencing). Signals are never skipped, so the sequence words stay in step.
__global__ void __launch_bounds__(64) k_seq_signal(uint32_t* word, uint32_t value)
{
    if (threadIdx.x == 0) __hip_atomic_store(word, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64) k_seq_wait(const uint32_t* word, uint32_t value, uint32_t* timed_out, uint32_t* host_flag, uint64_t timeout_ticks)
{
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    while (static_cast<int32_t>(__hip_atomic_load(word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - value) < 0) {
        if (wall_clock64() - t0 > timeout_ticks || __hip_atomic_load(timed_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
            __hip_atomic_store(timed_out, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (host_flag) __hip_atomic_store(host_flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Atlas clears (DDGINode.cpp:50-55) as 32-bit fills.
__global__ void k_fill_u32(uint32_t* __restrict__ p, uint64_t n, uint32_t value)
{
    for (uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; i < n; i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        p[i] = value;
}

// ---------------------------------------------------------------------------
// 5. AO / bent-normal bake (BakeAmbientOcclusionNode.cpp:15-131)
// ---------------------------------------------------------------------------
// Parameterization pass (bakeParameterization.vert/.frag) as a deterministic integer
// rasterizer of the mesh's UV layout: a vertex lands at (fract(u) * W, fract(v) * H)
// (the viewport transform of NDC = fract * 2 - 1), snapped to 1/256 texel with RNE
// (8-bit subpixel precision); a texel is covered when its centre is inside the
// triangle (exact 64-bit edge functions; a centre on an edge belongs to the triangle
// that runs the edge "up, or right when horizontal" in positive orientation, so a
// centre on an edge shared by two triangles is covered once). Where triangles
// overlap the later primitive wins (draw order, no depth test): atomicMax of
// triangle + 1. gl_BaryCoordEXT = edge function / area in fp32, stored RGBA16F.
// The CPU oracle (oracle/ddgi_oracle.cpp, bake section) restates the same rules.


__device__ __forceinline__ int64_t bakeSnap(float c, uint32_t extent)
{
    const float fr = c - floorf_(c); // GLSL fract
    return static_cast<int64_t>(rintf(fr * static_cast<float>(extent) * 256.0f));
}

__device__ __forceinline__ int64_t bakeEdge(int64_t ax, int64_t ay, int64_t bx, int64_t by, int64_t px, int64_t py)
{
    return (bx - ax) * (py - ay) - (by - ay) * (px - ax);
}

// tie rule for a centre exactly on edge (a -> b) of a positively oriented triangle
__device__ __forceinline__ bool bakeOwnsEdge(int64_t dx, int64_t dy) { return dy > 0 || (dy == 0 && dx > 0); }

struct BakeTri {
    int64_t x[3], y[3];
    int64_t area; // bakeEdge(v0, v1, v2); 0 = degenerate
};

__device__ __forceinline__ BakeTri bakeTriangle(const BakeArgs& b, uint32_t t)
{
    BakeTri r;
    for (int k = 0; k < 3; ++k) {
        const uint32_t idx = b.indices[static_cast<size_t>(b.first_index) + 3u * t + k];
        const float* vx = b.vertices + (static_cast<size_t>(b.first_vertex) + idx) * 9;
        r.x[k] = bakeSnap(vx[0], b.W);
        r.y[k] = bakeSnap(vx[1], b.H);
    }
    r.area = bakeEdge(r.x[0], r.y[0], r.x[1], r.y[1], r.x[2], r.y[2]);
    return r;
}

// edge functions at texel centre (px, py): w[k] is opposite vertex k; returns coverage
__device__ __forceinline__ bool bakeCover(const BakeTri& t, int px, int py, int64_t* w)
{
    const int64_t cx = 256 * static_cast<int64_t>(px) + 128, cy = 256 * static_cast<int64_t>(py) + 128;
    w[0] = bakeEdge(t.x[1], t.y[1], t.x[2], t.y[2], cx, cy);
    w[1] = bakeEdge(t.x[2], t.y[2], t.x[0], t.y[0], cx, cy);
    w[2] = bakeEdge(t.x[0], t.y[0], t.x[1], t.y[1], cx, cy);
    const int64_t s = t.area > 0 ? 1 : -1;
    bool in = true;
    for (int k = 0; k < 3; ++k) {
        const int a = (k + 1) % 3, c = (k + 2) % 3; // edge a -> c (as oriented when area > 0)
        const int64_t e = s * w[k];
        const int64_t dx = s * (t.x[c] - t.x[a]), dy = s * (t.y[c] - t.y[a]);
        in = in && (e > 0 || (e == 0 && bakeOwnsEdge(dx, dy)));
    }
    return in;
}

__global__ void __launch_bounds__(256) k_bake_raster(BakeArgs b)
{
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= b.tri_count) return;
    const BakeTri tr = bakeTriangle(b, t);
    if (tr.area == 0) return;
    const int64_t xmin = min(tr.x[0], min(tr.x[1], tr.x[2])), xmax = max(tr.x[0], max(tr.x[1], tr.x[2]));
    const int64_t ymin = min(tr.y[0], min(tr.y[1], tr.y[2])), ymax = max(tr.y[0], max(tr.y[1], tr.y[2]));
    // texel centres 256 p + 128 inside [min, max]
    const int px0 = static_cast<int>(max<int64_t>(0, (xmin - 128 + 255) >> 8));
    const int px1 = static_cast<int>(min<int64_t>(static_cast<int64_t>(b.W) - 1, (xmax - 128) >> 8));
    const int py0 = static_cast<int>(max<int64_t>(0, (ymin - 128 + 255) >> 8));
    const int py1 = static_cast<int>(min<int64_t>(static_cast<int64_t>(b.H) - 1, (ymax - 128) >> 8));
    for (int py = py0; py <= py1; ++py)
        for (int px = px0; px <= px1; ++px) {
            int64_t w[3];
            if (bakeCover(tr, px, py, w)) atomicMax(&b.tri_idx[static_cast<size_t>(py) * b.W + px], t + 1u);
        }
}

// barycentrics of the winning triangle; uncovered texels get their final output
// here (bakeAmbientOcclusion.rgen:44-51), covered ones join the AO work list
__global__ void __launch_bounds__(256) k_bake_bary(BakeArgs b)
{
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= b.W * b.H) return;
    const uint32_t t1 = b.tri_idx[p];
    uint2 packed = make_uint2(0u, 0u);
    if (t1 == 0) {
        if (b.bent) reinterpret_cast<uint32_t*>(b.out)[p] = 128u | (128u << 8) | (128u << 16) | (255u << 24);
        else b.out[p] = 0;
    } else {
        const BakeTri tr = bakeTriangle(b, t1 - 1u);
        int64_t w[3];
        bakeCover(tr, static_cast<int>(p % b.W), static_cast<int>(p / b.W), w);
        const float A = static_cast<float>(tr.area);
        const float b0 = static_cast<float>(w[0]) / A, b1 = static_cast<float>(w[1]) / A, b2 = static_cast<float>(w[2]) / A;
        packed.x = static_cast<uint32_t>(f32_to_f16(b0)) | (static_cast<uint32_t>(f32_to_f16(b1)) << 16);
        packed.y = static_cast<uint32_t>(f32_to_f16(b2)) | (0x3c00u << 16);
        b.pixels[atomicAdd(&b.counters[0], 1u)] = p;
    }
    reinterpret_cast<uint2*>(b.bary)[p] = packed;
}

__device__ __forceinline__ uint8_t unorm8(float x) { return static_cast<uint8_t>(rintf(saturate(x) * 255.0f)); }

// bakeAmbientOcclusion.rgen:93-98: one cosine-distributed direction by rejection,
// bounded to kBakeMaxDraws draws (then the normal): a texel whose seed hashes to 0
// (wang_hash(61) == 0) has a xorshift state stuck at 0 and would loop forever with a
// +z normal, which on the reference is a GPU hang (DESIGN.md §AO bake).
constexpr int kBakeMaxDraws = 16;
__device__ __forceinline__ V3 bakeSampleDirection(V3 normal, uint32_t& rng)
{
    V3 dir;
    int draws = 0;
    do {
        const float theta = kTwoPi * randomFloat(rng);
        const float u = 2.0f * randomFloat(rng) - 1.0f;
        const float sr = sqrtf_(1.0f - u * u);
        float s, c;
        sincosf_(theta, &s, &c);
        dir = normal + v3(sr * c, sr * s, u);
    } while (dot(dir, dir) <= 1e-4f && ++draws < kBakeMaxDraws);
    if (dot(dir, dir) <= 1e-4f) dir = normal;
    return normalize(dir);
}

// bakeAmbientOcclusion.rgen:33-118, persistent: every lane owns one texel and runs
// its sample_count rays one after the other (one any-hit traversal each over the
// three hit-mask classes, masked candidates alpha tested as .rahit does); lanes whose
// texel is done take the next covered texel from a wave-private pool.
template<int WPE>
__global__ void __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(WPE))) k_bake_ao(SceneArgs sc, BakeArgs b)
{
    __shared__ uint32_t ldsStack[kStackLds * 2 * kTraceBlock];
    __shared__ uint4 ldsNodes[kLdsNodes * 5];
    const NodeCache nc = loadNodeCache<kTraceBlock>(sc, ldsNodes);
    const uint32_t gtid = blockIdx.x * kTraceBlock + threadIdx.x;
    Stack<kTraceBlock> st { ldsStack + threadIdx.x, b.spill + gtid, gridDim.x * kTraceBlock, 0 };
    const uint32_t lane = threadIdx.x & 63u;
    const float tmin = 0.0005f, tmax = 100.0f;
    const uint32_t total = b.counters[0];
    const int32_t roots[3] = { sc.root_opaque, sc.root_masked, sc.root_blend };
    uint32_t cN = 0, cT = 0;

    uint32_t poolNext = 0, poolEnd = 0;
    bool exhausted = false, active = false;
    uint32_t pixel = 0, rng = 0, sampleIdx = 0;
    float aoAcc = 0.0f;
    V3 dirAcc = splat(0.0f), P = splat(0.0f), Nrm = splat(0.0f);
    int pass = 0;
    TravState ts { 0u, 0u, 0u, 0u };
    uint32_t oct = 0;
    V3 d = { 0, 0, 1 }, idir = { 0, 0, 1 };
    auto startRay = [&]() {
        d = bakeSampleDirection(Nrm, rng);
        idir = safeInv(d);
        oct = rayOctant(idir);
        st.depth = 0;
        pass = 0;
        while (pass < 3 && roots[pass] < 0) ++pass;
        ts = pass < 3 ? TravState { static_cast<uint32_t>(roots[pass]), rootGroupBits(), 0u, 0u } : TravState { 0u, 0u, 0u, 0u };
    };
    for (;;) {
        const uint64_t need = __ballot(!active);
        if (need != 0 && !exhausted) {
            const uint32_t n = static_cast<uint32_t>(__popcll(need));
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(need >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(need), 0u));
            const uint32_t avail = poolEnd - poolNext;
            uint32_t fb = 0, fe = 0;
            if (avail < n) {
                uint32_t s = 0;
                if (lane == 0) s = atomicAdd(&b.counters[32], 64u);
                fb = min(__shfl(s, 0), total);
                fe = min(fb + 64u, total);
            }
            if (!active) {
                uint32_t r = kNoHit;
                if (rank < avail) r = poolNext + rank;
                else if (fb + (rank - avail) < fe) r = fb + (rank - avail);
                if (r != kNoHit) {
                    // texel setup (bakeAmbientOcclusion.rgen:53-86)
                    pixel = b.pixels[r];
                    const uint32_t tri = b.tri_idx[pixel] - 1u;
                    const uint2 bw = reinterpret_cast<const uint2*>(b.bary)[pixel];
                    const V3 bc = v3(f16_to_f32(static_cast<uint16_t>(bw.x & 0xffffu)), f16_to_f32(static_cast<uint16_t>(bw.x >> 16)),
                                     f16_to_f32(static_cast<uint16_t>(bw.y & 0xffffu)));
                    V3 p[3], nn[3];
                    for (int k = 0; k < 3; ++k) {
                        const uint32_t idx = b.indices[static_cast<size_t>(b.first_index) + 3u * tri + k];
                        const size_t vi = static_cast<size_t>(b.first_vertex) + idx;
                        p[k] = v3(b.positions[vi * 3 + 0], b.positions[vi * 3 + 1], b.positions[vi * 3 + 2]);
                        const float* vx = b.vertices + vi * 9;
                        nn[k] = v3(vx[2], vx[3], vx[4]);
                    }
                    P = p[0] * bc.x + p[1] * bc.y + p[2] * bc.z;
                    Nrm = normalize(nn[0] * bc.x + nn[1] * bc.y + nn[2] * bc.z);
                    rng = wang_hash(pixel); // seedRandom(x + y * W)
                    sampleIdx = 0;
                    aoAcc = 0.0f;
                    dirAcc = splat(0.0f);
                    active = true;
                    startRay();
                }
            }
            if (avail < n) {
                if (fb >= fe) {
                    exhausted = true;
                    poolNext = poolEnd = 0;
                } else {
                    poolNext = min(fb + (n - avail), fe);
                    poolEnd = fe;
                }
            } else {
                poolNext += n;
            }
        }
        if (__ballot(active) == 0) break;
        if (active) {
            bool hit = false;
            if (!travDone(ts, st)) {
                Fetch fx;
                travFetch(sc, nc, ts, st, oct, fx);
                uint32_t inst, prim;
                float tt, uu, vv;
                bool bf;
                hit = travCompute(fx, ts, P, d, idir, oct, tmin, tmax, tt, uu, vv, bf, inst, prim, cN, cT) &&
                      !(pass == 1 && !alphaAccept(sc, inst, prim, uu, vv)); // masked.rahit ignoreIntersection
            }
            bool rayDone = hit;
            if (!hit && travDone(ts, st)) {
                ++pass;
                while (pass < 3 && roots[pass] < 0) ++pass;
                if (pass < 3) {
                    st.depth = 0;
                    ts = TravState { static_cast<uint32_t>(roots[pass]), rootGroupBits(), 0u, 0u };
                } else {
                    rayDone = true;
                }
            }
            if (rayDone) {
                // bakeAmbientOcclusion.rgen:101-106 (hit distance <= tmax iff an accepted hit)
                if (hit) aoAcc += 1.0f;
                else dirAcc = dirAcc + d;
                if (++sampleIdx < b.samples) {
                    startRay();
                } else {
                    if (b.bent) { // :109-114
                        const V3 bent = dirAcc / static_cast<float>(b.samples);
                        const float cone = (kPi / 2.0f) / (kPi / 2.0f);
                        const V3 enc = bent * v3(0.5f, 0.5f, 0.5f) + v3(0.5f, 0.5f, 0.5f);
                        reinterpret_cast<uint32_t*>(b.out)[pixel] = static_cast<uint32_t>(unorm8(enc.x)) | (static_cast<uint32_t>(unorm8(enc.y)) << 8) |
                                                                    (static_cast<uint32_t>(unorm8(enc.z)) << 16) | (static_cast<uint32_t>(unorm8(cone)) << 24);
                    } else { // :115-118
                        const float ao = aoAcc / static_cast<float>(b.samples);
                        b.out[pixel] = unorm8(1.0f - ao);
                    }
                    active = false;
                }
            }
        }
    }
}

#include "ddgi_compose.inc"
#include "ddgi_reflections.inc"

} // namespace dev

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
hipError_t launch_probe_slots(const FrameArgs& f, hipStream_t s)
{
    const uint32_t n = f.window > f.R ? f.window : f.R;
    hipLaunchKernelGGL(dev::k_probe_slots, dim3((n + 255u) / 256u), dim3(256), 0, s, f);
    return hipGetLastError();
}

// Persistent traversal at 6 waves/SIMD (80 VGPRs, no spill; round 1: 3.43 vs 3.61 ms
// at the compiler's 5 on C4, 8 spilled and took 5.4 ms); COUNT variants run at the
// compiler's occupancy.
// Dual-step traversal at 6 waves/SIMD (80 VGPRs): the only spills (4 VGPRs) sit in
// the masked pass's alpha test. C4: 2.39 ms, against 2.51 at 5 waves (96 VGPRs, no
// spill) and 2.65 for one step per iteration at 6 waves.
constexpr int kTraceWpe = 6, kShadowWpe = 6;
const void* kernel_trace_ptr(bool count)
{
    return count ? reinterpret_cast<const void*>(&dev::k_trace<true, 1>) : reinterpret_cast<const void*>(&dev::k_trace<false, kTraceWpe>);
}

hipError_t launch_trace(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s)
{
    void* args[] = { const_cast<SceneArgs*>(&sc), const_cast<FrameArgs*>(&f) };
    return hipLaunchKernel(kernel_trace_ptr(count), dim3(blocks), dim3(kTraceBlock), args, 0, s);
}

// Co-resident workgroups of a persistent kernel on this device (cached per kernel).
static uint32_t persistentBlocks(const void* fn, int block, uint32_t fallback)
{
    static thread_local std::vector<std::pair<const void*, uint32_t>> cache;
    for (const auto& c : cache)
        if (c.first == fn) return c.second;
    int dev = 0, cus = 0, occ = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, block, 0) != hipSuccess || occ <= 0 || cus <= 0)
        return fallback;
    cache.emplace_back(fn, static_cast<uint32_t>(occ * cus));
    return cache.back().second;
}

// One-pass shading at <= 128 VGPRs, 4 waves/SIMD, no spill (round 1: 0.57 -> 0.50 ms
// at C4 against the compiler's 133 VGPRs, 3 waves). Round 3: 5 waves (96 VGPRs)
// spills 30 and shades in 0.525 instead of 0.469 ms (profiles/r03_ak).
constexpr int kShadeWpe = 4;
hipError_t launch_shade(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s)
{
    if (count) {
        hipLaunchKernelGGL((dev::k_shade<true, 1>), dim3(blocks), dim3(kShadeBlock), 0, s, sc, f);
    } else {
        const void* fn = reinterpret_cast<const void*>(&dev::k_shade<false, kShadeWpe>);
        hipLaunchKernelGGL((dev::k_shade<false, kShadeWpe>), dim3(persistentBlocks(fn, kShadeBlock, blocks)), dim3(kShadeBlock), 0, s, sc, f);
    }
    return hipGetLastError();
}

// One launch: the sun's list through the light-space BVH (when k_shadow_gen split it
// off; then the other lights' list in the same launch, kShadowSunWorld), or every
// shadow ray through the world BVHs.
hipError_t launch_trace_shadow(const SceneArgs& sc, const FrameArgs& f, uint32_t blocks, bool count, hipStream_t s)
{
    void* args[] = { const_cast<SceneArgs*>(&sc), const_cast<FrameArgs*>(&f) };
    const void* fn = kernel_trace_shadow_ptr(count);
    if (f.sun_rays && f.light_count <= 1u)
        fn = count ? reinterpret_cast<const void*>(&dev::k_trace_shadow<true, 1, dev::kShadowSun>)
                   : reinterpret_cast<const void*>(&dev::k_trace_shadow<false, kShadowWpe, dev::kShadowSun>);
    else if (f.sun_rays)
        fn = count ? reinterpret_cast<const void*>(&dev::k_trace_shadow<true, 1, dev::kShadowSunWorld>)
                   : reinterpret_cast<const void*>(&dev::k_trace_shadow<false, kShadowWpe, dev::kShadowSunWorld>);
    return hipLaunchKernel(fn, dim3(blocks), dim3(kTraceBlock), args, 0, s);
}

hipError_t launch_shadow_gen(const SceneArgs& sc, const FrameArgs& f, hipStream_t s)
{
    const uint32_t blocks = (f.window_rays + dev::kGenSpan - 1u) / dev::kGenSpan;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_shadow_gen<false>, dim3(blocks), dim3(256), 0, s, sc, f);
    return hipGetLastError();
}

hipError_t launch_seq_signal(uint32_t* word, uint32_t value, hipStream_t s)
{
    hipLaunchKernelGGL(dev::k_seq_signal, dim3(1), dim3(64), 0, s, word, value);
    return hipGetLastError();
}

hipError_t launch_seq_wait(const uint32_t* word, uint32_t value, uint32_t* timedOut, uint32_t* hostFlag, uint64_t timeoutTicks, hipStream_t s)
{
    hipLaunchKernelGGL(dev::k_seq_wait, dim3(1), dim3(64), 0, s, word, value, timedOut, hostFlag, timeoutTicks);
    return hipGetLastError();
}

hipError_t launch_fill_u32(void* p, uint64_t count, uint32_t value, hipStream_t s)
{
    if (count == 0) return hipSuccess;
    uint64_t blocks = (count + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(dev::k_fill_u32, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, static_cast<uint32_t*>(p), count, value);
    return hipGetLastError();
}

const void* kernel_shade_ptr(bool count)
{
    return count ? reinterpret_cast<const void*>(&dev::k_shade<true, 1>) : reinterpret_cast<const void*>(&dev::k_shade<false, kShadeWpe>);
}

const void* kernel_trace_shadow_ptr(bool count)
{
    return count ? reinterpret_cast<const void*>(&dev::k_trace_shadow<true, 1>) : reinterpret_cast<const void*>(&dev::k_trace_shadow<false, kShadowWpe>);
}

hipError_t launch_bake(const SceneArgs& sc, const BakeArgs& b, uint32_t blocks, int stage, hipStream_t s)
{
    if (stage == 0) hipLaunchKernelGGL(dev::k_bake_raster, dim3((b.tri_count + 255) / 256), dim3(256), 0, s, b);
    else if (stage == 1) hipLaunchKernelGGL(dev::k_bake_bary, dim3((b.W * b.H + 255) / 256), dim3(256), 0, s, b);
    else hipLaunchKernelGGL((dev::k_bake_ao<6>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, b);
    return hipGetLastError();
}

hipError_t launch_probe_debug(const FrameArgs& f, const ArkProbeDebugDesc& d, hipStream_t s)
{
    if (d.count == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_probe_debug, dim3((d.count + 255u) / 256u), dim3(256), 0, s, f, d);
    return hipGetLastError();
}

hipError_t launch_rt_reflections(const SceneArgs& sc, const FrameArgs& f, const ArkReflectionsDesc& r, uint32_t traceBlocks, uint32_t shadowBlocks,
                                 hipStream_t s)
{
    const uint64_t pixels = static_cast<uint64_t>(r.width) * r.height;
    const uint64_t slots = static_cast<uint64_t>((r.width + 7u) / 8u) * ((r.height + 7u) / 8u) * 64u;
    hipLaunchKernelGGL(dev::k_refl_setup, dim3(static_cast<uint32_t>((slots + dev::kReflSetupSpan - 1) / dev::kReflSetupSpan)), dim3(256), 0, s, f, r,
                       const_cast<float4*>(f.ray_list), const_cast<uint32_t*>(f.list_count));
    void* args[] = { const_cast<SceneArgs*>(&sc), const_cast<FrameArgs*>(&f) };
    hipError_t e = hipLaunchKernel(reinterpret_cast<const void*>(&dev::k_trace<false, 6, dev::ListRays>), dim3(traceBlocks), dim3(kTraceBlock), args, 0, s);
    if (e != hipSuccess) return e;
    if (f.light_count > 0) {
        hipLaunchKernelGGL(dev::k_shadow_gen<true>, dim3(static_cast<uint32_t>((pixels + dev::kGenSpan - 1) / dev::kGenSpan)), dim3(256), 0, s, sc, f);
        e = launch_trace_shadow(sc, f, shadowBlocks, false, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dev::k_refl_shade, dim3(static_cast<uint32_t>((pixels + 255) / 256)), dim3(256), 0, s, sc, f, r);
    return hipGetLastError();
}

hipError_t launch_lighting_compose(const FrameArgs& f, const ArkComposeDesc& c, hipStream_t s)
{
    if (c.width == 0 || c.height == 0) return hipSuccess;
    const uint64_t tiles = static_cast<uint64_t>((c.width + 63u) / 64u) * ((c.height + 3u) / 4u); // 64 x 4 tiles (ddgi_compose.inc)
    if (tiles > (1ull << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dev::k_lighting_compose, dim3(static_cast<uint32_t>((tiles + 7u) / 8u * 8u)), dim3(256), 0, s, f, c);
    return hipGetLastError();
}

} // namespace ark

