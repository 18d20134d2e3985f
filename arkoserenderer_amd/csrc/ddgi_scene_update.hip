// ddgi_scene_update.hip — per-frame scene inputs on the device (include/ark_ddgi.h
// ark_ddgi_set_lights / ark_ddgi_set_instances), the reference's per-frame uploads of
// GpuScene::update (GpuScene.cpp:790-858 lights, :872-1009 TLAS instances + build).
//
//   k_store_lights   the context's spot lights from a by-value kernel argument into its
//                    device light buffer, in stream order (no host staging buffer whose
//                    reuse could race a copy still queued).
//   k_node_masks     the instances below each node (bit id mod 64), once per topology.
//   k_refit_nodes    one BVH8 level (deepest first), the nodes with a moved instance below
//                    them: the moved instances' records of their leaf slots re-transformed
//                    from the object-space pools in set_scene's fp32 operation order
//                    (ark_ddgi.cpp), each node's child boxes - leaf slots
//                    from their triangle records, internal children from the level below
//                    - inflated as the builder inflates them (bvh_builder.cpp writeNode),
//                    the node's quantization grid and outward-rounded child planes
//                    recomputed (quantGrid, collapse_bvh8). The world BVHs box world
//                    coordinates; the sun's light-space BVH its records' light
//                    coordinates, so it follows the motion instead of being dropped.
//   k_gather_records the shading records in an installed background rebuild's order.
// Every launch is stream-ordered behind the context's earlier work (ark_ddgi_set_instances_async):
// the boxes' inflation comes from the host with the launch (refitInflations: the
// instances' object-space boxes through their new transforms), no device round trip.
// Refitting never changes a hit: hits do not depend on the BVH's shape (the (instance,
// primitive) tie rule and conservative boxes), only on the triangle records,
// which equal a fresh set_scene's bit for bit.
#include <hip/hip_runtime.h>

#include "ddgi_kernels.h"

namespace ark {
namespace dev {

__global__ void __launch_bounds__(256) k_store_lights(LightBlock b, GpuSpotLight* __restrict__ dst)
{
    const uint32_t words = b.count * static_cast<uint32_t>(sizeof(GpuSpotLight) / 4u);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x) reinterpret_cast<uint32_t*>(dst)[i] = reinterpret_cast<const uint32_t*>(b.spots)[i];
}

// A dirty instance's triangle record re-transformed from its mesh's vertices in place
// (k_refit_nodes, for the triangles of the leaf slots it refits).
__device__ __forceinline__ void refitRecord(float4* rec, float4& t0, float4& t1, float4& t2, const RefitInstance& I, uint32_t prim,
                                            const uint32_t* __restrict__ indices, const float* __restrict__ positions)
{
    const float* M = I.m;
    float w[3][3];
    for (int k = 0; k < 3; ++k) {
        const uint32_t idx = indices[static_cast<size_t>(I.first_index) + 3u * prim + k];
        const float* P = positions + (static_cast<uint64_t>(static_cast<int64_t>(I.first_vertex)) + idx) * 3u;
        // ark_ddgi_set_scene's expression, left to right, no contraction
        w[k][0] = M[0] * P[0] + M[1] * P[1] + M[2] * P[2] + M[3];
        w[k][1] = M[4] * P[0] + M[5] * P[1] + M[6] * P[2] + M[7];
        w[k][2] = M[8] * P[0] + M[9] * P[1] + M[10] * P[2] + M[11];
    }
    // make_gpu_triangle: e1 = v1 - v0, e2 = v2 - v0
    const float e1x = w[1][0] - w[0][0], e1y = w[1][1] - w[0][1], e1z = w[1][2] - w[0][2];
    const float e2x = w[2][0] - w[0][0], e2y = w[2][1] - w[0][1], e2z = w[2][2] - w[0][2];
    t0 = make_float4(w[0][0], w[0][1], w[0][2], e1x);
    t1 = make_float4(e1y, e1z, e2x, e2y);
    t2.x = e2z;
    t2.w = __uint_as_float(I.flip);
    rec[0] = t0;
    rec[1] = t1;
    rec[2] = t2;
}

// The instances below each node (bit id mod 64 of every triangle's instance), one level
// per launch, deepest first, one thread per node: k_refit_nodes skips the nodes none of
// whose instances moved.
__global__ void __launch_bounds__(256) k_node_masks(const GpuBvh8Node* __restrict__ nodes, const GpuTriangle* __restrict__ tris, uint64_t* __restrict__ masks,
                                                    const uint32_t* __restrict__ order, uint32_t count)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= count) return;
    const uint32_t n = order[i];
    const GpuBvh8Node& nd = nodes[n];
    uint64_t m = 0;
    for (int s = 0; s < 8; ++s) {
        if ((nd.imask >> s) & 1u) {
            m |= masks[nd.child_base + static_cast<uint32_t>(__builtin_popcount(nd.imask & ((1u << s) - 1u)))];
        } else if ((nd.leaf_mask >> s) & 1u) {
            for (uint32_t k = 0; k < static_cast<uint32_t>(kBvh8MaxLeafSize); ++k) {
                const uint32_t pos = s + nd.tri_stride * k;
                if (pos >= 24u || !((nd.leaf_tris >> pos) & 1u)) break;
                const uint32_t id = __float_as_uint(reinterpret_cast<const float4*>(tris + nd.tri_base + pos)[2].y);
                m |= 1ull << (id & 63u);
            }
        }
    }
    masks[n] = m;
}

// The light coordinates of a record's three vertices as build_sun_bvh computes them
// (bvh_builder.cpp sunAddRecords: v0, v0 + e1, v0 + e2 in double, each rotated into the
// frame in double and rounded to fp32), and the largest |world coordinate|.
__device__ __forceinline__ void lightVertices(const float4 t0, const float4 t1, const float4 t2, const double* F, float L[3][3], float& maxAbs)
{
    double V[3][3];
    const double e1[3] = { t0.w, t1.x, t1.y }, e2[3] = { t1.z, t1.w, t2.x };
    V[0][0] = t0.x;
    V[0][1] = t0.y;
    V[0][2] = t0.z;
    maxAbs = 0.0f;
    for (int a = 0; a < 3; ++a) {
        V[1][a] = V[0][a] + e1[a];
        V[2][a] = V[0][a] + e2[a];
        maxAbs = fmaxf(maxAbs, static_cast<float>(fmax(fabs(V[0][a]), fmax(fabs(V[1][a]), fabs(V[2][a])))));
    }
    for (int k = 0; k < 3; ++k)
        for (int r = 0; r < 3; ++r) L[k][r] = static_cast<float>(F[3 * r + 0] * V[k][0] + F[3 * r + 1] * V[k][1] + F[3 * r + 2] * V[k][2]);
}

// bvh_builder.cpp writeNode's inflation of a child box: relative to its magnitude and
// extent, plus the scene's absolute inflation
__device__ __forceinline__ void inflateBox(float lo[3], float hi[3], float inflateAbs)
{
    float m = 0.0f, e = 0.0f;
    for (int a = 0; a < 3; ++a) {
        m = fmaxf(m, fmaxf(fabsf(lo[a]), fabsf(hi[a])));
        e = fmaxf(e, hi[a] - lo[a]);
    }
    const float eps = m * 2e-6f + e * 1e-5f + 1e-7f + inflateAbs;
    for (int a = 0; a < 3; ++a) {
        lo[a] -= eps;
        hi[a] += eps;
    }
}

// bvh_builder.cpp quantGrid: step 2^e, anchor p = k 2^e <= L with p + 255 2^e >= H and
// |k| + 256 < 2^24 (every plane p + q 2^e exact in fp32)
__device__ __forceinline__ void quantGrid(float L, float H, int& e, double& p)
{
    const double ext = static_cast<double>(H) - static_cast<double>(L);
    e = ext > 0.0 ? static_cast<int>(ceil(log2(ext / 255.0))) : -100;
    e = max(-100, e);
    for (;; ++e) {
        const double step = ldexp(1.0, e);
        const double k = floor(static_cast<double>(L) / step);
        if (fabs(k) + 256.0 >= 16777216.0) continue;
        p = k * step;
        if (p + 255.0 * step < static_cast<double>(H)) continue;
        return;
    }
}

// One level of the refit, eight lanes per node - lane s owns child slot s: its box (the
// child node's from the level below, or its leaf triangles'), the node's box by a
// reduction over the eight lanes, the node's grid (every lane alike), then the slot's
// outward-rounded planes. (One thread per node walked the eight slots and up to 24
// triangle records in a row: C4 refits took 4.0 ms, profiles/r06_f_refit_continuous_bg.log.)
__global__ void __launch_bounds__(128) k_refit_nodes(GpuBvh8Node* __restrict__ nodes, GpuTriangle* __restrict__ tris, float* __restrict__ boxes,
                                                     const uint32_t* __restrict__ order, uint32_t count, RefitBoxArgs ra, const uint64_t* __restrict__ masks,
                                                     const RefitInstance* __restrict__ inst, const uint32_t* __restrict__ indices,
                                                     const float* __restrict__ positions)
{
    // the refit runs beside the frame in flight's persistent kernels (the refit stream):
    // its few waves take the SIMDs' issue slots first, so that its chain of per-level
    // launches, which the next frame's traversal waits for, is not starved
    __builtin_amdgcn_s_setprio(3);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = t >> 3, s = t & 7u;
    const uint32_t n0 = i < count ? order[i] : 0u;
    // a node none of whose instances moved keeps its planes and its box (boxes[]) from
    // the last refit that reached it (the same transforms and inflation: RefitBoxArgs.dirty)
    const bool live = i < count && (masks[n0] & ra.dirty) != 0; // a node's eight lanes alike
    if (!__any(live)) return;
    const uint32_t n = live ? n0 : 0u;
    const float inflateAbs = ra.inflate;
    const uint4 hdr = live ? reinterpret_cast<const uint4*>(nodes + n)[1] : make_uint4(0u, 0u, 0u, 0u); // child_base, tri_base, leaf_tris, stride | leaf_mask << 8
    const uint32_t imask = live ? (reinterpret_cast<const uint32_t*>(nodes + n)[3] >> 24) : 0u;
    const uint32_t childBase = hdr.x, triBase = hdr.y, leafTris = hdr.z, stride = hdr.w & 0xffu, leafMask = (hdr.w >> 8) & 0xffu;
    float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    bool used = false;
    if ((imask >> s) & 1u) {
        // the child node's box (its level ran before this one), already inflated
        const float* b = boxes + 6u * static_cast<size_t>(childBase + static_cast<uint32_t>(__builtin_popcount(imask & ((1u << s) - 1u))));
        for (int a = 0; a < 3; ++a) {
            lo[a] = b[a];
            hi[a] = b[3 + a];
        }
        used = true;
    } else if ((leafMask >> s) & 1u) {
        // triangle k of the slot at tri_base + s + stride k, its row's consecutive bits
        for (uint32_t k = 0; k < static_cast<uint32_t>(kBvh8MaxLeafSize); ++k) {
            const uint32_t pos = s + stride * k;
            if (pos >= 24u || !((leafTris >> pos) & 1u)) break;
            float4* rec = reinterpret_cast<float4*>(tris + triBase + pos);
            float4 a = rec[0], b = rec[1], c = rec[2];
            // the record of a moved instance re-transformed here (each record is in one leaf slot)
            const RefitInstance& I = inst[__float_as_uint(c.y)];
            if (I.dirty) refitRecord(rec, a, b, c, I, __float_as_uint(c.z), indices, positions);
            if (ra.light) {
                // the light coordinates build_sun_bvh boxed
                float L[3][3], m;
                lightVertices(a, b, c, ra.frame, L, m);
                for (int ax = 0; ax < 3; ++ax) {
                    lo[ax] = fminf(lo[ax], fminf(L[0][ax], fminf(L[1][ax], L[2][ax])));
                    hi[ax] = fmaxf(hi[ax], fmaxf(L[0][ax], fmaxf(L[1][ax], L[2][ax])));
                }
                continue;
            }
            // the triangle Möller–Trumbore tests: v0, v0 + e1, v0 + e2
            const float v0[3] = { a.x, a.y, a.z }, e1[3] = { a.w, b.x, b.y }, e2[3] = { b.z, b.w, c.x };
            for (int ax = 0; ax < 3; ++ax) {
                const float p1 = v0[ax] + e1[ax], p2 = v0[ax] + e2[ax];
                lo[ax] = fminf(lo[ax], fminf(v0[ax], fminf(p1, p2)));
                hi[ax] = fmaxf(hi[ax], fmaxf(v0[ax], fmaxf(p1, p2)));
            }
        }
        inflateBox(lo, hi, inflateAbs);
        used = true;
    }
    // the node's box over its eight lanes (an unused slot contributes +-inf)
    float nlo[3] = { lo[0], lo[1], lo[2] }, nhi[3] = { hi[0], hi[1], hi[2] };
    for (int m = 1; m < 8; m <<= 1)
        for (int a = 0; a < 3; ++a) {
            nlo[a] = fminf(nlo[a], __shfl_xor(nlo[a], m, 8));
            nhi[a] = fmaxf(nhi[a], __shfl_xor(nhi[a], m, 8));
        }
    if (!live) return;
    // the node's grid (each lane alike) and this slot's planes, rounded outward (collapse_bvh8)
    GpuBvh8Node* nd = nodes + n;
    for (int a = 0; a < 3; ++a) {
        int e;
        double p;
        quantGrid(nlo[a], nhi[a], e, p);
        const double step = ldexp(1.0, e), inv = ldexp(1.0, -e); // exact: the step is a power of two
        if (s == 0) {
            nd->p[a] = static_cast<float>(p);
            nd->e[a] = static_cast<uint8_t>(e + 127);
        }
        if (!used) continue;
        double ql = floor((static_cast<double>(lo[a]) - p) * inv);
        double qh = ceil((static_cast<double>(hi[a]) - p) * inv);
        ql = fmin(255.0, fmax(0.0, ql));
        qh = fmin(255.0, fmax(0.0, qh));
        while (ql > 0.0 && static_cast<double>(static_cast<float>(p + ql * step)) > lo[a]) ql -= 1.0;
        while (qh < 255.0 && static_cast<double>(static_cast<float>(p + qh * step)) < hi[a]) qh += 1.0;
        nd->qlo[a][s] = static_cast<uint8_t>(ql);
        nd->qhi[a][s] = static_cast<uint8_t>(qh);
    }
    if (s == 0) {
        // this node's box as its parent's child box (inflated, as writeNode does per level)
        inflateBox(nlo, nhi, inflateAbs);
        float* b = boxes + 6u * static_cast<size_t>(n);
        for (int a = 0; a < 3; ++a) {
            b[a] = nlo[a];
            b[3 + a] = nhi[a];
        }
    }
}

// an installed rebuild's shading records in its record order: dst record i = src record
// perm[i] (holes: zeros), one float4 per thread
__global__ void __launch_bounds__(256) k_gather_records(float4* __restrict__ dst, const float4* __restrict__ src, const uint32_t* __restrict__ perm, uint64_t words)
{
    const uint64_t w = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    if (w >= words) return;
    const uint32_t from = perm[w >> 2];
    dst[w] = from == 0xffffffffu ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : src[static_cast<uint64_t>(from) * 4u + (w & 3u)];
}

} // namespace dev

hipError_t launch_store_lights(const LightBlock& b, GpuSpotLight* dst, hipStream_t s)
{
    if (b.count == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_store_lights, dim3(1), dim3(256), 0, s, b, dst);
    return hipGetLastError();
}

hipError_t launch_node_masks(const GpuBvh8Node* nodes, const GpuTriangle* tris, uint64_t* masks, const uint32_t* order, uint32_t count, hipStream_t s)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_node_masks, dim3((count + 255u) / 256u), dim3(256), 0, s, nodes, tris, masks, order, count);
    return hipGetLastError();
}

hipError_t launch_refit_nodes(GpuBvh8Node* nodes, GpuTriangle* tris, float* boxes, const uint32_t* order, uint32_t count, const RefitBoxArgs& a,
                              const uint64_t* masks, const RefitInstance* inst, const uint32_t* indices, const float* positions, hipStream_t s)
{
    if (count == 0) return hipSuccess;
    const uint64_t lanes = 8ull * count; // eight lanes per node
    hipLaunchKernelGGL(dev::k_refit_nodes, dim3(static_cast<uint32_t>((lanes + 127u) / 128u)), dim3(128), 0, s, nodes, tris, boxes, order, count, a, masks, inst, indices,
                       positions);
    return hipGetLastError();
}

hipError_t launch_gather_records(float4* dst, const float4* src, const uint32_t* perm, uint64_t count, hipStream_t s)
{
    if (count == 0) return hipSuccess;
    const uint64_t words = count * 4u; // four float4 per 64-B record
    hipLaunchKernelGGL(dev::k_gather_records, dim3(static_cast<uint32_t>((words + 255u) / 256u)), dim3(256), 0, s, dst, src, perm, words);
    return hipGetLastError();
}

} // namespace ark
