// ddgi_scene_update.hip — per-frame scene inputs on the device (include/ark_ddgi.h
// ark_ddgi_set_lights / ark_ddgi_set_instances), the reference's per-frame uploads of
// GpuScene::update (GpuScene.cpp:790-858 lights, :872-1009 TLAS instances + build).
//
//   k_store_lights   the context's spot lights from a by-value kernel argument into its
//                    device light buffer, in stream order (no host staging buffer whose
//                    reuse could race a copy still queued).
//   k_refit_tris     every world-space triangle record re-transformed from the object-
//                    space pools with the new instance transform, in set_scene's fp32
//                    operation order (ark_ddgi.cpp), + the scene bounds (for the boxes'
//                    absolute inflation).
//   k_refit_nodes    one BVH8 level (deepest first): each node's child boxes - leaf slots
//                    from their triangle records, internal children from the level below
//                    - inflated as the builder inflates them (bvh_builder.cpp writeNode),
//                    the node's quantization grid and outward-rounded child planes
//                    recomputed (quantGrid, collapse_bvh8).
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

// order-preserving float <-> u32 (for atomicMin / atomicMax of the scene bounds)
__device__ __forceinline__ uint32_t orderedBits(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(256) k_refit_tris(GpuTriangle* __restrict__ tris, uint32_t count, const RefitInstance* __restrict__ inst,
                                                    const uint32_t* __restrict__ indices, const float* __restrict__ positions, uint32_t* __restrict__ bounds)
{
    __shared__ uint32_t red[6];
    if (threadIdx.x < 6) red[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < count) {
        float4* rec = reinterpret_cast<float4*>(tris + i);
        float4 t2 = rec[2];
        const uint32_t id = __float_as_uint(t2.y), prim = __float_as_uint(t2.z);
        if (id != kHoleInstance) {
            const RefitInstance I = inst[id];
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
            rec[0] = make_float4(w[0][0], w[0][1], w[0][2], e1x);
            rec[1] = make_float4(e1y, e1z, e2x, e2y);
            t2.x = e2z;
            t2.w = __uint_as_float(I.flip);
            rec[2] = t2;
            for (int a = 0; a < 3; ++a) {
                const float lo = fminf(fminf(w[0][a], w[1][a]), w[2][a]), hi = fmaxf(fmaxf(w[0][a], w[1][a]), w[2][a]);
                atomicMin(&red[a], orderedBits(lo));
                atomicMax(&red[3 + a], orderedBits(hi));
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&bounds[threadIdx.x], red[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&bounds[threadIdx.x], red[threadIdx.x]);
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

__global__ void __launch_bounds__(128) k_refit_nodes(GpuBvh8Node* __restrict__ nodes, const GpuTriangle* __restrict__ tris, float* __restrict__ boxes,
                                                     const uint32_t* __restrict__ order, uint32_t count, float inflateAbs)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t n = order[i];
    GpuBvh8Node nd = nodes[n];
    float clo[8][3], chi[8][3];
    float nlo[3] = { INFINITY, INFINITY, INFINITY }, nhi[3] = { -INFINITY, -INFINITY, -INFINITY };
    uint32_t used = 0, internal = 0;
    for (int s = 0; s < 8; ++s) {
        float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
        if ((nd.imask >> s) & 1u) {
            // the child node's box (its level ran before this one), already inflated
            const float* b = boxes + 6u * static_cast<size_t>(nd.child_base + internal++);
            for (int a = 0; a < 3; ++a) {
                lo[a] = b[a];
                hi[a] = b[3 + a];
            }
        } else if ((nd.leaf_mask >> s) & 1u) {
            // triangle i of the slot at tri_base + s + stride i, its row's consecutive bits
            for (uint32_t k = 0; k < static_cast<uint32_t>(kBvh8MaxLeafSize); ++k) {
                const uint32_t pos = static_cast<uint32_t>(s) + nd.tri_stride * k;
                if (pos >= 24u || !((nd.leaf_tris >> pos) & 1u)) break;
                const float4* rec = reinterpret_cast<const float4*>(tris + nd.tri_base + pos);
                const float4 a = rec[0], b = rec[1], c = rec[2];
                // the triangle Möller–Trumbore tests: v0, v0 + e1, v0 + e2
                const float v0[3] = { a.x, a.y, a.z }, e1[3] = { a.w, b.x, b.y }, e2[3] = { b.z, b.w, c.x };
                for (int ax = 0; ax < 3; ++ax) {
                    const float p1 = v0[ax] + e1[ax], p2 = v0[ax] + e2[ax];
                    lo[ax] = fminf(lo[ax], fminf(v0[ax], fminf(p1, p2)));
                    hi[ax] = fmaxf(hi[ax], fmaxf(v0[ax], fmaxf(p1, p2)));
                }
            }
            inflateBox(lo, hi, inflateAbs);
        } else {
            continue;
        }
        used |= 1u << s;
        for (int a = 0; a < 3; ++a) {
            clo[s][a] = lo[a];
            chi[s][a] = hi[a];
            nlo[a] = fminf(nlo[a], lo[a]);
            nhi[a] = fmaxf(nhi[a], hi[a]);
        }
    }
    // the node's grid and its children's planes, rounded outward (collapse_bvh8)
    double step[3], p[3];
    for (int a = 0; a < 3; ++a) {
        int e;
        quantGrid(nlo[a], nhi[a], e, p[a]);
        step[a] = ldexp(1.0, e);
        nd.p[a] = static_cast<float>(p[a]);
        nd.e[a] = static_cast<uint8_t>(e + 127);
    }
    for (int s = 0; s < 8; ++s) {
        if (!((used >> s) & 1u)) continue;
        for (int a = 0; a < 3; ++a) {
            double ql = floor((static_cast<double>(clo[s][a]) - p[a]) / step[a]);
            double qh = ceil((static_cast<double>(chi[s][a]) - p[a]) / step[a]);
            ql = fmin(255.0, fmax(0.0, ql));
            qh = fmin(255.0, fmax(0.0, qh));
            while (ql > 0.0 && static_cast<double>(static_cast<float>(p[a] + ql * step[a])) > clo[s][a]) ql -= 1.0;
            while (qh < 255.0 && static_cast<double>(static_cast<float>(p[a] + qh * step[a])) < chi[s][a]) qh += 1.0;
            nd.qlo[a][s] = static_cast<uint8_t>(ql);
            nd.qhi[a][s] = static_cast<uint8_t>(qh);
        }
    }
    nodes[n] = nd;
    // this node's box as its parent's child box (inflated, as writeNode does per level)
    inflateBox(nlo, nhi, inflateAbs);
    float* b = boxes + 6u * static_cast<size_t>(n);
    for (int a = 0; a < 3; ++a) {
        b[a] = nlo[a];
        b[3 + a] = nhi[a];
    }
}

} // namespace dev

hipError_t launch_store_lights(const LightBlock& b, GpuSpotLight* dst, hipStream_t s)
{
    if (b.count == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_store_lights, dim3(1), dim3(256), 0, s, b, dst);
    return hipGetLastError();
}

hipError_t launch_refit_tris(GpuTriangle* tris, uint32_t count, const RefitInstance* inst, const uint32_t* indices, const float* positions, uint32_t* bounds,
                             hipStream_t s)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_refit_tris, dim3((count + 255u) / 256u), dim3(256), 0, s, tris, count, inst, indices, positions, bounds);
    return hipGetLastError();
}

hipError_t launch_refit_nodes(GpuBvh8Node* nodes, const GpuTriangle* tris, float* boxes, const uint32_t* order, uint32_t count, float inflateAbs, hipStream_t s)
{
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::k_refit_nodes, dim3((count + 127u) / 128u), dim3(128), 0, s, nodes, tris, boxes, order, count, inflateAbs);
    return hipGetLastError();
}

} // namespace ark
