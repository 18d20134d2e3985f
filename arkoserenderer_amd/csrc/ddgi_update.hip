// ddgi_update.hip — the probe update of the DDGI path (kernel 4 of ddgi_kernels.hip):
// irradiance + visibility blend (probeUpdateIrradiance.comp, probeUpdateVisibility.comp),
// tile border copy (probeBorderCopy*.comp) and probe offsets (probeUpdateOffset.comp).
//
// Own translation unit: it is built with -fno-slp-vectorize. The loops are VALU
// bound, and on gfx950 a packed v_pk_*_f32 op costs the issue time of two plain ones
// (MI355X_MICROARCH.md: 64 FLOP/clk/SIMD either way) while SLP packing adds the
// v_mov shuffles that feed it (measured: 69 VALU incl. 19 v_mov per two-ray
// irradiance iteration packed, 80 plain ones unpacked, 30 of them 2-cycle pk ops).

#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/ark_ddgi.h"
#include "ddgi_device.h"
#include "ddgi_kernels.h"

namespace ark {
namespace dev {

// probeBorderCopyCorners.comp / probeBorderCopyEdges.comp for one tile of side
// res+2, as a (dst <- src) map over the 4*res+4 border texels (tile-local).

__device__ __forceinline__ void borderSource(int res, int b, int* dx, int* dy, int* sx, int* sy)
{
    const int side = res + 2;
    if (b < 4) { // corners (probeBorderCopyCorners.comp:20-51)
        int cx = b & 1, cy = b >> 1;
        int scx = (cx + 1) % 2, scy = (cy + 1) % 2;
        *dx = cx * (side - 1);
        *dy = cy * (side - 1);
        *sx = scx * (side - 1) + (scx == 0 ? 1 : -1);
        *sy = scy * (side - 1) + (scy == 0 ? 1 : -1);
        return;
    }
    // edges (probeBorderCopyEdges.comp:20-56)
    b -= 4;
    const int sideIdx = b / res, step = b % res;
    const int cornerX[4] = { 0, 1, 1, 0 }, cornerY[4] = { 0, 0, 1, 1 };
    const int stepX[4] = { 1, 0, -1, 0 }, stepY[4] = { 0, 1, 0, -1 };
    const int inIdx = (sideIdx + 1) % 4;
    int cX = cornerX[sideIdx] * (side - 1), cY = cornerY[sideIdx] * (side - 1);
    *dx = cX + (step + 1) * stepX[sideIdx];
    *dy = cY + (step + 1) * stepY[sideIdx];
    *sx = (cX + stepX[inIdx]) + (res - step) * stepX[sideIdx];
    *sy = (cY + stepY[inIdx]) + (res - step) * stepY[sideIdx];
}

// ---------------------------------------------------------------------------
// Probe update: irradiance + visibility blend, border copy, probe offsets
// (probeUpdateIrradiance.comp:22-79, probeUpdateVisibility.comp:24-63,
// probeBorderCopyCorners.comp, probeBorderCopyEdges.comp, probeUpdateOffset.comp:27-96).
//
// Octahedral symmetry. A tile texel (a, b) (odd integer coordinates, a = 2*tx+1-res)
// decodes to the direction t; the texel (-a, b) decodes to the x-mirror t' =
// (-t.x, t.y, t.z) and the texel (-(res-|b|)*sgn a, -(res-|a|)*sgn b) to the
// antipode -t, exactly: every coordinate is a dyadic rational, the decode's fold
// and normalize are sign-symmetric (tests/test_oracle_kat.py pins both tables).
// So {t, t', -t, -t'} is an orbit of four texels, one of them in the quadrant
// tx, ty < res/2; for a ray r with p = t*r (per component) and the dot contracted
// as a shader compiler does (last product fused, the oracle's dotFma):
//     dot(t, r)   = fma(tz, rz, px + py) =  d1       dot(-t, r)  = -d1
//     dot(t', r)  = fma(tz, rz, py - px) =  d2       dot(-t', r) = -d2
// each the same IEEE operations as that dot on that texel (negation is exact and
// commutes with round-to-nearest-even; for z = 0 texels only the sign of a zero dot
// can differ, whose weight is 0 either way). Sums of weighted terms are fmas too. At most one of d and -d is positive, so one pow(|d|, sharpness)
// serves both texels of a pair: the texel on the negative side gets weight +0,
// which adds exactly nothing (finite distances; radiance is multiplied by the
// same +0 as in the reference). One lane owns one orbit: 3 products, 4 sums and
// 2 pows per ray for 4 texels, instead of 4 dots and 4 pows.
//
// Workgroup: 4 probes. Waves 0..3: visibility of probe w (64 orbits = 256 texels);
// wave 4: irradiance of the 4 probes (16 orbits = 64 texels each, 16 lanes per
// probe). Rays, surfels and clamped distances are staged in LDS. The probe offsets
// are k_probe_offsets' (below).
// ---------------------------------------------------------------------------

// powi_(x, N) for a constant N: the same binary-exponentiation multiply sequence
template<int N>
__device__ __forceinline__ float powiN(float x)
{
    float result = 1.0f, base = x;
    int n = N;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (n & 1) result = result * base;
        n >>= 1;
        if (n == 0) break;
        base = base * base;
    }
    return result;
}

// Visibility weight of a non-negative |dot|: pow(|d|, sharpness) in the kernel's
// modes. MODE 0: sharpness 50 (default), 1: integral 1..64, 2: other powf_pos_ domain.
template<int MODE>
__device__ __forceinline__ float visWeightAbs(float a, float sharp, int ns)
{
    if (MODE == 0) return powiN<50>(a);
    if (MODE == 1) return a > 0.0f ? powi_(a, ns) : 0.0f;
    return a > 0.0f ? powf_pos_(a, sharp) : 0.0f;
}

struct UpdateLds {
    float4* ray;    // [P][R + pad]  rotated direction + clamped distance
    float* d2;      // [P][R + pad]  clamped distance squared
    uint2* rad;     // [P][R + pad]  raw fp16 surfel: radiance rgb + signed distance
    uint32_t* vis;  // [P][18*18]    visibility tile (interior + border)
    uint2* irr;     // [P][10*10]    irradiance tile
    uint32_t stride; // per-probe stride of ray/d2/rad (elements)
};

__device__ __forceinline__ UpdateLds updateLds(uint32_t R)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    UpdateLds L;
    L.stride = R + 4; // +4 elements: the 4 probes' rows start on different LDS banks
    unsigned char* p = smem;
    L.ray = reinterpret_cast<float4*>(p);
    p += sizeof(float4) * kUpdateProbes * L.stride;
    L.rad = reinterpret_cast<uint2*>(p);
    p += sizeof(uint2) * kUpdateProbes * L.stride;
    L.irr = reinterpret_cast<uint2*>(p);
    p += sizeof(uint2) * kUpdateProbes * 100;
    L.vis = reinterpret_cast<uint32_t*>(p);
    p += sizeof(uint32_t) * kUpdateProbes * 324;
    L.d2 = reinterpret_cast<float*>(p);
    return L;
}

size_t probe_update_lds_bytes(uint32_t R)
{
    const size_t stride = R + 4;
    return kUpdateProbes * (stride * (16 + 8 + 4) + 100 * 8 + 324 * 4); // 37.6 KB at R = 256: 4 workgroups per CU
}

// the orbit of quadrant texel (qx, qy) of a res x res tile: t, x-mirror t', antipode -t, -t'
__device__ __forceinline__ void orbitTexels(int res, int qx, int qy, int* tx, int* ty)
{
    const int h = res / 2;
    tx[0] = qx;          ty[0] = qy;
    tx[1] = res - 1 - qx; ty[1] = qy;
    tx[2] = qy + h;      ty[2] = qx + h;
    tx[3] = h - 1 - qy;  ty[3] = qx + h;
}

__device__ __forceinline__ V3 texelDirection(int res, int tx, int ty)
{
    float uvx = (static_cast<float>(tx) + 0.5f) / static_cast<float>(res);
    float uvy = (static_cast<float>(ty) + 0.5f) / static_cast<float>(res);
    return octahedralDecode(2.0f * uvx - 1.0f, 2.0f * uvy - 1.0f);
}

template<int MODE>
__device__ __forceinline__ void visibilityOrbit(const UpdateLds& L, int p, uint32_t R, V3 t, float sharp, float* nv0, float* nv1, float* tw)
{
    const float4* ray = L.ray + p * L.stride;
    const float* d2 = L.d2 + p * L.stride;
    const int ns = static_cast<int>(sharp);
#pragma unroll 2
    for (uint32_t s = 0; s < R; ++s) {
        const float4 r = ray[s];
        const float dd2 = d2[s];
        const float px = t.x * r.x, py = t.y * r.y;
        const float d1 = fmaf(t.z, r.z, px + py);
        const float d2v = fmaf(t.z, r.z, py - px);
        const float w1 = visWeightAbs<MODE>(fabsf_(d1), sharp, ns);
        const float w2 = visWeightAbs<MODE>(fabsf_(d2v), sharp, ns);
        const float w0 = d1 > 0.0f ? w1 : 0.0f, w2n = d1 > 0.0f ? 0.0f : w1;
        const float w1p = d2v > 0.0f ? w2 : 0.0f, w3 = d2v > 0.0f ? 0.0f : w2;
        // texel order: t, t', -t, -t'
        nv0[0] = fmaf(w0, r.w, nv0[0]);  nv1[0] = fmaf(w0, dd2, nv1[0]);  tw[0] += w0;
        nv0[1] = fmaf(w1p, r.w, nv0[1]); nv1[1] = fmaf(w1p, dd2, nv1[1]); tw[1] += w1p;
        nv0[2] = fmaf(w2n, r.w, nv0[2]); nv1[2] = fmaf(w2n, dd2, nv1[2]); tw[2] += w2n;
        nv0[3] = fmaf(w3, r.w, nv0[3]);  nv1[3] = fmaf(w3, dd2, nv1[3]);  tw[3] += w3;
    }
}

// any sharpness: each texel's dot and pow evaluated as the reference does
__device__ __forceinline__ void visibilityOrbitGeneric(const UpdateLds& L, int p, uint32_t R, const V3* dir, float sharp, float* nv0, float* nv1, float* tw)
{
    const float4* ray = L.ray + p * L.stride;
    const float* d2 = L.d2 + p * L.stride;
    for (uint32_t s = 0; s < R; ++s) {
        const float4 r = ray[s];
        const V3 rd = v3(r.x, r.y, r.z);
        for (int k = 0; k < 4; ++k) {
            const float weight = powf_(fmaxf_(0.0f, fmaf(dir[k].z, rd.z, dir[k].x * rd.x + dir[k].y * rd.y)), sharp);
            nv0[k] = fmaf(weight, r.w, nv0[k]);
            nv1[k] = fmaf(weight, d2[s], nv1[k]);
            tw[k] += weight;
        }
    }
}

__global__ void __launch_bounds__(kUpdateBlock) k_probe_update(FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    constexpr int IR = ARK_DDGI_IRRADIANCE_RES, VR = ARK_DDGI_VISIBILITY_RES;
    const uint32_t R = f.R;
    const UpdateLds L = updateLds(R);
    const int tid = threadIdx.x;
    const uint32_t slot0 = blockIdx.x * kUpdateProbes;

    // --- stage rays / surfels of the block's probes ---------------------------
    {
        const float gridMaxSpacing = fmaxf_(f.spacing[0], fmaxf_(f.spacing[1], f.spacing[2]));
        const float maxDistance = 1.5f * gridMaxSpacing; // probeUpdateVisibility.comp:45-48
        for (uint32_t i = tid; i < kUpdateProbes * R; i += kUpdateBlock) {
            const uint32_t p = i / R, s = i - p * R;
            const uint32_t slot = slot0 + p;
            if (slot >= f.window_probes) break;
            const GpuProbeSlot& ps = f.slots[slot];
            const float4 fb = f.fib[s];
            const V3 d = rotate(v3(fb.x, fb.y, fb.z), v3(ps.axis[0], ps.axis[1], ps.axis[2]), ps.angle_sin, ps.angle_cos);
            const uint2 sv = reinterpret_cast<const uint2*>(f.surfels)[static_cast<size_t>(slot) * f.Rmax + s];
            const float a = f16_to_f32(static_cast<uint16_t>(sv.y >> 16));
            const float dd = fminf_(fabsf_(a), maxDistance);
            L.ray[p * L.stride + s] = make_float4(d.x, d.y, d.z, dd);
            L.d2[p * L.stride + s] = square(dd);
            L.rad[p * L.stride + s] = sv; // fp16 as stored: converted where used (exact)
        }
    }
    __syncthreads();
    const float epsilon = 1e-9f * static_cast<float>(R);
    const int wv = tid >> 6, ln = tid & 63;
    if (wv < kUpdateProbes) {
        // --- visibility of probe wv: lane = orbit of quadrant texel (ln & 7, ln >> 3)
        const uint32_t slot = slot0 + wv;
        if (slot < f.window_probes) {
            const uint32_t probeIdx = f.slots[slot].probe_index;
            int tx[4], ty[4];
            orbitTexels(VR, ln & 7, ln >> 3, tx, ty);
            float nv0[4] = { 0.0f, 0.0f, 0.0f, 0.0f }, nv1[4] = { 0.0f, 0.0f, 0.0f, 0.0f }, tw[4] = { 0.0f, 0.0f, 0.0f, 0.0f };
            const float sharp = f.visibility_sharpness;
            const V3 t = texelDirection(VR, tx[0], ty[0]);
            if (sharp == 50.0f) {
                visibilityOrbit<0>(L, wv, R, t, sharp, nv0, nv1, tw);
            } else if (is_small_int_(sharp)) {
                visibilityOrbit<1>(L, wv, R, t, sharp, nv0, nv1, tw);
            } else if (sharp > 0.0f && sharp <= 64.0f && !is_root_exp_(sharp)) {
                visibilityOrbit<2>(L, wv, R, t, sharp, nv0, nv1, tw);
            } else {
                V3 dir[4];
                for (int k = 0; k < 4; ++k) dir[k] = texelDirection(VR, tx[k], ty[k]);
                visibilityOrbitGeneric(L, wv, R, dir, sharp, nv0, nv1, tw);
            }
            const uint32_t tilesPerSheet = static_cast<uint32_t>(f.X * f.Z); // ddgi/common.glsl:53-67
            const uint32_t sheetProbeIdx = probeIdx % tilesPerSheet;
            const int py = static_cast<int>(probeIdx / tilesPerSheet);
            const int px = static_cast<int>(sheetProbeIdx % static_cast<uint32_t>(f.X));
            const int pz = static_cast<int>(sheetProbeIdx / static_cast<uint32_t>(f.X));
            const int tileX = px + py * f.X, tileY = pz;
            uint32_t* tile = L.vis + wv * 324;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float den = fmaxf_(tw[k], epsilon);
                float a0 = nv0[k] / den, a1 = nv1[k] / den;
                const int ax = 1 + tileX * (VR + 2) + tx[k], ay = 1 + tileY * (VR + 2) + ty[k];
                uint32_t* g = reinterpret_cast<uint32_t*>(f.vis) + static_cast<size_t>(ay) * f.Wv + ax;
                const uint32_t old = *g;
                a0 = mixf(a0, f16_to_f32(static_cast<uint16_t>(old & 0xffffu)), f.hysteresis_visibility);
                a1 = mixf(a1, f16_to_f32(static_cast<uint16_t>(old >> 16)), f.hysteresis_visibility);
                const uint32_t nw = static_cast<uint32_t>(f32_to_f16(a0)) | (static_cast<uint32_t>(f32_to_f16(a1)) << 16);
                *g = nw;
                tile[(ty[k] + 1) * (VR + 2) + tx[k] + 1] = nw;
            }
        }
    } else {
        // --- irradiance of the 4 probes: 16 lanes per probe, lane = orbit ----------
        const int p = ln >> 4, j = ln & 15;
        const uint32_t slot = slot0 + p;
        const bool live = slot < f.window_probes;
        if (live) {
            int tx[4], ty[4];
            orbitTexels(IR, j & 3, j >> 2, tx, ty);
            const V3 t = texelDirection(IR, tx[0], ty[0]);
            const float4* ray = L.ray + p * L.stride;
            const uint2* rad = L.rad + p * L.stride;
            V3 acc[4] = { splat(0.0f), splat(0.0f), splat(0.0f), splat(0.0f) };
            float tw[4] = { 0.0f, 0.0f, 0.0f, 0.0f };
#pragma unroll 2
            for (uint32_t s = 0; s < R; ++s) {
                const float4 r = ray[s];
                const uint2 cw = rad[s];
                const float4 c = make_float4(f16_to_f32(static_cast<uint16_t>(cw.x & 0xffffu)), f16_to_f32(static_cast<uint16_t>(cw.x >> 16)),
                                             f16_to_f32(static_cast<uint16_t>(cw.y & 0xffffu)), 0.0f);
                const float px = t.x * r.x, py = t.y * r.y;
                const float d1 = fmaf(t.z, r.z, px + py);
                const float d2 = fmaf(t.z, r.z, py - px);
                float w[4];
                w[0] = fmaxf_(0.0f, d1);
                w[1] = fmaxf_(0.0f, d2);
                w[2] = fmaxf_(0.0f, -d1);
                w[3] = fmaxf_(0.0f, -d2);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    acc[k] = v3(fmaf(w[k], c.x, acc[k].x), fmaf(w[k], c.y, acc[k].y), fmaf(w[k], c.z, acc[k].z));
                    tw[k] += w[k];
                }
            }
            const uint32_t probeIdx = f.slots[slot].probe_index;
            const uint32_t tilesPerSheet = static_cast<uint32_t>(f.X * f.Z);
            const uint32_t sheetProbeIdx = probeIdx % tilesPerSheet;
            const int py = static_cast<int>(probeIdx / tilesPerSheet);
            const int px = static_cast<int>(sheetProbeIdx % static_cast<uint32_t>(f.X));
            const int pz = static_cast<int>(sheetProbeIdx / static_cast<uint32_t>(f.X));
            const int tileX = px + py * f.X, tileY = pz;
            uint2* tile = L.irr + p * 100;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                V3 newIrr = acc[k] / fmaxf_(tw[k], epsilon);
                newIrr = pow3(newIrr, 1.0f / 5.0f);
                const int ax = 1 + tileX * (IR + 2) + tx[k], ay = 1 + tileY * (IR + 2) + ty[k];
                uint2* g = reinterpret_cast<uint2*>(f.irr) + static_cast<size_t>(ay) * f.Wi + ax;
                const uint2 old = *g;
                const V3 o = v3(f16_to_f32(static_cast<uint16_t>(old.x & 0xffffu)), f16_to_f32(static_cast<uint16_t>(old.x >> 16)),
                                f16_to_f32(static_cast<uint16_t>(old.y & 0xffffu)));
                newIrr = mix3(newIrr, o, f.hysteresis_irradiance);
                uint2 nw;
                nw.x = static_cast<uint32_t>(f32_to_f16(newIrr.x)) | (static_cast<uint32_t>(f32_to_f16(newIrr.y)) << 16);
                nw.y = static_cast<uint32_t>(f32_to_f16(newIrr.z)) | (static_cast<uint32_t>(f32_to_f16(0.0f)) << 16);
                *g = nw;
                tile[(ty[k] + 1) * (IR + 2) + tx[k] + 1] = nw;
            }
        }
    }
    __syncthreads();
    // --- border texels of the updated tiles ------------------------------------
    // Tiles not updated this frame already hold border == f(interior) since their
    // last update (or the uniform clear), so copying borders of updated tiles only
    // equals the reference's all-tile pass.
    constexpr int VB = 4 * VR + 4, IB = 4 * IR + 4;
    for (int i = tid; i < kUpdateProbes * (VB + IB); i += kUpdateBlock) {
        const int p = i / (VB + IB), b = i - p * (VB + IB);
        const uint32_t slot = slot0 + p;
        if (slot >= f.window_probes) break;
        const uint32_t probeIdx = f.slots[slot].probe_index;
        const uint32_t tilesPerSheet = static_cast<uint32_t>(f.X * f.Z);
        const uint32_t sheetProbeIdx = probeIdx % tilesPerSheet;
        const int py = static_cast<int>(probeIdx / tilesPerSheet);
        const int px = static_cast<int>(sheetProbeIdx % static_cast<uint32_t>(f.X));
        const int pz = static_cast<int>(sheetProbeIdx / static_cast<uint32_t>(f.X));
        const int tileX = px + py * f.X, tileY = pz;
        int dx, dy, sx, sy;
        if (b < VB) {
            borderSource(VR, b, &dx, &dy, &sx, &sy);
            const uint32_t val = L.vis[p * 324 + sy * (VR + 2) + sx];
            reinterpret_cast<uint32_t*>(f.vis)[static_cast<size_t>(tileY * (VR + 2) + dy) * f.Wv + tileX * (VR + 2) + dx] = val;
        } else {
            borderSource(IR, b - VB, &dx, &dy, &sx, &sy);
            const uint2 val = L.irr[p * 100 + sy * (IR + 2) + sx];
            reinterpret_cast<uint2*>(f.irr)[static_cast<size_t>(tileY * (IR + 2) + dy) * f.Wi + tileX * (IR + 2) + dx] = val;
        }
    }
}

// ---------------------------------------------------------------------------
// Probe offsets (probeUpdateOffset.comp:27-96). Their only reader is a later frame's
// slot table (raygen.rgen:117-118: the ray origins), and their inputs - the window's
// ray directions and hit distances, the current offsets - are final once the primary
// traversal is: the distance the shader reads back from the ray's surfel is the hit
// record's t (front face), t * 0.2 (back face, t stored negative) or zFar (miss),
// rounded to fp16 as the surfel stores it (raygen.rgen:108-139). So this kernel runs
// right after the traversal, and with frames in flight the next frame's slot table
// and traversal follow it on the traversal stream (ark_ddgi.cpp updateImpl).
// P probes per workgroup (P * R = 1,024 summands per kind). Phase 1, all 256 threads
// (their hit loads in flight together): each ray's class and rotated direction give
// the six summands of its probe's sums - direction component c % 3 of a class-1 ray
// (near front face, c < 3) or a class-2 ray (back face), +0 for the others, exactly the
// `m ? v : 0` the sum adds - staged in LDS, and the class counts (LDS atomics). Phase 2:
// lane 6q + c adds its summands in ray order, as the shader's loop does, one LDS read and
// one add per ray. (Until round 3 the summing lanes also rotated every direction
// themselves: 256 dependent iterations of ~35 VALU on one wave, 31 us per launch even
// for 2,048 probes, on the traversal stream's critical path.)
constexpr int kOffsetBlock = 256;

__host__ __device__ __forceinline__ uint32_t offsetProbesPerBlock(uint32_t R)
{
    const uint32_t p = R ? 1024u / R : 1u;
    return p < 1u ? 1u : (p > 32u ? 32u : p);
}


// LDS bytes of one workgroup
__host__ __device__ __forceinline__ size_t offsetLdsBytes(uint32_t P, uint32_t R)
{
    return sizeof(float) * (static_cast<size_t>(P) * (6u * R + 8u) + 6u * P) + sizeof(uint32_t) * 2u * P;
}

__global__ void __launch_bounds__(kOffsetBlock) k_probe_offsets(FrameArgs f)
{
    if (frameAborted(f.abort_word)) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t R = f.R;
    const uint32_t P = offsetProbesPerBlock(R);
    const uint32_t stride = 6u * R + 8u; // floats per probe: +8 puts the probes' rows on different LDS banks
    float* valL = reinterpret_cast<float*>(smem);               // [P][R][6] summands
    float* sumL = valL + P * stride;                              // [P][6] sums
    uint32_t* cntL = reinterpret_cast<uint32_t*>(sumL + 6u * P);  // [P][2] class-1 / class-2 counts
    const uint32_t tid = threadIdx.x;
    const uint32_t slot0 = blockIdx.x * P;
    const float minAxialSpacing = fminf_(f.spacing[0], fminf_(f.spacing[1], f.spacing[2]));
    const float maxOffset = minAxialSpacing / 2.0f;
    for (uint32_t i = tid; i < 2u * P; i += kOffsetBlock) cntL[i] = 0u;
    __syncthreads();
    // 4 records per thread in flight at once
    constexpr uint32_t kBatch = 4;
    for (uint32_t i0 = 0; i0 < P * R; i0 += kBatch * kOffsetBlock) {
        GpuHit h[kBatch];
        float4 fb[kBatch];
        bool ok[kBatch];
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            const uint32_t i = i0 + k * kOffsetBlock + tid;
            const uint32_t p = i / R, s = i - p * R;
            ok[k] = i < P * R && slot0 + p < f.window_probes;
            if (ok[k]) {
                h[k] = f.hits[static_cast<size_t>(slot0 + p) * R + s];
                fb[k] = f.fib[s];
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kBatch; ++k) {
            if (!ok[k]) continue;
            const uint32_t i = i0 + k * kOffsetBlock + tid;
            const uint32_t p = i / R, s = i - p * R;
            // the surfel's distance (k_shade: miss, back face, front face)
            const float dist = h[k].tri == kNoHit ? f.z_far : (h[k].t < 0.0f ? h[k].t * 0.2f : h[k].t);
            const float a = f16_to_f32(f32_to_f16(dist));
            const uint32_t cls = (a > 0.0f && a < maxOffset) ? 1u : (a < 0.0f ? 2u : 0u);
            const GpuProbeSlot& ps = f.slots[slot0 + p];
            const V3 d = rotate(v3(fb[k].x, fb[k].y, fb[k].z), v3(ps.axis[0], ps.axis[1], ps.axis[2]), ps.angle_sin, ps.angle_cos);
            float* v = valL + p * stride + 6u * s;
            v[0] = cls == 1u ? d.x : 0.0f;
            v[1] = cls == 1u ? d.y : 0.0f;
            v[2] = cls == 1u ? d.z : 0.0f;
            v[3] = cls == 2u ? d.x : 0.0f;
            v[4] = cls == 2u ? d.y : 0.0f;
            v[5] = cls == 2u ? d.z : 0.0f;
            if (cls) atomicAdd(cntL + 2u * p + (cls - 1u), 1u);
        }
    }
    __syncthreads();
    if (tid < 6u * P && slot0 + tid / 6u < f.window_probes) {
        const float* v = valL + (tid / 6u) * stride + tid % 6u;
        float acc = 0.0f;
#pragma unroll 8
        for (uint32_t s = 0; s < R; ++s) acc += v[6u * s];
        sumL[tid] = acc;
    }
    __syncthreads();
    const uint32_t slot = slot0 + tid;
    if (tid < P && slot < f.window_probes) {
        const float* sm = sumL + 6u * tid;
        const V3 accumNearFrontfaceDir = v3(sm[0], sm[1], sm[2]);
        const V3 accumBackfaceDir = v3(sm[3], sm[4], sm[5]);
        const uint32_t nc = cntL[2u * tid], bc = cntL[2u * tid + 1u];
        const uint32_t probeIdx = f.slots[slot].probe_index;
        float4 cur = f.offsets[probeIdx];
        V3 currentOffset = v3(cur.x, cur.y, cur.z);
        V3 offset = splat(0.0f);
        const float stepSize = 0.125f, lerpSpeed = 10.0f;
        if (static_cast<float>(bc) / static_cast<float>(R) >= 0.25f)
            offset = offset + normalize(accumBackfaceDir) * stepSize;
        else if (nc >= 1)
            offset = offset - normalize(accumNearFrontfaceDir) * stepSize;
        else
            offset = offset - currentOffset * stepSize;
        V3 newOffset = currentOffset + offset;
        if (length(newOffset) > maxOffset) newOffset = maxOffset * normalize(newOffset);
        newOffset = mix3(newOffset, currentOffset, exp2f_(-lerpSpeed * f.delta_time));
        f.offsets[probeIdx] = make_float4(newOffset.x, newOffset.y, newOffset.z, 0.0f);
    }
}

} // namespace dev

hipError_t launch_probe_offsets(const FrameArgs& f, hipStream_t s)
{
    if (f.window_probes == 0 || !f.update_offsets) return hipSuccess;
    const uint32_t P = dev::offsetProbesPerBlock(f.R);
    const uint32_t blocks = (f.window_probes + P - 1) / P;
    const size_t lds = dev::offsetLdsBytes(P, f.R);
    static size_t lds_set = 0;
    if (lds > 65536 && lds > lds_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dev::k_probe_offsets), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        if (e != hipSuccess) return e;
        lds_set = lds;
    }
    hipLaunchKernelGGL(dev::k_probe_offsets, dim3(blocks), dim3(dev::kOffsetBlock), lds, s, f);
    return hipGetLastError();
}

hipError_t launch_probe_update(const FrameArgs& f, hipStream_t s)
{
    if (f.window_probes == 0) return hipSuccess;
    const uint32_t blocks = (f.window_probes + kUpdateProbes - 1) / kUpdateProbes;
    const size_t lds = dev::probe_update_lds_bytes(f.R);
    static size_t lds_set = 0;
    if (lds > 65536 && lds > lds_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dev::k_probe_update), hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        if (e != hipSuccess) return e;
        lds_set = lds;
    }
    hipLaunchKernelGGL(dev::k_probe_update, dim3(blocks), dim3(kUpdateBlock), lds, s, f);
    return hipGetLastError();
}

} // namespace ark
