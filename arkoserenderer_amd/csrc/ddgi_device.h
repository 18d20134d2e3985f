// ddgi_device.h — device-side math for the DDGI kernels (gfx950).
//
// Every function restates the reference GLSL with the same per-component
// evaluation order as the CPU oracle (oracle/ddgi_oracle.cpp), so that with
// -ffp-contract=off and ark_fmath.h the HIP path is bit-exact against it.
// Reference citations are on each function.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ark_fmath.h"
#include "../../include/ark_ddgi.h"
#include "ddgi_types.h"

namespace ark {
namespace dev {

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return { x, y, z }; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return { a.x + b.x, a.y + b.y, a.z + b.z }; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
__device__ __forceinline__ V3 operator-(V3 a) { return { -a.x, -a.y, -a.z }; }
__device__ __forceinline__ V3 operator*(V3 a, V3 b) { return { a.x * b.x, a.y * b.y, a.z * b.z }; }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return { a.x * s, a.y * s, a.z * s }; }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return { s * a.x, s * a.y, s * a.z }; }
__device__ __forceinline__ V3 operator/(V3 a, float s) { return { a.x / s, a.y / s, a.z / s }; }
__device__ __forceinline__ V3 operator/(V3 a, V3 b) { return { a.x / b.x, a.y / b.y, a.z / b.z }; }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) { return { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x }; }
__device__ __forceinline__ float length(V3 a) { return sqrtf_(dot(a, a)); }
__device__ __forceinline__ V3 normalize(V3 a) { float s = 1.0f / sqrtf_(dot(a, a)); return a * s; }
__device__ __forceinline__ float saturate(float x) { return fminf_(fmaxf_(x, 0.0f), 1.0f); }
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf_(fmaxf_(x, lo), hi); }
__device__ __forceinline__ float square(float x) { return x * x; }
__device__ __forceinline__ float mixf(float x, float y, float a) { return x * (1.0f - a) + y * a; }
__device__ __forceinline__ V3 mix3(V3 x, V3 y, float a) { return { mixf(x.x, y.x, a), mixf(x.y, y.y, a), mixf(x.z, y.z, a) }; }
__device__ __forceinline__ V3 pow3(V3 v, float e) { return { powf_(v.x, e), powf_(v.y, e), powf_(v.z, e) }; }
__device__ __forceinline__ V3 splat(float s) { return { s, s, s }; }
__device__ __forceinline__ float lerpf(float a, float b, float t) { return a + (b - a) * t; }

// fp16 storage (RNE, NaN canonicalised to 0x7e00 like the oracle)
__device__ __forceinline__ uint16_t f32_to_f16(float f)
{
    // The empty asm makes the fp32 value opaque: without it the backend may fuse
    // the producing fmul/fma with the conversion (v_mad_mix* rounds the exact
    // product to f16 once), which differs from fp32-then-f16 on fp16 ties.
    asm volatile("" : "+v"(f));
    if (f != f) return 0x7e00u;
    return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) { return static_cast<float>(__builtin_bit_cast(_Float16, h)); }

// random.glsl:25-48
__device__ __forceinline__ uint32_t wang_hash(uint32_t seed)
{
    seed = (seed ^ 61u) ^ (seed >> 16);
    seed *= 9u;
    seed = seed ^ (seed >> 4);
    seed *= 0x27d4eb2du;
    seed = seed ^ (seed >> 15);
    return seed;
}
__device__ __forceinline__ uint32_t rand_xorshift(uint32_t state)
{
    state ^= (state << 13);
    state ^= (state >> 17);
    state ^= (state << 5);
    return state;
}
__device__ __forceinline__ float randomFloat(uint32_t& state)
{
    state = rand_xorshift(state);
    return static_cast<float>(state) * (1.0f / 4294967296.0f);
}

// axisAngleRotate (common.glsl:133-142) with sin/cos of the per-probe angle hoisted.
__device__ __forceinline__ V3 rotate(V3 v, V3 k, float s, float c)
{
    return v * c + cross(k, v) * s + k * dot(k, v) * (1.0f - c);
}

// octahedral.glsl:10-41
__device__ __forceinline__ float signNotZero(float f) { return (f >= 0.0f) ? 1.0f : -1.0f; }
__device__ __forceinline__ void octahedralEncode(V3 v, float* ox, float* oy)
{
    float l1norm = fabsf_(v.x) + fabsf_(v.y) + fabsf_(v.z);
    float inv = 1.0f / l1norm;
    float rx = v.x * inv, ry = v.y * inv;
    if (v.z < 0.0f) {
        float nx = (1.0f - fabsf_(ry)) * signNotZero(rx);
        float ny = (1.0f - fabsf_(rx)) * signNotZero(ry);
        rx = nx;
        ry = ny;
    }
    *ox = rx;
    *oy = ry;
}
__device__ __forceinline__ V3 octahedralDecode(float ox, float oy)
{
    V3 v = { ox, oy, 1.0f - fabsf_(ox) - fabsf_(oy) };
    if (v.z < 0.0f) {
        float nx = (1.0f - fabsf_(v.y)) * signNotZero(v.x);
        float ny = (1.0f - fabsf_(v.x)) * signNotZero(v.y);
        v.x = nx;
        v.y = ny;
    }
    return normalize(v);
}

// spherical.glsl:6-13
__device__ __forceinline__ void sphericalUvFromDirection(V3 d, float* u, float* v)
{
    float phi = atan2f_(d.z, d.x);
    float theta = acosf_(clampf(d.y, -1.0f, 1.0f));
    if (phi < 0.0f) phi += kTwoPi;
    *u = phi / kTwoPi;
    *v = theta / kPi;
}

// Texel wrap of one axis (GpuTextureInfo.wrap: s in bits 0-3, t in 4-7, normalised
// by ark_ddgi_set_scene): clamp to edge, mirrored repeat (period 2n, the second
// half reversed) or repeat.
__device__ __forceinline__ int wrapCoord(int i, int n, int wrap)
{
    if (wrap == ARK_WRAP_CLAMP_TO_EDGE) return min(max(i, 0), n - 1);
    if (wrap == ARK_WRAP_MIRRORED_REPEAT) {
        int m = i % (2 * n);
        m = m < 0 ? m + 2 * n : m;
        return m < n ? m : 2 * n - 1 - m;
    }
    int m = i % n;
    return m < 0 ? m + n : m;
}

// Bilinear LOD-0 fetch from a decoded float4 texture (see oracle sampleBilinear).
__device__ __forceinline__ float4 sampleTexture(const GpuTextureInfo* __restrict__ infos, const float4* __restrict__ texels, int idx, float u, float v)
{
    const GpuTextureInfo ti = infos[idx];
    float x = u * static_cast<float>(ti.width) - 0.5f;
    float y = v * static_cast<float>(ti.height) - 0.5f;
    float x0f = floorf_(x), y0f = floorf_(y);
    float fx = x - x0f, fy = y - y0f;
    int x0 = static_cast<int>(x0f), y0 = static_cast<int>(y0f);
    const int ws = ti.wrap & 0xf, wt = (ti.wrap >> 4) & 0xf;
    int xa = wrapCoord(x0, ti.width, ws), xb = wrapCoord(x0 + 1, ti.width, ws);
    int ya = wrapCoord(y0, ti.height, wt), yb = wrapCoord(y0 + 1, ti.height, wt);
    const float4* base = texels + ti.texel_offset;
    float4 t00 = base[static_cast<size_t>(ya) * ti.width + xa];
    float4 t10 = base[static_cast<size_t>(ya) * ti.width + xb];
    float4 t01 = base[static_cast<size_t>(yb) * ti.width + xa];
    float4 t11 = base[static_cast<size_t>(yb) * ti.width + xb];
    float4 r;
    r.x = lerpf(lerpf(t00.x, t10.x, fx), lerpf(t01.x, t11.x, fx), fy);
    r.y = lerpf(lerpf(t00.y, t10.y, fx), lerpf(t01.y, t11.y, fx), fy);
    r.z = lerpf(lerpf(t00.z, t10.z, fx), lerpf(t01.z, t11.z, fx), fy);
    r.w = lerpf(lerpf(t00.w, t10.w, fx), lerpf(t01.w, t11.w, fx), fy);
    return r;
}

// brdf.glsl:17-148 (Filament BRDF) -------------------------------------------
constexpr float kDielectricReflectance = 0.04f;

__device__ __forceinline__ float D_GGX(float NdotH, float a)
{
    float a2 = a * a;
    float f = (NdotH * a2 - NdotH) * NdotH + 1.0f;
    return a2 / (kPi * f * f + 1e-20f);
}
__device__ __forceinline__ float F_Schlick1(float VdotH, float f0) { return f0 + (1.0f - f0) * powf_(1.0f - VdotH, 5.0f); }
__device__ __forceinline__ V3 F_Schlick3(float VdotH, V3 f0)
{
    float p = powf_(1.0f - VdotH, 5.0f);
    return f0 + (splat(1.0f) - f0) * p;
}
__device__ __forceinline__ float V_SmithGGXCorrelated(float NdotV, float NdotL, float a)
{
    float a2 = a * a;
    float GGXL = NdotV * sqrtf_((-NdotL * a2 + NdotL) * NdotL + a2);
    float GGXV = NdotL * sqrtf_((-NdotV * a2 + NdotV) * NdotV + a2);
    return 0.5f / (GGXV + GGXL + 1e-20f);
}
__device__ __forceinline__ V3 evaluateDefaultBRDF(V3 L, V3 V, V3 N, V3 baseColor, float roughness, float metallic, float clearcoat, float ccRough)
{
    // clearcoatBRDF (brdf.glsl:55-68)
    V3 H = normalize(L + V);
    float NdotHc = saturate(dot(N, H));
    float LdotHc = saturate(dot(L, H));
    float ac = square(clampf(ccRough, 0.1f, 1.0f));
    float Dc = D_GGX(NdotHc, ac);
    float Vc = 0.25f / square(LdotHc);
    float F_c = F_Schlick1(LdotHc, kDielectricReflectance) * clearcoat;
    float Fr_c = Dc * Vc * F_c;
    // specularBRDF (brdf.glsl:70-89)
    V3 Hs = normalize(L + V);
    float NdotV = fabsf_(dot(N, V)) + 1e-5f;
    float NdotL = clampf(dot(N, L), 0.0f, 1.0f);
    float NdotH = clampf(dot(N, Hs), 0.0f, 1.0f);
    float LdotH = clampf(dot(L, Hs), 0.0f, 1.0f);
    float a = square(roughness);
    V3 f0 = mix3(splat(kDielectricReflectance), baseColor, metallic);
    V3 F_s = F_Schlick3(LdotH, f0);
    float D = D_GGX(NdotH, a);
    float Vv = V_SmithGGXCorrelated(NdotV, NdotL, a);
    V3 Fr_s = F_s * D * Vv;
    V3 diffuseColor = splat(1.0f - metallic) * baseColor;
    V3 Fr_d = diffuseColor * splat(1.0f / kPi);
    return (Fr_d * (splat(1.0f) - F_s) + Fr_s) * (1.0f - F_c) + splat(Fr_c);
}

} // namespace dev
} // namespace ark
