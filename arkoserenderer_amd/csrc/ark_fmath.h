// ark_fmath.h — deterministic fp32 scalar math for the DDGI path.
//
// The reference evaluates GLSL built-ins (sin, cos, acos, atan, pow, exp2) whose
// precision is implementation-defined (GLSL 4.60 §4.7.1 allows e.g. 2^-11 absolute
// error for sin/cos) and that differ between every GPU vendor and libm. To make the
// HIP kernels reproduce the CPU oracle bit for bit, both sides evaluate these
// functions with the SAME algorithm built only from IEEE-754 operations that are
// correctly rounded on gfx950 and x86-64 alike (+ - * / sqrt fma floor rint):
// Cody-Waite range reduction + minimax polynomials (Cephes single precision
// coefficients, S. L. Moshier). Accuracy vs. double-precision libm is pinned by
// tests/test_fmath.py (<= 2 ulp for sin/cos/acos/atan2/log2/exp2 on the ranges used).
//
// Both sides must be compiled with -ffp-contract=off so that only the explicit
// fmaf() calls below fuse.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define ARK_HD __host__ __device__ __forceinline__
#else
#define ARK_HD static inline
#endif

namespace ark {

constexpr float kPi = 0x1.921fb6p+1f;        // float(3.14159265358979323846) (common.glsl:4)
constexpr float kTwoPi = 0x1.921fb6p+2f;     // 2.0 * PI in fp32 (common.glsl:5), exact
constexpr float kHalfPi = 0x1.921fb6p+0f;
constexpr float kQuarterPi = 0x1.921fb6p-1f;
constexpr float kGoldenRatio = 1.618034f;    // common.glsl:7

ARK_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
ARK_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
ARK_HD float fmaf_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
ARK_HD float sqrtf_(float x) { return __builtin_sqrtf(x); }
ARK_HD float floorf_(float x) { return __builtin_floorf(x); }
ARK_HD float rintf_(float x) { return __builtin_rintf(x); }
ARK_HD float fabsf_(float x) { return __builtin_fabsf(x); }
ARK_HD bool isnan_(float x) { return x != x; }
ARK_HD float inf_() { return u2f(0x7f800000u); }
ARK_HD float nan_() { return u2f(0x7fc00000u); }

// GLSL max/min: NaN handling as fmaxf/fminf (a NaN operand yields the other operand).
ARK_HD float fmaxf_(float a, float b) { return __builtin_fmaxf(a, b); }
ARK_HD float fminf_(float a, float b) { return __builtin_fminf(a, b); }

// sin and cos of x, |x| < 2^17. Quadrant reduction by pi/2 split into three fp32
// parts; fmaf keeps each reduction step exactly rounded.
ARK_HD void sincosf_(float x, float* s, float* c)
{
    const float k = rintf_(x * 0x1.45f306p-1f); // x * 2/pi
    float r = fmaf_(-k, 0x1.921fb6p+0f, x);
    r = fmaf_(-k, -0x1.777a5cp-25f, r);
    r = fmaf_(-k, -0x1.ee59dap-50f, r);
    const int q = static_cast<int>(k) & 3;
    const float z = r * r;
    // Cephes sinf/cosf polynomials on [-pi/4, pi/4]
    float ps = fmaf_(z, -1.9515295891e-4f, 8.3321608736e-3f);
    ps = fmaf_(z, ps, -1.6666654611e-1f);
    const float sn = fmaf_(r * z, ps, r);
    float pc = fmaf_(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    pc = fmaf_(z, pc, 4.166664568298827e-2f);
    const float cs = fmaf_(z * z, pc, fmaf_(-0.5f, z, 1.0f));
    float so, co;
    switch (q) {
    case 0: so = sn; co = cs; break;
    case 1: so = cs; co = -sn; break;
    case 2: so = -sn; co = -cs; break;
    default: so = -cs; co = sn; break;
    }
    *s = so;
    *c = co;
}
ARK_HD float sinf_(float x) { float s, c; sincosf_(x, &s, &c); return s; }
ARK_HD float cosf_(float x) { float s, c; sincosf_(x, &s, &c); return c; }

// asin on [0, 0.5] (Cephes asinf polynomial)
ARK_HD float asin_core_(float x)
{
    const float z = x * x;
    float p = fmaf_(z, 4.2163199048e-2f, 2.4181311049e-2f);
    p = fmaf_(z, p, 4.5470025998e-2f);
    p = fmaf_(z, p, 7.4953002686e-2f);
    p = fmaf_(z, p, 1.6666752422e-1f);
    return fmaf_(x * z, p, x);
}

ARK_HD float acosf_(float x)
{
    if (isnan_(x) || x < -1.0f || x > 1.0f)
        return nan_();
    if (x < -0.5f)
        return kPi - 2.0f * asin_core_(sqrtf_(0.5f * (1.0f + x)));
    if (x > 0.5f)
        return 2.0f * asin_core_(sqrtf_(0.5f * (1.0f - x)));
    const float a = asin_core_(fabsf_(x));
    return kHalfPi - (x < 0.0f ? -a : a);
}

ARK_HD float atanf_(float x)
{
    const bool neg = x < 0.0f;
    float a = fabsf_(x);
    float y;
    if (a > 2.414213562373095f) {
        y = kHalfPi;
        a = -(1.0f / a);
    } else if (a > 0.4142135623730950f) {
        y = kQuarterPi;
        a = (a - 1.0f) / (a + 1.0f);
    } else {
        y = 0.0f;
    }
    const float z = a * a;
    float p = fmaf_(z, 8.05374449538e-2f, -1.38776856032e-1f);
    p = fmaf_(z, p, 1.99777106478e-1f);
    p = fmaf_(z, p, -3.33329491539e-1f);
    y = y + fmaf_(p * z, a, a);
    return neg ? -y : y;
}

// GLSL atan(y, x)
ARK_HD float atan2f_(float y, float x)
{
    if (isnan_(x) || isnan_(y))
        return nan_();
    if (x == 0.0f) {
        if (y < 0.0f) return -kHalfPi;
        if (y == 0.0f) return 0.0f;
        return kHalfPi;
    }
    if (y == 0.0f)
        return x < 0.0f ? kPi : 0.0f;
    float w = 0.0f;
    if (x < 0.0f)
        w = (y < 0.0f) ? -kPi : kPi;
    return w + atanf_(y / x);
}

// log2 (Cephes log2f)
ARK_HD float log2f_(float x)
{
    if (isnan_(x) || x < 0.0f) return nan_();
    if (x == 0.0f) return -inf_();
    if (x == inf_()) return x;
    int e = 0;
    if (x < 0x1p-126f) { x *= 0x1p+23f; e = -23; }
    const uint32_t u = f2u(x);
    e += static_cast<int>((u >> 23) & 0xffu) - 126;
    float m = u2f((u & 0x007fffffu) | 0x3f000000u); // [0.5, 1)
    if (m < 0.70710678118654752440f) {
        e -= 1;
        m = m + m - 1.0f;
    } else {
        m = m - 1.0f;
    }
    const float z = m * m;
    float p = fmaf_(m, 7.0376836292e-2f, -1.1514610310e-1f);
    p = fmaf_(m, p, 1.1676998740e-1f);
    p = fmaf_(m, p, -1.2420140846e-1f);
    p = fmaf_(m, p, 1.4249322787e-1f);
    p = fmaf_(m, p, -1.6668057665e-1f);
    p = fmaf_(m, p, 2.0000714765e-1f);
    p = fmaf_(m, p, -2.4999993993e-1f);
    p = fmaf_(m, p, 3.3333331174e-1f);
    float y = m * (z * p);
    y = fmaf_(-0.5f, z, y);
    // log2(1+m) = (m + y) * log2(e), with log2(e) = 1 + 0.44269504...
    const float LOG2EA = 0.44269504088896340736f;
    float r = y * LOG2EA;
    r = fmaf_(m, LOG2EA, r);
    r = r + y;
    r = r + m;
    return r + static_cast<float>(e);
}

// 2^x (Cephes exp2f)
ARK_HD float exp2f_(float x)
{
    if (isnan_(x)) return x;
    if (x > 128.0f) return inf_();
    if (x < -151.0f) return 0.0f;
    const float i = floorf_(x + 0.5f);
    const float f = x - i;
    float p = fmaf_(f, 1.535336188319500e-4f, 1.339887440266574e-3f);
    p = fmaf_(f, p, 9.618437357674640e-3f);
    p = fmaf_(f, p, 5.550332471162809e-2f);
    p = fmaf_(f, p, 2.402264791363012e-1f);
    p = fmaf_(f, p, 6.931472028550421e-1f);
    float r = fmaf_(f, p, 1.0f);
    int n = static_cast<int>(i);
    // scale by 2^n in at most two exact power-of-two steps
    if (n > 127) { r *= 0x1p+127f; n -= 127; }
    if (n < -126) { r *= 0x1p-126f; n += 126; }
    if (n < -126) return 0.0f;
    return r * u2f(static_cast<uint32_t>(n + 127) << 23);
}

// x^n for an integer n >= 1 by right-to-left binary exponentiation (exact
// multiply order fixed here; <= ~log2(n)+popcount(n) roundings).
ARK_HD float powi_(float x, int n)
{
    float result = 1.0f, base = x;
    for (;;) {
        if (n & 1) result = result * base;
        n >>= 1;
        if (n == 0) break;
        base = base * base;
    }
    return result;
}

ARK_HD bool is_small_int_(float y) { return y >= 1.0f && y <= 64.0f && floorf_(y) == y; }

// Exponents with a square-root form: 1/4, 1/2 and n + 1/2 for n in 1..16.
ARK_HD bool is_root_exp_(float y) { return y == 0.25f || y == 0.5f || (y > 1.0f && y <= 16.5f && floorf_(y) + 0.5f == y); }

// GLSL pow(x, y) for x >= 0 (x < 0 is undefined in GLSL; NaN here). Integral
// exponents 1..64 (Schlick's ^5, the visibility sharpness 50) use powi_: about as
// accurate as exp2(y*log2(x)) (tests/test_fmath.py bounds both) at a fraction of
// the instructions; other exponents use exp2f_/log2f_.
//
// Exponents 1/4, 1/2 and n + 1/2 (the DDGI smoothing pow(x, 0.25) and the
// irradiance decode pow(x, 2.5)) use correctly rounded square roots: sqrt(sqrt(x)),
// sqrt(x), powi_(x, n) * sqrt(x) (<= 2 ulp; GLSL leaves pow's precision to the
// implementation, this fixes one on both sides).
//
// Negative bases (GLSL: undefined) with an integral exponent are evaluated as the
// product, like a driver's expansion of pow(x, 5.0) into multiplies: Schlick's
// pow(1 - VdotH, 5) sees 1 - VdotH = -1.2e-7 on head-on hits (VdotH rounds to
// 1.0000001), and a NaN there would poison the atlases.
ARK_HD float powf_(float x, float y)
{
    if (y == 0.0f || x == 1.0f) return 1.0f;
    if (isnan_(x) || isnan_(y)) return nan_();
    if (is_small_int_(y)) return powi_(x, static_cast<int>(y));
    if (x < 0.0f) return nan_();
    if (is_root_exp_(y)) {
        if (y == 0.25f) return sqrtf_(sqrtf_(x));
        if (y == 0.5f) return sqrtf_(x);
        return powi_(x, static_cast<int>(y)) * sqrtf_(x);
    }
    if (x == 0.0f) return y > 0.0f ? 0.0f : inf_();
    if (x == inf_()) return y > 0.0f ? inf_() : 0.0f;
    return exp2f_(y * log2f_(x));
}

// powf_ restricted to x > 0 finite, y finite, not a small integer and not a
// square-root exponent (see powf_),
// with y*log2(x) < 127.5, written
// without branches (selects only) so it vectorises in the hot visibility loop.
// Bitwise identical to powf_ on that domain: the same IEEE operations in the
// same order (tests/test_fmath.py and tests/test_gpu_fmath.py pin this).
ARK_HD float powf_pos_(float x, float y)
{
    // log2f_ main path
    const bool den = x < 0x1p-126f;
    const float xs = den ? x * 0x1p+23f : x;
    const uint32_t u = f2u(xs);
    int e = (den ? -23 : 0) + static_cast<int>((u >> 23) & 0xffu) - 126;
    const float m0 = u2f((u & 0x007fffffu) | 0x3f000000u);
    const bool lo = m0 < 0.70710678118654752440f;
    e -= lo ? 1 : 0;
    const float m = lo ? (m0 + m0 - 1.0f) : (m0 - 1.0f);
    const float z2 = m * m;
    float p = fmaf_(m, 7.0376836292e-2f, -1.1514610310e-1f);
    p = fmaf_(m, p, 1.1676998740e-1f);
    p = fmaf_(m, p, -1.2420140846e-1f);
    p = fmaf_(m, p, 1.4249322787e-1f);
    p = fmaf_(m, p, -1.6668057665e-1f);
    p = fmaf_(m, p, 2.0000714765e-1f);
    p = fmaf_(m, p, -2.4999993993e-1f);
    p = fmaf_(m, p, 3.3333331174e-1f);
    float yy = m * (z2 * p);
    yy = fmaf_(-0.5f, z2, yy);
    const float LOG2EA = 0.44269504088896340736f;
    float r = yy * LOG2EA;
    r = fmaf_(m, LOG2EA, r);
    r = r + yy;
    r = r + m;
    const float l2 = r + static_cast<float>(e);
    // exp2f_ main path
    const float z = y * l2;
    const float i = floorf_(z + 0.5f);
    const float f = z - i;
    float q = fmaf_(f, 1.535336188319500e-4f, 1.339887440266574e-3f);
    q = fmaf_(f, q, 9.618437357674640e-3f);
    q = fmaf_(f, q, 5.550332471162809e-2f);
    q = fmaf_(f, q, 2.402264791363012e-1f);
    q = fmaf_(f, q, 6.931472028550421e-1f);
    float t = fmaf_(f, q, 1.0f);
    int n = static_cast<int>(i);
    const bool sub = n < -126;
    t = sub ? t * 0x1p-126f : t;
    n = sub ? n + 126 : n;
    const float res = t * u2f(static_cast<uint32_t>(n + 127) << 23);
    return (z < -151.0f || n < -126) ? 0.0f : res;
}

} // namespace ark
