// fmath_vs_libm.cpp — the probe-ray directions of one DDGI frame computed twice:
// with ark_fmath.h (the transcendental code that the HIP kernels and the CPU oracle
// share) and with glibc's sinf/cosf/acosf/sqrtf, same formula and operation order
// otherwise (ddgi/common.glsl:12-25, common.glsl:121-142, random.glsl:40-74).
// An independent witness for ark_fmath.h: prints the distance between the two
// direction sets as one JSON line.
//
//   fmath_vs_libm <X> <Y> <Z> <rays> <frame>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ark_fmath.h"

using namespace ark;

namespace {

constexpr float kTwoPi = 6.28318530717958647692f;
constexpr float kGoldenRatio = 1.618034f;

struct V { float x, y, z; };
struct V3d { double x, y, z; };

uint32_t wangHash(uint32_t s)
{
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    return s ^ (s >> 15);
}

uint32_t xorshift(uint32_t s)
{
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}

// the two math libraries behind one interface
struct Fmath {
    static void sincos(float x, float* s, float* c) { sincosf_(x, s, c); }
    static float acos(float x) { return acosf_(x); }
    static float sqrt(float x) { return sqrtf_(x); }
};
struct Libm {
    static void sincos(float x, float* s, float* c) { *s = ::sinf(x); *c = ::cosf(x); }
    static float acos(float x) { return ::acosf(x); }
    static float sqrt(float x) { return ::sqrtf(x); }
};

// the same formula in double precision from the same fp32 arguments (theta, u, angle
// as the fp32 code forms them): the exact direction both fp32 versions approximate
V3d directionExact(uint32_t probe, uint32_t sample, uint32_t n, uint32_t frame)
{
    const float theta = kTwoPi * static_cast<float>(sample) / kGoldenRatio;
    const double phi = std::acos(static_cast<double>(2.0f * (static_cast<float>(sample) / static_cast<float>(n)) - 1.0f));
    const V3d v = { std::cos(theta) * std::sin(phi), std::sin(theta) * std::sin(phi), std::cos(phi) };
    uint32_t s = wangHash(512u * probe + frame % 512u);
    auto rnd = [&]() { s = xorshift(s); return static_cast<float>(s) * (1.0f / 4294967296.0f); };
    const float th = kTwoPi * rnd();
    const float u = 2.0f * rnd() - 1.0f;
    const double sr = std::sqrt(1.0 - static_cast<double>(u) * u);
    const V3d k = { sr * std::cos(th), sr * std::sin(th), static_cast<double>(u) };
    const float angle = kTwoPi * rnd();
    const double sa = std::sin(angle), ca = std::cos(angle);
    const V3d kxv = { k.y * v.z - k.z * v.y, k.z * v.x - k.x * v.z, k.x * v.y - k.y * v.x };
    const double kv = k.x * v.x + k.y * v.y + k.z * v.z;
    return { v.x * ca + kxv.x * sa + k.x * kv * (1 - ca), v.y * ca + kxv.y * sa + k.y * kv * (1 - ca), v.z * ca + kxv.z * sa + k.z * kv * (1 - ca) };
}

double angleBetween(V3d a, V3d b)
{
    const double cx = a.y * b.z - a.z * b.y, cy = a.z * b.x - a.x * b.z, cz = a.x * b.y - a.y * b.x;
    return std::atan2(std::sqrt(cx * cx + cy * cy + cz * cz), a.x * b.x + a.y * b.y + a.z * b.z);
}

template<class M>
V direction(uint32_t probe, uint32_t sample, uint32_t n, uint32_t frame)
{
    // sphericalFibonacciSample (common.glsl:121-130)
    const float theta = kTwoPi * static_cast<float>(sample) / kGoldenRatio;
    const float phi = M::acos(2.0f * (static_cast<float>(sample) / static_cast<float>(n)) - 1.0f);
    float sp, cp, st, ct;
    M::sincos(phi, &sp, &cp);
    M::sincos(theta, &st, &ct);
    const V v = { ct * sp, st * sp, cp };
    // seedRandom / randomPointOnSphere / randomFloat (random.glsl:40-74)
    uint32_t s = wangHash(512u * probe + frame % 512u);
    auto rnd = [&]() { s = xorshift(s); return static_cast<float>(s) * (1.0f / 4294967296.0f); };
    const float th = kTwoPi * rnd();
    const float u = 2.0f * rnd() - 1.0f;
    const float sr = M::sqrt(1.0f - u * u);
    float s1, c1;
    M::sincos(th, &s1, &c1);
    const V k = { sr * c1, sr * s1, u };
    const float angle = kTwoPi * rnd();
    float sa, ca;
    M::sincos(angle, &sa, &ca);
    // axisAngleRotate (common.glsl:133-142): v c + (k x v) s + k (k . v)(1 - c)
    const V kxv = { k.y * v.z - k.z * v.y, k.z * v.x - k.x * v.z, k.x * v.y - k.y * v.x };
    const float kv = k.x * v.x + k.y * v.y + k.z * v.z;
    const float oc = 1.0f - ca;
    return { v.x * ca + kxv.x * sa + k.x * kv * oc, v.y * ca + kxv.y * sa + k.y * kv * oc, v.z * ca + kxv.z * sa + k.z * kv * oc };
}

// distance in units in the last place of the larger magnitude, floored at 1/8: a
// component near 0 comes out of a cancelling sum, where an absolute error of one
// ulp of the unit vector's other components is the meaningful scale
double ulps(float a, float b)
{
    const float m = std::fmax(0.125f, std::fmax(std::fabs(a), std::fabs(b)));
    int e;
    std::frexp(m, &e);
    return std::fabs(static_cast<double>(a) - static_cast<double>(b)) / std::ldexp(1.0, e - 24);
}

} // namespace

int main(int argc, char** argv)
{
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s X Y Z rays frame\n", argv[0]);
        return 2;
    }
    const uint32_t N = static_cast<uint32_t>(std::atoi(argv[1]) * std::atoi(argv[2]) * std::atoi(argv[3]));
    const uint32_t R = static_cast<uint32_t>(std::atoi(argv[4]));
    const uint32_t frame = static_cast<uint32_t>(std::atoi(argv[5]));
    double maxUlp = 0.0, maxAbs = 0.0, maxAngle = 0.0, sumUlp = 0.0, maxAngleFmath = 0.0, maxAngleLibm = 0.0;
    uint64_t identical = 0, total = 0, comps = 0;
    uint64_t hist[4] = { 0, 0, 0, 0 }; // component ulp distance 0, 1, 2-3, >= 4
    for (uint32_t p = 0; p < N; ++p)
        for (uint32_t i = 0; i < R; ++i) {
            const V a = direction<Fmath>(p, i, R, frame), b = direction<Libm>(p, i, R, frame);
            const float ca[3] = { a.x, a.y, a.z }, cb[3] = { b.x, b.y, b.z };
            bool same = true;
            for (int c = 0; c < 3; ++c) {
                const double u = ulps(ca[c], cb[c]);
                maxUlp = std::fmax(maxUlp, u);
                sumUlp += u;
                ++comps;
                hist[u == 0.0 ? 0 : u <= 1.0 ? 1 : u < 4.0 ? 2 : 3]++;
                maxAbs = std::fmax(maxAbs, std::fabs(static_cast<double>(ca[c]) - cb[c]));
                same = same && std::memcmp(&ca[c], &cb[c], 4) == 0;
            }
            identical += same;
            // angles (double precision): fmath vs glibc, and each vs the exact direction
            const V3d da = { a.x, a.y, a.z }, db = { b.x, b.y, b.z }, de = directionExact(p, i, R, frame);
            maxAngle = std::fmax(maxAngle, angleBetween(da, db));
            maxAngleFmath = std::fmax(maxAngleFmath, angleBetween(da, de));
            maxAngleLibm = std::fmax(maxAngleLibm, angleBetween(db, de));
            ++total;
        }
    std::printf("{\"rays\": %llu, \"identical_rays\": %llu, \"max_component_ulp\": %.3f, \"mean_component_ulp\": %.5f, "
                "\"max_abs\": %.3e, \"max_angle_rad\": %.3e, \"max_angle_fmath_vs_exact_rad\": %.3e, \"max_angle_libm_vs_exact_rad\": %.3e, "
                "\"ulp_hist\": [%llu, %llu, %llu, %llu]}\n",
                static_cast<unsigned long long>(total), static_cast<unsigned long long>(identical), maxUlp, sumUlp / static_cast<double>(comps), maxAbs,
                maxAngle, maxAngleFmath, maxAngleLibm, static_cast<unsigned long long>(hist[0]), static_cast<unsigned long long>(hist[1]), static_cast<unsigned long long>(hist[2]),
                static_cast<unsigned long long>(hist[3]));
    return 0;
}
