// bvh_trace_sim.cpp — host traversal simulator of the BVH8 set_scene builds (a tool,
// not part of libark_ddgi.so; VERDICT r05 "do this" #7). Moved out of
// arkoserenderer_amd/csrc/bvh_builder.cpp: it restates k_trace's visiting order on the
// host and the rejected packed-fp16 child tests (ARK_SIM_BOX), and its build and
// traversal experiments are steered by environment variables (ARK_SIM_*,
// ARK_BVH_PRESPLIT, ARK_BVH_AREA_W, ARK_BVH8_COLLAPSE, ARK_BVH8_TRI_COST,
// ARK_BVH_INTERSECTION_COST) that the product library does not read.
// Built into tools/lib/libark_bvhsim.so with the product's BVH builder (tools/sim/Makefile);
// used by tools/bvh_stats.py, tools/sun_bvh_stats.py and tests/test_box_f16.py.
#include "bvh_trace_sim.h"

#include "../../arkoserenderer_amd/csrc/bvh_builder.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

// Round to the nearest fp16 value (RNE; +-inf above the largest finite value),
// returned as a double: the host emulation of the packed-f16 box test below.
static double rn16(double x)
{
    const double ax = std::fabs(x);
    if (ax >= 65520.0) return x < 0 ? -INFINITY : INFINITY;
    if (ax == 0.0) return x;
    int e = std::ilogb(ax);
    if (e < -14) e = -14;
    const double ulp = std::ldexp(1.0, e - 10);
    return std::nearbyint(x / ulp) * ulp;
}

// Round to fp16 toward -inf (dir < 0) or +inf (dir > 0), as a double: the MODE
// register's directed rounding of ARK_NODE_F16 == 2 (a finite value never rounds to
// the infinity on the other side; beyond the largest finite value toward it, inf).
static double rd16(double x, int dir)
{
    if (x == 0.0 || std::isinf(x) || std::isnan(x)) return x;
    const double ax = std::fabs(x);
    int e = std::ilogb(ax);
    if (e < -14) e = -14;
    const double ulp = std::ldexp(1.0, e - 10);
    double r = (dir < 0 ? std::floor(x / ulp) : std::ceil(x / ulp)) * ulp;
    if (r > 65504.0) r = dir > 0 ? INFINITY : 65504.0;
    if (r < -65504.0) r = dir < 0 ? -INFINITY : -65504.0;
    return r;
}

// ark_ddgi_debug.h: traversal statistics of the BVH8 that set_scene would upload
// (host simulation of k_trace's closest-hit order: per node the hit children,
// those whose box holds the origin first, then octant order; a node's leaf
// triangles are tested right after it). For comparing BVH builds without a GPU.
extern "C" int ark_ddgi_debug_bvh8_trace_stats(const float* triangles, uint64_t n, const float* rays, uint64_t nRays, int threads, uint64_t* out,
                                                uint32_t* perRay)
{
    using namespace ark;
    std::vector<BuildTriangle> tris(n);
    for (uint64_t i = 0; i < n; ++i) {
        for (int a = 0; a < 3; ++a) {
            tris[i].v0[a] = triangles[9 * i + a];
            tris[i].v1[a] = triangles[9 * i + 3 + a];
            tris[i].v2[a] = triangles[9 * i + 6 + a];
        }
        tris[i].instance = 0;
        tris[i].primitive = static_cast<uint32_t>(i);
        tris[i].flip_facing = 0;
    }
    BvhBuildOptions opt;
    opt.max_leaf_size = kBvh8MaxLeafSize;
    opt.inflate_abs = bvh8_inflation(triangles, n);
    opt.threads = threads > 0 ? threads : 8;
    if (const char* e = std::getenv("ARK_BVH_INTERSECTION_COST")) opt.intersection_cost = std::max(0.05f, static_cast<float>(std::atof(e)));
    // ARK_BVH_PRESPLIT="levels,ratio": early split clipping (BvhBuildOptions::presplit_levels)
    if (const char* e = std::getenv("ARK_BVH_PRESPLIT")) std::sscanf(e, "%d,%f", &opt.presplit_levels, &opt.presplit_ratio);
    // ARK_BVH_AREA_W="xy,yz,zx": SAH face weights of both the BVH2 build and the collapse
    if (const char* e = std::getenv("ARK_BVH_AREA_W"))
        std::sscanf(e, "%f,%f,%f", &opt.area_w[0], &opt.area_w[1], &opt.area_w[2]);
    const BvhBuildResult r2 = build_bvh(tris, opt, 0u, 0u);
    Bvh8CollapseOptions copt;
    if (const char* e = std::getenv("ARK_BVH8_COLLAPSE")) copt.sah_optimal = std::strcmp(e, "sah") == 0;
    if (const char* e = std::getenv("ARK_BVH8_TRI_COST")) copt.tri_cost = std::max(0.01f, static_cast<float>(std::atof(e)));
    for (int k = 0; k < 3; ++k) copt.area_w[k] = opt.area_w[k];
    const Bvh8BuildResult r8 = collapse_bvh8(r2, 0u, 0u, copt);
    if (std::getenv("ARK_SIM_FILL")) {
        // children per node (internal + leaf slots) and leaf triangles per leaf child
        uint64_t hist[9] = {}, leafTris = 0, leaves = 0;
        for (const GpuBvh8Node& nd : r8.nodes) {
            hist[__builtin_popcount(static_cast<uint32_t>(nd.imask | nd.leaf_mask))]++;
            leaves += static_cast<uint64_t>(__builtin_popcount(nd.leaf_mask));
            leafTris += static_cast<uint64_t>(__builtin_popcount(nd.leaf_tris));
        }
        std::fprintf(stderr, "bvh8 fill: nodes %zu, children per node", r8.nodes.size());
        for (int k = 0; k <= 8; ++k) std::fprintf(stderr, " %d:%llu", k, static_cast<unsigned long long>(hist[k]));
        std::fprintf(stderr, ", leaves %llu, triangles per leaf %.3f\n", static_cast<unsigned long long>(leaves),
                     leaves ? static_cast<double>(leafTris) / static_cast<double>(leaves) : 0.0);
    }
    std::atomic<uint64_t> nodes { 0 }, triTests { 0 }, hits { 0 }, maxSteps { 0 }, boxViolations { 0 };
    // ARK_SIM_ORDER=distance: exact front-to-back child order (what octant order approximates)
    const bool sortByDistance = std::getenv("ARK_SIM_ORDER") && std::strcmp(std::getenv("ARK_SIM_ORDER"), "distance") == 0;
    // ARK_SIM_ANYHIT=1: shadow-ray statistics - tmin 0.025 (k_shadow_gen's), the ray
    // ends at its first hit (any-hit, k_trace_shadow)
    const bool anyHit = std::getenv("ARK_SIM_ANYHIT") && std::atoi(std::getenv("ARK_SIM_ANYHIT")) != 0;
    // ARK_SIM_BOX: the child box test. "exact" (default): decoded planes, (p - o) * idir;
    // "kernel32": k_trace's fp32 form t = fma(q, step * idir, (anchor - o) * idir);
    // "f16": the packed-f16 form (visitNode8 with ARK_NODE_F16): per-ray scale 2^-s,
    // t = RN16((1024 + q) * RN16(a) + RN16(b - 1024 a)), near/far reduced in f16, the
    // test tn <= RN16(tf * (1 + 2^-8) + 2E) with the per-node error bound E. In the
    // non-exact modes, a child that the exact test accepts and the chosen form rejects
    // is counted in out[8] (must stay 0: the form must be conservative).
    const char* boxEnv = std::getenv("ARK_SIM_BOX");
    // f16d: ARK_NODE_F16 == 2 - the f16s scales with the near planes' A, B and
    // distances rounded toward -inf and the far planes' toward +inf, no error bound
    const int boxMode = !boxEnv                           ? 0
                        : std::strcmp(boxEnv, "kernel32") == 0 ? 1
                        : std::strcmp(boxEnv, "f16") == 0      ? 2
                        : std::strcmp(boxEnv, "f16s") == 0     ? 3
                        : std::strcmp(boxEnv, "f16d") == 0     ? 4
                                                               : 0;
    // f16s: q as the fp16 subnormal q * 2^-24 (no 1024 bias), A = a * 2^(24 - s) with a
    // per-node scale s (ARK_NODE_F16's visitNode8)
    // the f16 form's error bound e = EA |a| + EB |B'| + 2^-22 (sensitivity runs only:
    // the defaults are the proven bound)
    const float simEA = std::getenv("ARK_SIM_E_A") ? static_cast<float>(std::atof(std::getenv("ARK_SIM_E_A"))) : (boxMode == 3 ? 0.3f : 1.3f);
    const float simEB = std::getenv("ARK_SIM_E_B") ? static_cast<float>(std::atof(std::getenv("ARK_SIM_E_B"))) : 0x1p-9f;
    // scene bounds of the anchors (every node box lies inside the root's planes)
    double sceneLo[3] = { 0, 0, 0 }, sceneHi[3] = { 0, 0, 0 };
    if (!r8.nodes.empty()) {
        const GpuBvh8Node& root = r8.nodes[0];
        for (int a = 0; a < 3; ++a) {
            sceneLo[a] = root.p[a];
            sceneHi[a] = root.p[a] + 255.0 * std::ldexp(1.0, static_cast<int>(root.e[a]) - 127);
        }
    }
    // ARK_SIM_STEP=1: k_trace's dual step (one pending leaf triangle and one node per
    // iteration, the node side paused while a second leaf group waits), per-ray
    // iterations in perRay / out[5]; =2: the same with two nodes per iteration (the next
    // two children of the group / stack, the second's children pushed below the first's
    // group, up to two waiting leaf groups). Exact box test, k-order (slot ^ octant).
    const int stepMode = std::getenv("ARK_SIM_STEP") ? std::atoi(std::getenv("ARK_SIM_STEP")) : 0;
    if (stepMode) {
        std::atomic<uint64_t> sumIter { 0 };
        auto stepWorker = [&](uint64_t r0, uint64_t r1) {
            uint64_t cn = 0, ct = 0, ch = 0, ms = 0, it = 0;
            struct Group { uint32_t base; uint32_t bits; uint32_t imask; };
            for (uint64_t r = r0; r < r1; ++r) {
                const float* ry = rays + 7 * r;
                const float o[3] = { ry[0], ry[1], ry[2] }, d[3] = { ry[3], ry[4], ry[5] };
                float tmax = ry[6];
                const float tmin = 1e-4f;
                float idir[3];
                for (int a = 0; a < 3; ++a) idir[a] = 1.0f / (std::fabs(d[a]) < 1e-20f ? (d[a] < 0.0f ? -1e-20f : 1e-20f) : d[a]);
                const uint32_t oct = (idir[0] < 0 ? 1u : 0u) | (idir[1] < 0 ? 2u : 0u) | (idir[2] < 0 ? 4u : 0u);
                bool hit = false;
                auto nextChild = [&](Group& g) {
                    const uint32_t k = static_cast<uint32_t>(__builtin_ctz(g.bits));
                    g.bits &= g.bits - 1u;
                    const uint32_t slot = k ^ oct;
                    return g.base + static_cast<uint32_t>(__builtin_popcount(g.imask & ((1u << slot) - 1u)));
                };
                // node visit: the group of hit internal children, the hit leaves' triangles
                auto visit = [&](uint32_t ni, Group& g, std::vector<uint32_t>& leafTris) {
                    const GpuBvh8Node& nd = r8.nodes[ni];
                    cn++;
                    g = Group { nd.child_base, 0u, nd.imask };
                    leafTris.clear();
                    for (int s = 0; s < 8; ++s) {
                        const bool internal = (nd.imask >> s) & 1u;
                        if (!internal && !((nd.leaf_mask >> s) & 1u)) continue;
                        float tn = tmin, tf = tmax;
                        for (int a = 0; a < 3; ++a) {
                            const float step = std::ldexp(1.0f, static_cast<int>(nd.e[a]) - 127);
                            const float lo = std::fma(static_cast<float>(nd.qlo[a][s]), step, nd.p[a]);
                            const float hi = std::fma(static_cast<float>(nd.qhi[a][s]), step, nd.p[a]);
                            float t0 = (lo - o[a]) * idir[a], t1 = (hi - o[a]) * idir[a];
                            if (t0 > t1) std::swap(t0, t1);
                            tn = std::max(tn, t0);
                            tf = std::min(tf, t1);
                        }
                        if (!(tn <= tf * 1.00001f + 1e-7f)) continue;
                        if (internal) g.bits |= 1u << (static_cast<uint32_t>(s) ^ oct);
                        else {
                            uint32_t st[kBvh8MaxLeafSize];
                            const int c = bvh8SlotTriangles(nd, s, st);
                            for (int i = 0; i < c; ++i) leafTris.push_back(st[i]);
                        }
                    }
                };
                auto testTri = [&](uint32_t t) {
                    ct++;
                    const GpuTriangle& g = r8.tris[t];
                    const float v0[3] = { g.t0[0], g.t0[1], g.t0[2] }, e1[3] = { g.t0[3], g.t1[0], g.t1[1] }, e2[3] = { g.t1[2], g.t1[3], g.t2[0] };
                    const float pv[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
                    const float det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
                    if (det == 0.0f) return;
                    const float inv = 1.0f / det;
                    const float sv[3] = { o[0] - v0[0], o[1] - v0[1], o[2] - v0[2] };
                    const float u = (sv[0] * pv[0] + sv[1] * pv[1] + sv[2] * pv[2]) * inv;
                    if (!(u >= 0.0f && u <= 1.0f)) return;
                    const float q[3] = { sv[1] * e1[2] - sv[2] * e1[1], sv[2] * e1[0] - sv[0] * e1[2], sv[0] * e1[1] - sv[1] * e1[0] };
                    const float v = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv;
                    if (!(v >= 0.0f && u + v <= 1.0f)) return;
                    const float tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
                    if (tt >= tmin && tt <= tmax) {
                        tmax = tt;
                        hit = true;
                    }
                };
                Group G { 0u, 1u, 0u }; // the root alone (k = 0, no internal mask: base + 0)
                std::vector<Group> S;
                std::vector<uint32_t> triQ, q1, q2, leafA, leafB;
                size_t triPos = 0;
                uint64_t iters = 0;
                auto addLeaves = [&](std::vector<uint32_t>& L) {
                    if (L.empty()) return;
                    if (triPos >= triQ.size()) { triQ.swap(L); triPos = 0; }
                    else if (q1.empty()) q1.swap(L);
                    else q2.swap(L);
                };
                for (;;) {
                    const bool doTri = triPos < triQ.size();
                    const bool room = stepMode == 2 ? (q1.empty() && q2.empty()) : q1.empty();
                    const bool doNode = room && (G.bits != 0 || !S.empty());
                    if (!doTri && !doNode) break;
                    iters++;
                    if (doTri) testTri(triQ[triPos++]);
                    if (doNode) {
                        if (G.bits == 0) { G = S.back(); S.pop_back(); }
                        const uint32_t A = nextChild(G);
                        bool haveB = false;
                        uint32_t B = 0;
                        if (stepMode == 2) {
                            if (G.bits != 0) { B = nextChild(G); haveB = true; }
                            else if (!S.empty()) {
                                Group& H = S.back();
                                B = nextChild(H);
                                haveB = true;
                                if (H.bits == 0) S.pop_back();
                            }
                        }
                        if (G.bits != 0) S.push_back(G);
                        Group GA {}, GB {};
                        visit(A, GA, leafA);
                        if (haveB) {
                            visit(B, GB, leafB);
                            if (GB.bits != 0) S.push_back(GB);
                        }
                        G = GA;
                        addLeaves(leafA);
                        if (haveB) addLeaves(leafB);
                    }
                    if (triPos >= triQ.size()) {
                        if (!q1.empty()) { triQ.swap(q1); q1.clear(); triPos = 0; if (!q2.empty()) { q1.swap(q2); q2.clear(); } }
                    }
                }
                ch += hit ? 1 : 0;
                it += iters;
                ms = std::max(ms, iters);
                if (perRay) perRay[r] = static_cast<uint32_t>(iters);
            }
            nodes += cn;
            triTests += ct;
            hits += ch;
            sumIter += it;
            uint64_t m = maxSteps.load();
            while (ms > m && !maxSteps.compare_exchange_weak(m, ms)) {}
        };
        const int T = std::max(1, threads);
        std::vector<std::thread> pool;
        for (int t = 0; t < T; ++t) pool.emplace_back(stepWorker, nRays * t / T, nRays * (t + 1) / T);
        for (auto& th : pool) th.join();
        if (out) {
            out[0] = nodes.load();
            out[1] = triTests.load();
            out[2] = hits.load();
            out[3] = r8.nodes.size();
            out[4] = sumIter.load(); // iterations (in place of the SAH cost)
            out[5] = maxSteps.load();
            out[6] = r8.max_depth;
            out[7] = r8.tris.size();
            out[8] = 0;
        }
        return 0;
    }
    auto worker = [&](uint64_t r0, uint64_t r1) {
        uint64_t cn = 0, ct = 0, ch = 0, ms = 0;
        for (uint64_t r = r0; r < r1; ++r) {
            const float* ry = rays + 7 * r;
            const float o[3] = { ry[0], ry[1], ry[2] }, d[3] = { ry[3], ry[4], ry[5] };
            float tmax = ry[6];
            const float tmin = anyHit ? 0.025f : 1e-4f;
            float idir[3];
            for (int a = 0; a < 3; ++a) idir[a] = 1.0f / (std::fabs(d[a]) < 1e-20f ? (d[a] < 0.0f ? -1e-20f : 1e-20f) : d[a]);
            const uint32_t oct = (idir[0] < 0 ? 1u : 0u) | (idir[1] < 0 ? 2u : 0u) | (idir[2] < 0 ? 4u : 0u);
            std::vector<uint32_t> stack { 0u };
            bool hit = false;
            uint64_t steps = 0;
            // f16 form: per-ray scale 2^-s so that |b - 1024 a| and every t fit fp16
            int sExp = 0;
            if (boxMode == 2) {
                double m = 0.0;
                for (int a = 0; a < 3; ++a)
                    m = std::max(m, std::max(std::fabs(sceneHi[a] - o[a]), std::fabs(sceneLo[a] - o[a])) * std::fabs(static_cast<double>(idir[a])));
                sExp = std::max(0, std::ilogb(std::max(m * 10.0, 1e-30)) + 1 - 15);
            }
            while (!stack.empty() && !(anyHit && hit)) {
                const uint32_t ni = stack.back();
                stack.pop_back();
                const GpuBvh8Node& nd = r8.nodes[ni];
                cn++;
                steps++;
                struct C { float tn; uint32_t k; bool inside; int s; };
                C hitc[8];
                int nh = 0;
                // per-node terms of the kernel forms
                float a32[3], b32[3];
                double A16[3], Bn16[3], Bf16[3], An16[3], Af16[3];
                double tmin16 = 0.0, tmax16 = 0.0;
                for (int a = 0; a < 3; ++a) {
                    a32[a] = std::ldexp(idir[a], static_cast<int>(nd.e[a]) - 127);
                    b32[a] = (nd.p[a] - o[a]) * idir[a];
                }
                if (boxMode == 2) {
                    for (int a = 0; a < 3; ++a) {
                        // per axis: B' = b - 1024 a (fp32), its error bound e (the rounding
                        // of A over 1279 steps, of B', of the result and of B' +- e),
                        // and the near / far biases B' -+ e (the planes move outward)
                        const float as = std::ldexp(a32[a], -sExp), bs = std::ldexp(b32[a], -sExp);
                        const float Bp = std::fma(-1024.0f, as, bs);
                        const float e = std::fma(std::fabs(as), simEA, std::fma(std::fabs(Bp), simEB, 0x1p-22f));
                        A16[a] = rn16(as);
                        const bool flip = idir[a] < 0.0f;
                        // near planes (the smaller t) move down, far planes up; with a
                        // negative a the near plane is qhi's, still the smaller t
                        Bn16[a] = rn16(static_cast<double>(Bp - e));
                        Bf16[a] = rn16(static_cast<double>(Bp + e));
                        (void)flip;
                    }
                    tmin16 = rn16(std::ldexp(static_cast<double>(tmin), -sExp) * (1.0 - 0x1p-9));
                    tmax16 = rn16(std::ldexp(static_cast<double>(tmax), -sExp) * (1.0 + 0x1p-9));
                }
                if (boxMode == 3) {
                    // per-node scale 2^-s (visitNode8 with ARK_NODE_F16): the largest
                    // A = a * 2^(24 - s) of the node stays below 2^15
                    int L = 0;
                    (void)std::frexp(std::max({ std::fabs(idir[0]), std::fabs(idir[1]), std::fabs(idir[2]) }), &L);
                    const int emax = std::max({ static_cast<int>(nd.e[0]), static_cast<int>(nd.e[1]), static_cast<int>(nd.e[2]) });
                    const int sN = std::max(0, emax - 127 + L + 9);
                    for (int a = 0; a < 3; ++a) {
                        const float Aa = std::ldexp(idir[a], static_cast<int>(nd.e[a]) - 103 - sN);
                        const float bs = std::ldexp(b32[a], -sN);
                        const float e = std::fma(std::fabs(Aa), simEA * 0x1p-24f, std::fma(std::fabs(bs), simEB, 0x1p-22f));
                        A16[a] = rn16(Aa);
                        // (B, e) rounded to fp16 first, then one packed add each way
                        const double b16 = rn16(bs), e16 = rn16(e);
                        Bn16[a] = rn16(b16 - e16);
                        Bf16[a] = rn16(b16 + e16);
                    }
                    tmin16 = 0.0;  // the kernel does not apply tmin (conservative)
                    tmax16 = rn16(static_cast<double>(std::ldexp(tmax, -sN) * (1.0f + 0x1p-9f)));
                }
                if (boxMode == 4) {
                    int L = 0;
                    (void)std::frexp(std::max({ std::fabs(idir[0]), std::fabs(idir[1]), std::fabs(idir[2]) }), &L);
                    const int emax = std::max({ static_cast<int>(nd.e[0]), static_cast<int>(nd.e[1]), static_cast<int>(nd.e[2]) });
                    const int sN = std::max(0, emax - 127 + L + 9);
                    for (int a = 0; a < 3; ++a) {
                        const float Aa = std::ldexp(idir[a], static_cast<int>(nd.e[a]) - 103 - sN);
                        const float bs = std::ldexp(b32[a], -sN);
                        An16[a] = rd16(Aa, -1);
                        Af16[a] = rd16(Aa, 1);
                        Bn16[a] = rd16(bs, -1);
                        Bf16[a] = rd16(bs, 1);
                    }
                    tmin16 = 0.0;
                    tmax16 = rd16(static_cast<double>(std::ldexp(tmax, -sN) * (1.0f + 0x1p-16f)), 1);
                }
                for (int s = 0; s < 8; ++s) {
                    const bool internal = (nd.imask >> s) & 1u;
                    if (!internal && !((nd.leaf_mask >> s) & 1u)) continue;
                    float tn = tmin, tf = tmax;
                    for (int a = 0; a < 3; ++a) {
                        const float step = std::ldexp(1.0f, static_cast<int>(nd.e[a]) - 127);
                        const float lo = std::fma(static_cast<float>(nd.qlo[a][s]), step, nd.p[a]);
                        const float hi = std::fma(static_cast<float>(nd.qhi[a][s]), step, nd.p[a]);
                        float t0 = (lo - o[a]) * idir[a], t1 = (hi - o[a]) * idir[a];
                        if (t0 > t1) std::swap(t0, t1);
                        tn = std::max(tn, t0);
                        tf = std::min(tf, t1);
                    }
                    const bool exactHit = tn <= tf * 1.00001f + 1e-7f;
                    bool accept = exactHit;
                    if (boxMode == 1) {
                        float kn = tmin, kf = tmax;
                        for (int a = 0; a < 3; ++a) {
                            const bool flip = idir[a] < 0.0f;
                            const float qn = static_cast<float>(flip ? nd.qhi[a][s] : nd.qlo[a][s]);
                            const float qf = static_cast<float>(flip ? nd.qlo[a][s] : nd.qhi[a][s]);
                            kn = std::max(kn, std::fma(qn, a32[a], b32[a]));
                            kf = std::min(kf, std::fma(qf, a32[a], b32[a]));
                        }
                        accept = kn <= std::fma(kf, 1.00001f, 1e-7f);
                    } else if (boxMode == 4) {
                        double kn = 0.0, kf = tmax16;
                        for (int a = 0; a < 3; ++a) {
                            const bool flip = idir[a] < 0.0f;
                            const double qn = (flip ? nd.qhi[a][s] : nd.qlo[a][s]) * 0x1p-24;
                            const double qf = (flip ? nd.qlo[a][s] : nd.qhi[a][s]) * 0x1p-24;
                            kn = std::max(kn, rd16(qn * An16[a] + Bn16[a], -1));
                            kf = std::min(kf, rd16(qf * Af16[a] + Bf16[a], 1));
                        }
                        accept = kn <= kf;
                    } else if (boxMode >= 2) {
                        double kn = -INFINITY, kf = INFINITY;
                        const double bias = boxMode == 2 ? 1024.0 : 0.0, qs = boxMode == 2 ? 1.0 : 0x1p-24;
                        for (int a = 0; a < 3; ++a) {
                            const bool flip = idir[a] < 0.0f;
                            const double qn = (bias + (flip ? nd.qhi[a][s] : nd.qlo[a][s])) * qs;
                            const double qf = (bias + (flip ? nd.qlo[a][s] : nd.qhi[a][s])) * qs;
                            kn = std::max(kn, rn16(qn * A16[a] + Bn16[a]));
                            kf = std::min(kf, rn16(qf * A16[a] + Bf16[a]));
                        }
                        kn = std::max(kn, tmin16);
                        kf = std::min(kf, tmax16);
                        accept = kn <= kf;
                    }
                    if (exactHit && !accept) boxViolations++;
                    if (accept) hitc[nh++] = { tn, static_cast<uint32_t>(s) ^ oct, tn <= tmin, s };
                }
                // leaf triangles of this node now, internal children by (inside first, k order)
                uint32_t internalBefore[8];
                uint32_t cntInt = 0;
                for (int s = 0; s < 8; ++s) {
                    internalBefore[s] = cntInt;
                    if ((nd.imask >> s) & 1u) cntInt++;
                }
                for (int i = 0; i < nh && !(anyHit && hit); ++i) {
                    const int s = hitc[i].s;
                    if ((nd.imask >> s) & 1u) continue;
                    uint32_t slotTris[kBvh8MaxLeafSize];
                    const int cnt = bvh8SlotTriangles(nd, s, slotTris);
                    for (int ti = 0; ti < cnt; ++ti) {
                        const uint32_t t = slotTris[ti];
                        ct++;
                        steps++;
                        const GpuTriangle& g = r8.tris[t];
                        const float v0[3] = { g.t0[0], g.t0[1], g.t0[2] }, e1[3] = { g.t0[3], g.t1[0], g.t1[1] }, e2[3] = { g.t1[2], g.t1[3], g.t2[0] };
                        const float pv[3] = { d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0] };
                        const float det = e1[0] * pv[0] + e1[1] * pv[1] + e1[2] * pv[2];
                        if (det == 0.0f) continue;
                        const float inv = 1.0f / det;
                        const float sv[3] = { o[0] - v0[0], o[1] - v0[1], o[2] - v0[2] };
                        const float u = (sv[0] * pv[0] + sv[1] * pv[1] + sv[2] * pv[2]) * inv;
                        if (!(u >= 0.0f && u <= 1.0f)) continue;
                        const float q[3] = { sv[1] * e1[2] - sv[2] * e1[1], sv[2] * e1[0] - sv[0] * e1[2], sv[0] * e1[1] - sv[1] * e1[0] };
                        const float v = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) * inv;
                        if (!(v >= 0.0f && u + v <= 1.0f)) continue;
                        const float tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) * inv;
                        if (tt >= tmin && tt <= tmax) {
                            tmax = tt;
                            hit = true;
                            if (anyHit) break;
                        }
                    }
                }
                // push internal children so that the first to visit is on top
                if (sortByDistance) std::sort(hitc, hitc + nh, [](const C& a, const C& b) { return a.tn < b.tn; });
                else std::sort(hitc, hitc + nh, [](const C& a, const C& b) { return a.inside != b.inside ? a.inside : a.k < b.k; });
                for (int i = nh - 1; i >= 0; --i) {
                    const int s = hitc[i].s;
                    if (((nd.imask >> s) & 1u) && hitc[i].tn <= tmax * 1.00001f + 1e-7f) stack.push_back(nd.child_base + internalBefore[s]);
                }
            }
            ch += hit ? 1 : 0;
            ms = std::max(ms, steps);
            if (perRay) perRay[r] = static_cast<uint32_t>(steps);
        }
        nodes += cn;
        triTests += ct;
        hits += ch;
        uint64_t m = maxSteps.load();
        while (ms > m && !maxSteps.compare_exchange_weak(m, ms)) {}
    };
    const int T = std::max(1, threads);
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(worker, nRays * t / T, nRays * (t + 1) / T);
    for (auto& th : pool) th.join();
    if (out) {
        out[0] = nodes.load();
        out[1] = triTests.load();
        out[2] = hits.load();
        out[3] = r8.nodes.size();
        out[4] = static_cast<uint64_t>(static_cast<double>(r8.sah_cost) * 1e6);
        out[5] = maxSteps.load();
        out[6] = r8.max_depth;
        out[7] = r8.tris.size();
        out[8] = boxViolations.load();
    }
    return 0;
}
