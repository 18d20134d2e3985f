// Host timing of set_scene's BVH path on the C4 soup (no GPU): world BVH2 build,
// BVH8 collapse, the sun's light-space BVH and its cost sampling.
// g++ -O3 -std=c++17 -pthread -I../../include tools/probe/build_timing.cpp
//     arkoserenderer_amd/csrc/bvh_builder.cpp arkoserenderer_amd/csrc/scene_gen.cpp
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../arkoserenderer_amd/csrc/bvh_builder.h"
#include "../../include/ark_scene.h"

using namespace ark;
using Clock = std::chrono::steady_clock;
static double ms(Clock::time_point a) { return std::chrono::duration<double, std::milli>(Clock::now() - a).count(); }

int main(int argc, char** argv)
{
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 10000000ull;
    const int threads = argc > 2 ? std::atoi(argv[2]) : 16;
    ArkSoupParams sp;
    ark_soup_default_params(&sp);
    sp.triangle_count = n;
    ArkSoupScene* soup = nullptr;
    auto t = Clock::now();
    if (ark_soup_generate(&sp, &soup) != 0) return 1;
    const ArkDdgiScene* s = ark_soup_scene_view(soup);
    std::printf("soup %.0f ms\n", ms(t));
    t = Clock::now();
    std::vector<BuildTriangle> cls;
    cls.reserve(n);
    for (uint32_t ii = 0; ii < s->instance_count; ++ii) {
        const ArkRTInstance& inst = s->instances[ii];
        const ArkRTTriangleMesh& m = s->meshes[inst.rt_mesh_index];
        const float* M = inst.object_to_world;
        for (uint32_t p = 0; p < inst.triangle_count; ++p) {
            BuildTriangle bt;
            float* w[3] = { bt.v0, bt.v1, bt.v2 };
            for (int k = 0; k < 3; ++k) {
                const uint32_t idx = s->indices[static_cast<size_t>(m.first_index) + 3u * p + k];
                const float* P = &s->positions[(static_cast<uint64_t>(m.first_vertex) + idx) * 3];
                w[k][0] = M[0] * P[0] + M[1] * P[1] + M[2] * P[2] + M[3];
                w[k][1] = M[4] * P[0] + M[5] * P[1] + M[6] * P[2] + M[7];
                w[k][2] = M[8] * P[0] + M[9] * P[1] + M[10] * P[2] + M[11];
            }
            bt.instance = ii;
            bt.primitive = p;
            bt.flip_facing = 0;
            cls.push_back(bt);
        }
    }
    std::printf("world triangles %.0f ms\n", ms(t));
    BvhBuildOptions opt;
    opt.max_leaf_size = kBvh8MaxLeafSize;
    opt.threads = threads;
    float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    for (const BuildTriangle& b : cls)
        for (const float* v : { b.v0, b.v1, b.v2 })
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::fmin(lo[a], v[a]);
                hi[a] = std::fmax(hi[a], v[a]);
            }
    opt.inflate_abs = bvh8_inflation_box(lo, hi);
    SunBvhInput sunIn;
    sun_frame(s->directional_light.world_space_direction, sunIn.frame);
    t = Clock::now();
    sun_add_triangles(sunIn, cls, threads);
    std::printf("sun input %.0f ms\n", ms(t));
    t = Clock::now();
    BvhBuildResult r2 = build_bvh(cls, opt, 0u, 0u);
    std::printf("world BVH2 %.0f ms (%zu nodes, depth %u)\n", ms(t), r2.nodes.size(), r2.max_depth);
    t = Clock::now();
    Bvh8CollapseOptions copt;
    copt.threads = threads;
    Bvh8BuildResult r8 = collapse_bvh8(r2, 0u, 0u, copt);
    std::printf("world collapse %.0f ms (%zu nodes)\n", ms(t), r8.nodes.size());
    t = Clock::now();
    Bvh8BuildResult rs;
    build_sun_bvh(sunIn, opt, copt, rs);
    std::printf("sun BVH (BVH2 + collapse) %.0f ms (%zu nodes)\n", ms(t), rs.nodes.size());
    t = Clock::now();
    const float* sd = s->directional_light.world_space_direction;
    const float isc = 1.0f / std::sqrt(sd[0] * sd[0] + sd[1] * sd[1] + sd[2] * sd[2]);
    const float L[3] = { -(sd[0] * isc), -(sd[1] * isc), -(sd[2] * isc) };
    std::vector<float> origins;
    sun_sample_origins(r8.tris, L, 4096u, origins);
    const int32_t roots[3] = { 0, -1, -1 }, sroot = 0;
    const double cw = sun_shadow_cost(r8.nodes, r8.tris, roots, 3, nullptr, L, origins);
    const double cl = sun_shadow_cost(rs.nodes, rs.tris, &sroot, 1, sunIn.frame, L, origins);
    std::printf("sun cost sampling %.0f ms (world %.2f, light %.2f)\n", ms(t), cw, cl);
    // the background rebuild's input: the world BVH's records in leaf order (holes skipped)
    SunBvhInput recIn;
    sun_frame(s->directional_light.world_space_direction, recIn.frame);
    t = Clock::now();
    sun_add_records(recIn, r8.tris, threads);
    Bvh8BuildResult rr;
    build_sun_bvh(recIn, opt, copt, rr);
    const double cr = sun_shadow_cost(rr.nodes, rr.tris, &sroot, 1, recIn.frame, L, origins);
    std::printf("sun BVH from the world records %.0f ms (%zu nodes, depth %u vs %u), light cost %.2f\n", ms(t), rr.nodes.size(), rr.max_depth, rs.max_depth, cr);
    ark_soup_free(soup);
    return 0;
}
