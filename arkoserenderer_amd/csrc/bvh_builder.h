// bvh_builder.h — binned-SAH BVH2 builder producing the 64 B node / 48 B triangle
// HBM layout consumed by the traversal kernels (ddgi_types.h). Replaces the
// acceleration structure build the Vulkan driver performs for the reference
// (VulkanAccelerationStructureKHR.cpp, build flag PREFER_FAST_TRACE).
#pragma once

#include <stdint.h>
#include <vector>

#include "ddgi_types.h"

namespace ark {

struct BuildTriangle {
    float v0[3], v1[3], v2[3]; // world space
    uint32_t instance;
    uint32_t primitive;
    uint32_t flip_facing; // the instance's det(ObjectToWorld) < 0, stored in GpuTriangle t2.w
};

struct BvhBuildOptions {
    int max_leaf_size = 4;   // <= kMaxLeafSize
    int bins = 32;
    int max_depth = 60;      // hard cap: splits fall back to object median near it
    int threads = 0;         // 0 = hardware concurrency
    float inflate_abs = 0.0f; // absolute box inflation on top of the relative one (see collapse_bvh8 / visitNode8)
    float traversal_cost = 1.0f;
    float intersection_cost = 1.0f;
    float area_w[3] = { 1.0f, 1.0f, 1.0f }; // SAH face weights {xy, yz, zx} (surface area: all 1)
    // Early split clipping (Ernst & Greiner 2007): a triangle whose box surface exceeds
    // presplit_ratio x twice its area enters the build as up to 2^presplit_levels
    // references, the bounds of its pieces clipped at the box's longest-axis midpoints
    // (rounded outward) (0: off)
    int presplit_levels = 0;
    float presplit_ratio = 8.0f;
};

struct BvhBuildResult {
    std::vector<GpuBvhNode> nodes; // node 0 is the root (always an internal node)
    std::vector<GpuTriangle> tris; // leaf order
    uint32_t max_depth = 0;
    uint32_t max_leaf = 0;
    float sah_cost = 0.0f;
};

// Builds one BVH over `tris` (all of one hit-mask class). Node indices and
// triangle indices are offset by node_base / tri_base so several BVHs can share
// one node array and one triangle array.
BvhBuildResult build_bvh(const std::vector<BuildTriangle>& tris, const BvhBuildOptions& opt, uint32_t node_base, uint32_t tri_base);

struct Bvh8BuildResult {
    std::vector<GpuBvh8Node> nodes; // node 0 (+ node_base) is the root
    std::vector<GpuTriangle> tris;  // leaf triangle rows (GpuBvh8Node), holes included
    uint32_t max_depth = 0;
    uint32_t leaf_children = 0;
    uint64_t triangles = 0; // records of `tris` that are not holes
    float sah_cost = 0.0f; // SAH cost (node 1, triangle Bvh8CollapseOptions::tri_cost) relative to the root
};

// Collapses a BVH2 (built with max_leaf_size <= kBvh8MaxLeafSize, node_base 0,
// tri_base 0) into the 8-wide quantized layout: every node adopts the largest-area
// internal descendants of its BVH2 node until it has 8 children (or the SAH-optimal
// set, Bvh8CollapseOptions::sah_optimal), children are
// placed in octant slots, and the triangles of each node's leaf children are
// stored contiguously. Node/triangle indices are offset by node_base/tri_base.
struct Bvh8CollapseOptions {
    // true: the SAH-optimal child selection of Ylitie et al. 2017 (dynamic programming
    // over BVH2 subtrees, also merging subtrees of <= kBvh8MaxLeafSize triangles into
    // one leaf slot; the default: C4 traversal 2.26 -> 2.24 ms, shadow 0.74 -> 0.70 ms,
    // 2,148 -> 2,174 Mrays/s, profiles/r03_h_ab); false: greedy largest-area opening
    bool sah_optimal = true;
    float node_cost = 1.0f; // SAH cost of visiting a BVH8 node (8 box tests)
    float tri_cost = 1.0f;  // SAH cost of one triangle test
    float area_w[3] = { 1.0f, 1.0f, 1.0f }; // SAH face weights {xy, yz, zx}, as BvhBuildOptions::area_w
    // -1: internal children in octant slots (visited in slot ^ ray octant order);
    // 0-2: in slots 0, 1, ... by their box's lower bound along that axis (a BVH that
    // only rays along +axis traverse: the sun's light-space BVH, slot order = octant 0)
    int slot_sort_axis = -1;
    int threads = 0; // subtrees collapsed in parallel (0 = hardware concurrency)
};
Bvh8BuildResult collapse_bvh8(const BvhBuildResult& bvh2, uint32_t node_base, uint32_t tri_base, const Bvh8CollapseOptions& opt);

// The 48-B triangle record of a build triangle (v0, e1 = v1 - v0, e2 = v2 - v0 in
// fp32, instance, primitive, facing flip): what the traversal's Möller–Trumbore reads.
GpuTriangle make_gpu_triangle(const BuildTriangle& t);

// Hole records of the triangle rows (kHoleInstance)
GpuTriangle holeTriangle();
bool isHoleTriangle(const GpuTriangle& t);
// Triangle indices of leaf slot s of a node (tri_base + s + stride * i for the
// consecutive set bits of its row from i = 0); 0 for a slot that is not a leaf, -1
// when a leaf slot has no triangle, an internal slot is marked leaf, or the slot's
// spread reaches another slot's triangle (GpuBvh8Node)
int bvh8SlotTriangles(const GpuBvh8Node& nd, int s, uint32_t out[kBvh8MaxLeafSize]);

// Absolute box inflation for the BVH8 slab test: 1e-6 of the diagonal of the
// bounding box of nTriangles world-space triangles (9 floats each). It bounds
// the rounding of (p - o) * idir for anchors p and ray origins o in the scene
// (about 2 ulp of the diagonal, i.e. 2.4e-7 of it) with a 4x margin.
float bvh8_inflation(const float* xyz, uint64_t nTriangles);
float bvh8_inflation_box(const float lo[3], const float hi[3]);

// The sun's light-space BVH (k_trace_shadow<SUN>): every triangle of every hit-mask
// class in the frame (u, v, w = the shadow rays' direction L = -normalize(sun dir) as
// the kernels compute it in fp32), leaves holding the world-space records.
struct SunBvhInput {
    std::vector<BuildTriangle> tris;  // light-space vertices; primitive = index into world
    std::vector<GpuTriangle> world;   // world-space records (make_gpu_triangle)
    double frame[3][3] = {};          // rows u, v, w
    float maxAbs = 0.0f;              // largest |world coordinate|
    float inflateAbs = 0.0f;          // out (build_sun_bvh): the boxes' absolute inflation (the refit's floor)
};
void sun_frame(const float sun_dir[3], double frame[3][3]);
void sun_add_triangles(SunBvhInput& in, const std::vector<BuildTriangle>& world_tris, int threads = 0);
// The same from world-space triangle records as the world BVHs hold them (holes skipped):
// the background rebuild after a sun-direction change or a refit (ark_ddgi.cpp)
void sun_add_records(SunBvhInput& in, const std::vector<GpuTriangle>& records, int threads = 0);
// Builds the BVH2 (opt; its inflation replaced by the light-space bound), the BVH8
// (copt, slots sorted by w) and swaps in the world records; consumes in.tris and
// in.world. False when a BVH2 leaf exceeds kBvh8MaxLeafSize.
bool build_sun_bvh(SunBvhInput& in, const BvhBuildOptions& opt, const Bvh8CollapseOptions& copt, Bvh8BuildResult& out);
// Whether the light-space BVH pays for a scene: n sample sun shadow rays (points on
// triangles whose front face faces the sun, deterministic) traced any-hit on the host
// through both structures (exact decoded planes, tmin 0.025; frame == nullptr: the
// world BVHs and their roots, else the light frame with rays along +w), cost = node
// visits + triangle tests per ray - the persistent traversals' steps. Large
// axis-aligned surfaces (walls, a ground plane: C5's city block) become long slanted
// boxes in light space, where the world BVH culls them.
void sun_sample_origins(const std::vector<GpuTriangle>& tris, const float L[3], uint32_t n, std::vector<float>& out_xyz);
double sun_shadow_cost(const std::vector<GpuBvh8Node>& nodes, const std::vector<GpuTriangle>& tris, const int32_t* roots, int nRoots,
                       const double (*frame)[3], const float L[3], const std::vector<float>& origins_xyz);
// The light-space traversal has no LDS node cache, but its node test is a handful of
// byte compares: at C4's sampled ratio 0.948 it is the faster one (shadow phase 0.705 ->
// 0.669 ms, K = 2048 windows 1,384 -> 1,471 Mrays/s, profiles/r04_c_bench_step7/8), so
// it is chosen unless it saves less than 2 % of the sampled steps.
inline bool sun_bvh_pays(double costWorld, double costLight) { return costLight < 0.98 * costWorld; }

} // namespace ark
