// bvh_trace_sim.h — host traversal simulator of the BVH8 (tools/lib/libark_bvhsim.so).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Traversal statistics of that BVH8 on the host (a scalar simulation of k_trace's
 * closest-hit order: hit children, origin-containing first, then octant order; the
 * leaf triangles of a node right after it): nRays rays of 7 floats (origin,
 * direction, tmax) over `threads` host threads. out[9] = {node visits, triangle
 * tests, hits, BVH8 nodes, SAH cost x 1e6, max steps of one ray, max depth,
 * triangle records (leaf triangle rows, holes included), children the exact box
 * test accepts and the ARK_SIM_BOX form (kernel32 | f16) rejects (must be 0)};
 * per_ray_steps (if not NULL) gets each ray's node visits + triangle tests.
 * For comparing BVH builds (ARK_BVH8_COLLAPSE, ARK_BVH8_TRI_COST,
 * ARK_BVH_INTERSECTION_COST) without a GPU: tools/bvh_stats.py. */
int ark_ddgi_debug_bvh8_trace_stats(const float* triangles, uint64_t n, const float* rays, uint64_t n_rays, int threads, uint64_t* out,
                                    uint32_t* per_ray_steps /* nullable: node visits + triangle tests of each ray */);

#ifdef __cplusplus
}
#endif
