/*
 * ark_ddgi_debug.h — diagnostic entry points of libark_ddgi (not used by the
 * DDGI node). They exist so tests can pin the device side of the deterministic
 * math (ark_fmath.h) against the CPU side bit for bit.
 */
#ifndef ARK_DDGI_DEBUG_H
#define ARK_DDGI_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Extra resource id for ark_ddgi_read: the primary-pass hit records of the last
 * update, 16 B each ({float t (negative = backface, +inf = miss), u, v, uint32
 * leaf-order triangle}) at slot * rays_per_probe + sample (slot = window slot,
 * sample = the ray's Fibonacci sample index). */
#define ARK_DDGI_DEBUG_HITS 100

/* Extra resource id for ark_ddgi_read: the traversal iterations (both passes) of
 * every probe ray of the last counting update (ark_ddgi_set_counting), uint16 at
 * the ray's hit-record index (slot * rays_per_probe + sample), saturating at 65535;
 * sized max_probe_updates x max_rays_per_probe. For the launch-tail analysis
 * (tools/ray_cost.py); counting is enabled first. */
#define ARK_DDGI_DEBUG_RAY_STEPS 101

/* Evaluates op (0 sin, 1 cos, 2 acos, 3 atan2(x,y), 4 log2, 5 exp2, 6 pow(x,y),
 * 7 fp32->fp16->fp32 round trip, 8 powf_pos_(x,y)) on `device` for n inputs (host arrays). */
int ark_ddgi_debug_fmath(int device, int op, const float* x, const float* y, float* out, uint64_t n);

/* Host-side evaluation of the same functions (for comparison with the device). */
int ark_ddgi_debug_fmath_host(int op, const float* x, const float* y, float* out, uint64_t n);

/* sizeof() of the ABI structs, in this order: ArkDdgiDesc, ArkRTVertex,
 * ArkRTTriangleMesh, ArkShaderMaterial, ArkTexture, ArkRTInstance,
 * ArkDirectionalLight, ArkSpotLight, ArkDdgiScene, ArkDdgiFrameParams,
 * ArkDdgiCounters, ArkDdgiDeviceViews, ArkDdgiBvhStats. Returns the count written. */
int ark_ddgi_debug_struct_sizes(uint32_t* out, int n);

/* Builds the BVH used by ark_ddgi_set_scene (binned-SAH BVH2 with leaves of at most
 * 3 triangles, collapsed into 8-wide quantized nodes) over n world-space triangles
 * (9 floats each) on the host and checks it: every triangle in exactly one leaf,
 * every quantized plane exactly representable, every triangle vertex inside the
 * decoded boxes of its leaf and of all its ancestors. out[8] = {nodes, leaf
 * children, max depth, violations, triangles, bvh2 nodes, internal children, BVH8
 * SAH cost x 1e6 (node cost 1)}. The BVH8 child selection is set_scene's (SAH-optimal
 * collapse, default triangle cost); _opts selects the greedy collapse (sah_optimal 0)
 * or another triangle cost (tri_cost > 0), for comparing builds.
 * Returns 0 when the check passes, 1 when it found violations. No GPU. */
int ark_ddgi_debug_bvh8_check(const float* triangles, uint64_t n, uint64_t* out);
int ark_ddgi_debug_bvh8_check_opts(const float* triangles, uint64_t n, int sah_optimal, float tri_cost, uint64_t* out);

/* The host traversal simulator (ark_ddgi_debug_bvh8_trace_stats) is a tool, not part
 * of this library: tools/sim/bvh_trace_sim.h, tools/lib/libark_bvhsim.so. */

/* The sun's light-space BVH (the one set_scene builds for k_trace_shadow<SUN>) built
 * on the host from n world triangles (9 floats each) and checked without a GPU: a sun
 * shadow ray from each of n_rays origins (3 floats) along L = -normalize(sun_dir),
 * [0.025, tmax], any hit through the BVH with a host restatement of the kernel's
 * light-space node test, and against every triangle. out[8] = {rays, occluded (brute
 * force), occluded (BVH), mismatches, node visits, triangle tests, BVH8 nodes, max
 * stack depth}. Returns 0 when no ray differs, 2 on a mismatch, 1 on a build error. */
int ark_ddgi_debug_sun_bvh_check(const float* triangles, uint64_t n, const float* sun_dir, const float* origins, uint64_t n_rays, float tmax,
                                 uint64_t* out);

/* set_scene's choice of structure for the sun's shadow rays (ark_ddgi.cpp, ARK_SUN_BVH
 * unset): the world BVH8 and the light-space BVH8 of the triangles are built, sample
 * sun shadow rays from sun-facing points traced any-hit through both on the host;
 * out[4] = {world steps per ray, light-space steps per ray, 1 if the light-space BVH
 * is chosen, samples}. No GPU. */
int ark_ddgi_debug_sun_choice(const float* triangles, uint64_t n, const float* sun_dir, uint32_t n_samples, double* out);

/* FNV-1a 64 digests of the geometry the context's kernels read now (the front copy,
 * after everything it enqueued): out[4] = {world BVH8 nodes, world triangle records,
 * light-space sun BVH8 nodes, its records} (the sun's 0 without one). For the refit
 * tests: refits that reach only the nodes of moved instances leave the same bytes as
 * one that reaches every node. Synchronous. */
int ark_ddgi_debug_scene_digest(struct ArkDdgiCtx* ctx, uint64_t* out);

#ifdef __cplusplus
}
#endif

#endif /* ARK_DDGI_DEBUG_H */
