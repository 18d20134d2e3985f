// ddgi_types.h — HBM layouts shared by the HIP kernels and the host side of
// libark_ddgi (BVH builder, context). Plain structs, no HIP types.
#pragma once

#include <stdint.h>

namespace ark {

// BVH2 node, 64 B = 4 x 16 B (one half of a 128 B line). Child boxes are stored in
// the parent ("Aila–Laine" layout) so one node fetch tests both children:
//   n0 = (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)
//   n1 = (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//   n2 = (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
//   n3 = (child0, child1, 0, 0) as int32: >= 0 internal node index,
//        < 0 leaf: ~((firstTri << kLeafCountBits) | (count - 1)).
struct alignas(16) GpuBvhNode {
    float n0[4];
    float n1[4];
    float n2[4];
    int32_t child[4];
};
static_assert(sizeof(GpuBvhNode) == 64, "node is 64 B");

constexpr int kLeafCountBits = 3;           // up to 8 triangles per leaf
constexpr int kMaxLeafSize = 1 << kLeafCountBits;

// 8-wide BVH node with quantized child boxes, 80 B = 5 x 16 B (compressed wide
// BVH: one fetch tests 8 children). Child boxes are stored as 8-bit offsets on a
// per-axis power-of-two grid anchored at p:
//     plane = p + q * 2^(e - 127),  q in [0, 255]
// p is an exact multiple of the grid step and |p / step| + 255 < 2^24, so every
// plane decodes EXACTLY in fp32 (one fma), and q is rounded outward, so a decoded
// child box contains the (already inflated) BVH2 child box it replaces.
//   w0..2  p.xyz            w3  e.x | e.y << 8 | e.z << 16 | imask << 24
//   w4     child_base       w5  tri_base          w6  leaf_tris   w7  stride | leaf_mask << 8
//   w8,9   qlo.x[8]         w10,11 qlo.y[8]       w12,13 qlo.z[8]
//   w14,15 qhi.x[8]         w16,17 qhi.y[8]       w18,19 qhi.z[8]
// Slot s of a node holds its child whose centre lies on the (s & 1 ? + : -) x,
// (s & 2 ? + : -) y, (s & 4 ? + : -) z side of the node centre, as far as the
// children allow, so visiting hit slots in increasing (s ^ rayOctant) order is
// roughly front to back. imask bit s: internal child, stored at
// child_base + popcount(imask & ((1 << s) - 1)). leaf_mask bit s: leaf child.
// Leaf triangles in strided rows: triangle i (< kBvh8MaxLeafSize) of leaf slot s is
// at tri_base + s + stride * i, and bit s + stride * i of leaf_tris marks it, so the
// triangles of a set H of hit leaf slots are
//     (H | H << stride | H << 2 stride) & leaf_tris
// (three VALU; a per-slot offset/count code cost ~40). The builder picks the
// smallest stride (1..8; 8 always works) for which no position s' + stride * i'
// (i' < 3) of a leaf s' belongs to another slot's triangle, which keeps a node's
// triangles close together (stride 8 for all nodes spread them over 24 records:
// +42 % HBM traffic, profiles/r03_k). Nodes' rows interleave in the triangle array
// (first fit), and a position nothing uses is a hole record (kHoleInstance) that no
// leaf references.
struct alignas(16) GpuBvh8Node {
    float p[3];
    uint8_t e[3];
    uint8_t imask;
    uint32_t child_base;
    uint32_t tri_base;
    uint32_t leaf_tris;
    uint8_t tri_stride;
    uint8_t leaf_mask;
    uint8_t pad[2];
    uint8_t qlo[3][8];
    uint8_t qhi[3][8];
};
static_assert(sizeof(GpuBvh8Node) == 80, "BVH8 node is 80 B");
constexpr int kBvh8MaxLeafSize = 3;
// the positions of leaf slot s's row (bits s, s + stride, s + 2 stride), unmasked
inline constexpr uint32_t bvh8SlotRow(uint32_t stride, int s) { return (1u | 1u << stride | 1u << (2u * stride)) << s; }

// World-space triangle record, 48 B = 3 x 16 B, in leaf order:
//   t0 = (v0.x, v0.y, v0.z, e1.x)   t1 = (e1.y, e1.z, e2.x, e2.y)
//   t2 = (e2.z, instance, primitive, flip)  (e1 = v1 - v0, e2 = v2 - v0; flip = 1
//        when the instance's det(ObjectToWorld) < 0, i.e. its facing is mirrored)
// Closest-hit ties are broken on (instance, primitive), i.e. the global triangle
// id, so the hit does not depend on the BVH shape (same rule in the oracle).
// A hole of the BVH8 triangle rows (GpuBvh8Node) is all zero but instance =
// kHoleInstance.
constexpr uint32_t kHoleInstance = 0xffffffffu;
struct alignas(16) GpuTriangle {
    float t0[4];
    float t1[4];
    float t2[4];
};
static_assert(sizeof(GpuTriangle) == 48, "triangle is 48 B");

// Per-instance shading data (TLAS instance + RT mesh), 64 B.
struct alignas(16) GpuInstance {
    float normal_matrix[12]; // mat3(ObjectToWorld) as 3 rows of 4 (w unused)
    int32_t rt_mesh_index;
    int32_t flip_facing;     // det(ObjectToWorld) < 0
    int32_t hit_mask;
    int32_t material_index;  // meshes[rt_mesh_index].material_index, resolved at upload
};

struct GpuTextureInfo {
    int32_t width, height, wrap, _pad;
    uint64_t texel_offset; // in float4 texels into the texel pool
};

// Spot light as consumed by the closest hit (LightData.h:19-40 subset), 80 B.
struct alignas(16) GpuSpotLight {
    float color[4];
    float direction[4];
    float right[4];
    float up[4];
    float position[4]; // w = outer cone half angle
    int32_t ies_texture;
    int32_t _pad[3];
};

// One probe of the current window (slot), 32 B: position (+offset), rotation.
struct alignas(16) GpuProbeSlot {
    float pos[3];
    uint32_t probe_index;
    float axis[3];
    float angle_sin;
    float angle_cos;
    float _pad[3];
};

// Hit record of the primary pass, 16 B: signed t (negative = backface, +inf =
// miss), barycentrics (u, v) and the leaf-order triangle index.
struct alignas(16) GpuHit {
    float t;
    float u;
    float v;
    uint32_t tri;
};

} // namespace ark
