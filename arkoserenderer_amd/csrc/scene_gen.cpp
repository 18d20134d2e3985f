// scene_gen.cpp — deterministic synthetic triangle-strip soup.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/ark_scene.h"

namespace {

// PCG32 (O'Neill, pcg32_srandom / pcg32_random / bounded float)
struct Pcg32 {
    uint64_t state = 0, inc = 0;
    Pcg32(uint64_t initstate, uint64_t initseq)
    {
        inc = (initseq << 1u) | 1u;
        next();
        state += initstate;
        next();
    }
    uint32_t next()
    {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t xorshifted = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = static_cast<uint32_t>(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((-rot) & 31u));
    }
    float uniform() { return static_cast<float>(next() >> 8) * (1.0f / 16777216.0f); } // [0,1)
    float uniform(float a, float b) { return a + (b - a) * uniform(); }
};

struct V { float x, y, z; };
V sub(V a, V b) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
V add(V a, V b) { return { a.x + b.x, a.y + b.y, a.z + b.z }; }
V mul(V a, float s) { return { a.x * s, a.y * s, a.z * s }; }
float dotv(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V crossv(V a, V b) { return { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x }; }
V norm(V a) { float l = std::sqrt(dotv(a, a)); return mul(a, 1.0f / l); }
V sphere(Pcg32& r)
{
    float z = 2.0f * r.uniform() - 1.0f;
    float phi = 6.2831853f * r.uniform();
    float s = std::sqrt(std::max(0.0f, 1.0f - z * z));
    return { s * std::cos(phi), s * std::sin(phi), z };
}

} // namespace

struct ArkSoupScene {
    std::vector<float> positions;
    std::vector<ArkRTVertex> vertices;
    std::vector<uint32_t> indices;
    std::vector<ArkRTTriangleMesh> meshes;
    std::vector<ArkShaderMaterial> materials;
    std::vector<ArkRTInstance> instances;
    ArkDdgiScene view {};
};

extern "C" {

void ark_soup_default_params(ArkSoupParams* p)
{
    std::memset(p, 0, sizeof(*p));
    p->struct_size = sizeof(ArkSoupParams);
    p->triangle_count = 10000000ull;
    p->extent = 31.0f;
    p->step_min = 0.05f;
    p->step_max = 0.3f;
    p->width_min = 0.05f;
    p->width_max = 0.3f;
    p->seed = 0xA2C05E00ull;
    p->stream = 1;
    p->material_count = 16;
    p->sun_color[0] = p->sun_color[1] = p->sun_color[2] = 3.0f;
    V d = norm(V { 0.5f, -1.0f, 0.2f });
    p->sun_direction[0] = d.x;
    p->sun_direction[1] = d.y;
    p->sun_direction[2] = d.z;
    p->has_sun = 1;
}

int ark_soup_generate(const ArkSoupParams* p, ArkSoupScene** out)
{
    if (!p || !out || p->struct_size != sizeof(ArkSoupParams) || p->material_count == 0) return ARK_DDGI_E_INVALID_ARGUMENT;
    const uint64_t strips = p->triangle_count / 16;
    if (strips == 0) return ARK_DDGI_E_INVALID_ARGUMENT;
    auto* s = new ArkSoupScene();
    Pcg32 rng(p->seed, p->stream);
    const uint32_t M = p->material_count;
    // materials: baseColor ~ U(0.05,0.95)^3, metallic 0, roughness 0.5, default textures
    for (uint32_t m = 0; m < M; ++m) {
        ArkShaderMaterial mat;
        std::memset(&mat, 0, sizeof(mat));
        mat.base_color = mat.normal_map = mat.metallic_roughness = mat.emissive = -1;
        mat.occlusion = mat.bent_normal_map = -1;
        mat.blend_mode = ARK_BLEND_MODE_OPAQUE;
        mat.mask_cutoff = 1.0f;
        mat.metallic_factor = 0.0f;
        mat.roughness_factor = 0.5f;
        mat.dielectric_reflectance = 0.04f;
        for (int c = 0; c < 3; ++c) mat.color_tint[c] = rng.uniform(0.05f, 0.95f);
        mat.color_tint[3] = 1.0f;
        s->materials.push_back(mat);
    }
    s->positions.reserve(strips * 18 * 3);
    s->vertices.reserve(strips * 18);
    s->indices.reserve(strips * 48);
    const uint64_t perMesh = (strips + M - 1) / M;
    for (uint32_t m = 0; m < M; ++m) {
        const uint64_t k0 = m * perMesh, k1 = std::min<uint64_t>(strips, k0 + perMesh);
        if (k0 >= k1) break;
        ArkRTTriangleMesh mesh { static_cast<int32_t>(s->positions.size() / 3), static_cast<int32_t>(s->indices.size()), static_cast<int32_t>(m) };
        s->meshes.push_back(mesh);
        uint32_t local = 0;
        for (uint64_t k = k0; k < k1; ++k) {
            V o = { rng.uniform() * p->extent, rng.uniform() * p->extent, rng.uniform() * p->extent };
            V d = sphere(rng);
            V w;
            do {
                V a = sphere(rng);
                w = sub(a, mul(d, dotv(a, d)));
            } while (dotv(w, w) < 1e-6f);
            w = norm(w);
            float step = rng.uniform(p->step_min, p->step_max);
            float width = rng.uniform(p->width_min, p->width_max);
            V n = norm(crossv(w, d)); // geometric normal of the CCW triangles below
            for (int j = 0; j < 9; ++j) {
                V a = add(o, mul(d, step * j));
                V b = add(a, mul(w, width));
                for (int e = 0; e < 2; ++e) {
                    const V q = e ? b : a;
                    s->positions.insert(s->positions.end(), { q.x, q.y, q.z });
                    ArkRTVertex vx;
                    std::memset(&vx, 0, sizeof(vx));
                    vx.tex_coord[0] = static_cast<float>(j) / 8.0f;
                    vx.tex_coord[1] = static_cast<float>(e);
                    vx.normal[0] = n.x;
                    vx.normal[1] = n.y;
                    vx.normal[2] = n.z;
                    vx.tangent[0] = d.x;
                    vx.tangent[1] = d.y;
                    vx.tangent[2] = d.z;
                    vx.tangent[3] = 1.0f;
                    s->vertices.push_back(vx);
                }
            }
            for (uint32_t j = 0; j < 8; ++j) {
                uint32_t b = local + 2 * j;
                s->indices.insert(s->indices.end(), { b, b + 1, b + 2, b + 1, b + 3, b + 2 });
            }
            local += 18;
        }
        ArkRTInstance inst;
        std::memset(&inst, 0, sizeof(inst));
        inst.object_to_world[0] = inst.object_to_world[5] = inst.object_to_world[10] = 1.0f;
        inst.rt_mesh_index = static_cast<uint32_t>(s->meshes.size() - 1);
        inst.triangle_count = static_cast<uint32_t>((k1 - k0) * 16);
        inst.hit_mask = ARK_RT_HIT_MASK_OPAQUE;
        s->instances.push_back(inst);
    }
    ArkDdgiScene& v = s->view;
    std::memset(&v, 0, sizeof(v));
    v.struct_size = sizeof(ArkDdgiScene);
    v.indices = s->indices.data();
    v.index_count = s->indices.size();
    v.positions = s->positions.data();
    v.vertex_count = s->vertices.size();
    v.vertices = s->vertices.data();
    v.meshes = s->meshes.data();
    v.mesh_count = static_cast<uint32_t>(s->meshes.size());
    v.materials = s->materials.data();
    v.material_count = static_cast<uint32_t>(s->materials.size());
    v.instances = s->instances.data();
    v.instance_count = static_cast<uint32_t>(s->instances.size());
    v.has_directional_light = p->has_sun;
    for (int c = 0; c < 3; ++c) {
        v.directional_light.color[c] = p->sun_color[c];
        v.directional_light.world_space_direction[c] = p->sun_direction[c];
    }
    v.environment_texture = -1;
    *out = s;
    return ARK_DDGI_OK;
}

const ArkDdgiScene* ark_soup_scene_view(const ArkSoupScene* s) { return s ? &s->view : nullptr; }

void ark_soup_free(ArkSoupScene* s) { delete s; }

} // extern "C"
