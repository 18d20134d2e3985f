// ASan + UBSan run of the host-side code on the path (SURVEY §5 "race detection /
// sanitizers"): the CPU oracle (frames with offsets, the AO bake, lighting compose),
// the synthetic soup generator and the BVH2 -> BVH8 builder with its structural check.
// Built by tests/test_sanitizers.py with g++ -fsanitize=address,undefined
// -fno-sanitize-recover=all; any report aborts with a non-zero status.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/ark_ddgi.h"
#include "../../include/ark_ddgi_debug.h"
#include "../../include/ark_scene.h"

extern "C" {
void* oracle_create(const ArkDdgiDesc* desc);
void oracle_destroy(void* ctx);
int oracle_set_scene(void* ctx, const ArkDdgiScene* s, int threads);
int oracle_update(void* ctx, const ArkDdgiFrameParams* p, int threads);
int oracle_read(void* ctx, int which, void* dst, uint64_t bytes);
int oracle_bake_ao(void* ctx, uint32_t instance, uint32_t W, uint32_t H, uint32_t samples, int bent, uint32_t row0, uint32_t row1,
                   uint32_t* triOut, uint16_t* baryOut, uint8_t* out, int threads);
}

#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

int main()
{
    ArkSoupParams sp;
    ark_soup_default_params(&sp);
    sp.triangle_count = 4096;
    sp.extent = 6.0f;
    ArkSoupScene* soup = nullptr;
    CHECK(ark_soup_generate(&sp, &soup) == 0);
    const ArkDdgiScene* scene = ark_soup_scene_view(soup);

    // BVH8 build + structural check over the soup's world-space triangles
    std::vector<float> tri(static_cast<size_t>(scene->index_count) * 3);
    uint64_t nTri = 0;
    for (uint32_t mi = 0; mi < scene->mesh_count; ++mi) {
        const ArkRTTriangleMesh& m = scene->meshes[mi];
        const uint64_t end = mi + 1 < scene->mesh_count ? static_cast<uint64_t>(scene->meshes[mi + 1].first_index) : scene->index_count;
        for (uint64_t k = static_cast<uint64_t>(m.first_index); k < end; ++k) {
            const uint32_t v = static_cast<uint32_t>(m.first_vertex) + scene->indices[k];
            for (int a = 0; a < 3; ++a) tri[nTri * 3 + a] = scene->positions[3 * static_cast<size_t>(v) + a];
            ++nTri;
        }
    }
    nTri /= 3;
    uint64_t stats[8] = {};
    CHECK(ark_ddgi_debug_bvh8_check(tri.data(), nTri, stats) == 0);
    CHECK(stats[3] == 0 && stats[4] == nTri); // no violations, every triangle in a leaf
    std::printf("bvh8: %llu triangles, %llu nodes\n", static_cast<unsigned long long>(nTri), static_cast<unsigned long long>(stats[0]));

    // oracle: 4x4x4 probes x 64 rays, offsets on, three frames
    ArkDdgiDesc d;
    std::memset(&d, 0, sizeof(d));
    d.struct_size = sizeof(d);
    d.grid_dims[0] = d.grid_dims[1] = d.grid_dims[2] = 4;
    for (int k = 0; k < 3; ++k) {
        d.probe_spacing[k] = 1.5f;
        d.offset_to_first[k] = 0.5f;
    }
    d.max_rays_per_probe = 64;
    d.max_probe_updates = 64;
    d.z_far = 100.0f;
    d.clear_overflow_mode = ARK_DDGI_CLEAR_OVERFLOW_INF;
    d.shard_count = 1;
    void* o = oracle_create(&d);
    CHECK(o != nullptr);
    CHECK(oracle_set_scene(o, scene, 2) == 0);
    for (uint32_t frame = 0; frame < 3; ++frame) {
        ArkDdgiFrameParams p;
        std::memset(&p, 0, sizeof(p));
        p.struct_size = sizeof(p);
        p.rays_per_probe = 64;
        p.probe_updates = 64;
        p.first_probe_index = 0;
        p.frame_index = frame;
        p.hysteresis_irradiance = frame ? 0.98f : 0.0f;
        p.hysteresis_visibility = frame ? 0.98f : 0.0f;
        p.visibility_sharpness = 50.0f;
        p.environment_multiplier = 1.0f;
        p.ambient_amount = 0.0f;
        p.delta_time = 1.0f / 60.0f;
        p.update_offsets = 1;
        CHECK(oracle_update(o, &p, 2) == 0);
    }
    std::vector<uint16_t> irr(4 * 10 * 4 * 4 * 10 * 4);
    CHECK(oracle_read(o, ARK_DDGI_ATLAS_IRRADIANCE, irr.data(), irr.size() * 2) == 0);
    // AO bake of the soup's first instance, a small texture
    const uint32_t W = 32, H = 32;
    std::vector<uint32_t> bt(W * H);
    std::vector<uint16_t> bb(W * H * 4);
    std::vector<uint8_t> bo(W * H * 4);
    CHECK(oracle_bake_ao(o, 0, W, H, 4, 1, 0, H, bt.data(), bb.data(), bo.data(), 2) == 0);
    oracle_destroy(o);
    ark_soup_free(soup);
    std::printf("OK\n");
    return 0;
}
