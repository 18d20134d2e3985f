// CPU test of the GpuScene -> ArkDdgiScene adapter (host/rendering/GpuScene.cpp):
// GpuScene.cpp:872-929 (RT meshes + TLAS instances per LOD segment, hit mask by
// blend mode, segments without a BLAS skipped) and :790-858 (light data). Built and
// run by tests/test_gpuscene_adapter.py with g++ (no GPU, no HIP).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "core/Logging.h"
#include "rendering/GpuScene.h"

namespace ark {
int& errorCounter() { static int n = 0; return n; }
const char* logLevelName(LogLevel l) { return l == LogLevel::Fatal ? "Fatal" : "Log"; }
}

static int failures = 0;
#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++failures; } } while (0)

int main()
{
    GpuScene gs(*reinterpret_cast<HipBackend*>(&failures)); // the adapter never touches the backend
    gs.camera().setExposure(0.25f);
    // two segments of geometry through the VertexManager path
    const float p0[9] = { 0, 0, 0, 1, 0, 0, 0, 1, 0 };
    const float p1[12] = { 0, 0, 1, 1, 0, 1, 1, 1, 1, 0, 1, 1 };
    ArkRTVertex v[4] {};
    const uint32_t i0[3] = { 0, 1, 2 }, i1[6] = { 0, 1, 2, 0, 2, 3 };
    VertexAllocation a0 = gs.allocateVertices(p0, v, 3, i0, 3);
    VertexAllocation a1 = gs.allocateVertices(p1, v, 4, i1, 6);
    CHECK(a0.firstVertex == 0 && a0.firstIndex == 0 && a1.firstVertex == 3 && a1.firstIndex == 3 && a1.indexCount == 6);
    ArkShaderMaterial m {};
    m.blend_mode = ARK_BLEND_MODE_OPAQUE;
    const int32_t opaque = gs.registerMaterial(m);
    m.blend_mode = ARK_BLEND_MODE_MASKED;
    const int32_t masked = gs.registerMaterial(m);
    m.blend_mode = ARK_BLEND_MODE_TRANSLUCENT;
    const int32_t blend = gs.registerMaterial(m);
    // mesh A: LOD0 = {a0 opaque, a1 masked}, LOD1 = {a0 translucent}; mesh B: {a1 opaque (no BLAS yet), a0 opaque}
    StaticMesh A;
    A.LODs.push_back(StaticMeshLOD { { StaticMeshSegment { a0, opaque, true }, StaticMeshSegment { a1, masked, true } } });
    A.LODs.push_back(StaticMeshLOD { { StaticMeshSegment { a0, blend, true } } });
    StaticMesh B;
    B.LODs.push_back(StaticMeshLOD { { StaticMeshSegment { a1, opaque, false }, StaticMeshSegment { a0, opaque, true } } });
    const uint32_t ha = gs.addStaticMesh(A), hb = gs.addStaticMesh(B);
    StaticMeshInstance ia {}, ib {};
    ia.mesh = ha;
    ib.mesh = hb;
    for (int k = 0; k < 16; ++k) ia.worldMatrix[k] = ib.worldMatrix[k] = (k % 5 == 0) ? 1.0f : 0.0f;
    ib.worldMatrix[12] = 5.0f; // column-major translation x
    ib.worldMatrix[1] = 2.0f;  // column 0, row 1
    gs.addStaticMeshInstance(ia);
    gs.addStaticMeshInstance(ib);
    ManagedDirectionalLight sun;
    sun.color[0] = 0.5f; sun.color[1] = 0.25f; sun.color[2] = 1.0f;
    sun.intensity = 8.0f;
    sun.forward[0] = 0.0f; sun.forward[1] = -1.0f; sun.forward[2] = 0.0f;
    gs.setDirectionalLight(sun);
    ManagedSpotLight spot;
    spot.color[0] = spot.color[1] = spot.color[2] = 1.0f;
    spot.intensity = 100.0f;
    spot.position[1] = 3.0f;
    spot.outerConeAngle = 1.5f;
    spot.iesLut = 7;
    gs.addSpotLight(spot);
    gs.updateLightData();
    const ArkDdgiScene& s = gs.rtScene();
    CHECK(s.struct_size == sizeof(ArkDdgiScene));
    // A: 3 segments over 2 LODs, B: 1 (the BLAS-less segment is skipped)
    CHECK(s.instance_count == 4 && s.mesh_count == 4);
    const uint32_t masks[4] = { ARK_RT_HIT_MASK_OPAQUE, ARK_RT_HIT_MASK_MASKED, ARK_RT_HIT_MASK_BLEND, ARK_RT_HIT_MASK_OPAQUE };
    const uint32_t tris[4] = { 1, 2, 1, 1 };
    for (uint32_t i = 0; i < 4 && i < s.instance_count; ++i) {
        CHECK(s.instances[i].rt_mesh_index == i); // customInstanceId = RT mesh index
        CHECK(s.instances[i].hit_mask == masks[i]);
        CHECK(s.instances[i].triangle_count == tris[i]);
    }
    CHECK(s.meshes[1].first_vertex == 3 && s.meshes[1].first_index == 3 && s.meshes[1].material_index == masked);
    CHECK(s.meshes[3].first_vertex == 0 && s.meshes[3].material_index == opaque);
    // instance B: row-major 3x4 of the column-major matrix
    CHECK(s.instances[3].object_to_world[3] == 5.0f && s.instances[3].object_to_world[4] == 2.0f && s.instances[3].object_to_world[0] == 1.0f);
    // lights: colour * intensity * preExposure, half the outer cone angle, IES LUT handle
    CHECK(s.has_directional_light == 1);
    CHECK(s.directional_light.color[0] == 0.5f * 8.0f * 0.25f && s.directional_light.color[2] == 1.0f * 8.0f * 0.25f);
    CHECK(s.directional_light.world_space_direction[1] == -1.0f);
    CHECK(s.spot_light_count == 1 && s.spot_lights[0].color[1] == 100.0f * 0.25f && s.spot_lights[0].outer_cone_half_angle == 0.75f);
    CHECK(s.spot_lights[0].ies_profile_index == 7 && s.spot_lights[0].world_space_position[1] == 3.0f);
    CHECK(s.index_count == 9 && s.vertex_count == 7 && s.material_count == 3 && s.environment_texture == -1);
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
