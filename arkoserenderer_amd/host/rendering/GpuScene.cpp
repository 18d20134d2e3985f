#include "GpuScene.h"

#include <cstring>

#include "core/Logging.h"

VertexAllocation GpuScene::allocateVertices(const float* positions, const ArkRTVertex* nonPositionVertices, uint32_t vertexCount,
                                            const uint32_t* indices, uint32_t indexCount)
{
    // VertexManager::allocateMeshDataForSegment: the segment's vertices and indices are
    // appended to the shared pools; indices stay local to the segment's first vertex
    VertexAllocation a;
    a.firstVertex = static_cast<int32_t>(m_nonPosition.size());
    a.vertexCount = vertexCount;
    a.firstIndex = static_cast<uint32_t>(m_indices.size());
    a.indexCount = indexCount;
    m_positions.insert(m_positions.end(), positions, positions + 3 * static_cast<size_t>(vertexCount));
    m_nonPosition.insert(m_nonPosition.end(), nonPositionVertices, nonPositionVertices + vertexCount);
    m_indices.insert(m_indices.end(), indices, indices + indexCount);
    return a;
}

void GpuScene::setVertexPools(std::vector<uint32_t> indices, std::vector<float> positions, std::vector<ArkRTVertex> nonPositionVertices)
{
    m_indices = std::move(indices);
    m_positions = std::move(positions);
    m_nonPosition = std::move(nonPositionVertices);
}

int32_t GpuScene::registerMaterial(const ArkShaderMaterial& material)
{
    m_materials.push_back(material);
    return static_cast<int32_t>(m_materials.size() - 1);
}

int32_t GpuScene::registerTexture(int32_t width, int32_t height, int32_t format, int32_t wrap, std::vector<uint8_t> pixels)
{
    m_texturePixels.push_back(std::move(pixels));
    m_textures.push_back(ArkTexture { width, height, format, wrap, nullptr });
    // re-point every view: the pixel vectors may have moved
    for (size_t t = 0; t < m_textures.size(); ++t) m_textures[t].data = m_texturePixels[t].data();
    return static_cast<int32_t>(m_textures.size() - 1);
}

uint32_t GpuScene::addStaticMesh(StaticMesh mesh)
{
    m_staticMeshes.push_back(std::move(mesh));
    return static_cast<uint32_t>(m_staticMeshes.size() - 1);
}

void GpuScene::addStaticMeshInstance(const StaticMeshInstance& instance)
{
    if (instance.mesh >= m_staticMeshes.size()) ARKOSE_LOG(Fatal, "GpuScene: static mesh instance of unknown mesh %u", instance.mesh);
    m_instances.push_back(instance);
}

void GpuScene::updateLightData()
{
    // GpuScene.cpp:790-858: colour * intensity * lightPreExposure; directions are the
    // light transform's forward / right / up, positions its world position; the
    // outer cone half angle is half the light's outer cone angle
    const float pre = lightPreExposure();
    m_dirLightData.clear();
    m_spotLightData.clear();
    if (m_directional) {
        const ManagedDirectionalLight& l = *m_directional;
        DirectionalLightData d {};
        for (int k = 0; k < 3; ++k) {
            d.color[k] = l.color[k] * l.intensity * pre;
            d.worldSpaceDirection[k] = l.forward[k];
        }
        d.exposure = pre;
        m_dirLightData.push_back(d);
    }
    for (const ManagedSpotLight& l : m_spots) {
        SpotLightData s {};
        for (int k = 0; k < 3; ++k) {
            s.color[k] = l.color[k] * l.intensity * pre;
            s.worldSpaceDirection[k] = l.forward[k];
            s.worldSpaceRight[k] = l.right[k];
            s.worldSpaceUp[k] = l.up[k];
            s.worldSpacePosition[k] = l.position[k];
        }
        s.exposure = pre;
        s.outerConeHalfAngle = l.outerConeAngle / 2.0f;
        s.iesProfileIndex = l.iesLut;
        m_spotLightData.push_back(s);
    }
}

void GpuScene::setLightData(std::vector<DirectionalLightData> directional, std::vector<SpotLightData> spots)
{
    m_dirLightData = std::move(directional);
    m_spotLightData = std::move(spots);
    m_lightsManaged = false;
}

void GpuScene::setManagedLights(std::optional<ManagedDirectionalLight> directional, std::vector<ManagedSpotLight> spots)
{
    m_directional = directional;
    m_spots = std::move(spots);
    m_lightsManaged = true;
}

void GpuScene::setInstanceTransform(size_t index, const float worldMatrix[16])
{
    if (index >= m_instances.size()) ARKOSE_LOG(Fatal, "GpuScene: no static mesh instance %zu", index);
    std::memcpy(m_instances[index].worldMatrix, worldMatrix, sizeof(m_instances[index].worldMatrix));
    ++m_instanceVersion;
}

void GpuScene::update()
{
    // m_lightPreExposure = camera().exposure() (:792), then the light buffers (:795-858)
    if (m_lightsManaged) updateLightData();
}

void GpuScene::buildRtInstances()
{
    // GpuScene.cpp:872-929 (the TLAS update): every LOD of every static mesh instance,
    // every segment whose BLAS exists, becomes one RT mesh (firstVertex, firstIndex,
    // material) and one TLAS instance at the instance's transform whose custom
    // index is that RT mesh, hit mask and SBT offset by the material's blend mode
    // (VertexManager.cpp:1298-1329: the BLAS is the segment's indexed triangles at an
    // identity geometry transform).
    m_rtMeshes.clear();
    m_rtInstances.clear();
    for (const StaticMeshInstance& inst : m_instances) {
        for (const StaticMeshLOD& lod : m_staticMeshes[inst.mesh].LODs) {
            for (const StaticMeshSegment& seg : lod.meshSegments) {
                if (!seg.blasBuilt) continue; // not yet loaded
                const uint32_t rtMeshIndex = static_cast<uint32_t>(m_rtMeshes.size());
                m_rtMeshes.push_back(ArkRTTriangleMesh { seg.vertexAllocation.firstVertex, static_cast<int32_t>(seg.vertexAllocation.firstIndex), seg.material });
                uint32_t hitMask = 0;
                if (seg.material >= 0 && static_cast<size_t>(seg.material) < m_materials.size()) {
                    switch (m_materials[seg.material].blend_mode) {
                    case ARK_BLEND_MODE_OPAQUE: hitMask = ARK_RT_HIT_MASK_OPAQUE; break;      // SBT offset 0
                    case ARK_BLEND_MODE_MASKED: hitMask = ARK_RT_HIT_MASK_MASKED; break;      // SBT offset 1
                    case ARK_BLEND_MODE_TRANSLUCENT: hitMask = ARK_RT_HIT_MASK_BLEND; break;  // SBT offset 2
                    default: ARKOSE_LOG(Fatal, "GpuScene: material %d has no blend mode", seg.material);
                    }
                }
                if (hitMask == 0) ARKOSE_LOG(Fatal, "GpuScene: segment without a material (ARKOSE_ASSERT(hitMask != 0))");
                ArkRTInstance ri {};
                // VkTransformMatrixKHR rows of the column-major world matrix
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 4; ++c) ri.object_to_world[r * 4 + c] = inst.worldMatrix[c * 4 + r];
                ri.rt_mesh_index = rtMeshIndex;
                ri.triangle_count = seg.vertexAllocation.indexCount / 3;
                ri.hit_mask = hitMask;
                m_rtInstances.push_back(ri);
            }
        }
    }
}

void GpuScene::buildArkLights()
{
    // SceneLightSet (lighting.glsl:8-17): at most one directional light (GpuScene.cpp:797)
    if (m_dirLightData.size() > 1) ARKOSE_LOG(Fatal, "GpuScene: we only support 0 or 1 directional lights in a scene");
    m_arkSpots.clear();
    for (const SpotLightData& s : m_spotLightData) {
        ArkSpotLight a {};
        for (int k = 0; k < 3; ++k) {
            a.color[k] = s.color[k];
            a.world_space_direction[k] = s.worldSpaceDirection[k];
            a.world_space_right[k] = s.worldSpaceRight[k];
            a.world_space_up[k] = s.worldSpaceUp[k];
            a.world_space_position[k] = s.worldSpacePosition[k];
        }
        a.outer_cone_half_angle = s.outerConeHalfAngle;
        a.ies_profile_index = s.iesProfileIndex;
        m_arkSpots.push_back(a);
    }
}

const std::vector<ArkRTInstance>& GpuScene::rtInstances()
{
    buildRtInstances();
    return m_rtInstances;
}

const ArkDdgiLights& GpuScene::rtLights()
{
    buildArkLights();
    ArkDdgiLights& v = m_lightsView;
    std::memset(&v, 0, sizeof(v));
    v.struct_size = sizeof(ArkDdgiLights);
    v.has_directional_light = m_dirLightData.empty() ? 0 : 1;
    if (!m_dirLightData.empty())
        for (int k = 0; k < 3; ++k) {
            v.directional_light.color[k] = m_dirLightData[0].color[k];
            v.directional_light.world_space_direction[k] = m_dirLightData[0].worldSpaceDirection[k];
        }
    v.spot_lights = m_arkSpots.data();
    v.spot_light_count = static_cast<uint32_t>(m_arkSpots.size());
    return v;
}

const ArkDdgiScene& GpuScene::rtScene()
{
    buildRtInstances();
    buildArkLights();
    ArkDdgiScene& v = m_view;
    std::memset(&v, 0, sizeof(v));
    v.struct_size = sizeof(ArkDdgiScene);
    v.indices = m_indices.data();
    v.index_count = m_indices.size();
    v.positions = m_positions.data();
    v.vertex_count = m_nonPosition.size();
    v.vertices = m_nonPosition.data();
    v.meshes = m_rtMeshes.data();
    v.mesh_count = static_cast<uint32_t>(m_rtMeshes.size());
    v.materials = m_materials.data();
    v.material_count = static_cast<uint32_t>(m_materials.size());
    v.textures = m_textures.data();
    v.texture_count = static_cast<uint32_t>(m_textures.size());
    v.instances = m_rtInstances.data();
    v.instance_count = static_cast<uint32_t>(m_rtInstances.size());
    v.has_directional_light = m_dirLightData.empty() ? 0 : 1;
    if (!m_dirLightData.empty())
        for (int k = 0; k < 3; ++k) {
            v.directional_light.color[k] = m_dirLightData[0].color[k];
            v.directional_light.world_space_direction[k] = m_dirLightData[0].worldSpaceDirection[k];
        }
    v.spot_lights = m_arkSpots.data();
    v.spot_light_count = static_cast<uint32_t>(m_arkSpots.size());
    v.environment_texture = m_environmentTexture;
    return v;
}
