// GpuScene.h — the scene side of the engine that the DDGI node reads, shaped as the
// reference holds it (arkose/rendering/GpuScene.h:38-333 subset): VertexManager
// pools (u32 indices, Position3F positions, RTVertex non-position data), static
// meshes as LODs of segments with their vertex allocations and material handles,
// static mesh instances with world transforms, the bindless material and texture
// tables, managed lights, the environment map, the camera and the scene's probe
// grid. rtScene() is the adapter from that contract to the C-ABI's ArkDdgiScene:
// the RT mesh table and TLAS instances exactly as GpuScene::update builds them
// (GpuScene.cpp:872-929) and the light buffers as it uploads them (:790-858).
#pragma once

#include <cstdint>
#include <optional>
#include <vector>

#include "../../../include/ark_ddgi.h"

struct ProbeGrid {
    int gridDimensions[3] {};  // x = width, y = height, z = depth (arkcore/scene/ProbeGrid.h:6-15)
    float probeSpacing[3] {};
    float offsetToFirst[3] {};
    int probeCount() const { return gridDimensions[0] * gridDimensions[1] * gridDimensions[2]; }
};

class Scene {
public:
    bool hasProbeGrid() const { return m_probeGrid.has_value(); }
    const ProbeGrid& probeGrid() const { return *m_probeGrid; }
    void setProbeGrid(const ProbeGrid& g) { m_probeGrid = g; } // Scene.h:124
    float ambientIlluminance() const { return m_ambientLx; }
    void setAmbientIlluminance(float lx) { m_ambientLx = lx; }
    float environmentBrightness() const { return m_envBrightness; }
    void setEnvironmentBrightness(float b) { m_envBrightness = b; }

private:
    std::optional<ProbeGrid> m_probeGrid;
    float m_ambientLx { 0.0f };
    float m_envBrightness { 1.0f };
};

class Camera {
public:
    float farClipPlane() const { return m_zFar; }
    void setFarClipPlane(float z) { m_zFar = z; }
    // Camera::calculateManualExposure (Camera.cpp:203-214) is applied by the caller
    float exposure() const { return m_exposure; }
    void setExposure(float e) { m_exposure = e; }

private:
    float m_zFar { 10000.0f };
    float m_exposure { 1.0f };
};

// DrawCallDescription::fromVertexAllocation of one mesh segment: its vertices start at
// firstVertex in the vertex pools, its indices (local to firstVertex) at firstIndex.
struct VertexAllocation {
    int32_t firstVertex { 0 };
    uint32_t vertexCount { 0 };
    uint32_t firstIndex { 0 };
    uint32_t indexCount { 0 };
};

struct StaticMeshSegment {
    VertexAllocation vertexAllocation;
    int32_t material { -1 };  // MaterialHandle (index into the material table)
    bool blasBuilt { true };  // `meshSegment.blas != nullptr`: segments still loading are skipped
};

struct StaticMeshLOD {
    std::vector<StaticMeshSegment> meshSegments;
};

struct StaticMesh {
    std::vector<StaticMeshLOD> LODs;
};

struct StaticMeshInstance {
    uint32_t mesh { 0 };        // StaticMeshHandle
    float worldMatrix[16] {};   // Transform::worldMatrix(), column-major (ark::mat4)
};

// Lights as the scene manages them (DirectionalLight / SpotLight + their Transform).
struct ManagedDirectionalLight {
    float color[3] { 1.0f, 1.0f, 1.0f };
    float intensity { 1.0f };     // intensityValue()
    float forward[3] { 0.0f, -1.0f, 0.0f };
};

struct ManagedSpotLight {
    float color[3] { 1.0f, 1.0f, 1.0f };
    float intensity { 1.0f };
    float forward[3] {}, right[3] {}, up[3] {}, position[3] {};
    float outerConeAngle { 1.0f };
    int32_t iesLut { -1 };        // texture handle of the profile's LUT
};

// The light buffers as GpuScene uploads them (shared/LightData.h:4-42), the fields a
// closest hit reads.
struct DirectionalLightData {
    float color[3];             // colour * intensity * lightPreExposure
    float exposure;
    float worldSpaceDirection[4];
};

struct SpotLightData {
    float color[3];
    float exposure;
    float worldSpaceDirection[4];
    float worldSpaceRight[4];
    float worldSpaceUp[4];
    float worldSpacePosition[4];
    float outerConeHalfAngle;
    int32_t iesProfileIndex;
};

class HipBackend;

class GpuScene {
public:
    explicit GpuScene(HipBackend& backend) : m_backend(backend) {}
    Scene& scene() { return m_scene; }
    const Scene& scene() const { return m_scene; }
    Camera& camera() { return m_camera; }
    HipBackend& backend() { return m_backend; }
    float lightPreExposure() const { return m_camera.exposure(); }                                                            // GpuScene.h:148
    float preExposedEnvironmentBrightnessFactor() const { return m_scene.environmentBrightness() * lightPreExposure(); }    // GpuScene.h:150

    // VertexManager: append one segment's geometry (indices local to its first vertex)
    VertexAllocation allocateVertices(const float* positions, const ArkRTVertex* nonPositionVertices, uint32_t vertexCount,
                                      const uint32_t* indices, uint32_t indexCount);
    // ... or adopt packed pools whole (a loader whose allocations are already known)
    void setVertexPools(std::vector<uint32_t> indices, std::vector<float> positions, std::vector<ArkRTVertex> nonPositionVertices);

    int32_t registerMaterial(const ArkShaderMaterial& material);                            // MaterialHandle
    // bindless texture slot; `pixels` is kept alive by the scene (ArkTexture.data points into it)
    int32_t registerTexture(int32_t width, int32_t height, int32_t format, int32_t wrap, std::vector<uint8_t> pixels);
    uint32_t addStaticMesh(StaticMesh mesh);                                                  // StaticMeshHandle
    void addStaticMeshInstance(const StaticMeshInstance& instance);
    void setEnvironmentMap(int32_t textureHandle) { m_environmentTexture = textureHandle; }  // -1: the 1x1 white default

    void setDirectionalLight(const ManagedDirectionalLight& light) { m_directional = light; m_lightsManaged = true; }
    void addSpotLight(const ManagedSpotLight& light) { m_spots.push_back(light); m_lightsManaged = true; }
    // the scene's lights as they are this frame (a light that moved, turned or changed colour)
    void setManagedLights(std::optional<ManagedDirectionalLight> directional, std::vector<ManagedSpotLight> spots);
    // GpuScene::update's light data from the managed lights (GpuScene.cpp:790-858)
    void updateLightData();
    // light data recorded as uploaded (a loader of captured frames); replaces the managed lights
    void setLightData(std::vector<DirectionalLightData> directional, std::vector<SpotLightData> spots);
    // Transform::setWorldMatrix of instance i (column-major ark::mat4): the TLAS instance
    // data of the next frame changes (GpuScene.cpp:901-928)
    void setInstanceTransform(size_t index, const float worldMatrix[16]);
    uint32_t instanceVersion() const { return m_instanceVersion; }

    // The per-frame part of GpuScene::update (GpuScene.cpp:790-1009): the exposure is read
    // (:792) and the light data re-computed from the managed lights with it (recorded
    // light data stays as recorded); the TLAS instance data follow the transforms
    // (rtInstances()).
    void update();

    // The adapter: the C-ABI scene view of this GpuScene (valid until the next change).
    const ArkDdgiScene& rtScene();
    uint32_t rtMeshCount() const { return static_cast<uint32_t>(m_rtMeshes.size()); }
    // this frame's light set for ark_ddgi_set_lights (valid until the next call)
    const ArkDdgiLights& rtLights();
    // this frame's TLAS instances (GpuScene.cpp:901-928) for ark_ddgi_set_instances
    const std::vector<ArkRTInstance>& rtInstances();

private:
    HipBackend& m_backend;
    Scene m_scene;
    Camera m_camera;
    std::vector<uint32_t> m_indices;
    std::vector<float> m_positions;
    std::vector<ArkRTVertex> m_nonPosition;
    std::vector<ArkShaderMaterial> m_materials;
    std::vector<ArkTexture> m_textures;
    std::vector<std::vector<uint8_t>> m_texturePixels;
    std::vector<StaticMesh> m_staticMeshes;
    std::vector<StaticMeshInstance> m_instances;
    int32_t m_environmentTexture { -1 };
    std::optional<ManagedDirectionalLight> m_directional;
    std::vector<ManagedSpotLight> m_spots;
    std::vector<DirectionalLightData> m_dirLightData;
    std::vector<SpotLightData> m_spotLightData;
    bool m_lightsManaged { false }; // update() recomputes the light data from the managed lights
    uint32_t m_instanceVersion { 0 };
    // adapter output
    void buildRtInstances(); // m_rtMeshes + m_rtInstances from the instances
    void buildArkLights();   // m_arkSpots from the light data
    std::vector<ArkRTTriangleMesh> m_rtMeshes;
    std::vector<ArkRTInstance> m_rtInstances;
    std::vector<ArkSpotLight> m_arkSpots;
    ArkDdgiScene m_view {};
    ArkDdgiLights m_lightsView {};
};
