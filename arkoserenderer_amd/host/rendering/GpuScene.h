// GpuScene.h — the RT-scene data contract the DDGI node consumes (GpuScene.h:38-333
// subset): the ArkDdgiScene arrays (RT mesh table, index/position/RTVertex pools,
// materials, textures, TLAS instances, lights, environment), the camera far plane,
// the light pre-exposure and the scene's probe grid. The arrays are host views
// owned by the caller; the DDGI context copies them to HBM at construct.
#pragma once

#include <optional>

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

class HipBackend;

class GpuScene {
public:
    GpuScene(HipBackend& backend, const ArkDdgiScene& rtScene) : m_backend(backend), m_rtScene(rtScene) {}
    Scene& scene() { return m_scene; }
    const Scene& scene() const { return m_scene; }
    Camera& camera() { return m_camera; }
    HipBackend& backend() { return m_backend; }
    const ArkDdgiScene& rtScene() const { return m_rtScene; }
    float lightPreExposure() const { return m_camera.exposure(); }                                                            // GpuScene.h:148
    float preExposedEnvironmentBrightnessFactor() const { return m_scene.environmentBrightness() * lightPreExposure(); }    // GpuScene.h:150

private:
    HipBackend& m_backend;
    ArkDdgiScene m_rtScene;
    Scene m_scene;
    Camera m_camera;
};
