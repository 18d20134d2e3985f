// DDGINode.h — drop-in DDGI node on the HIP backend. Same name ("DDGI"), same
// members and defaults as arkose/rendering/nodes/DDGINode.h:10-39, same published
// resource ("DDGISamplingSet" = {grid CB, probe offsets SB, irradiance atlas,
// visibility atlas}, DDGINode.cpp:62-66). The GPU work is the C-ABI of
// libark_ddgi (include/ark_ddgi.h) instead of a Vulkan RT pipeline.
#pragma once

#include "../GpuScene.h"
#include "../RenderPipelineNode.h"
#include "../backend/hip/SlabExchange.h"

#include <cstdint>
#include <vector>

class DDGINode final : public RenderPipelineNode {
public:
    std::string name() const override { return "DDGI"; }
    void drawGui() override {}

    ExecuteCallback construct(GpuScene&, Registry&) override;

    // Settings the reference edits through ImGui (DDGINode.cpp:17-35); exposed as setters here.
    void setRaysPerProbe(int r) { m_raysPerProbeInt = r; }
    void setProbeUpdatesPerFrame(int n) { m_probeUpdatesPerFrame = n; }
    void setHysteresis(float irradiance, float visibility) { m_hysteresisIrradiance = irradiance; m_hysteresisVisibility = visibility; }
    void setVisibilitySharpness(float s) { m_visibilitySharpness = s; }
    void setComputeProbeOffsets(bool c) { m_computeProbeOffsets = c; }
    void setApplyProbeOffsets(bool a) { m_applyProbeOffsets = a; }
    void setMaxProbeUpdates(int n) { m_maxProbeUpdates = n; }
    void setShard(int rank, int count) { m_shardRank = rank; m_shardCount = count; }
    // Z-slab ranks: the atlas exchange after each update (RCCL all-gather, or device
    // copies for contexts in one process); frame n+1's shading waits for frame n's.
    void setSlabExchange(SlabExchange* exchange) { m_exchange = exchange; }
    // the event the last exchange completes (null without an exchange): consumers of
    // DDGISamplingSet on other ranks' bands wait on it
    void* pendingExchange() const { return m_exchangePending; }
    ArkDdgiCtx* context() const { return m_ctx; }
    int probeUpdateIdx() const { return m_probeUpdateIdx; }
    void setProbeUpdateIdx(int idx) { m_probeUpdateIdx = idx; }
    // DDGI history checkpoint (ark_ddgi_save_state / _load_state): atlases, offsets and
    // the rolling window position, so a resumed node continues where it stopped
    bool saveState(std::vector<uint8_t>& out) const;
    bool loadState(const std::vector<uint8_t>& blob);

    // we can dynamically choose to do fewer samples or probes, but not more since it defines the fixed image size
    static constexpr int MaxNumProbeSamples { ARK_DDGI_MAX_RAYS_PER_PROBE };
    static constexpr int MaxNumProbeUpdates { ARK_DDGI_REFERENCE_MAX_PROBE_UPDATES };

private:
    int m_raysPerProbeInt = 256;
    float m_hysteresisIrradiance { 0.93f };
    float m_hysteresisVisibility { 0.93f };

    float m_visibilitySharpness { 50.0f };

    int m_probeUpdatesPerFrame { 2048 };
    int m_probeUpdateIdx { 0 };

    bool m_computeProbeOffsets { true };
    bool m_applyProbeOffsets { true };

    bool m_useSceneAmbient { true };
    float m_injectedAmbientLx { 100.0f };

    // MI355X: the window may cover the whole grid (288 GB of HBM; the reference caps at 4096)
    int m_maxProbeUpdates { MaxNumProbeUpdates };
    int m_shardRank { 0 };
    int m_shardCount { 1 };
    ArkDdgiCtx* m_ctx { nullptr };
    uint32_t m_instanceVersion { 0 }; // GpuScene::instanceVersion() the context's BVHs follow
    SlabExchange* m_exchange { nullptr };
    void* m_updateDone { nullptr };      // hipEvent_t recorded after each update
    void* m_exchangePending { nullptr }; // hipEvent_t of the last exchange
public:
    ~DDGINode() override;
};
