#include "DDGINode.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "core/Logging.h"

// DDGIProbeGridData (arkose/shaders/shared/DDGIData.h:11-15), std140
struct DDGIProbeGridData {
    int gridDimensions[4];
    float probeSpacing[4];
    float offsetToFirst[4];
};

DDGINode::~DDGINode()
{
    if (m_updateDone) (void)hipEventDestroy(static_cast<hipEvent_t>(m_updateDone));
}

bool DDGINode::saveState(std::vector<uint8_t>& out) const
{
    uint64_t bytes = 0;
    if (!m_ctx || ark_ddgi_state_size(m_ctx, &bytes) != ARK_DDGI_OK) return false;
    out.resize(bytes);
    if (int rc = ark_ddgi_save_state(m_ctx, out.data(), bytes); rc != ARK_DDGI_OK) {
        ARKOSE_LOG(Error, "DDGINode: ark_ddgi_save_state failed (%d): %s", rc, ark_ddgi_last_error(m_ctx));
        return false;
    }
    return true;
}

bool DDGINode::loadState(const std::vector<uint8_t>& blob)
{
    if (!m_ctx) return false;
    if (int rc = ark_ddgi_load_state(m_ctx, blob.data(), blob.size()); rc != ARK_DDGI_OK) {
        ARKOSE_LOG(Error, "DDGINode: ark_ddgi_load_state failed (%d): %s", rc, ark_ddgi_last_error(m_ctx));
        return false;
    }
    uint32_t next = 0;
    if (ark_ddgi_get_next_probe_index(m_ctx, &next) != ARK_DDGI_OK) return false;
    m_probeUpdateIdx = static_cast<int>(next);
    return true;
}

RenderPipelineNode::ExecuteCallback DDGINode::construct(GpuScene& scene, Registry& reg)
{
    // DDGINode.cpp:39-42
    if (!scene.scene().hasProbeGrid()) {
        ARKOSE_LOG(Error, "DDGINode is used but no probe grid is available, will no-op");
        return RenderPipelineNode::NullExecuteCallback;
    }

    const ProbeGrid& probeGrid = scene.scene().probeGrid();
    DDGIProbeGridData probeGridData {};
    for (int k = 0; k < 3; ++k) {
        probeGridData.gridDimensions[k] = probeGrid.gridDimensions[k];
        probeGridData.probeSpacing[k] = probeGrid.probeSpacing[k];
        probeGridData.offsetToFirst[k] = probeGrid.offsetToFirst[k];
    }
    Buffer& probeGridDataBuffer = reg.createBufferForData(probeGridData, Buffer::Usage::ConstantBuffer);

    // Atlases (RGBA16F irradiance cleared to 0, RG16F visibility cleared to (zFar, zFar^2)),
    // probe offsets (zeros) and the surfel store live in the context; reused across
    // pipeline rebuilds like createOrReuseTexture2D (DDGINode.cpp:50-55, Registry.cpp:120-150).
    ArkDdgiDesc desc {};
    desc.struct_size = sizeof(ArkDdgiDesc);
    for (int k = 0; k < 3; ++k) {
        desc.grid_dims[k] = probeGrid.gridDimensions[k];
        desc.probe_spacing[k] = probeGrid.probeSpacing[k];
        desc.offset_to_first[k] = probeGrid.offsetToFirst[k];
    }
    desc.z_far = scene.camera().farClipPlane();
    desc.max_rays_per_probe = MaxNumProbeSamples;
    desc.max_probe_updates = std::min(m_maxProbeUpdates, probeGrid.probeCount());
    desc.device = scene.backend().device();
    desc.clear_overflow_mode = ARK_DDGI_CLEAR_OVERFLOW_INF;
    desc.shard_rank = m_shardRank;
    desc.shard_count = m_shardCount;
    auto created = reg.createOrReuseDdgiContext("ddgi", desc);
    ArkDdgiCtx* ctx = created.first;
    if (!ctx) {
        ARKOSE_LOG(Error, "DDGINode: could not create the DDGI context, will no-op");
        return RenderPipelineNode::NullExecuteCallback;
    }
    m_ctx = ctx;
    if (created.second == Registry::ReuseMode::Reused) {
        // atlases carry over; the offsets buffer is created anew with zeros (DDGINode.cpp:57-60)
        uint64_t bytes = 0;
        ark_ddgi_resource_size(ctx, ARK_DDGI_PROBE_OFFSETS, &bytes);
        std::vector<uint8_t> zeros(bytes, 0);
        ark_ddgi_write(ctx, ARK_DDGI_PROBE_OFFSETS, zeros.data(), bytes);
    }
    if (int rc = ark_ddgi_set_scene(ctx, &scene.rtScene()); rc != ARK_DDGI_OK) {
        ARKOSE_LOG(Error, "DDGINode: ark_ddgi_set_scene failed (%d): %s", rc, ark_ddgi_last_error(ctx));
        return RenderPipelineNode::NullExecuteCallback;
    }
    m_instanceVersion = scene.instanceVersion(); // set_scene built the BVHs at these transforms

    ArkDdgiDeviceViews views {};
    ark_ddgi_get_device_views(ctx, &views);
    Buffer& probeOffsetBuffer = reg.wrapBuffer(views.probe_offsets, views.probe_offsets_bytes, Buffer::Usage::StorageBuffer);
    probeOffsetBuffer.setName("DDGIProbeOffsetBuffer");
    probeOffsetBuffer.setStride(16);
    Texture& irradiance = reg.wrapTexture("ddgi-irradiance", views.irradiance_atlas, views.irradiance_width, views.irradiance_height, Texture::Format::RGBA16F);
    Texture& visibility = reg.wrapTexture("ddgi-visibility", views.visibility_atlas, views.visibility_width, views.visibility_height, Texture::Format::RG16F);
    BindingSet& ddgiSamplingBindingSet = reg.createBindingSet({ ShaderBinding::constantBuffer(probeGridDataBuffer),
                                                                ShaderBinding::storageBuffer(probeOffsetBuffer),
                                                                ShaderBinding::sampledTexture(irradiance),
                                                                ShaderBinding::sampledTexture(visibility) });
    reg.publish("DDGISamplingSet", ddgiSamplingBindingSet);

    // DDGINode.cpp:132-259
    return [&, ctx](const AppState& appState, CommandList& cmdList, UploadBuffer&) {
        const ProbeGrid& grid = scene.scene().probeGrid();
        const uint32_t frameIdx = appState.frameIndex();
        const uint32_t raysPerProbe = static_cast<uint32_t>(m_raysPerProbeInt);
        const float ambientLx = m_useSceneAmbient ? scene.scene().ambientIlluminance() : m_injectedAmbientLx;
        const uint32_t probeUpdatesThisFrame = static_cast<uint32_t>(std::min(m_probeUpdatesPerFrame, grid.probeCount()));
        const uint32_t firstProbeIdx = static_cast<uint32_t>(m_probeUpdateIdx);

        ArkDdgiFrameParams p {};
        p.struct_size = sizeof(ArkDdgiFrameParams);
        p.frame_index = frameIdx;                       // parameter1 / frameIdx
        p.first_probe_index = firstProbeIdx;            // parameter3
        p.probe_updates = probeUpdatesThisFrame;
        p.rays_per_probe = raysPerProbe;                // parameter2
        p.hysteresis_irradiance = appState.isFirstFrame() ? 0.0f : m_hysteresisIrradiance;
        p.hysteresis_visibility = appState.isFirstFrame() ? 0.0f : m_hysteresisVisibility;
        p.visibility_sharpness = m_visibilitySharpness;
        p.ambient_amount = ambientLx * scene.lightPreExposure();
        p.environment_multiplier = scene.preExposedEnvironmentBrightnessFactor();
        p.delta_time = appState.deltaTime();
        p.update_offsets = (m_computeProbeOffsets && m_applyProbeOffsets) ? 1 : 0;
        // GpuScene::update's per-frame uploads, which the reference's trace reads through
        // the SceneLightSet and the TLAS: the light buffers with this frame's
        // pre-exposure (GpuScene.cpp:792-858; the context keeps its device copy when
        // nothing changed), and the TLAS instance data + build when a transform moved
        // (:872-1009; here a device refit of the flattened BVHs, and a background rebuild
        // installed when ready - the reference's full build every 60 frames)
        if (int rc = ark_ddgi_set_lights(ctx, &scene.rtLights()); rc != ARK_DDGI_OK)
            ARKOSE_LOG(Error, "DDGINode: ark_ddgi_set_lights failed (%d): %s", rc, ark_ddgi_last_error(ctx));
        if (scene.instanceVersion() != m_instanceVersion) {
            const std::vector<ArkRTInstance>& instances = scene.rtInstances();
            // enqueued on this frame's stream ahead of the update (no host wait)
            int rc = ark_ddgi_set_instances_async(ctx, instances.data(), static_cast<uint32_t>(instances.size()), cmdList.hipStream());
            if (rc != ARK_DDGI_OK) {
                // a refit cannot follow this change (the topology changed: another mesh,
                // triangle count or hit mask): build the scene anew, as construct() does
                // (never keep the old transforms for good)
                ARKOSE_LOG(Warning, "DDGINode: ark_ddgi_set_instances failed (%d): %s; rebuilding the scene", rc, ark_ddgi_last_error(ctx));
                rc = ark_ddgi_set_scene(ctx, &scene.rtScene());
                if (rc != ARK_DDGI_OK) ARKOSE_LOG(Error, "DDGINode: ark_ddgi_set_scene failed (%d): %s", rc, ark_ddgi_last_error(ctx));
            }
            // the context follows this version only once it holds it (else: retried next frame)
            if (rc == ARK_DDGI_OK) m_instanceVersion = scene.instanceVersion();
        }
        if (m_exchange) {
            // Z-slab rank: traversal goes ahead, shading waits for the previous exchange;
            // this update's bands are then exchanged on the exchange's side stream
            if (!m_exchange->readyForNextUpdate(m_shardRank))
                ARKOSE_LOG(Fatal, "DDGINode: rank %d updates again before every rank's %s exchange of its previous frame", m_shardRank, m_exchange->name());
            if (!m_updateDone) {
                hipEvent_t e;
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) ARKOSE_LOG(Fatal, "DDGINode: event creation failed");
                m_updateDone = e;
            }
            if (int rc = ark_ddgi_update_overlapped(ctx, &p, cmdList.hipStream(), m_exchangePending, m_updateDone); rc != ARK_DDGI_OK)
                ARKOSE_LOG(Error, "DDGINode: ark_ddgi_update_overlapped failed (%d): %s", rc, ark_ddgi_last_error(ctx));
            m_exchangePending = m_exchange->exchange(m_shardRank, m_updateDone);
            if (!m_exchangePending) ARKOSE_LOG(Error, "DDGINode: %s slab exchange failed", m_exchange->name());
        } else if (int rc = ark_ddgi_update(ctx, &p, cmdList.hipStream()); rc != ARK_DDGI_OK) {
            ARKOSE_LOG(Error, "DDGINode: ark_ddgi_update failed (%d): %s", rc, ark_ddgi_last_error(ctx));
        }

        m_probeUpdateIdx = static_cast<int>((m_probeUpdateIdx + probeUpdatesThisFrame) % static_cast<uint32_t>(grid.probeCount()));
    };
}
