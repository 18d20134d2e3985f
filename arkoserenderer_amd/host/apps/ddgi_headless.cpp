// ddgi_headless.cpp — headless driver of the C++ DDGI node: loads a scene into the
// engine-shaped GpuScene (vertex pools, static meshes of LOD segments, instances,
// materials, textures, uploaded light data), builds a RenderPipeline {DDGINode} on
// the HIP backend, runs F frames the way MeshViewerApp::performAmbientOcclusionBake
// submits a pipeline (MeshViewerApp.cpp:845-893), optionally rebuilds the pipeline
// mid-run (history carried through the Registry like Registry.cpp:120-150), and
// dumps the DDGISamplingSet contents as raw files for comparison. The node reads the
// scene through GpuScene::rtScene(), the GpuScene -> ArkDdgiScene adapter.
//
//   ddgi_headless --scene s.arkscn | --soup N   --grid X Y Z --spacing sx sy sz --origin ox oy oz
//                 [--rays R] [--updates K] [--frames F] [--zfar Z] [--exposure E] [--env B]
//                 [--ambient LX] [--offsets 0|1] [--rebuild-at F] [--device D] --out PREFIX
//                 [--shards P]                          Z-slab ranks as P contexts in this process,
//                                                       bands exchanged by device copies (one GPU)
//                 [--world P --rank r --nccl-id FILE]   rank r of P processes (one per GPU), bands
//                 [--nccl-nonce S]                      exchanged by RCCL all-gather; rank 0 writes
//                                                       the ncclUniqueId (+ nonce S) to FILE, the
//                                                       others read it (a file without S is stale:
//                                                       they wait). S is required for P > 1 (one
//                                                       value per launch, the same on every rank)
//                 [--save-state FILE] [--load-state FILE] [--first-frame F]
//                 [--frame-script FILE]                 per-frame scene changes (ARKFRM1): the
//                                                       camera exposure, the managed lights and
//                                                       the instance transforms of each frame,
//                                                       applied before GpuScene::update()
//                                                       checkpoint of the (unsharded) node after the
//                                                       last frame / before the first; frame indices
//                                                       start at F (DDGINode::saveState/loadState)
//                 [--exchange-timeout SEC]              deadline of the exchange watchdog
//                 [--exchange-deadline-test]            1-rank RCCL: stalls the exchange stream for
//                                                       1.5 s under a 0.2 s deadline; the watchdog
//                                                       must end the process with exit code 14
// Sharded runs dump the (exchanged, therefore complete) atlases of rank 0 / this rank
// and the probe offsets of this rank's slab ("--shards": merged over the owners).
#include <sys/stat.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <memory>
#include <thread>
#include <string>
#include <vector>

#include "../../../include/ark_ddgi.h"
#include "../../../include/ark_scene.h"
#include "core/Logging.h"
#include "rendering/GpuScene.h"
#include "rendering/RenderPipeline.h"
#include "rendering/backend/hip/SlabExchange.h"
#include "rendering/nodes/DDGINode.h"

#include <hip/hip_runtime.h>

namespace {

struct SceneFile {
    std::vector<uint32_t> indices;
    std::vector<float> positions;
    std::vector<ArkRTVertex> vertices;
    std::vector<ArkRTTriangleMesh> meshes;
    std::vector<ArkShaderMaterial> materials;
    std::vector<ArkRTInstance> instances;
    std::vector<ArkSpotLight> spots;
    std::vector<ArkTexture> textures;
    std::vector<std::vector<uint8_t>> texData;
    ArkDdgiScene view {};
};

template<typename T>
bool readVec(FILE* f, std::vector<T>& v, uint64_t n)
{
    v.resize(n);
    return n == 0 || std::fread(v.data(), sizeof(T), n, f) == n;
}

// ARKSCN1 container written by arkoserenderer_amd/scene.py (SceneData.save_binary)
bool loadScene(const char* path, SceneFile& s)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    char magic[8];
    uint64_t n[7];
    int32_t hasSun, envTex;
    float sun[6];
    bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "ARKSCN1", 7) == 0 && std::fread(n, 8, 7, f) == 7 &&
              std::fread(&hasSun, 4, 1, f) == 1 && std::fread(sun, 4, 6, f) == 6 && std::fread(&envTex, 4, 1, f) == 1;
    ok = ok && readVec(f, s.indices, n[0]) && readVec(f, s.positions, n[1] * 3) && readVec(f, s.vertices, n[1]) && readVec(f, s.meshes, n[2]) &&
         readVec(f, s.materials, n[3]) && readVec(f, s.instances, n[4]) && readVec(f, s.spots, n[6]);
    for (uint64_t t = 0; ok && t < n[5]; ++t) {
        int32_t hdr[4];
        ok = std::fread(hdr, 4, 4, f) == 4;
        if (!ok) break;
        size_t bytes = static_cast<size_t>(hdr[0]) * hdr[1] * (hdr[2] == ARK_TEX_R32F ? 4 : hdr[2] == ARK_TEX_RGBA32F ? 16 : 4);
        s.texData.emplace_back(bytes);
        ok = std::fread(s.texData.back().data(), 1, bytes, f) == bytes;
        s.textures.push_back(ArkTexture { hdr[0], hdr[1], hdr[2], hdr[3], nullptr });
    }
    std::fclose(f);
    if (!ok) return false;
    for (size_t t = 0; t < s.textures.size(); ++t) s.textures[t].data = s.texData[t].data();
    ArkDdgiScene& v = s.view;
    v.struct_size = sizeof(ArkDdgiScene);
    v.indices = s.indices.data(); v.index_count = s.indices.size();
    v.positions = s.positions.data(); v.vertex_count = s.vertices.size();
    v.vertices = s.vertices.data();
    v.meshes = s.meshes.data(); v.mesh_count = static_cast<uint32_t>(s.meshes.size());
    v.materials = s.materials.data(); v.material_count = static_cast<uint32_t>(s.materials.size());
    v.textures = s.textures.data(); v.texture_count = static_cast<uint32_t>(s.textures.size());
    v.instances = s.instances.data(); v.instance_count = static_cast<uint32_t>(s.instances.size());
    v.has_directional_light = hasSun;
    for (int k = 0; k < 3; ++k) {
        v.directional_light.color[k] = sun[k];
        v.directional_light.world_space_direction[k] = sun[3 + k];
    }
    v.spot_lights = s.spots.data(); v.spot_light_count = static_cast<uint32_t>(s.spots.size());
    v.environment_texture = envTex;
    return true;
}

// The flat RT arrays of a scene file (or the soup generator) as the engine holds them:
// the pools as VertexManager's, one static mesh per TLAS instance with one LOD of one
// segment (its RT mesh's vertex allocation and material), the instance transform as a
// column-major world matrix, the lights as the uploaded light buffers (the file holds
// pre-exposed colours, as GpuScene uploads them).
void populate(GpuScene& gs, const ArkDdgiScene& s)
{
    gs.setVertexPools(std::vector<uint32_t>(s.indices, s.indices + s.index_count),
                      std::vector<float>(s.positions, s.positions + 3 * s.vertex_count),
                      std::vector<ArkRTVertex>(s.vertices, s.vertices + s.vertex_count));
    for (uint32_t m = 0; m < s.material_count; ++m) gs.registerMaterial(s.materials[m]);
    for (uint32_t t = 0; t < s.texture_count; ++t) {
        const ArkTexture& tx = s.textures[t];
        const size_t texel = tx.format == ARK_TEX_RGBA32F ? 16 : 4;
        const uint8_t* p = static_cast<const uint8_t*>(tx.data);
        gs.registerTexture(tx.width, tx.height, tx.format, tx.wrap, std::vector<uint8_t>(p, p + static_cast<size_t>(tx.width) * tx.height * texel));
    }
    for (uint32_t i = 0; i < s.instance_count; ++i) {
        const ArkRTInstance& ri = s.instances[i];
        const ArkRTTriangleMesh& rm = s.meshes[ri.rt_mesh_index];
        StaticMeshSegment seg;
        seg.vertexAllocation.firstVertex = rm.first_vertex;
        seg.vertexAllocation.firstIndex = static_cast<uint32_t>(rm.first_index);
        seg.vertexAllocation.indexCount = 3 * ri.triangle_count;
        seg.material = rm.material_index;
        StaticMesh mesh;
        mesh.LODs.push_back(StaticMeshLOD { { seg } });
        StaticMeshInstance inst;
        inst.mesh = gs.addStaticMesh(std::move(mesh));
        for (int r = 0; r < 4; ++r)
            for (int c = 0; c < 4; ++c) inst.worldMatrix[c * 4 + r] = r < 3 ? ri.object_to_world[r * 4 + c] : (c == 3 ? 1.0f : 0.0f);
        gs.addStaticMeshInstance(inst);
    }
    std::vector<DirectionalLightData> dir;
    if (s.has_directional_light) {
        DirectionalLightData d {};
        for (int k = 0; k < 3; ++k) {
            d.color[k] = s.directional_light.color[k];
            d.worldSpaceDirection[k] = s.directional_light.world_space_direction[k];
        }
        dir.push_back(d);
    }
    std::vector<SpotLightData> spots;
    for (uint32_t l = 0; l < s.spot_light_count; ++l) {
        const ArkSpotLight& a = s.spot_lights[l];
        SpotLightData d {};
        for (int k = 0; k < 3; ++k) {
            d.color[k] = a.color[k];
            d.worldSpaceDirection[k] = a.world_space_direction[k];
            d.worldSpaceRight[k] = a.world_space_right[k];
            d.worldSpaceUp[k] = a.world_space_up[k];
            d.worldSpacePosition[k] = a.world_space_position[k];
        }
        d.outerConeHalfAngle = a.outer_cone_half_angle;
        d.iesProfileIndex = a.ies_profile_index;
        spots.push_back(d);
    }
    gs.setLightData(std::move(dir), std::move(spots));
    gs.setEnvironmentMap(s.environment_texture);
}

std::vector<uint8_t> readResource(ArkDdgiCtx* ctx, int which)
{
    uint64_t bytes = 0;
    if (ark_ddgi_resource_size(ctx, which, &bytes) != 0) return {};
    std::vector<uint8_t> buf(bytes);
    if (ark_ddgi_read(ctx, which, buf.data(), bytes) != 0) return {};
    return buf;
}

bool writeFile(const std::string& path, const std::vector<uint8_t>& buf)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    std::fclose(f);
    return ok;
}

// rendezvous of the RCCL ranks through a shared file: rank 0 removes any old file,
// then publishes the 128-byte id followed by the launch nonce (written then renamed,
// so readers never see a partial file). A reader takes only a file with this
// launch's nonce (a file left by an earlier run holds a dead id, and ncclCommInitRank
// on it would hang). The nonce is required for P > 1 (main); a 1-rank run reads
// nothing, so without a nonce the file only has to be newer than the process start.
bool shareUniqueId(const std::string& path, int rank, const std::string& nonce, std::time_t startedAt, std::vector<uint8_t>& id)
{
    if (rank == 0) {
        std::remove(path.c_str());
        if (!RcclSlabExchange::createUniqueId(id)) return false;
        std::vector<uint8_t> blob(id);
        blob.insert(blob.end(), nonce.begin(), nonce.end());
        const std::string tmp = path + ".tmp";
        return writeFile(tmp, blob) && std::rename(tmp.c_str(), path.c_str()) == 0;
    }
    for (int tries = 0; tries < 600; ++tries) {
        struct stat st {};
        if (stat(path.c_str(), &st) == 0 && (!nonce.empty() || st.st_mtime + 1 >= startedAt)) {
            if (FILE* f = std::fopen(path.c_str(), "rb")) {
                std::vector<uint8_t> blob(128 + nonce.size() + 1);
                const size_t n = std::fread(blob.data(), 1, blob.size(), f);
                std::fclose(f);
                if (n == 128 + nonce.size() && std::equal(nonce.begin(), nonce.end(), blob.begin() + 128)) {
                    id.assign(blob.begin(), blob.begin() + 128);
                    return true;
                }
            }
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    return false;
}

// A bounded stall of a stream (the exchange deadline test): one lane sleeps until
// `ticks` of the constant wall clock have passed, then the kernel ends.
__global__ void k_stall(uint64_t ticks)
{
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// Per-frame scene changes (--frame-script): "ARKFRM1\0", u32 frames, u32 instances, then
// per frame: f32 exposure; i32 has_sun, f32 colour[3], intensity, forward[3]; u32 spots,
// per spot f32 colour[3], intensity, forward[3], right[3], up[3], position[3], outer
// cone angle, i32 IES LUT texture; u32 moved, and when 1 the instances' object-to-world
// rows (12 f32 each).
struct FrameChange {
    float exposure = 1.0f;
    std::optional<ManagedDirectionalLight> sun;
    std::vector<ManagedSpotLight> spots;
    std::vector<float> transforms; // instances x 12, empty = unchanged
};

bool loadFrameScript(const char* path, std::vector<FrameChange>& out)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    auto rd = [&](void* p, size_t n) { return std::fread(p, 1, n, f) == n; };
    char magic[8];
    uint32_t frames = 0, instances = 0;
    bool ok = rd(magic, 8) && std::memcmp(magic, "ARKFRM1\0", 8) == 0 && rd(&frames, 4) && rd(&instances, 4);
    for (uint32_t i = 0; ok && i < frames; ++i) {
        FrameChange c;
        int32_t hasSun = 0;
        float sun[7];
        ok = rd(&c.exposure, 4) && rd(&hasSun, 4) && rd(sun, sizeof(sun));
        if (ok && hasSun) {
            ManagedDirectionalLight d;
            for (int k = 0; k < 3; ++k) {
                d.color[k] = sun[k];
                d.forward[k] = sun[4 + k];
            }
            d.intensity = sun[3];
            c.sun = d;
        }
        uint32_t n = 0;
        ok = ok && rd(&n, 4) && n <= ARK_DDGI_MAX_SPOT_LIGHTS;
        for (uint32_t l = 0; ok && l < n; ++l) {
            float v[17];
            int32_t ies = -1;
            ok = rd(v, sizeof(v)) && rd(&ies, 4);
            ManagedSpotLight sl;
            for (int k = 0; k < 3; ++k) {
                sl.color[k] = v[k];
                sl.forward[k] = v[4 + k];
                sl.right[k] = v[7 + k];
                sl.up[k] = v[10 + k];
                sl.position[k] = v[13 + k];
            }
            sl.intensity = v[3];
            sl.outerConeAngle = v[16];
            sl.iesLut = ies;
            c.spots.push_back(sl);
        }
        uint32_t moved = 0;
        ok = ok && rd(&moved, 4);
        if (ok && moved) {
            c.transforms.resize(static_cast<size_t>(instances) * 12);
            ok = rd(c.transforms.data(), c.transforms.size() * 4);
        }
        out.push_back(std::move(c));
    }
    std::fclose(f);
    return ok;
}

bool dump(ArkDdgiCtx* ctx, int which, const std::string& path)
{
    uint64_t bytes = 0;
    if (ark_ddgi_resource_size(ctx, which, &bytes) != 0) return false;
    std::vector<uint8_t> buf(bytes);
    if (ark_ddgi_read(ctx, which, buf.data(), bytes) != 0) return false;
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    bool ok = std::fwrite(buf.data(), 1, bytes, f) == bytes;
    std::fclose(f);
    return ok;
}

} // namespace

int main(int argc, char** argv)
{
    std::string scenePath, out = "ddgi";
    uint64_t soupTris = 0;
    ProbeGrid grid;
    int rays = 64, updates = 512, frames = 4, device = 0, offsets = 1, rebuildAt = -1;
    int shards = 1, world = 1, rank = 0;
    std::string ncclIdPath, ncclNonce;
    double exchangeTimeout = 0.0;
    std::string saveStatePath, loadStatePath, frameScriptPath;
    int firstFrame = 0;
    bool deadlineTest = false;
    const std::time_t startedAt = std::time(nullptr);
    float zFar = 10000.0f, exposure = 1.0f, env = 1.0f, ambient = 0.0f;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) ARKOSE_LOG(Fatal, "missing value for %s", a.c_str());
            return argv[++i];
        };
        if (a == "--scene") scenePath = next();
        else if (a == "--soup") soupTris = std::strtoull(next(), nullptr, 10);
        else if (a == "--grid") for (int k = 0; k < 3; ++k) grid.gridDimensions[k] = std::atoi(next());
        else if (a == "--spacing") for (int k = 0; k < 3; ++k) grid.probeSpacing[k] = std::strtof(next(), nullptr);
        else if (a == "--origin") for (int k = 0; k < 3; ++k) grid.offsetToFirst[k] = std::strtof(next(), nullptr);
        else if (a == "--rays") rays = std::atoi(next());
        else if (a == "--updates") updates = std::atoi(next());
        else if (a == "--frames") frames = std::atoi(next());
        else if (a == "--zfar") zFar = std::strtof(next(), nullptr);
        else if (a == "--exposure") exposure = std::strtof(next(), nullptr);
        else if (a == "--env") env = std::strtof(next(), nullptr);
        else if (a == "--ambient") ambient = std::strtof(next(), nullptr);
        else if (a == "--offsets") offsets = std::atoi(next());
        else if (a == "--rebuild-at") rebuildAt = std::atoi(next());
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--shards") shards = std::atoi(next());
        else if (a == "--world") world = std::atoi(next());
        else if (a == "--rank") rank = std::atoi(next());
        else if (a == "--nccl-id") ncclIdPath = next();
        else if (a == "--nccl-nonce") ncclNonce = next();
        else if (a == "--exchange-timeout") exchangeTimeout = std::strtod(next(), nullptr);
        else if (a == "--exchange-deadline-test") deadlineTest = true;
        else if (a == "--save-state") saveStatePath = next();
        else if (a == "--load-state") loadStatePath = next();
        else if (a == "--first-frame") firstFrame = std::atoi(next());
        else if (a == "--frame-script") frameScriptPath = next();
        else ARKOSE_LOG(Fatal, "unknown argument %s", a.c_str());
    }
    SceneFile file;
    ArkSoupScene* soup = nullptr;
    const ArkDdgiScene* rt = nullptr;
    if (!scenePath.empty()) {
        if (!loadScene(scenePath.c_str(), file)) ARKOSE_LOG(Fatal, "cannot read scene %s", scenePath.c_str());
        rt = &file.view;
    } else {
        ArkSoupParams sp;
        ark_soup_default_params(&sp);
        sp.triangle_count = soupTris ? soupTris : 1000000;
        if (ark_soup_generate(&sp, &soup) != 0) ARKOSE_LOG(Fatal, "soup generation failed");
        rt = ark_soup_scene_view(soup);
    }

    HipBackend backend(device);
    GpuScene scene(backend);
    populate(scene, *rt);
    if (scene.rtScene().instance_count != rt->instance_count) ARKOSE_LOG(Fatal, "GpuScene adapter dropped instances");
    scene.scene().setProbeGrid(grid);
    scene.scene().setAmbientIlluminance(ambient);
    scene.scene().setEnvironmentBrightness(env);
    scene.camera().setFarClipPlane(zFar);
    scene.camera().setExposure(exposure);

    if (world > 1 && ncclNonce.empty())
        ARKOSE_LOG(Fatal, "--world %d needs --nccl-nonce S (one value per launch, the same on every rank): a rendezvous file's age "
                          "cannot tell this launch's id from a stale one", world);
    if (shards < 1 || world < 1 || rank < 0 || rank >= world || (shards > 1 && world > 1) || (world > 1 && ncclIdPath.empty()))
        ARKOSE_LOG(Fatal, "bad sharding arguments (--shards %d, --world %d --rank %d)", shards, world, rank);
    const bool rccl = !ncclIdPath.empty();
    const int ranksHere = shards;                    // contexts in this process
    const int slabCount = rccl ? world : shards;     // Z-slab ranks in total

    auto makePipeline = [&](int shardRank) {
        auto pipeline = std::make_unique<RenderPipeline>(&scene);
        DDGINode& node = pipeline->addNode<DDGINode>();
        node.setRaysPerProbe(rays);
        node.setProbeUpdatesPerFrame(updates);
        node.setComputeProbeOffsets(offsets != 0);
        node.setMaxProbeUpdates(updates);
        if (slabCount > 1) node.setShard(shardRank, slabCount);
        return pipeline;
    };
    auto nodeOf = [](RenderPipeline& p) {
        RenderPipelineNode* n = nullptr;
        p.forEachNodeInResolvedOrder([&](RenderPipelineNode& node, const RenderPipelineNode::ExecuteCallback&) { n = &node; });
        return static_cast<DDGINode*>(n);
    };
    std::vector<std::unique_ptr<RenderPipeline>> pipelines;
    std::vector<std::unique_ptr<Registry>> registries;
    for (int r = 0; r < ranksHere; ++r) {
        pipelines.push_back(makePipeline(rccl ? rank : r));
        registries.push_back(std::make_unique<Registry>(backend, nullptr));
        pipelines.back()->constructAll(*registries.back());
    }
    // the slab exchange over the constructed contexts
    std::unique_ptr<SlabExchange> exchange;
    if (slabCount > 1 || rccl) {
        std::string err;
        if (rccl) {
            SlabBands bands;
            if (!SlabBands::fromContext(nodeOf(*pipelines[0])->context(), rank, world, bands, err)) ARKOSE_LOG(Fatal, "%s", err.c_str());
            std::vector<uint8_t> id;
            if (!shareUniqueId(ncclIdPath, rank, ncclNonce, startedAt, id)) ARKOSE_LOG(Fatal, "cannot share the ncclUniqueId through %s", ncclIdPath.c_str());
            auto ex = std::make_unique<RcclSlabExchange>(device, rank, world, id.data(), bands, deadlineTest ? 0.2 : exchangeTimeout);
            if (!ex->ok()) ARKOSE_LOG(Fatal, "RCCL: %s", ex->error().c_str());
            if (deadlineTest) {
                if (world != 1) ARKOSE_LOG(Fatal, "--exchange-deadline-test runs with --world 1");
                // frame 0's all-gather queues behind a 1.5 s stall; frame 3's exchange waits
                // for it with a 0.2 s deadline. The handler lets the bounded stall finish
                // (so no kernel is left running), then takes the default failure path.
                RcclSlabExchange* rx = ex.get();
                rx->watchdog().setFailureHandler([rx](const std::string& why) {
                    std::printf("ddgi_headless: watchdog fired: %s\n", why.c_str());
                    (void)hipDeviceSynchronize();
                    ExchangeWatchdog::abortAndExit(rx->comm(), why);
                });
                int khz = 0;
                if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
                hipLaunchKernelGGL(k_stall, dim3(1), dim3(1), 0, static_cast<hipStream_t>(rx->stream()), static_cast<uint64_t>(khz) * 1500u);
                if (hipGetLastError() != hipSuccess) ARKOSE_LOG(Fatal, "stall kernel launch failed");
            }
            exchange = std::move(ex);
        } else {
            std::vector<SlabBands> all(ranksHere);
            for (int r = 0; r < ranksHere; ++r)
                if (!SlabBands::fromContext(nodeOf(*pipelines[r])->context(), r, ranksHere, all[r], err)) ARKOSE_LOG(Fatal, "%s", err.c_str());
            exchange = std::make_unique<DeviceCopySlabExchange>(std::move(all));
        }
        for (auto& p : pipelines) nodeOf(*p)->setSlabExchange(exchange.get());
    }
    if (!loadStatePath.empty()) {
        if (ranksHere != 1 || exchange) ARKOSE_LOG(Fatal, "--load-state is for unsharded runs");
        FILE* fh = std::fopen(loadStatePath.c_str(), "rb");
        if (!fh) ARKOSE_LOG(Fatal, "cannot read %s", loadStatePath.c_str());
        std::vector<uint8_t> blob;
        uint8_t buf[1 << 16];
        for (size_t n; (n = std::fread(buf, 1, sizeof(buf), fh)) > 0;) blob.insert(blob.end(), buf, buf + n);
        std::fclose(fh);
        if (!nodeOf(*pipelines[0])->loadState(blob)) ARKOSE_LOG(Fatal, "DDGINode::loadState failed");
        std::printf("ddgi_headless: resumed at probe %d\n", nodeOf(*pipelines[0])->probeUpdateIdx());
    }
    std::vector<FrameChange> script;
    if (!frameScriptPath.empty() && !loadFrameScript(frameScriptPath.c_str(), script)) ARKOSE_LOG(Fatal, "cannot read frame script %s", frameScriptPath.c_str());
    for (int f = firstFrame; f < firstFrame + frames; ++f) {
        if (static_cast<size_t>(f - firstFrame) < script.size()) {
            // this frame's camera exposure, lights and instance transforms
            const FrameChange& c = script[static_cast<size_t>(f - firstFrame)];
            scene.camera().setExposure(c.exposure);
            scene.setManagedLights(c.sun, c.spots);
            for (size_t i = 0; i < c.transforms.size() / 12; ++i) {
                float m[16];
                for (int r = 0; r < 4; ++r)
                    for (int col = 0; col < 4; ++col) m[col * 4 + r] = r < 3 ? c.transforms[i * 12 + r * 4 + col] : (col == 3 ? 1.0f : 0.0f);
                scene.setInstanceTransform(i, m);
            }
        }
        scene.update(); // GpuScene::update: the exposure and light data of this frame
        if (f == rebuildAt) {
            // pipeline rebuild (VulkanBackend::reconstructRenderPipelineResources,
            // VulkanBackend.cpp:2327-2347): same nodes, new Registry that adopts the
            // previous one's DDGI history
            if (ranksHere != 1 || exchange) ARKOSE_LOG(Fatal, "--rebuild-at is for unsharded runs");
            auto nextReg = std::make_unique<Registry>(backend, registries[0].get());
            pipelines[0]->constructAll(*nextReg);
            registries[0] = std::move(nextReg);
        }
        for (auto& p : pipelines) p->executeFrame(AppState(1.0f / 60.0f, f / 60.0f, static_cast<uint32_t>(f), f == 0), backend);
    }
    backend.synchronize();
    if (exchange && !exchange->drain()) ARKOSE_LOG(Error, "slab exchange did not complete");
    if (hipDeviceSynchronize() != hipSuccess) ARKOSE_LOG(Error, "device synchronize failed");  // the exchange's side stream
    for (auto& reg : registries) {
        BindingSet* set = reg->getBindingSet("DDGISamplingSet");
        if (!set || set->bindings().size() != 4) ARKOSE_LOG(Fatal, "DDGISamplingSet not published");
    }
    ArkDdgiCtx* ctx = nodeOf(*pipelines[0])->context();
    if (!saveStatePath.empty()) {
        std::vector<uint8_t> blob;
        if (!nodeOf(*pipelines[0])->saveState(blob) || !writeFile(saveStatePath, blob)) ARKOSE_LOG(Fatal, "cannot save the DDGI state");
    }
    bool ok = dump(ctx, ARK_DDGI_ATLAS_IRRADIANCE, out + ".irr") && dump(ctx, ARK_DDGI_ATLAS_VISIBILITY, out + ".vis") &&
              dump(ctx, ARK_DDGI_SURFELS, out + ".surf");
    if (ranksHere > 1) {
        // every context holds the complete atlases after the exchange
        const std::vector<uint8_t> irr0 = readResource(ctx, ARK_DDGI_ATLAS_IRRADIANCE), vis0 = readResource(ctx, ARK_DDGI_ATLAS_VISIBILITY);
        for (int r = 1; r < ranksHere; ++r) {
            ArkDdgiCtx* c = nodeOf(*pipelines[r])->context();
            if (readResource(c, ARK_DDGI_ATLAS_IRRADIANCE) != irr0 || readResource(c, ARK_DDGI_ATLAS_VISIBILITY) != vis0) {
                ARKOSE_LOG(Error, "shard %d: atlases differ from shard 0 after the exchange", r);
                ok = false;
            }
        }
        // offsets are owner-only: probe i from the rank whose slab holds its z
        std::vector<float> merged(readResource(ctx, ARK_DDGI_PROBE_OFFSETS).size() / 4, 0.0f);
        const int X = grid.gridDimensions[0], Z = grid.gridDimensions[2];
        for (int r = 0; r < ranksHere; ++r) {
            const std::vector<uint8_t> raw = readResource(nodeOf(*pipelines[r])->context(), ARK_DDGI_PROBE_OFFSETS);
            const float* o = reinterpret_cast<const float*>(raw.data());
            for (size_t i = 0; i < merged.size() / 4; ++i) {
                const int z = static_cast<int>((i % static_cast<size_t>(X * Z)) / static_cast<size_t>(X));
                if (z * ranksHere / Z == r)
                    for (int k = 0; k < 4; ++k) merged[i * 4 + k] = o[i * 4 + k];
            }
        }
        std::vector<uint8_t> bytes(merged.size() * 4);
        std::memcpy(bytes.data(), merged.data(), bytes.size());
        ok = ok && writeFile(out + ".off", bytes);
    } else {
        ok = ok && dump(ctx, ARK_DDGI_PROBE_OFFSETS, out + ".off");
    }
    if (exchange) std::printf("ddgi_headless: %d Z-slab ranks, %s exchange\n", slabCount, exchange->name());
    pipelines.clear();
    exchange.reset();
    registries.clear();
    if (soup) ark_soup_free(soup);
    std::printf("ddgi_headless: %d frames, %s\n", frames, ok ? "dumped" : "DUMP FAILED");
    return ok && ark::errorCounter() == 0 ? 0 : 1;
}
