// ark_ddgi.cpp — the C-ABI context of the MI355X DDGI path (include/ark_ddgi.h).
//
// Owns all device memory of one DDGI node instance on one GPU: the persistent
// atlases/offsets (the DDGISamplingSet, DDGINode.cpp:62-66), the per-update
// working set (slot table, hit records, surfels) and the scene (BVH + RT mesh
// data + materials + lights). Every update is enqueued on one HIP stream.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ark_ddgi.h"
#include "../../include/ark_ddgi_debug.h"
#include "ark_fmath.h"
#include "bvh_builder.h"
#include "ddgi_kernels.h"

using namespace ark;

namespace {

// pipelined windows below this many probe rays trace at half occupancy (ctx->pipeTraceBlocks)
constexpr uint32_t kPipeHalfRays = 5u << 20;
constexpr int kPipeTracePerCu = 3; // traversal workgroups per CU of such a window (ctx->pipeTraceBlocks; 2, 4, 5 measured slower)
// Idle traversal lanes are refilled in batches of >= kRefillMin (the refill then stalls
// a wave once per 16 finished rays, and the rays it starts descend from the root
// together: C4 2.98 vs 3.30 ms at 1 in round 1; with the fetches outside branches 16
// is the best: step 3.53 -> 3.46 ms against 4, 24 and 32, profiles/r03_as, r03_at). The
// sun's any-hit rays in the light-space BVH are short: 32 (profiles/r05_q: C4 shadow
// phase 0.648 -> 0.630 ms, K = 2048 0.327 -> 0.320 ms; the world BVHs' shadow rays keep
// 16: 32 there made C5's shadow phase 1.92 -> 2.07 ms). kGrabChunk: rays per
// partition-head grab, 64 = a probe quarter of direction-clustered rays per wave pool
// (16 and 8 measured slower on 1/8 slabs).
constexpr uint32_t kRefillMin = 16, kSunRefillMin = 32, kGrabChunk = 64;

// roctx range over a scope (host-side enqueue markers, named after the reference's
// ScopedDebugZone labels, DDGINode.cpp:152-247); end() closes it early.
class RoctxRange {
public:
    explicit RoctxRange(const char* name) { roctxRangePushA(name); }
    ~RoctxRange() { end(); }
    void end()
    {
        if (m_open) roctxRangePop();
        m_open = false;
    }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;

private:
    bool m_open { true };
};

struct DeviceBuffer {
    void* ptr = nullptr;
    size_t bytes = 0;
    hipError_t alloc(size_t n)
    {
        release();
        bytes = n;
        if (n == 0) return hipSuccess;
        return hipMalloc(&ptr, n);
    }
    void release()
    {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template<typename T> T* as() const { return static_cast<T*>(ptr); }
};

uint16_t f32_to_f16_host(float f)
{
    // host-side RNE conversion for the clear values (matches v_cvt_f16_f32)
    _Float16 h = static_cast<_Float16>(f);
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

// Traversal order of a probe's R samples: groups of 64 (one wave's refill pool)
// with nearby directions, so the lanes of a wave descend similar BVH paths.
// Balanced greedy clustering around ceil(R/64) spherical-Fibonacci centres.
// Only the lane -> sample assignment changes; every sample is traced exactly
// once and its hit record is stored at its own index, so results do not depend
// on the order.
void sampleTraversalOrder(uint32_t R, std::vector<uint32_t>& order)
{
    order.resize(R);
    for (uint32_t i = 0; i < R; ++i) order[i] = i;
    const uint32_t G = (R + 63) / 64;
    if (G <= 1) return;
    auto fib = [](uint32_t i, uint32_t n, double* d) { // same point set as sphericalFibonacci (math accuracy irrelevant here)
        const double phi = 2.0 * M_PI * std::fmod(i * 0.6180339887498949, 1.0);
        const double z = 1.0 - (2.0 * i + 1.0) / n, r = std::sqrt(std::max(0.0, 1.0 - z * z));
        d[0] = std::cos(phi) * r; d[1] = std::sin(phi) * r; d[2] = z;
    };
    std::vector<double> pts(3 * R), ctr(3 * G);
    for (uint32_t i = 0; i < R; ++i) fib(i, R, &pts[3 * i]);
    for (uint32_t g = 0; g < G; ++g) fib(g, G, &ctr[3 * g]);
    struct Pair { double d; uint32_t i, g; };
    std::vector<Pair> pairs;
    pairs.reserve(static_cast<size_t>(R) * G);
    for (uint32_t i = 0; i < R; ++i)
        for (uint32_t g = 0; g < G; ++g)
            pairs.push_back({ pts[3 * i] * ctr[3 * g] + pts[3 * i + 1] * ctr[3 * g + 1] + pts[3 * i + 2] * ctr[3 * g + 2], i, g });
    std::stable_sort(pairs.begin(), pairs.end(), [](const Pair& a, const Pair& b) { return a.d > b.d; });
    std::vector<int> groupOf(R, -1);
    std::vector<uint32_t> room(G, 64u);
    room[G - 1] = R - 64u * (G - 1);
    for (const Pair& q : pairs)
        if (groupOf[q.i] < 0 && room[q.g] > 0) { groupOf[q.i] = static_cast<int>(q.g); room[q.g]--; }
    uint32_t k = 0;
    for (uint32_t g = 0; g < G; ++g)
        for (uint32_t i = 0; i < R; ++i)
            if (groupOf[i] == static_cast<int>(g)) order[k++] = i;
}

} // namespace

// The nodes of a BVH8 by depth, deepest first (a node's internal children are one level
// deeper): the refit's launch order, order[offsets[i] .. offsets[i + 1]) one level.
static bool bvhLevelOrder(const GpuBvh8Node* h, uint64_t n, const int32_t* roots, int nRoots, std::vector<uint32_t>& order, std::vector<uint32_t>& offsets)
{
    std::vector<std::vector<uint32_t>> byDepth;
    std::vector<std::pair<uint32_t, uint32_t>> work; // (node, depth)
    for (int r = 0; r < nRoots; ++r)
        if (roots[r] >= 0) work.push_back({ static_cast<uint32_t>(roots[r]), 0u });
    while (!work.empty()) {
        const auto [node, d] = work.back();
        work.pop_back();
        if (node >= n) return false;
        if (byDepth.size() <= d) byDepth.resize(d + 1);
        byDepth[d].push_back(node);
        const uint32_t internal = static_cast<uint32_t>(__builtin_popcount(h[node].imask));
        for (uint32_t k = 0; k < internal; ++k) work.push_back({ h[node].child_base + k, d + 1 });
    }
    order.clear();
    order.reserve(n);
    offsets.assign(1, 0u);
    for (size_t d = byDepth.size(); d-- > 0;) {
        std::sort(byDepth[d].begin(), byDepth[d].end());
        order.insert(order.end(), byDepth[d].begin(), byDepth[d].end());
        offsets.push_back(static_cast<uint32_t>(order.size()));
    }
    return true;
}

// The scene of a context on the device (ark_ddgi_set_scene): BVH nodes + triangles,
// shading records, RT mesh data, materials, textures, lights. Reference-counted:
// ark_ddgi_share_scene lets the Z-slab contexts of one GPU use one copy.
// A background rebuild of the sun's light-space BVH (sunRebuildStep): a host thread
// waits for a device snapshot of the world BVHs' triangle records (taken in stream
// order behind the refits, `snap` / `evSnap`), builds the BVH for `dir` and uploads it
// into `buf`; `done` set last (release).
struct SunJob {
    std::thread t;
    std::atomic<bool> done { false };
    float dir[3] {};
    uint32_t version = 0; // SceneStore::version of the snapshot
    uint32_t refitsAt = 0; // SceneStore::refitCount of the snapshot (later refits: refitted forward at install)
    DeviceBuffer snap;    // the records it builds from
    hipEvent_t evSnap = nullptr;
    DeviceBuffer buf;     // nodes, then the triangle records at triOffset
    size_t triOffset = 0;
    uint64_t nodes = 0, triRecords = 0;
    uint32_t depth = 0;
    float frame[9] {};
    double frameD[9] {};
    float inflateAbs = 0.0f;
    std::vector<uint32_t> levelOrder, levelOffsets;
    float ms = 0.0f;
    bool ok = false;
    ~SunJob()
    {
        if (t.joinable()) t.join();
        buf.release(); // not installed (an installed buffer was moved to the scene)
        snap.release();
        if (evSnap) (void)hipEventDestroy(evSnap);
    }
};

// A background rebuild of the world BVHs after refits (worldCollect / worldStart; the reference
// rebuilds its TLAS in full every 60 frames, GpuScene.cpp:998-1010): a host thread takes
// a device snapshot of the refitted triangle records, builds the three hit-mask classes'
// BVHs anew from them (set_scene's builder), keeps every record's words as they were
// (so hits stay bit-identical) and uploads nodes + records, the new record order's
// source indices (perm, for the shading records) and the refit's level order.
struct WorldJob {
    std::thread t;
    std::atomic<bool> done { false };
    uint32_t version = 0, refitsAt = 0;
    DeviceBuffer snap;
    hipEvent_t evSnap = nullptr;
    uint64_t snapRecords = 0;
    std::vector<int> classOf; // instance -> hit-mask class (0 opaque, 1 masked, 2 blend)
    DeviceBuffer buf, perm, order;
    size_t triOffset = 0;
    uint64_t nodes = 0, triRecords = 0, triangles = 0;
    int32_t roots[3] { -1, -1, -1 };
    uint32_t opaqueNodes = 0, depth = 0, maxLeaf = 0;
    float sah = 0.0f;
    std::vector<uint32_t> levelOffsets;
    float ms = 0.0f;
    bool ok = false;
    std::string error;
    ~WorldJob()
    {
        if (t.joinable()) t.join();
        for (DeviceBuffer* b : { &buf, &perm, &order, &snap }) b->release();
        if (evSnap) (void)hipEventDestroy(evSnap);
    }
};

// A buffer replaced while launches enqueued before may still read it: freed once `done`
// (recorded behind them) has completed.
struct Retired {
    DeviceBuffer buf;
    hipEvent_t done = nullptr;
};

struct SceneStore {
    int device = 0;
    DeviceBuffer nodes, triNormals, indices, vertices, positions, meshes, materials, instances, texInfos, texels;
    DeviceBuffer sunNodes; // light-space BVH8 of the sun's shadow rays + its world-space triangle records
    uint64_t sunBvhNodes = 0;
    float sunCostWorld = 0.0f, sunCostLight = 0.0f; // sampled sun shadow-ray steps per ray (sun_shadow_cost)
    std::vector<ArkRTInstance> instHost;     // the AO bake (instance -> mesh segment), set_instances' topology check
    std::vector<ArkRTTriangleMesh> meshHost;
    SceneArgs args {};    // the world BVHs, pools, materials, textures (lights: per context, deriveSceneArgs)
    SceneArgs sunArgs {}; // sun_nodes / sun_tris / sun_root / sun_frame of the light-space BVH (sun_root -1: none)
    float sunDirBuilt[3] { 0, 0, 0 }; // the sun direction the light-space BVH was built for
    // the scene's lights as set_scene got them: a context's lights until ark_ddgi_set_lights
    int32_t hasSunScene = 0;
    ArkDirectionalLight sunScene {};
    std::vector<GpuSpotLight> spotsScene;
    ArkDdgiBvhStats bvhStats {};
    uint32_t bvhMaxDepth = 0; // deepest of the world BVHs and the sun's (traversal spill)
    uint32_t worldDepth = 0, sunDepth = 0;
    // ark_ddgi_set_instances: bumped by every refit and install (a sharing context
    // re-derives its SceneArgs); the builder's absolute inflation; the refit's buffers
    uint32_t version = 0;
    float inflateAbs = 0.0f;
    uint64_t triRecords = 0; // triangle records of the world BVHs (holes included)
    DeviceBuffer refitInst, refitBoxes, refitOrder;
    std::vector<uint32_t> levelOffsets; // refitOrder[levelOffsets[i] .. [i + 1]): the nodes of one depth, deepest first
    // the light-space BVH follows the motion: refitted with the world BVHs (its records
    // re-transformed, its boxes of their light coordinates)
    DeviceBuffer sunRefitOrder, sunRefitBoxes;
    std::vector<uint32_t> sunLevelOffsets;
    uint64_t sunTriRecords = 0;
    float sunInflateAbs = 0.0f;
    double sunFrameD[9] {};
    // the refit's transforms: the last ones uploaded (dirty = changed since the records
    // were written); pinned staging of the stream-ordered uploads, two sets in turn
    std::vector<RefitInstance> refitHost;
    // pinned staging of the per-frame uploads, a ring: a slot is reused once its copy (a
    // few calls back) has run, so the host runs up to kStageSlots / 2 frames of
    // set_instances_async ahead of the device (two slots: one frame, and every call
    // waited for the previous frame's refit)
    static constexpr int kStageSlots = 8;
    void* stage[kStageSlots] {};
    size_t stageBytes[kStageSlots] {};
    hipEvent_t stageDone[kStageSlots] {};
    int stageNext = 0;
    // object-space bounds of every instance's triangles (set_scene): the refit's world and
    // light-space bounds, for its box inflation, from the instances' transforms on the host
    std::vector<std::array<float, 6>> instObjBox;
    // The geometry a refit writes comes in three copies: the front one (nodes, sunNodes,
    // instances above: what the kernels read) and two spares. A refit brings the next
    // spare from the transforms it holds (xf[slot]) to the new ones on the context's
    // refit stream and makes it the front one: it waits only for the operations that read
    // that copy while it was the front one, two refits before (the frame before last),
    // so that it runs beside the frame in flight's traversal and the next traversal does
    // not wait for it (with two copies it waited for the previous frame's shading, and
    // the frames ran one after the other: C4 4.3 ms per moving frame, static 3.3). An
    // install (a new topology) drops the spares; the next refit copies the front one.
    struct Spare {
        DeviceBuffer nodes, sunNodes, instances;
        bool valid = false;
        int slot = 0;
    };
    Spare spare[2]; // spare[0]: the next refit's target
    // the refit's node masks (k_node_masks: per topology) and the inflations each copy's
    // boxes hold; refitFull: the next refit reaches every node (a new topology, or boxes
    // scratch not of this one)
    DeviceBuffer nodeMasks, sunNodeMasks;
    bool masksValid = false, sunMasksValid = false, refitFull = true;
    float inflCopy[3][2] {};
    int front = 0; // slot of the front copy (xf index)
    std::vector<std::array<float, 12>> xf[3];
    // the light-space BVH follows the sun: set_scene chose it (sunWanted), and after a
    // sun-direction change it is rebuilt in the background (sunRebuildStep)
    bool sunWanted = false;
    int buildThreads = 16;
    std::unique_ptr<SunJob> sunJob;
    uint32_t sunRebuilds = 0;
    // rebuild requests (sunRebuildStep): the sun direction the contexts sharing this scene
    // asked for last and how many calls in a row asked for it; a rebuild starts only on a
    // stable request (>= 2), so contexts under different suns never start rebuilds that
    // undo each other. A failed build is remembered (direction and
    // scene version) and not retried until either changes.
    float sunReqDir[3] { 0, 0, 0 };
    uint32_t sunReqStreak = 0;
    bool sunFailed = false;
    float sunFailedDir[3] { 0, 0, 0 };
    uint32_t sunFailedVersion = 0;
    uint32_t sunFailures = 0;
    // the world BVHs' background rebuild (worldCollect / worldStart): refits since the installed
    // BVHs were built, the running job, rebuilds installed
    uint32_t refitsSinceBuild = 0, sunRefitsSinceBuild = 0;
    std::unique_ptr<WorldJob> worldJob;
    uint32_t worldRebuilds = 0, refitCount = 0;
    bool worldRebuildFailed = false;
    // the background build started last (loosenedTurn: loosened BVHs take turns)
    enum : uint8_t { kBackgroundNone, kBackgroundWorld, kBackgroundSun };
    uint8_t lastBackground = kBackgroundNone;
    std::vector<Retired> retired;
    SceneStore() = default;
    SceneStore(const SceneStore&) = delete;
    SceneStore& operator=(const SceneStore&) = delete;
    ~SceneStore()
    {
        (void)hipSetDevice(device);
        sunJob.reset(); // joins them: the jobs read snapshots freed below
        worldJob.reset();
        (void)hipDeviceSynchronize();
        for (Retired& r : retired) {
            r.buf.release();
            if (r.done) (void)hipEventDestroy(r.done);
        }
        for (int i = 0; i < kStageSlots; ++i) {
            if (stage[i]) (void)hipHostFree(stage[i]);
            if (stageDone[i]) (void)hipEventDestroy(stageDone[i]);
        }
        for (DeviceBuffer* b : { &nodes, &triNormals, &indices, &vertices, &positions, &meshes, &materials, &instances, &texInfos, &texels, &sunNodes, &refitInst,
                                 &refitBoxes, &refitOrder, &sunRefitOrder, &sunRefitBoxes, &spare[0].nodes, &spare[0].sunNodes,
                                 &spare[0].instances, &spare[1].nodes, &spare[1].sunNodes, &spare[1].instances,
                                 &nodeMasks, &sunNodeMasks })
            b->release();
    }
};

struct ArkDdgiCtx {
    ArkDdgiDesc desc {};
    std::string lastError;
    hipStream_t stream = nullptr; // internal (clears); synchronous use only
    // Call order across streams: every operation records evOrder on its stream when
    // enqueued, and the next one waits for it when given another stream (orderBegin).
    hipEvent_t evOrder = nullptr;
    hipStream_t orderStream = nullptr;
    bool orderValid = false;
    // traversal refill batch (probe and shadow rays, the sun's), rays per partition-head grab
    uint32_t refillMin = kRefillMin, sunRefillMin = kSunRefillMin, grabChunk = kGrabChunk;
    int device = 0;
    int cuCount = 0;
    int X = 0, Y = 0, Z = 0, N = 0;
    int Wi = 0, Hi = 0, Wv = 0, Hv = 0;
    int Kmax = 0, Rmax = 0;
    int slabZ0 = 0, slabZ1 = 0;
    // persistent resources
    DeviceBuffer irr, vis, offsets;
    // working set
    DeviceBuffer slots, slotOrder, fib, fibOrder, order, hits, surfels, spill, rayCounter, counters, shadeWork, reflWork;
    DeviceBuffer raySteps; // counting updates: u16 traversal iterations per probe ray (ARK_DDGI_DEBUG_RAY_STEPS)
    std::vector<uint32_t> orderHost; // traversal order of the samples for orderR
    uint32_t orderR = 0;
    uint32_t lightCount = 0;
    uint32_t spillEntries = 0;
    uint32_t traceBlocks = 0, shadeBlocks = 0, shadowBlocks = 0, shadowBlocksPerCu = 1;
    // Frames in flight (updateImpl): the per-frame buffers the traversal writes come in
    // two sets (slot table, slot order, sample directions, hit records, work counters);
    // frame n uses set n & 1. Frame n's slot table, primary traversal and probe offsets
    // run on traceStream as soon as frame n - 2 (the previous user of the set) is done,
    // after frame n - 1's offsets (same stream), overlapping frame n - 1's shadow
    // rays, shading and probe update on the caller's stream.
    bool pipelining = true;        // ARK_DDGI_FLAG_SERIAL_FRAMES: every update runs serially
    int sunBvh = -1;               // ArkDdgiDesc.sun_bvh: 0 the sun's shadow rays traverse the world BVHs, 1 the light-space BVH, -1: by cost (sun_bvh_pays)
    uint32_t pipeTraceBlocks = 0; // primary-traversal grid of a pipelined window below kPipeHalfRays rays
    bool pipeReady = false;        // the previous context operation was an update
    uint32_t parity = 0;           // buffer set of the next update
    uint32_t prevR = 0;
    bool prevPipelined = false;    // the previous update's offsets ran on traceStream
    hipStream_t traceStream = nullptr;
    hipEvent_t evTraced = nullptr, evFrameDone[2] = {};
    bool frameDoneValid[2] = { false, false };
    // Device-side frame sequencing of pipelined frames (k_seq_signal / k_seq_wait
    // instead of cross-queue event waits): seqWords [0] = the last frame whose
    // traversal-stream part (slot table, traversal, offsets) is done, [32] = the last
    // frame whose caller-stream part is done, [64] = a wait timed out (a signal folded
    // into the last kernel - its last workgroup storing the word after a device-scope
    // fence per workgroup - measured slower: the fences write back L2, K = 2048 frames
    // 0.371 -> 0.387 ms, profiles/r03_y). setSeq[b] = the
    // frame that last used buffer set b, when that frame was sequenced this way
    // (else its evFrameDone[b] is recorded). ark_ddgi_set_sequencing(ctx, 0, ...): events throughout.
    bool seqSync = true;
    DeviceBuffer seqWords;
    uint32_t frameSeq = 0;
    uint32_t setSeq[2] = { 0, 0 };
    bool setSeqValid[2] = { false, false };
    uint64_t seqTimeoutTicks = 0;
    uint32_t seqTimeoutMs = 10000;
    uint64_t wallClockKhz = 100000;
    // fail-closed sequencing: a k_seq_wait that gives up sets seqWords[64] (every path
    // kernel then skips: frameAborted) and this host-mapped word, which the next
    // update / exchange_begin / synchronize polls (checkSequencing)
    uint32_t* hostAbort = nullptr;    // host pointer (hipHostMalloc, coherent)
    uint32_t* hostAbortDev = nullptr; // its device address
    uint32_t seqTimeouts = 0;         // timeouts reported so far
    // Z-slab exchange sequencing (ark_ddgi_exchange_begin/_end, ark_ddgi_update_exchanged):
    // seqWords [96] = the last exchange completed on the caller's exchange stream
    uint32_t lastMainSeq = 0;        // the last update's caller-stream sequence number (0: not sequenced)
    hipStream_t lastStream = nullptr; // the last update's stream
    hipEvent_t evExchangeSrc = nullptr; // exchange_begin after an unsequenced update
    hipEvent_t evExchangeDone = nullptr; // exchange_end without sequence words (seqSync off)
    uint32_t exchSeq = 0;            // exchanges ended so far
    uint32_t pendingExchange = 0;    // the exchange the next update_exchanged waits for before shading
    uint32_t lastParity = 0;       // buffer set of the last update (debug hit records)
    uint32_t fibR[2] = { 0, 0 };
    uint64_t spillRegionWords = 0; // spill region 1 = the primary traversal's
    // scene
    bool hasScene = false;
    std::shared_ptr<SceneStore> sceneStore; // device scene (possibly shared with other contexts)
    uint32_t sceneVersion = 0;              // sceneStore->version that `scene` was derived at
    // Per-frame lights (ark_ddgi_set_lights; set_scene / share_scene start them with the
    // scene's): the sun travels in `scene` (kernel arguments), the spots in `lights` on
    // the device, stored there in stream order ahead of the next operation that reads
    // them (flushLights) when lightsDirty
    DeviceBuffer lights; // GpuSpotLight[kMaxLights - 1]
    std::vector<GpuSpotLight> spotHost;
    int32_t hasSun = 0;
    float sunColor[3] { 0, 0, 0 }, sunDir[3] { 0, 0, 0 };
    bool lightsDirty = false;
    // AO bake results (ark_ddgi_bake_ao)
    DeviceBuffer bakeTri, bakeBary, bakeOut, bakePixels, bakeCounters;
    uint32_t bakeW = 0, bakeH = 0;
    int bakeBent = 0;
    SceneArgs scene {};          // = sceneStore->args
    ArkDdgiBvhStats bvhStats {}; // = sceneStore->bvhStats
    uint32_t bvhMaxDepth = 0;
    // instrumentation
    bool counting = false;
    bool timing = false;
    hipEvent_t ev[6] = {};
    float lastMs[5] = {};
    bool timingValid = false;
    ArkDdgiCounters lastCounters {};
    bool countersPending = false;
    uint64_t lastRays = 0, lastProbes = 0;
    uint32_t nextProbeIndex = 0; // (first + K) % N of the last update, or of a loaded state
    uint32_t lastFirst = 0, lastK = 0; // the last update's window (ark_ddgi_window_exchange_info)
    // a refit or an installed rebuild enqueued on a caller's stream (ark_ddgi_set_instances_async,
    // worldCollect): the next update's traversal on the traversal stream waits for it
    hipEvent_t evRefit = nullptr;
    bool refitPending = false;
    // ark_ddgi_set_instances_async's refits run on refitStream (SceneStore::spare):
    // evFree[slot] ends with the operations that read that slot's copy while it was the
    // front one (recorded when a refit swapped it out, on the stream of the last
    // operation, which follows the others); evInstalled with the last install (a rebuild
    // installed on a caller's stream writes the front copy)
    hipStream_t refitStream = nullptr;
    hipEvent_t evFree[3] = {};
    bool freeValid[3] = { false, false, false };
    hipEvent_t evInstalled = nullptr;
    bool installValid = false;

    int fail(int code, const char* fmt, ...)
    {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        std::vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        lastError = buf;
        return code;
    }
    int hipFail(hipError_t e, const char* what)
    {
        return fail(ARK_DDGI_E_DEVICE, "%s: %s", what, hipGetErrorString(e));
    }
};

#define ARK_HIP(expr)                                                   \
    do {                                                                \
        hipError_t _e = (expr);                                         \
        if (_e != hipSuccess) return ctx->hipFail(_e, #expr);           \
    } while (0)

namespace {

int clearHistory(ArkDdgiCtx* ctx)
{
    // DDGINode.cpp:50-55: irradiance cleared to 0, visibility to (zFar, zFar^2) in RG16F;
    // zFar^2 = 1e8 overflows fp16: +inf by RNE, or 65504 if saturating.
    uint16_t zf = f32_to_f16_host(ctx->desc.z_far);
    uint16_t zf2 = f32_to_f16_host(ctx->desc.z_far * ctx->desc.z_far);
    if (ctx->desc.clear_overflow_mode == ARK_DDGI_CLEAR_OVERFLOW_MAX_FINITE) {
        if ((zf & 0x7fffu) == 0x7c00u) zf = static_cast<uint16_t>((zf & 0x8000u) | 0x7bffu);
        if ((zf2 & 0x7fffu) == 0x7c00u) zf2 = static_cast<uint16_t>((zf2 & 0x8000u) | 0x7bffu);
    }
    ARK_HIP(hipMemsetAsync(ctx->irr.ptr, 0, ctx->irr.bytes, ctx->stream));
    ARK_HIP(launch_fill_u32(ctx->vis.ptr, ctx->vis.bytes / 4, static_cast<uint32_t>(zf) | (static_cast<uint32_t>(zf2) << 16), ctx->stream));
    ARK_HIP(hipMemsetAsync(ctx->offsets.ptr, 0, ctx->offsets.bytes, ctx->stream));
    ARK_HIP(hipMemsetAsync(ctx->surfels.ptr, 0, ctx->surfels.bytes, ctx->stream));
    ARK_HIP(hipStreamSynchronize(ctx->stream));
    return ARK_DDGI_OK;
}

hipError_t drainContext(ArkDdgiCtx* ctx);

int ensureSpill(ArkDdgiCtx* ctx)
{
    // a node group is pushed at most once per BVH8 level: depth + 2 entries of 2 words
    uint32_t need = std::max<uint32_t>(1u, ctx->bvhMaxDepth + 2u > static_cast<uint32_t>(kStackLds) ? ctx->bvhMaxDepth + 2u - kStackLds : 1u);
    uint32_t threads = std::max(ctx->traceBlocks, ctx->shadowBlocks) * kTraceBlock; // the traversal kernels
    const uint64_t words = static_cast<uint64_t>(need) * 2 * threads;
    const size_t bytes = 2 * words * sizeof(uint32_t); // region 0: all but the primary traversal
    if (ctx->spill.bytes >= bytes) {
        ctx->spillRegionWords = words;
        return ARK_DDGI_OK;
    }
    if (ctx->spill.ptr) ARK_HIP(drainContext(ctx)); // a deeper BVH (a rebuilt sun BVH): frames in flight use it
    ctx->spillRegionWords = words;
    ARK_HIP(ctx->spill.alloc(bytes));
    ctx->spillEntries = need;
    return ARK_DDGI_OK;
}

// The stream of an asynchronous entry point: NULL is the legacy default (null)
// stream, which orders against every blocking stream of the process (torch's
// default stream among them), like any other HIP API taking a stream.
hipStream_t streamOf(void* h) { return static_cast<hipStream_t>(h); }

// Operations of one context execute in call order, whatever streams they are given
// (they share the traversal spill area, the hit records and the atlases): an
// operation on another stream than the previous one first waits for it.
hipError_t orderBegin(ArkDdgiCtx* ctx, hipStream_t s)
{
    if (ctx->orderValid && ctx->orderStream != s) return hipStreamWaitEvent(s, ctx->evOrder, 0);
    return hipSuccess;
}

hipError_t orderEnd(ArkDdgiCtx* ctx, hipStream_t s)
{
    const hipError_t e = hipEventRecord(ctx->evOrder, s);
    ctx->orderStream = s;
    ctx->orderValid = e == hipSuccess;
    return e;
}

// Shading work set for the largest window: per-ray light bits, then k_shadow_gen's
// shadow-ray list (at most one ray per probe ray and light).
struct ShadeWorkLayout {
    uint64_t bits, list, total;
};

ShadeWorkLayout shadeWorkLayout(const ArkDdgiCtx* ctx)
{
    auto al = [](uint64_t b) { return (b + 255) & ~static_cast<uint64_t>(255); };
    const uint64_t rays = static_cast<uint64_t>(ctx->Kmax) * ctx->Rmax;
    const uint64_t entries = rays * ctx->lightCount;
    ShadeWorkLayout w {};
    w.bits = 0;
    w.list = al(rays * 4);
    w.total = w.list + al(entries * sizeof(ShadowRay));
    return w;
}

int ensureShadeWork(ArkDdgiCtx* ctx)
{
    const uint64_t rays = static_cast<uint64_t>(ctx->Kmax) * ctx->Rmax;
    if (rays >= (1ull << 28) && ctx->lightCount > 0)
        return ctx->fail(ARK_DDGI_E_UNSUPPORTED, "%llu rays per update: shadow-ray owners pack (ray << 4) | light in 32 bits", static_cast<unsigned long long>(rays));
    const ShadeWorkLayout w = shadeWorkLayout(ctx);
    if (ctx->shadeWork.bytes < w.total) ARK_HIP(ctx->shadeWork.alloc(w.total));
    return ARK_DDGI_OK;
}

// RT reflections' ray-list work set for `pixels` rays (ark_ddgi_rt_reflections)
// Workgroups of the persistent shadow traversal for `rays` closest-hit rays (~0.25
// shadow rays each on C4): the launch is a tail of the longest shadow rays when
// there are few, and fewer co-resident waves shorten each one's iterations
// (measured on C4: K = 2048 windows 0.228 -> 0.180 ms at 3 workgroups per CU,
// K = 4096 0.246 -> 0.225, the full grid (8.4 M rays) unchanged from 5 to 6).
constexpr uint64_t kShadowMinPerCu = 3; // 1 and 2 measured slower or within noise (profiles/r04_p)
uint32_t shadowBlocksFor(const ArkDdgiCtx* ctx, uint64_t rays)
{
    const uint64_t perCu = std::min<uint64_t>(ctx->shadowBlocksPerCu, std::max<uint64_t>(kShadowMinPerCu, rays >> 20));
    return static_cast<uint32_t>(perCu * ctx->cuCount);
}

int ensureReflWork(ArkDdgiCtx* ctx, uint64_t pixels)
{
    if (pixels >= (1ull << 28) && ctx->lightCount > 0)
        return ctx->fail(ARK_DDGI_E_UNSUPPORTED, "%llu reflection rays: shadow-ray owners pack (ray << 4) | light in 32 bits", static_cast<unsigned long long>(pixels));
    auto al = [](uint64_t b) { return (b + 255) & ~static_cast<uint64_t>(255); };
    const uint64_t bytes = al(pixels * 32) + al(pixels * sizeof(GpuHit)) + al(pixels * 4) + al((kRayCounterWords + kRayCounterStride) * 4) +
                           al(pixels * ctx->lightCount * sizeof(ShadowRay));
    if (ctx->reflWork.bytes < bytes) ARK_HIP(ctx->reflWork.alloc(bytes));
    return ARK_DDGI_OK;
}

template<typename T>
int upload(ArkDdgiCtx* ctx, DeviceBuffer& buf, const T* data, size_t count)
{
    size_t bytes = count * sizeof(T);
    ARK_HIP(buf.alloc(std::max<size_t>(bytes, 16)));
    if (bytes) ARK_HIP(hipMemcpy(buf.ptr, data, bytes, hipMemcpyHostToDevice));
    return ARK_DDGI_OK;
}

static_assert(ARK_DDGI_MAX_SPOT_LIGHTS == kMaxLights - 1, "spot light capacity");

// SpotLightData as the closest hit reads it (GpuScene.cpp:844-858: the fields of
// LightData.h:19-40 the DDGI path uses)
GpuSpotLight gpuSpotLight(const ArkSpotLight& sl)
{
    GpuSpotLight g;
    std::memset(&g, 0, sizeof(g));
    for (int k = 0; k < 3; ++k) {
        g.color[k] = sl.color[k];
        g.direction[k] = sl.world_space_direction[k];
        g.right[k] = sl.world_space_right[k];
        g.up[k] = sl.world_space_up[k];
        g.position[k] = sl.world_space_position[k];
    }
    g.position[3] = sl.outer_cone_half_angle;
    g.ies_texture = sl.ies_profile_index;
    return g;
}

// f(begin, end) over [0, n) in `threads` contiguous chunks (one when n is small)
template<class F>
void parallelFor(size_t n, int threads, F f)
{
    const int T = std::max(1, std::min<int>(threads, static_cast<int>(n >> 16) + 1));
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T); });
    f(0, n / T);
    for (std::thread& th : pool) th.join();
}

// sRGB EOTF applied per texel before filtering (Vulkan sRGB formats).
float srgbToLinear(float c)
{
    return c <= 0.04045f ? c / 12.92f : powf_((c + 0.055f) / 1.055f, 2.4f);
}

// The context's kernel view of its scene: the store's world BVHs, pools and tables with
// the context's own lights (sun by value, spots in its light buffer); the light-space
// sun BVH only while it is valid and the sun points the way it was built for (any other
// direction traces the sun's shadow rays through the world BVHs: same results).
void deriveSceneArgs(ArkDdgiCtx* ctx)
{
    const SceneStore& st = *ctx->sceneStore;
    SceneArgs sc = st.args;
    sc.has_sun = ctx->hasSun;
    for (int k = 0; k < 3; ++k) {
        sc.sun_color[k] = ctx->sunColor[k];
        sc.sun_dir[k] = ctx->sunDir[k];
    }
    sc.spot_count = static_cast<int32_t>(ctx->spotHost.size());
    sc.spots = ctx->lights.as<GpuSpotLight>();
    const bool sunOk = ctx->hasSun && st.sunArgs.sun_root >= 0 && std::memcmp(ctx->sunDir, st.sunDirBuilt, sizeof(ctx->sunDir)) == 0;
    sc.sun_nodes = sunOk ? st.sunArgs.sun_nodes : nullptr;
    sc.sun_tris = sunOk ? st.sunArgs.sun_tris : nullptr;
    sc.sun_root = sunOk ? st.sunArgs.sun_root : -1;
    std::memcpy(sc.sun_frame, st.sunArgs.sun_frame, sizeof(sc.sun_frame));
    ctx->scene = sc;
    ctx->lightCount = (ctx->hasSun ? 1u : 0u) + static_cast<uint32_t>(ctx->spotHost.size());
    ctx->bvhStats = st.bvhStats;
    ctx->bvhMaxDepth = st.bvhMaxDepth;
    ctx->sceneVersion = st.version;
}

// deriveSceneArgs plus a traversal spill area deep enough for every BVH the derived
// args reach. Every caller goes through here: a sharing context may
// have installed a deeper sun BVH, and marking the store's version as seen without
// growing the spill area would let the next traversal overrun it.
int refreshScene(ArkDdgiCtx* ctx)
{
    deriveSceneArgs(ctx);
    return ensureSpill(ctx);
}

// The context's spot lights reach the device in stream order on `s`, ahead of the
// operation that reads them (a by-value kernel argument: no host buffer to keep alive).
hipError_t flushLights(ArkDdgiCtx* ctx, hipStream_t s)
{
    if (!ctx->lightsDirty) return hipSuccess;
    LightBlock b {};
    b.count = static_cast<uint32_t>(ctx->spotHost.size());
    std::copy(ctx->spotHost.begin(), ctx->spotHost.end(), b.spots);
    const hipError_t e = launch_store_lights(b, ctx->lights.as<GpuSpotLight>(), s);
    if (e == hipSuccess) ctx->lightsDirty = false;
    return e;
}

// Waits for every operation of the context enqueued so far (both of its streams).
hipError_t drainContext(ArkDdgiCtx* ctx)
{
    hipError_t e = hipStreamSynchronize(ctx->traceStream);
    if (e == hipSuccess && ctx->orderValid) e = hipEventSynchronize(ctx->evOrder);
    return e;
}

// --- scene maintenance: stream-ordered refits, background rebuilds ------------------

// A buffer the launches enqueued so far on `s` (and, through orderBegin, everything the
// context enqueued before) may read: freed by collectRetired once they are done.
hipError_t retireBuffer(SceneStore& st, DeviceBuffer& b, hipStream_t s)
{
    if (!b.ptr) return hipSuccess;
    Retired r;
    hipError_t e = hipEventCreateWithFlags(&r.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(r.done, s);
    if (e != hipSuccess) {
        if (r.done) (void)hipEventDestroy(r.done);
        (void)hipStreamSynchronize(s); // cannot defer: wait, then free
        b.release();
        return e;
    }
    r.buf = b;
    b = DeviceBuffer {};
    st.retired.push_back(r);
    return hipSuccess;
}

void collectRetired(SceneStore& st)
{
    for (size_t i = 0; i < st.retired.size();) {
        Retired& r = st.retired[i];
        if (hipEventQuery(r.done) == hipSuccess) {
            r.buf.release();
            (void)hipEventDestroy(r.done);
            st.retired[i] = st.retired.back();
            st.retired.pop_back();
        } else {
            ++i;
        }
    }
}

// `bytes` of host data into `dst` in stream order on `s`, through the store's pinned
// staging ring (a slot is reused once its previous copy has run).
hipError_t stagedUpload(SceneStore& st, void* dst, const void* src, size_t bytes, hipStream_t s)
{
    if (bytes == 0) return hipSuccess;
    const int i = st.stageNext;
    st.stageNext = (i + 1) % SceneStore::kStageSlots;
    hipError_t e = hipSuccess;
    if (!st.stageDone[i] && (e = hipEventCreateWithFlags(&st.stageDone[i], hipEventDisableTiming)) != hipSuccess) return e;
    if (st.stageBytes[i]) (void)hipEventSynchronize(st.stageDone[i]); // its last copy (an earlier frame's) has run
    if (st.stageBytes[i] < bytes) {
        if (st.stage[i]) (void)hipHostFree(st.stage[i]);
        st.stage[i] = nullptr;
        st.stageBytes[i] = 0;
        if ((e = hipHostMalloc(&st.stage[i], bytes, hipHostMallocDefault)) != hipSuccess) return e;
        st.stageBytes[i] = bytes;
    }
    std::memcpy(st.stage[i], src, bytes);
    if ((e = hipMemcpyAsync(dst, st.stage[i], bytes, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    return hipEventRecord(st.stageDone[i], s);
}

// The boxes' absolute inflations of a refit, as set_scene and build_sun_bvh derive them
// from the records' bounds (world: bvh8_inflation_box, 1e-6 |diagonal|; light space:
// 2 x 1e-6 |light diagonal| + 2e-6 max |world coordinate|), here from bounds that
// contain the records: every instance's object-space box (st.instObjBox) through its
// current transform (st.refitHost), corner by corner in double, and those corners in the
// sun's frame. Never less than the build's (st.inflateAbs, st.sunInflateAbs). Larger
// bounds only loosen the boxes; the hits do not depend on them.
void refitInflations(const SceneStore& st, float& world, float& light)
{
    double lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
    double llo[3] = { INFINITY, INFINITY, INFINITY }, lhi[3] = { -INFINITY, -INFINITY, -INFINITY };
    double maxAbs = 0.0;
    const size_t n = std::min(st.instObjBox.size(), st.refitHost.size());
    for (size_t i = 0; i < n; ++i) {
        const std::array<float, 6>& b = st.instObjBox[i];
        if (!(b[0] <= b[3])) continue; // no triangles
        const float* M = st.refitHost[i].m;
        for (int c = 0; c < 8; ++c) {
            const double P[3] = { b[(c & 1) ? 3 : 0], b[(c & 2) ? 4 : 1], b[(c & 4) ? 5 : 2] };
            double w[3];
            for (int r = 0; r < 3; ++r) {
                w[r] = double(M[4 * r]) * P[0] + double(M[4 * r + 1]) * P[1] + double(M[4 * r + 2]) * P[2] + double(M[4 * r + 3]);
                lo[r] = std::min(lo[r], w[r]);
                hi[r] = std::max(hi[r], w[r]);
                maxAbs = std::max(maxAbs, std::fabs(w[r]));
            }
            for (int r = 0; r < 3; ++r) {
                const double L = st.sunFrameD[3 * r] * w[0] + st.sunFrameD[3 * r + 1] * w[1] + st.sunFrameD[3 * r + 2] * w[2];
                llo[r] = std::min(llo[r], L);
                lhi[r] = std::max(lhi[r], L);
            }
        }
    }
    auto box = [](const double* l, const double* h) {
        double d2 = 0.0;
        for (int a = 0; a < 3; ++a)
            if (h[a] >= l[a]) d2 += (h[a] - l[a]) * (h[a] - l[a]);
        return 1e-6 * std::sqrt(d2);
    };
    // rounded up to fp32 (the bounds' own rounding to fp32 in the builds is within it)
    world = std::max(st.inflateAbs, std::nextafter(static_cast<float>(box(lo, hi)), INFINITY));
    light = std::max(st.sunInflateAbs, std::nextafter(static_cast<float>(2.0 * box(llo, lhi) + 2e-6 * maxAbs), INFINITY));
}

// The refit of every BVH of the scene on `s`: the records of dirty instances re-transformed
// (st.refitInst), the world BVHs' boxes level by level, and the light-space sun BVH's
// records and light-space boxes. The boxes' inflations from the instances' bounds
// (refitInflations, host).
struct RefitTarget {
    GpuBvh8Node* nodes;
    GpuBvh8Node* sunNodes; // the light-space BVH's buffer (its records at the front copy's offset)
};
RefitTarget frontTarget(SceneStore& st) { return { st.nodes.as<GpuBvh8Node>(), st.sunNodes.as<GpuBvh8Node>() }; }
RefitTarget spareTarget(SceneStore::Spare& c) { return { c.nodes.as<GpuBvh8Node>(), c.sunNodes.as<GpuBvh8Node>() }; }

// The instance masks of a BVH's nodes (k_node_masks), level by level on `s`, into `masks`
int computeMasks(ArkDdgiCtx* ctx, SceneStore& st, DeviceBuffer& masks, const GpuBvh8Node* nodes, const GpuTriangle* tris, uint64_t nodeCount,
                 const DeviceBuffer& order, const std::vector<uint32_t>& offsets, hipStream_t s)
{
    if (masks.bytes < std::max<uint64_t>(8, nodeCount * 8)) {
        ARK_HIP(retireBuffer(st, masks, s));
        ARK_HIP(masks.alloc(std::max<uint64_t>(8, nodeCount * 8)));
    }
    for (size_t l = 0; l + 1 < offsets.size(); ++l)
        ARK_HIP(launch_node_masks(nodes, tris, masks.as<uint64_t>(), order.as<uint32_t>() + offsets[l], offsets[l + 1] - offsets[l], s));
    return ARK_DDGI_OK;
}

// The inflation of the refitted boxes rounded up to a power of two: it changes only when
// the scene's extent crosses one, so that a refit rarely has to touch the nodes of the
// instances that did not move (a change refits every node).
float inflationStep(float x) { return x > 0.0f ? std::ldexp(1.0f, static_cast<int>(std::ceil(std::log2(static_cast<double>(x))))) : x; }

// The refit of the copy `t` (slot: the transforms and inflations it holds) of every BVH
// of the scene on `s`, level by level, the nodes with a moved instance below them
// (st.refitInst's dirty flags: the instances whose transform differs from the copy's):
// their moved records re-transformed, their boxes and planes recomputed. Every node after
// an install or a new scene (refitFull) or a change of the inflation.
int enqueueRefit(ArkDdgiCtx* ctx, SceneStore& st, hipStream_t s, const RefitTarget& t, int slot)
{
    float inflateWorld = 0.0f, inflateLight = 0.0f;
    refitInflations(st, inflateWorld, inflateLight);
    inflateWorld = inflationStep(inflateWorld);
    inflateLight = inflationStep(inflateLight);
    uint64_t dirty = 0;
    for (size_t i = 0; i < st.refitHost.size(); ++i)
        if (st.refitHost[i].dirty) dirty |= 1ull << (i & 63u);
    GpuTriangle* tris = reinterpret_cast<GpuTriangle*>(reinterpret_cast<char*>(t.nodes) + st.args.tri_byte_offset);
    const RefitInstance* inst = st.refitInst.as<RefitInstance>();
    if (!st.masksValid) {
        if (const int rc = computeMasks(ctx, st, st.nodeMasks, t.nodes, tris, st.bvhStats.node_count, st.refitOrder, st.levelOffsets, s)) return rc;
        st.masksValid = true;
    }
    RefitBoxArgs world {};
    world.inflate = inflateWorld;
    world.light = 0;
    world.dirty = (st.refitFull || inflateWorld != st.inflCopy[slot][0]) ? ~0ull : dirty;
    const uint32_t* order = st.refitOrder.as<uint32_t>();
    for (size_t l = 0; l + 1 < st.levelOffsets.size(); ++l)
        ARK_HIP(launch_refit_nodes(t.nodes, tris, st.refitBoxes.as<float>(), order + st.levelOffsets[l], st.levelOffsets[l + 1] - st.levelOffsets[l],
                                   world, st.nodeMasks.as<uint64_t>(), inst, st.indices.as<uint32_t>(), st.positions.as<float>(), s));
    st.inflCopy[slot][0] = inflateWorld;
    if (st.sunArgs.sun_root >= 0 && st.sunTriRecords && !st.sunLevelOffsets.empty()) {
        const size_t sunTriOffset = reinterpret_cast<const char*>(st.sunArgs.sun_tris) - static_cast<const char*>(st.sunNodes.ptr);
        GpuTriangle* stris = reinterpret_cast<GpuTriangle*>(reinterpret_cast<char*>(t.sunNodes) + sunTriOffset);
        if (!st.sunMasksValid) {
            if (const int rc = computeMasks(ctx, st, st.sunNodeMasks, t.sunNodes, stris, st.sunBvhNodes, st.sunRefitOrder, st.sunLevelOffsets, s)) return rc;
            st.sunMasksValid = true;
        }
        RefitBoxArgs light {};
        std::memcpy(light.frame, st.sunFrameD, sizeof(light.frame));
        light.inflate = inflateLight;
        light.light = 1;
        light.dirty = (st.refitFull || inflateLight != st.inflCopy[slot][1]) ? ~0ull : dirty;
        const uint32_t* so = st.sunRefitOrder.as<uint32_t>();
        for (size_t l = 0; l + 1 < st.sunLevelOffsets.size(); ++l)
            ARK_HIP(launch_refit_nodes(t.sunNodes, stris, st.sunRefitBoxes.as<float>(), so + st.sunLevelOffsets[l], st.sunLevelOffsets[l + 1] - st.sunLevelOffsets[l],
                                       light, st.sunNodeMasks.as<uint64_t>(), inst, st.indices.as<uint32_t>(), st.positions.as<float>(), s));
        st.inflCopy[slot][1] = inflateLight;
    }
    st.refitFull = false;
    return ARK_DDGI_OK;
}

// The refit's transforms of `instances` on the device (stream-ordered), every one dirty
// (have = nullptr: the records are of an older version, an installed rebuild) or those
// whose transform differs from the one the target copy's records hold (`have`).
int uploadRefitInstances(ArkDdgiCtx* ctx, SceneStore& st, const ArkRTInstance* instances, uint32_t count, const std::vector<std::array<float, 12>>* have,
                         hipStream_t s)
{
    bool allDirty = !have || have->size() != count;
    if (st.refitHost.size() != count) st.refitHost.assign(count, RefitInstance {});
    if (!st.refitInst.ptr || st.refitInst.bytes < std::max<size_t>(16, count * sizeof(RefitInstance))) ARK_HIP(st.refitInst.alloc(std::max<size_t>(16, count * sizeof(RefitInstance))));
    for (uint32_t ii = 0; ii < count; ++ii) {
        const float* M = instances[ii].object_to_world;
        const float det = M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) + M[2] * (M[4] * M[9] - M[5] * M[8]);
        const ArkRTTriangleMesh& mesh = st.meshHost[instances[ii].rt_mesh_index];
        RefitInstance& q = st.refitHost[ii];
        const bool moved = allDirty || std::memcmp((*have)[ii].data(), M, sizeof(q.m)) != 0;
        std::memcpy(q.m, M, sizeof(q.m));
        q.first_vertex = mesh.first_vertex;
        q.first_index = static_cast<uint32_t>(mesh.first_index);
        q.flip = det < 0.0f ? 1u : 0u;
        q.dirty = moved ? 1u : 0u;
    }
    ARK_HIP(stagedUpload(st, st.refitInst.ptr, st.refitHost.data(), count * sizeof(RefitInstance), s));
    return ARK_DDGI_OK;
}

// A BVH of the scene was replaced (an install): its node masks are recomputed and the
// next refit reaches every node.
void markTopologyChanged(SceneStore& st)
{
    st.masksValid = false;
    st.sunMasksValid = false;
    st.refitFull = true;
}

// The spare geometry copies retired behind everything enqueued on `s` so far.
hipError_t dropSpares(SceneStore& st, hipStream_t s)
{
    hipError_t e = hipSuccess;
    for (SceneStore::Spare& c : st.spare) {
        for (DeviceBuffer* b : { &c.nodes, &c.sunNodes, &c.instances })
            if (e == hipSuccess) e = retireBuffer(st, *b, s);
        c.valid = false;
    }
    return e;
}

// An install replaced a BVH of the front copy (a new topology, refitted forward on `s`):
// the back copy is dropped - retired behind everything enqueued so far - and copied anew
// from the front one by the next refit, which waits for the install (evInstalled).
hipError_t installedGeometry(ArkDdgiCtx* ctx, SceneStore& st, hipStream_t s)
{
    hipError_t e = dropSpares(st, s);
    markTopologyChanged(st); // (again: the boxes scratch is of the old topology without a forward refit)
    std::vector<std::array<float, 12>>& xf = st.xf[st.front];
    xf.resize(st.instHost.size());
    for (size_t i = 0; i < st.instHost.size(); ++i) std::memcpy(xf[i].data(), st.instHost[i].object_to_world, sizeof(float) * 12);
    if (e == hipSuccess) e = hipEventRecord(ctx->evInstalled, s);
    ctx->installValid = e == hipSuccess;
    return e;
}

// Background builds' host-thread inputs: a snapshot of the world records on `s` behind
// every refit enqueued so far (the refits run on the callers' streams; a thread reading
// the live records could see a half-refitted set).
hipError_t snapshotRecords(SceneStore& st, DeviceBuffer& snap, hipEvent_t& ev, hipStream_t s)
{
    const size_t bytes = st.triRecords * sizeof(GpuTriangle);
    hipError_t e = snap.alloc(std::max<size_t>(bytes, 16));
    if (e == hipSuccess && bytes)
        e = hipMemcpyAsync(snap.ptr, static_cast<const char*>(st.nodes.ptr) + st.args.tri_byte_offset, bytes, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess && !ev) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, s);
    return e;
}

// The sun rebuild's thread: the snapshot of the world records, the light-space BVH of
// job->dir on the host (as set_scene builds it), uploaded into job->buf.
void runSunJob(SunJob* job, int device, uint64_t count, int threads)
{
    const auto t0 = std::chrono::steady_clock::now();
    bool ok = hipSetDevice(device) == hipSuccess;
    hipStream_t s = nullptr;
    ok = ok && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventSynchronize(job->evSnap) == hipSuccess;
    std::vector<GpuTriangle> rec(ok ? count : 0);
    ok = ok && hipMemcpyAsync(rec.data(), job->snap.ptr, count * sizeof(GpuTriangle), hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
    Bvh8BuildResult r;
    if (ok) {
        SunBvhInput in;
        sun_frame(job->dir, in.frame);
        sun_add_records(in, rec, threads);
        std::vector<GpuTriangle>().swap(rec);
        BvhBuildOptions opt;
        opt.threads = threads;
        Bvh8CollapseOptions copt;
        copt.threads = threads;
        ok = build_sun_bvh(in, opt, copt, r) && !r.nodes.empty();
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) {
                job->frame[i * 3 + k] = static_cast<float>(in.frame[i][k]);
                job->frameD[i * 3 + k] = in.frame[i][k];
            }
        job->inflateAbs = in.inflateAbs;
        const int32_t root = 0;
        ok = ok && bvhLevelOrder(r.nodes.data(), r.nodes.size(), &root, 1, job->levelOrder, job->levelOffsets);
    }
    if (ok) {
        const size_t nb = r.nodes.size() * sizeof(GpuBvh8Node);
        job->triOffset = (nb + 255) & ~static_cast<size_t>(255);
        job->triRecords = r.tris.size();
        r.tris.push_back(GpuTriangle {}); // padding record (five-load fetch)
        ok = job->buf.alloc(job->triOffset + r.tris.size() * sizeof(GpuTriangle)) == hipSuccess &&
             hipMemcpyAsync(job->buf.ptr, r.nodes.data(), nb, hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(static_cast<char*>(job->buf.ptr) + job->triOffset, r.tris.data(), r.tris.size() * sizeof(GpuTriangle), hipMemcpyHostToDevice, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        job->nodes = r.nodes.size();
        job->depth = r.max_depth;
    }
    if (s) (void)hipStreamDestroy(s);
    job->ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    job->ok = ok;
    job->done.store(true, std::memory_order_release);
}

// Structural check of a BVH8 before anything reaches the GPU: every node is
// referenced once from a root-reachable parent (no cycles, no sharing), every leaf's
// triangles lie inside the triangle array and every triangle (every record but the
// holes of the rows) is covered once.
bool checkBvh8Structure(const std::vector<GpuBvh8Node>& allNodes, const std::vector<GpuTriangle>& allTris, const int32_t* roots, int nRoots, std::string& why)
{
    char buf[128];
    auto bad = [&](const char* fmt, uint64_t v) {
        std::snprintf(buf, sizeof(buf), fmt, static_cast<unsigned long long>(v));
        why = buf;
        return false;
    };
    std::vector<uint8_t> seenNode(allNodes.size(), 0);
    std::vector<uint8_t> seenTri(allTris.size(), 0);
    std::vector<uint32_t> work;
    for (int c = 0; c < nRoots; ++c)
        if (roots[c] >= 0) work.push_back(static_cast<uint32_t>(roots[c]));
    while (!work.empty()) {
        const uint32_t n = work.back();
        work.pop_back();
        if (n >= allNodes.size() || seenNode[n]) return bad("BVH invalid: node %llu", n);
        seenNode[n] = 1;
        const GpuBvh8Node& nd = allNodes[n];
        uint32_t internal = 0;
        if ((nd.leaf_tris >> 24) || (nd.leaf_mask & nd.imask)) return bad("BVH invalid: node %llu leaf rows", n);
        for (int sl = 0; sl < 8; ++sl) {
            const bool isInternal = (nd.imask >> sl) & 1u;
            uint32_t slotTris[kBvh8MaxLeafSize];
            const int cnt = bvh8SlotTriangles(nd, sl, slotTris);
            if (cnt < 0) return bad("BVH invalid: node %llu slot", n);
            if (isInternal) work.push_back(nd.child_base + internal++);
            for (int i = 0; i < cnt; ++i) {
                const uint32_t t = slotTris[i];
                if (t >= allTris.size() || isHoleTriangle(allTris[t])) return bad("BVH invalid: leaf range%.0llu", 0);
                if (seenTri[t]) return bad("BVH invalid: triangle %llu in two leaves", t);
                seenTri[t] = 1;
            }
            for (int a = 0; a < 3; ++a)
                if ((isInternal || cnt > 0) && nd.qlo[a][sl] > nd.qhi[a][sl]) return bad("BVH invalid: child box%.0llu", 0);
        }
    }
    for (size_t t = 0; t < seenTri.size(); ++t)
        if (!seenTri[t] && !isHoleTriangle(allTris[t])) return bad("BVH invalid: triangle %llu unreachable", t);
    return true;
}


// The world rebuild's thread: the three classes' BVHs from the snapshot's records (their
// vertices v0, v0 + e1, v0 + e2; each leaf record then replaced by its source record,
// bit for bit), the record order's source indices and the refit's level order.
void runWorldJob(WorldJob* job, int device, int threads)
{
    const auto t0 = std::chrono::steady_clock::now();
    bool ok = hipSetDevice(device) == hipSuccess;
    hipStream_t s = nullptr;
    ok = ok && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventSynchronize(job->evSnap) == hipSuccess;
    std::vector<GpuTriangle> rec(ok ? job->snapRecords : 0);
    ok = ok && hipMemcpyAsync(rec.data(), job->snap.ptr, rec.size() * sizeof(GpuTriangle), hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
    if (!ok) job->error = "snapshot download failed";
    std::vector<BuildTriangle> cls[3];
    if (ok) {
        for (size_t i = 0; i < rec.size(); ++i) {
            const GpuTriangle& g = rec[i];
            if (isHoleTriangle(g)) continue;
            uint32_t inst, flip;
            std::memcpy(&inst, &g.t2[1], 4);
            std::memcpy(&flip, &g.t2[3], 4);
            if (inst >= job->classOf.size()) {
                ok = false;
                job->error = "record of an unknown instance";
                break;
            }
            BuildTriangle t;
            const float e1[3] = { g.t0[3], g.t1[0], g.t1[1] }, e2[3] = { g.t1[2], g.t1[3], g.t2[0] };
            for (int a = 0; a < 3; ++a) {
                t.v0[a] = g.t0[a];
                t.v1[a] = g.t0[a] + e1[a];
                t.v2[a] = g.t0[a] + e2[a];
            }
            t.instance = inst;
            t.primitive = static_cast<uint32_t>(i); // the source record (replaced below)
            t.flip_facing = flip;
            cls[job->classOf[inst]].push_back(t);
        }
    }
    std::vector<GpuBvh8Node> allNodes;
    std::vector<GpuTriangle> allTris;
    if (ok) {
        BvhBuildOptions opt;
        opt.max_leaf_size = kBvh8MaxLeafSize;
        opt.threads = threads;
        {
            float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
            for (int c = 0; c < 3; ++c)
                for (const BuildTriangle& t : cls[c])
                    for (const float* v : { t.v0, t.v1, t.v2 })
                        for (int a = 0; a < 3; ++a) {
                            lo[a] = std::min(lo[a], v[a]);
                            hi[a] = std::max(hi[a], v[a]);
                        }
            opt.inflate_abs = bvh8_inflation_box(lo, hi);
        }
        Bvh8CollapseOptions copt;
        copt.threads = threads;
        for (int c = 0; c < 3 && ok; ++c) {
            if (cls[c].empty()) continue;
            BvhBuildResult r2 = build_bvh(cls[c], opt, 0u, 0u);
            std::vector<BuildTriangle>().swap(cls[c]);
            if (r2.max_leaf > static_cast<uint32_t>(kBvh8MaxLeafSize)) {
                ok = false;
                job->error = "BVH2 leaf over the leaf size";
                break;
            }
            if (c == 0) job->sah = r2.sah_cost;
            job->maxLeaf = std::max(job->maxLeaf, r2.max_leaf);
            Bvh8BuildResult r = collapse_bvh8(r2, static_cast<uint32_t>(allNodes.size()), static_cast<uint32_t>(allTris.size()), copt);
            job->roots[c] = static_cast<int32_t>(allNodes.size());
            if (c == 0) job->opaqueNodes = static_cast<uint32_t>(r.nodes.size());
            job->depth = std::max(job->depth, r.max_depth);
            job->triangles += r.triangles;
            allNodes.insert(allNodes.end(), r.nodes.begin(), r.nodes.end());
            allTris.insert(allTris.end(), r.tris.begin(), r.tris.end());
        }
    }
    std::vector<uint32_t> perm;
    if (ok) {
        perm.assign(allTris.size(), 0xffffffffu);
        for (size_t i = 0; i < allTris.size(); ++i) {
            GpuTriangle& g = allTris[i];
            if (isHoleTriangle(g)) continue;
            uint32_t src;
            std::memcpy(&src, &g.t2[2], 4);
            perm[i] = src;
            g = rec[src];
        }
        ok = checkBvh8Structure(allNodes, allTris, job->roots, 3, job->error);
    }
    std::vector<uint32_t> order;
    ok = ok && bvhLevelOrder(allNodes.data(), allNodes.size(), job->roots, 3, order, job->levelOffsets);
    if (ok) {
        const size_t nb = allNodes.size() * sizeof(GpuBvh8Node);
        job->triOffset = (nb + 255) & ~static_cast<size_t>(255);
        job->triRecords = allTris.size();
        job->nodes = allNodes.size();
        allTris.push_back(GpuTriangle {}); // padding record (five-load fetch)
        ok = job->triOffset + allTris.size() * sizeof(GpuTriangle) < (1ull << 32) &&
             job->buf.alloc(job->triOffset + allTris.size() * sizeof(GpuTriangle)) == hipSuccess &&
             job->perm.alloc(std::max<size_t>(16, perm.size() * 4)) == hipSuccess && job->order.alloc(std::max<size_t>(16, order.size() * 4)) == hipSuccess &&
             hipMemcpyAsync(job->buf.ptr, allNodes.data(), nb, hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(static_cast<char*>(job->buf.ptr) + job->triOffset, allTris.data(), allTris.size() * sizeof(GpuTriangle), hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(job->perm.ptr, perm.data(), perm.size() * 4, hipMemcpyHostToDevice, s) == hipSuccess &&
             hipMemcpyAsync(job->order.ptr, order.data(), order.size() * 4, hipMemcpyHostToDevice, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
        if (!ok && job->error.empty()) job->error = "upload failed";
    }
    if (s) (void)hipStreamDestroy(s);
    job->ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    job->ok = ok;
    job->done.store(true, std::memory_order_release);
}

// Frames in flight may read what an install replaces: a shared scene waits for the
// device (every context's work); otherwise the caller's stream `s` waits for the
// context's earlier operations (orderBegin) and the old buffers are retired behind it.
hipError_t installBarrier(ArkDdgiCtx* ctx, hipStream_t s)
{
    if (ctx->sceneStore.use_count() > 1) return hipDeviceSynchronize();
    return orderBegin(ctx, s);
}

// The end of a refit or an install on `s`: with a shared scene the other contexts'
// next traversals do not wait for this context's streams, so the work completes here.
hipError_t installDone(ArkDdgiCtx* ctx, hipStream_t s)
{
    if (ctx->sceneStore.use_count() > 1) return hipStreamSynchronize(s);
    return hipSuccess;
}

// The light-space sun BVH follows the context's sun (called by every update and by
// set_lights / set_instances, on the stream `s` of the call): a finished rebuild for
// this context's sun is installed - stream-ordered behind the frames that may read the
// old one, and refitted forward when refits came in between - and a new one is started
// when the scene chose the light-space BVH at set_scene but holds none for this
// direction. Until it is installed the sun's shadow rays traverse the world BVHs
// (deriveSceneArgs), with the same results. sunCollect: the request streak and a
// finished rebuild; sunStartKind / sunStart: a new one.
int sunCollect(ArkDdgiCtx* ctx, hipStream_t s)
{
    SceneStore& st = *ctx->sceneStore;
    auto sameDir = [](const float* a, const float* b) { return std::memcmp(a, b, 3 * sizeof(float)) == 0; };
    if (ctx->hasSun) {
        if (st.sunReqStreak && sameDir(st.sunReqDir, ctx->sunDir)) {
            st.sunReqStreak = std::min<uint32_t>(st.sunReqStreak + 1u, 1u << 30);
        } else {
            std::memcpy(st.sunReqDir, ctx->sunDir, sizeof(st.sunReqDir));
            st.sunReqStreak = 1;
        }
    }
    if (st.sunJob && st.sunJob->done.load(std::memory_order_acquire)) {
        SunJob& j = *st.sunJob;
        if (!j.ok) {
            // remembered: not started again for this direction and scene version
            st.sunFailed = true;
            std::memcpy(st.sunFailedDir, j.dir, sizeof(j.dir));
            st.sunFailedVersion = j.version;
            st.bvhStats.sun_rebuild_failures = ++st.sunFailures;
            j.t.join();
            st.sunJob.reset();
        } else if (st.sunReqStreak >= 2 && !sameDir(j.dir, st.sunReqDir)) {
            // stale: the scene's contexts settled on another sun
            j.t.join();
            st.sunJob.reset();
        } else if (ctx->hasSun && sameDir(j.dir, ctx->sunDir)) {
            std::unique_ptr<SunJob> job = std::move(st.sunJob);
            job->t.join();
            ARK_HIP(installBarrier(ctx, s));
            ARK_HIP(retireBuffer(st, st.sunNodes, s));
            ARK_HIP(retireBuffer(st, st.sunRefitOrder, s));
            st.sunNodes = job->buf;
            job->buf = DeviceBuffer {};
            st.sunArgs.sun_nodes = st.sunNodes.as<GpuBvh8Node>();
            st.sunArgs.sun_tris = reinterpret_cast<const GpuTriangle*>(static_cast<const char*>(st.sunNodes.ptr) + job->triOffset);
            st.sunArgs.sun_root = 0;
            std::memcpy(st.sunArgs.sun_frame, job->frame, sizeof(job->frame));
            std::memcpy(st.sunFrameD, job->frameD, sizeof(job->frameD));
            std::memcpy(st.sunDirBuilt, job->dir, sizeof(job->dir));
            st.sunInflateAbs = job->inflateAbs;
            st.sunTriRecords = job->triRecords;
            st.sunLevelOffsets = job->levelOffsets;
            ARK_HIP(st.sunRefitOrder.alloc(std::max<size_t>(16, job->levelOrder.size() * 4)));
            ARK_HIP(hipMemcpy(st.sunRefitOrder.ptr, job->levelOrder.data(), job->levelOrder.size() * 4, hipMemcpyHostToDevice));
            if (st.sunRefitBoxes.bytes < job->nodes * 6 * sizeof(float)) {
                ARK_HIP(retireBuffer(st, st.sunRefitBoxes, s));
                ARK_HIP(st.sunRefitBoxes.alloc(std::max<size_t>(16, job->nodes * 6 * sizeof(float) * 5 / 4)));
            }
            st.sunBvhNodes = job->nodes;
            st.sunDepth = job->depth;
            st.bvhMaxDepth = std::max(st.bvhMaxDepth, job->depth);
            st.bvhStats.max_depth = st.bvhMaxDepth;
            st.bvhStats.sun_node_count = job->nodes;
            st.bvhStats.sun_max_depth = job->depth;
            st.bvhStats.sun_rebuilds = ++st.sunRebuilds;
            st.bvhStats.sun_build_ms = job->ms;
            st.sunRefitsSinceBuild = st.refitCount - job->refitsAt;
            st.bvhStats.sun_built_refit_version = job->refitsAt;
            markTopologyChanged(st);
            if (st.sunRefitsSinceBuild) {
                // refits came in while it was built: its records follow them (every
                // instance re-transformed, the light-space boxes refitted)
                if (const int rc = uploadRefitInstances(ctx, st, st.instHost.data(), static_cast<uint32_t>(st.instHost.size()), nullptr, s)) return rc;
                if (const int rc = enqueueRefit(ctx, st, s, frontTarget(st), st.front)) return rc;
            }
            ARK_HIP(retireBuffer(st, job->snap, s));
            ARK_HIP(installedGeometry(ctx, st, s));
            ARK_HIP(hipEventRecord(ctx->evRefit, s));
            ARK_HIP(installDone(ctx, s));
            ctx->refitPending = true;
            ++st.version;
            if (const int rc = refreshScene(ctx)) return rc;
        }
        // else: built for another context's sun; that context installs it
    }
    return ARK_DDGI_OK;
}

// The sun rebuild this context's sun asks for: kSunNone; kSunMissing when the scene holds
// no light-space BVH for it (started at once, even beside a world rebuild); kSunLoosened
// when the installed one was built for it and refits have loosened it since (a
// background rebuild like the world BVHs', one at a time with them, not with
// ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD). Only on a stable request, and not again after a
// failure for the same direction and scene version.
enum SunStart { kSunNone, kSunLoosened, kSunMissing };
SunStart sunStartKind(const ArkDdgiCtx* ctx)
{
    const SceneStore& st = *ctx->sceneStore;
    auto sameDir = [](const float* a, const float* b) { return std::memcmp(a, b, 3 * sizeof(float)) == 0; };
    if (!st.sunWanted || !ctx->hasSun || st.sunJob || st.sunReqStreak < 2 || !sameDir(st.sunReqDir, ctx->sunDir)) return kSunNone;
    if (st.sunFailed && st.sunFailedVersion == st.version && sameDir(st.sunFailedDir, ctx->sunDir)) return kSunNone;
    if (st.sunArgs.sun_root >= 0 && sameDir(ctx->sunDir, st.sunDirBuilt))
        return (st.sunRefitsSinceBuild == 0 || (ctx->desc.flags & ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD)) ? kSunNone : kSunLoosened;
    return kSunMissing;
}

// A world rebuild is wanted while refits have loosened the installed BVHs (and none
// failed, and background rebuilds are on).
bool worldStartWanted(const ArkDdgiCtx* ctx)
{
    const SceneStore& st = *ctx->sceneStore;
    return !st.worldJob && st.refitsSinceBuild != 0 && !st.worldRebuildFailed && !(ctx->desc.flags & ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD);
}

int sunStart(ArkDdgiCtx* ctx, hipStream_t s)
{
    SceneStore& st = *ctx->sceneStore;
    auto job = std::make_unique<SunJob>();
    std::memcpy(job->dir, ctx->sunDir, sizeof(job->dir));
    job->version = st.version;
    job->refitsAt = st.refitCount;
    ARK_HIP(orderBegin(ctx, s));
    ARK_HIP(snapshotRecords(st, job->snap, job->evSnap, s));
    job->t = std::thread(runSunJob, job.get(), st.device, st.triRecords, std::max(1, st.buildThreads / 2));
    st.sunJob = std::move(job);
    st.lastBackground = SceneStore::kBackgroundSun;
    return ARK_DDGI_OK;
}

// A loosened BVH's rebuild starts when no other background build runs; when both the
// world BVHs and the light-space one are loosened they take turns (under continuous
// motion each would otherwise start again the moment its last one is installed).
bool loosenedTurn(const SceneStore& st, uint8_t mine, bool otherWanted)
{
    if (st.worldJob || st.sunJob) return false;
    return !otherWanted || st.lastBackground != mine;
}

// sunCollect, then a sun rebuild to start (set_lights: the world BVHs' rebuilds are
// left to the next update or set_instances)
int sunRebuildStep(ArkDdgiCtx* ctx, hipStream_t s)
{
    if (const int rc = sunCollect(ctx, s)) return rc;
    const SunStart k = sunStartKind(ctx);
    if (k == kSunMissing || (k == kSunLoosened && loosenedTurn(*ctx->sceneStore, SceneStore::kBackgroundSun, worldStartWanted(ctx))))
        return sunStart(ctx, s);
    return ARK_DDGI_OK;
}

// The world BVHs' background rebuild after refits (the reference's full TLAS build every
// 60 frames restores tightness, GpuScene.cpp:998-1010; a refit keeps the old topology,
// whose boxes loosen as instances move): a finished rebuild is installed on `s` -
// behind the frames that may read the old BVHs, its shading records gathered into its
// record order, and refitted forward when refits came in while it was built - and,
// while refits have loosened the installed one, a new one is started (worldStart).
int worldCollect(ArkDdgiCtx* ctx, hipStream_t s)
{
    SceneStore& st = *ctx->sceneStore;
    if (st.worldJob && st.worldJob->done.load(std::memory_order_acquire)) {
        std::unique_ptr<WorldJob> job = std::move(st.worldJob);
        job->t.join();
        if (!job->ok) {
            // the refitted BVHs stay (results do not depend on the tree); no more
            // background rebuilds of this scene (a set_scene builds anew), reported in
            // the stats and last_error, the update goes on
            st.worldRebuildFailed = true;
            st.bvhStats.bvh_rebuild_failures++;
            ctx->lastError = "background BVH rebuild failed: " + job->error;
            return ARK_DDGI_OK;
        }
        ARK_HIP(installBarrier(ctx, s));
        // the shading records in the new record order (before the old ones are retired)
        DeviceBuffer tn;
        ARK_HIP(tn.alloc(std::max<size_t>(64, job->triRecords * 64)));
        ARK_HIP(launch_gather_records(tn.as<float4>(), st.triNormals.as<float4>(), job->perm.as<uint32_t>(), job->triRecords, s));
        ARK_HIP(retireBuffer(st, st.triNormals, s));
        ARK_HIP(retireBuffer(st, st.nodes, s));
        ARK_HIP(retireBuffer(st, st.refitOrder, s));
        ARK_HIP(retireBuffer(st, job->perm, s));
        ARK_HIP(retireBuffer(st, job->snap, s));
        st.triNormals = tn;
        st.nodes = job->buf;
        job->buf = DeviceBuffer {};
        st.refitOrder = job->order;
        job->order = DeviceBuffer {};
        st.levelOffsets = job->levelOffsets;
        if (st.refitBoxes.bytes < job->nodes * 6 * sizeof(float)) {
            ARK_HIP(retireBuffer(st, st.refitBoxes, s));
            ARK_HIP(st.refitBoxes.alloc(std::max<size_t>(16, job->nodes * 6 * sizeof(float) * 5 / 4)));
        }
        SceneArgs& sc = st.args;
        sc.nodes = st.nodes.as<GpuBvh8Node>();
        sc.tris = reinterpret_cast<const GpuTriangle*>(static_cast<const char*>(st.nodes.ptr) + job->triOffset);
        sc.tri_byte_offset = static_cast<uint32_t>(job->triOffset);
        sc.tri_normals = st.triNormals.as<float4>();
        sc.root_opaque = job->roots[0];
        sc.root_masked = job->roots[1];
        sc.root_blend = job->roots[2];
        sc.opaque_nodes = job->opaqueNodes;
        st.triRecords = job->triRecords;
        st.worldDepth = job->depth;
        st.bvhMaxDepth = std::max(job->depth, st.sunArgs.sun_root >= 0 ? st.sunDepth : 0u);
        st.bvhStats.node_count = job->nodes;
        st.bvhStats.max_depth = st.bvhMaxDepth;
        st.bvhStats.max_leaf_size = job->maxLeaf;
        st.bvhStats.sah_cost = job->sah;
        st.bvhStats.node_bytes = job->nodes * sizeof(GpuBvh8Node);
        st.bvhStats.triangle_bytes = job->triRecords * sizeof(GpuTriangle);
        st.bvhStats.bvh_rebuilds = ++st.worldRebuilds;
        st.bvhStats.bvh_rebuild_ms = job->ms;
        st.refitsSinceBuild = st.refitCount - job->refitsAt; // refits since its snapshot
        st.bvhStats.bvh_built_refit_version = job->refitsAt;
        markTopologyChanged(st);
        if (st.refitsSinceBuild) {
            if (const int rc = uploadRefitInstances(ctx, st, st.instHost.data(), static_cast<uint32_t>(st.instHost.size()), nullptr, s)) return rc;
            if (const int rc = enqueueRefit(ctx, st, s, frontTarget(st), st.front)) return rc;
        }
        ARK_HIP(installedGeometry(ctx, st, s));
        ARK_HIP(hipEventRecord(ctx->evRefit, s));
        ARK_HIP(installDone(ctx, s));
        ctx->refitPending = true;
        ++st.version;
        if (const int rc = refreshScene(ctx)) return rc;
    }
    return ARK_DDGI_OK;
}

int worldStart(ArkDdgiCtx* ctx, hipStream_t s)
{
    SceneStore& st = *ctx->sceneStore;
    auto job = std::make_unique<WorldJob>();
    job->version = st.version;
    job->refitsAt = st.refitCount;
    job->snapRecords = st.triRecords;
    job->classOf.resize(st.instHost.size());
    for (size_t i = 0; i < st.instHost.size(); ++i) {
        const uint32_t m = st.instHost[i].hit_mask;
        job->classOf[i] = (m & ARK_RT_HIT_MASK_OPAQUE) ? 0 : (m & ARK_RT_HIT_MASK_MASKED) ? 1 : 2;
    }
    ARK_HIP(orderBegin(ctx, s));
    ARK_HIP(snapshotRecords(st, job->snap, job->evSnap, s));
    // half the host threads: the other half stays with the frames being enqueued meanwhile
    job->t = std::thread(runWorldJob, job.get(), st.device, std::max(1, st.buildThreads / 2));
    st.worldJob = std::move(job);
    st.lastBackground = SceneStore::kBackgroundWorld;
    st.refitsSinceBuild = 0;
    return ARK_DDGI_OK;
}

// Everything an operation on `s` does to the scene first: buffers retired by earlier
// installs freed, finished rebuilds installed, new ones started.
int sceneMaintenance(ArkDdgiCtx* ctx, hipStream_t s)
{
    collectRetired(*ctx->sceneStore);
    if (const int rc = worldCollect(ctx, s)) return rc;
    if (const int rc = sunCollect(ctx, s)) return rc;
    const SunStart k = sunStartKind(ctx);
    if (k == kSunMissing) {
        if (const int rc = sunStart(ctx, s)) return rc;
    }
    const bool world = worldStartWanted(ctx), sun = k == kSunLoosened;
    if (world && loosenedTurn(*ctx->sceneStore, SceneStore::kBackgroundWorld, sun)) return worldStart(ctx, s);
    if (sun && loosenedTurn(*ctx->sceneStore, SceneStore::kBackgroundSun, world)) return sunStart(ctx, s);
    return ARK_DDGI_OK;
}

// Makes `st` the context's scene with the scene's lights: the per-context work sets
// follow its light count and BVH depth.
int adoptScene(ArkDdgiCtx* ctx, std::shared_ptr<SceneStore> st)
{
    ctx->hasSun = st->hasSunScene;
    for (int k = 0; k < 3; ++k) {
        ctx->sunColor[k] = st->sunScene.color[k];
        ctx->sunDir[k] = st->sunScene.world_space_direction[k];
    }
    ctx->spotHost = st->spotsScene;
    ctx->sceneStore = std::move(st);
    if (!ctx->lights.ptr) ARK_HIP(ctx->lights.alloc((kMaxLights - 1) * sizeof(GpuSpotLight)));
    if (!ctx->spotHost.empty()) ARK_HIP(hipMemcpy(ctx->lights.ptr, ctx->spotHost.data(), ctx->spotHost.size() * sizeof(GpuSpotLight), hipMemcpyHostToDevice));
    ctx->lightsDirty = false;
    deriveSceneArgs(ctx);
    int rc;
    if ((rc = ensureShadeWork(ctx)) != 0) return rc;
    if ((rc = ensureSpill(ctx)) != 0) return rc;
    ctx->hasScene = true;
    return ARK_DDGI_OK;
}

} // namespace

extern "C" {

int32_t ark_ddgi_abi_version(void) { return ARK_DDGI_ABI_VERSION; }

int ark_ddgi_create(const ArkDdgiDesc* desc, ArkDdgiCtx** outCtx)
{
    if (!desc || !outCtx || desc->struct_size != sizeof(ArkDdgiDesc)) return ARK_DDGI_E_INVALID_ARGUMENT;
    *outCtx = nullptr;
    if (desc->grid_dims[0] <= 0 || desc->grid_dims[1] <= 0 || desc->grid_dims[2] <= 0) return ARK_DDGI_E_NO_PROBE_GRID;
    auto* ctx = new ArkDdgiCtx();
    ctx->desc = *desc;
    ctx->X = desc->grid_dims[0];
    ctx->Y = desc->grid_dims[1];
    ctx->Z = desc->grid_dims[2];
    ctx->N = ctx->X * ctx->Y * ctx->Z;
    ctx->Rmax = desc->max_rays_per_probe > 0 ? desc->max_rays_per_probe : ARK_DDGI_MAX_RAYS_PER_PROBE;
    ctx->Kmax = desc->max_probe_updates > 0 ? desc->max_probe_updates : ARK_DDGI_REFERENCE_MAX_PROBE_UPDATES;
    const int shards = desc->shard_count > 0 ? desc->shard_count : 1;
    if (ctx->Rmax > ARK_DDGI_MAX_RAYS_PER_PROBE || ctx->Z % shards != 0 || desc->shard_rank < 0 || desc->shard_rank >= shards ||
        desc->sun_bvh < ARK_DDGI_SUN_BVH_AUTO || desc->sun_bvh > ARK_DDGI_SUN_BVH_LIGHT_SPACE || (desc->flags & ~(ARK_DDGI_FLAG_SERIAL_FRAMES | ARK_DDGI_FLAG_NO_BACKGROUND_REBUILD)) ||
        desc->build_threads < 0) {
        delete ctx;
        return ARK_DDGI_E_INVALID_ARGUMENT;
    }
    ctx->desc.shard_count = shards;
    ctx->slabZ0 = desc->shard_rank * (ctx->Z / shards);
    ctx->slabZ1 = ctx->slabZ0 + ctx->Z / shards;
    const int si = ARK_DDGI_IRRADIANCE_RES + 2 * ARK_DDGI_ATLAS_PADDING;
    const int sv = ARK_DDGI_VISIBILITY_RES + 2 * ARK_DDGI_ATLAS_PADDING;
    ctx->Wi = ctx->X * si * ctx->Y;
    ctx->Hi = ctx->Z * si;
    ctx->Wv = ctx->X * sv * ctx->Y;
    ctx->Hv = ctx->Z * sv;
    auto bad = [&](hipError_t e, const char* what) {
        std::fprintf(stderr, "ark_ddgi_create: %s: %s\n", what, hipGetErrorString(e));
        delete ctx;
        return ARK_DDGI_E_DEVICE;
    };
    hipError_t e = hipSetDevice(desc->device);
    if (e != hipSuccess) return bad(e, "hipSetDevice");
    ctx->device = desc->device;
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, desc->device);
    if (e != hipSuccess) return bad(e, "hipGetDeviceProperties");
    ctx->cuCount = prop.multiProcessorCount;
    if ((e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    if ((e = hipEventCreateWithFlags(&ctx->evOrder, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    // the desc's options (ArkDdgiDesc.sun_bvh / flags); the traversal's refill and grab
    // sizes are the constants kRefillMin / kSunRefillMin / kGrabChunk
    ctx->pipelining = (desc->flags & ARK_DDGI_FLAG_SERIAL_FRAMES) == 0;
    ctx->sunBvh = desc->sun_bvh == ARK_DDGI_SUN_BVH_WORLD ? 0 : desc->sun_bvh == ARK_DDGI_SUN_BVH_LIGHT_SPACE ? 1 : -1;
    // a counter-collecting profiler (rocprofv3 --pmc) runs one kernel at a time across
    // queues: a polling wait could then hold the GPU while the kernel it waits for queues
    // behind it: it would give up after its bound and fail closed (checkSequencing),
    // dropping frames; such a context starts with events instead (the profiler's own
    // environment, not a tuning knob; ark_ddgi_set_sequencing overrides it)
    if (const char* pc = std::getenv("ROCPROF_COUNTER_COLLECTION"))
        if (*pc && std::strcmp(pc, "0") != 0 && std::strcmp(pc, "false") != 0) ctx->seqSync = false;
    if ((e = hipStreamCreateWithFlags(&ctx->traceStream, hipStreamNonBlocking)) != hipSuccess) return bad(e, "hipStreamCreate");
    // stream-order events of the frames in flight
    const unsigned syncFlags = hipEventDisableTiming;
    if ((e = hipEventCreateWithFlags(&ctx->evTraced, syncFlags)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->evExchangeSrc, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->evExchangeDone, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->evRefit, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    if ((e = hipEventCreateWithFlags(&ctx->evInstalled, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    for (auto& ev : ctx->evFree)
        if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return bad(e, "hipEventCreate");
    {
        // the refit stream at the device's highest priority: its per-level launches are
        // dispatched ahead of the frame in flight's work when both wait for a CU
        int lo = 0, hi = 0;
        if ((e = hipDeviceGetStreamPriorityRange(&lo, &hi)) != hipSuccess) return bad(e, "hipDeviceGetStreamPriorityRange");
        if ((e = hipStreamCreateWithPriority(&ctx->refitStream, hipStreamNonBlocking, hi)) != hipSuccess) return bad(e, "hipStreamCreateWithPriority");
    }
    for (auto& ev : ctx->evFrameDone)
        if ((e = hipEventCreateWithFlags(&ev, syncFlags)) != hipSuccess) return bad(e, "hipEventCreate");
    for (auto& ev : ctx->ev)
        if ((e = hipEventCreate(&ev)) != hipSuccess) return bad(e, "hipEventCreate");
    const size_t K = static_cast<size_t>(ctx->Kmax), R = static_cast<size_t>(ctx->Rmax);
    if ((e = ctx->irr.alloc(static_cast<size_t>(ctx->Wi) * ctx->Hi * 8)) != hipSuccess) return bad(e, "alloc irradiance");
    if ((e = ctx->vis.alloc(static_cast<size_t>(ctx->Wv) * ctx->Hv * 4)) != hipSuccess) return bad(e, "alloc visibility");
    if ((e = ctx->offsets.alloc(static_cast<size_t>(ctx->N) * 16)) != hipSuccess) return bad(e, "alloc offsets");
    if ((e = ctx->slots.alloc(2 * K * sizeof(GpuProbeSlot))) != hipSuccess) return bad(e, "alloc slots");
    if ((e = ctx->slotOrder.alloc(2 * K * 4)) != hipSuccess) return bad(e, "alloc slot order");
    if ((e = ctx->fib.alloc(2 * R * 16)) != hipSuccess) return bad(e, "alloc fib");
    if ((e = ctx->order.alloc(R * 4)) != hipSuccess) return bad(e, "alloc order");
    if ((e = ctx->fibOrder.alloc(2 * R * 16)) != hipSuccess) return bad(e, "alloc fib order");
    if ((e = ctx->hits.alloc(2 * K * R * sizeof(GpuHit))) != hipSuccess) return bad(e, "alloc hits");
    if ((e = ctx->surfels.alloc(K * R * 8)) != hipSuccess) return bad(e, "alloc surfels");
    if ((e = ctx->rayCounter.alloc(2 * kRayCounterWords * 4)) != hipSuccess) return bad(e, "alloc counter");
    if ((e = ctx->counters.alloc(8 * sizeof(unsigned long long))) != hipSuccess) return bad(e, "alloc counters");
    if ((e = ctx->seqWords.alloc(128 * 4)) != hipSuccess) return bad(e, "alloc sequence words");
    if ((e = hipMemset(ctx->seqWords.ptr, 0, ctx->seqWords.bytes)) != hipSuccess) return bad(e, "clear sequence words");
    {
        // k_seq_wait's bound: 10 s of the device wall clock (kHz attribute)
        int rateKhz = 0;
        if (hipDeviceGetAttribute(&rateKhz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || rateKhz <= 0) rateKhz = 100000;
        ctx->wallClockKhz = static_cast<uint64_t>(rateKhz);
        ctx->seqTimeoutTicks = ctx->wallClockKhz * ctx->seqTimeoutMs;
    }
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&ctx->hostAbort), 64, hipHostMallocCoherent | hipHostMallocMapped)) != hipSuccess)
        return bad(e, "hipHostMalloc sequencing flag");
    *reinterpret_cast<volatile uint32_t*>(ctx->hostAbort) = 0u;
    if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->hostAbortDev), ctx->hostAbort, 0)) != hipSuccess)
        return bad(e, "hipHostGetDevicePointer sequencing flag");
    // persistent grids: as many workgroups as are co-resident
    int occT = 0, occS = 0, occW = 0;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occT, kernel_trace_ptr(false), kTraceBlock, 0)) != hipSuccess) return bad(e, "occupancy trace");
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occS, kernel_shade_ptr(false), kShadeBlock, 0)) != hipSuccess) return bad(e, "occupancy shade");
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occW, kernel_trace_shadow_ptr(false), kTraceBlock, 0)) != hipSuccess) return bad(e, "occupancy shadow");
    ctx->traceBlocks = static_cast<uint32_t>(std::max(1, occT) * ctx->cuCount);
    // a pipelined update's traversal shares the GPU with the previous frame's shadow
    // rays, shading and probe update: below kPipeHalfRays rays, 3 workgroups per CU
    // (half the occupancy) leave them room (tools/shard_proxy.py,
    // tools/window_proxy.py, profiles/r02_m13-15: Z-slab steps P = 8 0.705 -> 0.640 ms,
    // P = 4 1.21 -> 1.11, P = 2 2.22 -> 2.10; K = 4096 windows 0.72 -> 0.65, K = 2048
    // 0.43 unchanged; 2 per CU: P = 8 0.72, 4 per CU: 0.69). The whole C4 grid (8.4 M
    // rays) keeps the full grid: 4.059 vs 4.067 ms per step at 3 (profiles/r02_m17_ab).
    ctx->pipeTraceBlocks = static_cast<uint32_t>(std::min(kPipeTracePerCu, std::max(1, occT)) * ctx->cuCount);
    ctx->shadeBlocks = static_cast<uint32_t>(std::max(1, occS) * ctx->cuCount);
    ctx->shadowBlocks = static_cast<uint32_t>(std::max(1, occW) * ctx->cuCount);
    ctx->shadowBlocksPerCu = static_cast<uint32_t>(std::max(1, occW));
    if (clearHistory(ctx) != ARK_DDGI_OK) {
        std::fprintf(stderr, "ark_ddgi_create: %s\n", ctx->lastError.c_str());
        delete ctx;
        return ARK_DDGI_E_DEVICE;
    }
    *outCtx = ctx;
    return ARK_DDGI_OK;
}

void ark_ddgi_destroy(ArkDdgiCtx* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    for (DeviceBuffer* b : { &ctx->irr, &ctx->vis, &ctx->offsets, &ctx->slots, &ctx->slotOrder, &ctx->fib, &ctx->fibOrder, &ctx->order, &ctx->hits, &ctx->surfels, &ctx->spill, &ctx->rayCounter, &ctx->seqWords, &ctx->shadeWork, &ctx->reflWork,
                             &ctx->raySteps, &ctx->counters, &ctx->lights, &ctx->bakeTri, &ctx->bakeBary, &ctx->bakeOut, &ctx->bakePixels, &ctx->bakeCounters })
        b->release();
    ctx->sceneStore.reset();
    for (auto& ev : ctx->ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->evOrder) (void)hipEventDestroy(ctx->evOrder);
    if (ctx->evTraced) (void)hipEventDestroy(ctx->evTraced);
    if (ctx->evExchangeSrc) (void)hipEventDestroy(ctx->evExchangeSrc);
    if (ctx->evExchangeDone) (void)hipEventDestroy(ctx->evExchangeDone);
    if (ctx->evRefit) (void)hipEventDestroy(ctx->evRefit);
    if (ctx->evInstalled) (void)hipEventDestroy(ctx->evInstalled);
    for (auto& ev : ctx->evFree)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->refitStream) (void)hipStreamDestroy(ctx->refitStream);
    for (auto& ev : ctx->evFrameDone)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->traceStream) (void)hipStreamDestroy(ctx->traceStream);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->hostAbort) (void)hipHostFree(ctx->hostAbort);
    delete ctx;
}

const char* ark_ddgi_last_error(const ArkDdgiCtx* ctx) { return ctx ? ctx->lastError.c_str() : "null context"; }

static int checkBvh8(ArkDdgiCtx* ctx, const std::vector<GpuBvh8Node>& allNodes, const std::vector<GpuTriangle>& allTris, const int32_t* roots, int nRoots)
{
    std::string why;
    if (!checkBvh8Structure(allNodes, allTris, roots, nRoots, why)) return ctx->fail(ARK_DDGI_E_DEVICE, "%s", why.c_str());
    return ARK_DDGI_OK;
}

int ark_ddgi_set_scene(ArkDdgiCtx* ctx, const ArkDdgiScene* s)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->pipeReady = false; // the next update's traversal waits for this
    if (!s || s->struct_size != sizeof(ArkDdgiScene)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkDdgiScene");
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    // the previous scene goes first (its memory is reused), unless another context
    // shares it; a failure below leaves the context without a scene
    ctx->hasScene = false;
    ctx->sceneStore.reset();
    auto st = std::make_shared<SceneStore>();
    st->device = ctx->device;
    const auto t0 = std::chrono::steady_clock::now();
    // validate
    for (uint32_t i = 0; i < s->instance_count; ++i) {
        const ArkRTInstance& inst = s->instances[i];
        if (inst.rt_mesh_index >= s->mesh_count) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "instance %u: rt_mesh_index out of range", i);
        const ArkRTTriangleMesh& m = s->meshes[inst.rt_mesh_index];
        if (m.material_index < 0 || static_cast<uint32_t>(m.material_index) >= s->material_count)
            return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "mesh %u: material_index out of range", inst.rt_mesh_index);
        if (static_cast<uint64_t>(m.first_index) + 3ull * inst.triangle_count > s->index_count)
            return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "instance %u: indices out of range", i);
    }
    if (s->spot_light_count > ARK_DDGI_MAX_SPOT_LIGHTS || (s->spot_light_count && !s->spot_lights))
        return ctx->fail(ARK_DDGI_E_UNSUPPORTED, "at most %d spot lights (GpuScene.cpp:430)", ARK_DDGI_MAX_SPOT_LIGHTS);
    // World-space triangles per hit-mask class (GpuScene.cpp:883-929: one TLAS
    // instance per mesh segment; flattened here into one BVH per class).
    std::vector<BuildTriangle> cls[3];
    std::vector<GpuInstance> ginst(s->instance_count);
    for (uint32_t ii = 0; ii < s->instance_count; ++ii) {
        const ArkRTInstance& inst = s->instances[ii];
        const ArkRTTriangleMesh& m = s->meshes[inst.rt_mesh_index];
        const float* M = inst.object_to_world;
        const float det = M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) + M[2] * (M[4] * M[9] - M[5] * M[8]);
        GpuInstance& g = ginst[ii];
        std::memset(&g, 0, sizeof(g));
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) g.normal_matrix[r * 4 + c] = M[r * 4 + c];
        g.rt_mesh_index = static_cast<int32_t>(inst.rt_mesh_index);
        g.flip_facing = det < 0.0f ? 1 : 0;
        g.hit_mask = static_cast<int32_t>(inst.hit_mask);
        g.material_index = m.material_index;
        const int c = (inst.hit_mask & ARK_RT_HIT_MASK_OPAQUE) ? 0 : (inst.hit_mask & ARK_RT_HIT_MASK_MASKED) ? 1 : 2;
        for (uint32_t p = 0; p < inst.triangle_count; ++p) {
            BuildTriangle t;
            float* w[3] = { t.v0, t.v1, t.v2 };
            for (int k = 0; k < 3; ++k) {
                const uint32_t idx = s->indices[static_cast<size_t>(m.first_index) + 3u * p + k];
                const uint64_t vi = static_cast<uint64_t>(m.first_vertex) + idx;
                if (vi >= s->vertex_count) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "instance %u prim %u: vertex out of range", ii, p);
                const float* P = &s->positions[vi * 3];
                w[k][0] = M[0] * P[0] + M[1] * P[1] + M[2] * P[2] + M[3];
                w[k][1] = M[4] * P[0] + M[5] * P[1] + M[6] * P[2] + M[7];
                w[k][2] = M[8] * P[0] + M[9] * P[1] + M[10] * P[2] + M[11];
            }
            t.instance = ii;
            t.primitive = p;
            t.flip_facing = static_cast<uint32_t>(g.flip_facing);
            cls[c].push_back(t);
        }
    }
    BvhBuildOptions opt;
    opt.max_leaf_size = kBvh8MaxLeafSize;
    {
        float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
        for (int c = 0; c < 3; ++c)
            for (const BuildTriangle& t : cls[c])
                for (const float* v : { t.v0, t.v1, t.v2 })
                    for (int a = 0; a < 3; ++a) {
                        lo[a] = std::min(lo[a], v[a]);
                        hi[a] = std::max(hi[a], v[a]);
                    }
        opt.inflate_abs = bvh8_inflation_box(lo, hi); // one inflation for all classes (shadow rays test all)
    }
    // host threads for the build (ArkDdgiDesc.build_threads; 0: the box's CPU share per
    // GPU, 16 cores)
    opt.threads = ctx->desc.build_threads > 0 ? ctx->desc.build_threads : 16;
    // BVH2 -> BVH8 child selection: SAH-optimal (Ylitie et al. 2017 DP) with the default
    // node / triangle costs (a lower triangle cost and the greedy collapse measured no
    // better)
    Bvh8CollapseOptions copt;
    copt.threads = opt.threads;
    // the sun's light-space BVH input, before the class builds free their triangles; the
    // build itself on its own thread beside the class builds (each build's top levels
    // leave cores idle: C4 setup 13.5 -> s)
    const bool sunBvh = s->has_directional_light && ctx->sunBvh != 0;
    SunBvhInput sunIn;
    Bvh8BuildResult r; // the sun's
    bool sunBuilt = false, sunOk = true;
    float sunBuildMs = 0.0f;
    struct Joiner {
        std::thread t;
        ~Joiner()
        {
            if (t.joinable()) t.join();
        }
    } sunThread;
    if (sunBvh) {
        const auto ts0 = std::chrono::steady_clock::now();
        sun_frame(s->directional_light.world_space_direction, sunIn.frame);
        for (int c = 0; c < 3; ++c) sun_add_triangles(sunIn, cls[c], opt.threads);
        sunBuilt = !sunIn.tris.empty();
        if (sunBuilt)
            sunThread.t = std::thread([&sunIn, &opt, &copt, &r, &sunOk, &sunBuildMs, ts0] {
                sunOk = build_sun_bvh(sunIn, opt, copt, r);
                sunBuildMs = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - ts0).count();
            });
    }
    std::vector<GpuBvh8Node> allNodes;
    std::vector<GpuTriangle> allTris;
    int32_t roots[3] = { -1, -1, -1 };
    uint32_t opaqueNodes = 0;
    uint32_t maxDepth = 0, maxLeaf = 0;
    uint64_t triangles = 0;
    float sah = 0.0f;
    for (int c = 0; c < 3; ++c) {
        if (cls[c].empty()) continue;
        BvhBuildResult r2 = build_bvh(cls[c], opt, 0u, 0u);
        std::vector<BuildTriangle>().swap(cls[c]);
        if (r2.max_leaf > static_cast<uint32_t>(kBvh8MaxLeafSize)) return ctx->fail(ARK_DDGI_E_DEVICE, "BVH2 leaf of %u triangles", r2.max_leaf);
        if (c == 0) sah = r2.sah_cost;
        maxLeaf = std::max(maxLeaf, r2.max_leaf);
        Bvh8BuildResult r = collapse_bvh8(r2, static_cast<uint32_t>(allNodes.size()), static_cast<uint32_t>(allTris.size()), copt);
        roots[c] = static_cast<int32_t>(allNodes.size());
        if (c == 0) opaqueNodes = static_cast<uint32_t>(r.nodes.size());
        maxDepth = std::max(maxDepth, r.max_depth);
        triangles += r.triangles;
        allNodes.insert(allNodes.end(), r.nodes.begin(), r.nodes.end());
        allTris.insert(allTris.end(), r.tris.begin(), r.tris.end());
    }
    if (allNodes.size() >= (1ull << 31) || allTris.size() >= (1ull << 31)) return ctx->fail(ARK_DDGI_E_UNSUPPORTED, "scene too large for 31-bit BVH indices");
    if (const int rc = checkBvh8(ctx, allNodes, allTris, roots, 3)) return rc;
    // textures: decoded to float4 texels (sRGB EOTF per texel), + trailing 1x1 white
    std::vector<GpuTextureInfo> infos;
    std::vector<float> texels;
    for (uint32_t i = 0; i <= s->texture_count; ++i) {
        GpuTextureInfo ti {};
        ti.texel_offset = texels.size() / 4;
        if (i == s->texture_count) {
            ti.width = ti.height = 1;
            ti.wrap = ARK_WRAP_REPEAT;
            texels.insert(texels.end(), { 1.0f, 1.0f, 1.0f, 1.0f });
        } else {
            const ArkTexture& t = s->textures[i];
            if (t.width <= 0 || t.height <= 0 || !t.data) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "texture %u invalid", i);
            ti.width = t.width;
            ti.height = t.height;
            // per-axis wrap, s in bits 0-3 and t in 4-7 (ARK_WRAP_AXES)
            const int ws = (t.wrap & ARK_WRAP_PER_AXIS) ? (t.wrap & 0xf) : t.wrap, wt = (t.wrap & ARK_WRAP_PER_AXIS) ? ((t.wrap >> 4) & 0xf) : t.wrap;
            if (ws < ARK_WRAP_REPEAT || ws > ARK_WRAP_MIRRORED_REPEAT || wt < ARK_WRAP_REPEAT || wt > ARK_WRAP_MIRRORED_REPEAT ||
                ((t.wrap & ARK_WRAP_PER_AXIS) && (t.wrap & ~0x1ff)))
                return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "texture %u: unknown wrap mode 0x%x", i, t.wrap);
            ti.wrap = ws | (wt << 4);
            const size_t n = static_cast<size_t>(t.width) * t.height;
            for (size_t p = 0; p < n; ++p)
                for (int c = 0; c < 4; ++c) {
                    float v = 0.0f;
                    switch (t.format) {
                    case ARK_TEX_RGBA8_UNORM: v = static_cast<float>(static_cast<const uint8_t*>(t.data)[p * 4 + c]) / 255.0f; break;
                    case ARK_TEX_RGBA8_SRGB:
                        v = static_cast<float>(static_cast<const uint8_t*>(t.data)[p * 4 + c]) / 255.0f;
                        if (c < 3) v = srgbToLinear(v);
                        break;
                    case ARK_TEX_R32F: v = c == 0 ? static_cast<const float*>(t.data)[p] : (c == 3 ? 1.0f : 0.0f); break;
                    case ARK_TEX_RGBA32F: v = static_cast<const float*>(t.data)[p * 4 + c]; break;
                    default: return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "texture %u: unknown format", i);
                    }
                    texels.push_back(v);
                }
        }
        infos.push_back(ti);
    }
    std::vector<GpuSpotLight> gspots(s->spot_light_count);
    for (uint32_t i = 0; i < s->spot_light_count; ++i) gspots[i] = gpuSpotLight(s->spot_lights[i]);
    int rc;
    // nodes and triangles in ONE allocation (triangles after the nodes, 256-B aligned):
    // the traversal addresses both through one buffer resource with a per-lane
    // byte offset (32 bits: the pair must stay below 4 GiB)
    const size_t nodeBytes = allNodes.size() * sizeof(GpuBvh8Node);
    const size_t triOffset = (nodeBytes + 255) & ~static_cast<size_t>(255);
    const size_t triBytes = (allTris.size() + 1) * sizeof(GpuTriangle); // + padding record
    if (triOffset + triBytes >= (1ull << 32)) return ctx->fail(ARK_DDGI_E_UNSUPPORTED, "BVH nodes + triangles exceed 4 GiB");
    ARK_HIP(st->nodes.alloc(triOffset + triBytes));
    ARK_HIP(hipMemcpy(st->nodes.ptr, allNodes.data(), nodeBytes, hipMemcpyHostToDevice));
    allTris.push_back(GpuTriangle {}); // padding: a five-load fetch of the last triangle stays in bounds (ARK_FETCH5)
    ARK_HIP(hipMemcpy(static_cast<char*>(st->nodes.ptr) + triOffset, allTris.data(), allTris.size() * sizeof(GpuTriangle), hipMemcpyHostToDevice));
    allTris.pop_back();
    uint64_t sunNodeCount = 0;
    uint32_t sunMaxDepth = 0;
    size_t sunTriOffset = 0;
    if (sunThread.t.joinable()) sunThread.t.join();
    const auto ts0 = std::chrono::steady_clock::now();
    if (sunBuilt) {
        if (!sunOk) return ctx->fail(ARK_DDGI_E_DEVICE, "sun BVH2 leaf over %d triangles", kBvh8MaxLeafSize);
        const int32_t sroot = 0;
        if (const int rc2 = checkBvh8(ctx, r.nodes, r.tris, &sroot, 1)) return rc2;
        // by cost unless forced: sample sun shadow rays through both structures on the host
        const float* sd = s->directional_light.world_space_direction;
        const float dd = sd[0] * sd[0] + sd[1] * sd[1] + sd[2] * sd[2];
        const float isc = 1.0f / std::sqrt(dd);
        const float L[3] = { -(sd[0] * isc), -(sd[1] * isc), -(sd[2] * isc) };
        std::vector<float> origins;
        sun_sample_origins(allTris, L, 4096u, origins);
        st->sunCostWorld = static_cast<float>(sun_shadow_cost(allNodes, allTris, roots, 3, nullptr, L, origins));
        st->sunCostLight = static_cast<float>(sun_shadow_cost(r.nodes, r.tris, &sroot, 1, sunIn.frame, L, origins));
    }
    const uint32_t worldDepth = maxDepth;
    if (sunBuilt && (ctx->sunBvh == 1 || sun_bvh_pays(st->sunCostWorld, st->sunCostLight))) {
        const size_t nb = r.nodes.size() * sizeof(GpuBvh8Node);
        sunTriOffset = (nb + 255) & ~static_cast<size_t>(255);
        // what its refits need (enqueueRefit): the level order, the build's inflation and
        // frame, the record count (padding excluded)
        {
            const int32_t sroot = 0;
            std::vector<uint32_t> order;
            if (!bvhLevelOrder(r.nodes.data(), r.nodes.size(), &sroot, 1, order, st->sunLevelOffsets)) return ctx->fail(ARK_DDGI_E_DEVICE, "sun BVH: a node outside it");
            if ((rc = upload(ctx, st->sunRefitOrder, order.data(), order.size())) != 0) return rc;
            ARK_HIP(st->sunRefitBoxes.alloc(std::max<size_t>(16, r.nodes.size() * 6 * sizeof(float) * 5 / 4)));
            st->sunTriRecords = r.tris.size();
            st->sunInflateAbs = sunIn.inflateAbs;
            for (int i = 0; i < 3; ++i)
                for (int k = 0; k < 3; ++k) st->sunFrameD[i * 3 + k] = sunIn.frame[i][k];
            st->sunDepth = r.max_depth;
        }
        r.tris.push_back(GpuTriangle {}); // padding record (five-load fetch)
        ARK_HIP(st->sunNodes.alloc(sunTriOffset + r.tris.size() * sizeof(GpuTriangle)));
        ARK_HIP(hipMemcpy(st->sunNodes.ptr, r.nodes.data(), nb, hipMemcpyHostToDevice));
        ARK_HIP(hipMemcpy(static_cast<char*>(st->sunNodes.ptr) + sunTriOffset, r.tris.data(), r.tris.size() * sizeof(GpuTriangle), hipMemcpyHostToDevice));
        sunNodeCount = r.nodes.size();
        // the sun's traversal pushes onto the same spill area (its depth counts)
        maxDepth = std::max(maxDepth, r.max_depth);
        sunMaxDepth = r.max_depth;
    }
    sunBuildMs += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - ts0).count();
    std::vector<GpuTriangle>().swap(sunIn.world);
    if ((rc = upload(ctx, st->indices, s->indices, s->index_count)) != 0) return rc;
    if ((rc = upload(ctx, st->vertices, reinterpret_cast<const float*>(s->vertices), s->vertex_count * 9)) != 0) return rc;
    if ((rc = upload(ctx, st->positions, s->positions, s->vertex_count * 3)) != 0) return rc;
    st->instHost.assign(s->instances, s->instances + s->instance_count);
    // the transforms both geometry copies hold (the back one is made at the first refit)
    st->xf[0].resize(s->instance_count);
    for (uint32_t ii = 0; ii < s->instance_count; ++ii) std::memcpy(st->xf[0][ii].data(), s->instances[ii].object_to_world, sizeof(float) * 12);
    st->xf[1] = st->xf[2] = st->xf[0];
    st->spare[0].slot = 1;
    st->spare[1].slot = 2;
    st->meshHost.assign(s->meshes, s->meshes + s->mesh_count);
    // every instance's object-space box (refitInflations)
    st->instObjBox.assign(s->instance_count, { INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY });
    for (uint32_t ii = 0; ii < s->instance_count; ++ii) {
        const ArkRTInstance& in = s->instances[ii];
        const ArkRTTriangleMesh& mesh = s->meshes[in.rt_mesh_index];
        std::array<float, 6>& box = st->instObjBox[ii];
        std::mutex mu;
        parallelFor(static_cast<size_t>(in.triangle_count) * 3u, opt.threads, [&](size_t b, size_t e) {
            float lo[3] = { INFINITY, INFINITY, INFINITY }, hi[3] = { -INFINITY, -INFINITY, -INFINITY };
            for (size_t k = b; k < e; ++k) {
                const float* P = s->positions + (static_cast<int64_t>(mesh.first_vertex) + s->indices[static_cast<size_t>(mesh.first_index) + k]) * 3;
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::min(lo[a], P[a]);
                    hi[a] = std::max(hi[a], P[a]);
                }
            }
            std::lock_guard<std::mutex> g(mu);
            for (int a = 0; a < 3; ++a) {
                box[a] = std::min(box[a], lo[a]);
                box[3 + a] = std::max(box[3 + a], hi[a]);
            }
        });
    }
    if ((rc = upload(ctx, st->meshes, s->meshes, s->mesh_count)) != 0) return rc;
    if ((rc = upload(ctx, st->materials, s->materials, s->material_count)) != 0) return rc;
    if ((rc = upload(ctx, st->instances, ginst.data(), ginst.size())) != 0) return rc;
    if ((rc = upload(ctx, st->texInfos, infos.data(), infos.size())) != 0) return rc;
    if ((rc = upload(ctx, st->texels, texels.data(), texels.size())) != 0) return rc;
    {
        // per-triangle shading records (GpuTriangle order, 64 B): the three vertex
        // normals, the instance and the three UVs, copied from the vertex pool, so
        // the shading and shadow-ray kernels reach a hit's surface in one fetch
        // instead of instance -> mesh -> indices -> vertices
        std::vector<float> tn(allTris.size() * 16, 0.0f);
        parallelFor(allTris.size(), opt.threads, [&](size_t b, size_t e) {
            for (size_t t = b; t < e; ++t) {
                if (isHoleTriangle(allTris[t])) continue; // never hit: no record
                uint32_t inst, prim;
                std::memcpy(&inst, &allTris[t].t2[1], 4);
                std::memcpy(&prim, &allTris[t].t2[2], 4);
                const ArkRTTriangleMesh& mesh = s->meshes[s->instances[inst].rt_mesh_index];
                float* o = tn.data() + t * 16;
                for (int q = 0; q < 3; ++q) {
                    const uint32_t idx = s->indices[static_cast<size_t>(mesh.first_index) + 3u * prim + q];
                    const float* v = reinterpret_cast<const float*>(s->vertices) + (static_cast<size_t>(mesh.first_vertex) + idx) * 9;
                    for (int k = 0; k < 3; ++k) o[q * 3 + k] = v[2 + k];
                    o[10 + 2 * q] = v[0];
                    o[11 + 2 * q] = v[1];
                }
                std::memcpy(o + 9, &inst, 4);
            }
        });
        if (tn.empty()) tn.assign(16, 0.0f);
        if ((rc = upload(ctx, st->triNormals, tn.data(), tn.size())) != 0) return rc;
    }
    SceneArgs& sc = st->args;
    sc.nodes = st->nodes.as<GpuBvh8Node>();
    sc.tris = reinterpret_cast<const GpuTriangle*>(static_cast<const char*>(st->nodes.ptr) + triOffset);
    sc.tri_byte_offset = static_cast<uint32_t>(triOffset);
    sc.tri_normals = st->triNormals.as<float4>();
    sc.root_opaque = roots[0];
    sc.root_masked = roots[1];
    sc.root_blend = roots[2];
    sc.opaque_nodes = opaqueNodes;
    sc.texture_count = static_cast<int32_t>(s->texture_count);
    sc.indices = st->indices.as<uint32_t>();
    sc.vertices = st->vertices.as<float>();
    sc.meshes = st->meshes.as<ArkRTTriangleMesh>();
    sc.materials = st->materials.as<ArkShaderMaterial>();
    sc.instances = st->instances.as<GpuInstance>();
    sc.tex_infos = st->texInfos.as<GpuTextureInfo>();
    sc.texels = st->texels.as<float4>();
    sc.white_texture = static_cast<int32_t>(s->texture_count);
    sc.env_texture = (s->environment_texture >= 0 && static_cast<uint32_t>(s->environment_texture) < s->texture_count) ? s->environment_texture : sc.white_texture;
    // lights: the scene's are each context's until ark_ddgi_set_lights (deriveSceneArgs)
    st->hasSunScene = s->has_directional_light ? 1 : 0;
    st->sunScene = s->directional_light;
    st->spotsScene = std::move(gspots);
    sc.sun_root = -1;
    st->sunArgs.sun_root = -1;
    if (sunNodeCount) {
        st->sunArgs.sun_nodes = st->sunNodes.as<GpuBvh8Node>();
        st->sunArgs.sun_tris = reinterpret_cast<const GpuTriangle*>(static_cast<const char*>(st->sunNodes.ptr) + sunTriOffset);
        st->sunArgs.sun_root = 0;
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) st->sunArgs.sun_frame[r * 3 + k] = static_cast<float>(sunIn.frame[r][k]);
        for (int k = 0; k < 3; ++k) st->sunDirBuilt[k] = s->directional_light.world_space_direction[k];
    }
    st->sunBvhNodes = sunNodeCount;
    st->sunWanted = sunNodeCount > 0;
    st->buildThreads = opt.threads;
    st->bvhMaxDepth = maxDepth;
    st->worldDepth = worldDepth;
    st->inflateAbs = opt.inflate_abs;
    st->triRecords = allTris.size();
    const auto t1 = std::chrono::steady_clock::now();
    st->bvhStats.node_count = allNodes.size();
    st->bvhStats.triangle_count = triangles;
    st->bvhStats.max_depth = maxDepth;
    st->bvhStats.max_leaf_size = maxLeaf;
    st->bvhStats.sah_cost = sah;
    st->bvhStats.build_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
    st->bvhStats.node_bytes = allNodes.size() * sizeof(GpuBvh8Node);
    st->bvhStats.triangle_bytes = allTris.size() * sizeof(GpuTriangle);
    st->bvhStats.sun_node_count = sunNodeCount;
    st->bvhStats.sun_max_depth = sunMaxDepth;
    st->bvhStats.sun_cost_world = st->sunCostWorld;
    st->bvhStats.sun_cost_light = st->sunCostLight;
    st->bvhStats.sun_build_ms = sunBuildMs;
    return adoptScene(ctx, std::move(st));
}

int ark_ddgi_share_scene(ArkDdgiCtx* ctx, const ArkDdgiCtx* src)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->pipeReady = false; // the next update's traversal waits for this
    if (!src || src == ctx || !src->hasScene || !src->sceneStore) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "share_scene: the source context has no scene");
    if (src->device != ctx->device) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "share_scene: contexts on devices %d and %d", src->device, ctx->device);
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    std::shared_ptr<SceneStore> st = src->sceneStore;
    ctx->hasScene = false;
    ctx->sceneStore.reset();
    return adoptScene(ctx, std::move(st));
}

int ark_ddgi_set_lights(ArkDdgiCtx* ctx, const ArkDdgiLights* L)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!L || L->struct_size != sizeof(ArkDdgiLights)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkDdgiLights");
    if (!ctx->hasScene) return ctx->fail(ARK_DDGI_E_NO_SCENE, "ark_ddgi_set_lights before ark_ddgi_set_scene");
    if (L->spot_light_count > ARK_DDGI_MAX_SPOT_LIGHTS) return ctx->fail(ARK_DDGI_E_UNSUPPORTED, "at most %d spot lights (GpuScene.cpp:430)", ARK_DDGI_MAX_SPOT_LIGHTS);
    if (L->spot_light_count && !L->spot_lights) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "set_lights: null spot_lights");
    std::vector<GpuSpotLight> spots(L->spot_light_count);
    for (uint32_t i = 0; i < L->spot_light_count; ++i) spots[i] = gpuSpotLight(L->spot_lights[i]);
    const uint32_t count = (L->has_directional_light ? 1u : 0u) + L->spot_light_count;
    ARK_HIP(hipSetDevice(ctx->device));
    if (count > ctx->lightCount) {
        // the shadow-ray list holds one ray per probe ray and light: grow it once the
        // frames in flight (which use it) are done
        const ShadeWorkLayout need = [&] {
            const uint32_t keep = ctx->lightCount;
            ctx->lightCount = count;
            const ShadeWorkLayout w = shadeWorkLayout(ctx);
            ctx->lightCount = keep;
            return w;
        }();
        if (ctx->shadeWork.bytes < need.total) {
            ARK_HIP(drainContext(ctx));
            const uint32_t keep = ctx->lightCount;
            ctx->lightCount = count;
            const int rc = ensureShadeWork(ctx);
            ctx->lightCount = keep;
            if (rc) return rc;
        }
    }
    ctx->hasSun = L->has_directional_light ? 1 : 0;
    for (int k = 0; k < 3; ++k) {
        ctx->sunColor[k] = ctx->hasSun ? L->directional_light.color[k] : 0.0f;
        ctx->sunDir[k] = ctx->hasSun ? L->directional_light.world_space_direction[k] : 0.0f;
    }
    if (spots.size() != ctx->spotHost.size() || (!spots.empty() && std::memcmp(spots.data(), ctx->spotHost.data(), spots.size() * sizeof(GpuSpotLight)) != 0)) {
        ctx->spotHost = std::move(spots);
        ctx->lightsDirty = true;
    }
    if (const int rc = refreshScene(ctx)) return rc;
    // a sun rebuild to start or install: on the context's internal stream, in call order
    // (orderBegin / orderEnd) only when one is, so that a frame with no rebuild costs the
    // next update no cross-stream wait
    SceneStore& st = *ctx->sceneStore;
    const bool sunWork = st.sunWanted && ctx->hasSun && (st.sunJob ? st.sunJob->done.load(std::memory_order_acquire) : true);
    if (!sunWork) return sunRebuildStep(ctx, nullptr);
    const uint32_t v = st.version;
    const bool hadJob = static_cast<bool>(st.sunJob);
    ARK_HIP(orderBegin(ctx, ctx->stream));
    if (const int rc = sunRebuildStep(ctx, ctx->stream)) return rc;
    if (st.version != v || static_cast<bool>(st.sunJob) != hadJob) ARK_HIP(orderEnd(ctx, ctx->stream));
    return ARK_DDGI_OK;
}

namespace {
// ark_ddgi_set_instances' first use of a scene: the world BVHs' nodes by depth, deepest
// first, and the refit's work buffers (a topology download: refits never change it)
int prepareRefit(ArkDdgiCtx* ctx, SceneStore& st)
{
    const uint64_t n = st.bvhStats.node_count;
    std::vector<GpuBvh8Node> h(n);
    if (n) ARK_HIP(hipMemcpy(h.data(), st.nodes.ptr, n * sizeof(GpuBvh8Node), hipMemcpyDeviceToHost));
    const int32_t roots[3] = { st.args.root_opaque, st.args.root_masked, st.args.root_blend };
    std::vector<uint32_t> order;
    if (!bvhLevelOrder(h.data(), n, roots, 3, order, st.levelOffsets)) return ctx->fail(ARK_DDGI_E_DEVICE, "refit: a node outside the BVH");
    int rc;
    if ((rc = upload(ctx, st.refitOrder, order.data(), order.size())) != 0) return rc;
    ARK_HIP(st.refitBoxes.alloc(std::max<size_t>(16, n * 6 * sizeof(float))));
    return ARK_DDGI_OK;
}
} // namespace

namespace {
// The refitted spare becomes the front copy (SceneStore::spare), the front one the last
// spare: the kernel views follow.
void rotateGeometry(SceneStore& st)
{
    const bool sun = st.sunArgs.sun_root >= 0 && st.sunNodes.ptr;
    const size_t sunTriOffset = sun ? static_cast<size_t>(reinterpret_cast<const char*>(st.sunArgs.sun_tris) - static_cast<const char*>(st.sunNodes.ptr)) : 0;
    SceneStore::Spare old;
    old.nodes = st.nodes;
    old.sunNodes = st.sunNodes;
    old.instances = st.instances;
    old.valid = true;
    old.slot = st.front;
    st.nodes = st.spare[0].nodes;
    st.sunNodes = st.spare[0].sunNodes;
    st.instances = st.spare[0].instances;
    st.front = st.spare[0].slot;
    st.spare[0] = st.spare[1];
    st.spare[1] = old;
    st.args.nodes = st.nodes.as<GpuBvh8Node>();
    st.args.tris = reinterpret_cast<const GpuTriangle*>(static_cast<const char*>(st.nodes.ptr) + st.args.tri_byte_offset);
    st.args.instances = st.instances.as<GpuInstance>();
    if (sun) {
        st.sunArgs.sun_nodes = st.sunNodes.as<GpuBvh8Node>();
        st.sunArgs.sun_tris = reinterpret_cast<const GpuTriangle*>(static_cast<const char*>(st.sunNodes.ptr) + sunTriOffset);
    }
}
} // namespace

static int checkSequencing(ArkDdgiCtx* ctx);

int ark_ddgi_set_instances_async(ArkDdgiCtx* ctx, const ArkRTInstance* instances, uint32_t count, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!ctx->hasScene) return ctx->fail(ARK_DDGI_E_NO_SCENE, "ark_ddgi_set_instances before ark_ddgi_set_scene");
    SceneStore& st = *ctx->sceneStore;
    if (count != st.instHost.size() || (count && !instances))
        return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "set_instances: %u instances, the scene has %zu", count, st.instHost.size());
    for (uint32_t i = 0; i < count; ++i) {
        const ArkRTInstance &a = instances[i], &b = st.instHost[i];
        if (a.rt_mesh_index != b.rt_mesh_index || a.triangle_count != b.triangle_count || a.hit_mask != b.hit_mask)
            return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "set_instances: instance %u changed its mesh, triangle count or hit mask (a set_scene builds a new scene)", i);
        for (float v : a.object_to_world)
            if (!std::isfinite(v)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "set_instances: instance %u: non-finite transform", i);
    }
    const auto t0 = std::chrono::steady_clock::now();
    const hipStream_t s = streamOf(hipStream);
    ARK_HIP(hipSetDevice(ctx->device));
    if (const int r = checkSequencing(ctx)) return r;
    // with a shared scene every context's launches may read either copy: all of them end
    // first (and the refit below before returning)
    const bool shared = ctx->sceneStore.use_count() > 1;
    if (shared) ARK_HIP(hipDeviceSynchronize());
    int rc;
    if (st.levelOffsets.empty() && (rc = prepareRefit(ctx, st)) != 0) return rc;
    // everything this context enqueued so far ends with its last operation (orderBegin
    // chains the others into it): the front copy's readers among them. Events that mark
    // that point are recorded on `s` behind it (orderBegin) - not on the last operation's
    // stream, which the caller may have destroyed since, nor on a stream of the
    // context's own (one more stream on the process's few hardware queues; measured no
    // better under motion, profiles/r06_ab2_refit_ordering/)
    ARK_HIP(orderBegin(ctx, s));
    const hipStream_t last = s;
    // a light-space sun BVH without a refit order (none recorded) cannot follow: dropped
    if (st.sunArgs.sun_root >= 0 && st.sunLevelOffsets.empty()) {
        st.sunArgs.sun_root = -1;
        st.sunArgs.sun_nodes = nullptr;
        st.sunArgs.sun_tris = nullptr;
        ARK_HIP(retireBuffer(st, st.sunNodes, last));
        ARK_HIP(dropSpares(st, last));
        st.sunBvhNodes = 0;
        st.bvhStats.sun_node_count = 0;
        st.bvhStats.sun_max_depth = 0;
    }
    // The refit writes the next spare copy on the refit stream, after the operations that
    // read it (while it was the front one: evFree) and the last install; the frames in
    // flight keep reading the front copy. The copy swapped out here is free once the
    // operations enqueued so far are done.
    SceneStore::Spare& tgt = st.spare[0];
    const int fs = st.front, ts = tgt.slot;
    const hipStream_t rs = ctx->refitStream;
    ARK_HIP(hipEventRecord(ctx->evFree[fs], last));
    ctx->freeValid[fs] = true;
    if (ctx->freeValid[ts]) ARK_HIP(hipStreamWaitEvent(rs, ctx->evFree[ts], 0));
    if (ctx->installValid) {
        ARK_HIP(hipStreamWaitEvent(rs, ctx->evInstalled, 0));
        ctx->installValid = false;
    }
    if (!tgt.valid) {
        // a copy of the front one (a new scene or an installed rebuild)
        auto copy = [&](DeviceBuffer& dst, const DeviceBuffer& src) -> hipError_t {
            if (!src.ptr) return retireBuffer(st, dst, last);
            hipError_t e = hipSuccess;
            if (dst.bytes != src.bytes) {
                if ((e = retireBuffer(st, dst, last)) != hipSuccess) return e;
                if ((e = dst.alloc(src.bytes)) != hipSuccess) return e;
            }
            return hipMemcpyAsync(dst.ptr, src.ptr, src.bytes, hipMemcpyDeviceToDevice, rs);
        };
        ARK_HIP(copy(tgt.nodes, st.nodes));
        ARK_HIP(copy(tgt.sunNodes, st.sunNodes));
        ARK_HIP(copy(tgt.instances, st.instances));
        st.xf[ts] = st.xf[fs];
        st.inflCopy[ts][0] = st.inflCopy[fs][0];
        st.inflCopy[ts][1] = st.inflCopy[fs][1];
        tgt.valid = true;
    }
    // the instance table of the shading kernels (set_scene's determinant and rows)
    std::vector<GpuInstance> ginst(count);
    for (uint32_t ii = 0; ii < count; ++ii) {
        const float* M = instances[ii].object_to_world;
        const float det = M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) + M[2] * (M[4] * M[9] - M[5] * M[8]);
        const ArkRTTriangleMesh& mesh = st.meshHost[instances[ii].rt_mesh_index];
        GpuInstance& g = ginst[ii];
        std::memset(&g, 0, sizeof(g));
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) g.normal_matrix[r * 4 + c] = M[r * 4 + c];
        g.rt_mesh_index = static_cast<int32_t>(instances[ii].rt_mesh_index);
        g.flip_facing = det < 0.0f ? 1 : 0;
        g.hit_mask = static_cast<int32_t>(instances[ii].hit_mask);
        g.material_index = mesh.material_index;
    }
    ARK_HIP(stagedUpload(st, tgt.instances.ptr, ginst.data(), count * sizeof(GpuInstance), rs));
    if ((rc = uploadRefitInstances(ctx, st, instances, count, &st.xf[ts], rs)) != 0) return rc;
    if ((rc = enqueueRefit(ctx, st, rs, spareTarget(tgt), ts)) != 0) return rc;
    ARK_HIP(hipEventRecord(ctx->evRefit, rs));
    if (shared) ARK_HIP(hipStreamSynchronize(rs));
    // the refitted copy becomes the front one
    st.xf[ts].resize(count);
    for (uint32_t ii = 0; ii < count; ++ii) std::memcpy(st.xf[ts][ii].data(), instances[ii].object_to_world, sizeof(float) * 12);
    rotateGeometry(st);
    // the caller's stream follows the refit (what it runs next sees the new geometry); the
    // next update's traversal on the traversal stream waits for it too (refitPending)
    ARK_HIP(hipStreamWaitEvent(s, ctx->evRefit, 0));
    ctx->refitPending = true;
    for (uint32_t ii = 0; ii < count; ++ii) std::memcpy(st.instHost[ii].object_to_world, instances[ii].object_to_world, sizeof(float) * 12);
    ++st.version;
    ++st.refitsSinceBuild;
    ++st.sunRefitsSinceBuild;
    st.bvhStats.refit_version = ++st.refitCount;
    if ((rc = refreshScene(ctx)) != 0) return rc;
    // background rebuilds of the loosened BVHs (world and light-space), from a snapshot
    // taken on s behind this refit
    if ((rc = sceneMaintenance(ctx, s)) != 0) return rc;
    ARK_HIP(orderEnd(ctx, s));
    st.bvhStats.refit_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return ARK_DDGI_OK;
}

int ark_ddgi_debug_scene_digest(ArkDdgiCtx* ctx, uint64_t* out)
{
    if (!ctx || !out) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!ctx->hasScene) return ctx->fail(ARK_DDGI_E_NO_SCENE, "scene digest before ark_ddgi_set_scene");
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    const SceneStore& st = *ctx->sceneStore;
    auto digest = [&](const void* dev, size_t bytes, uint64_t& h) -> hipError_t {
        h = 1469598103934665603ull;
        if (!dev || !bytes) return hipSuccess;
        std::vector<unsigned char> b(bytes);
        const hipError_t e = hipMemcpy(b.data(), dev, bytes, hipMemcpyDeviceToHost);
        for (unsigned char c : b) h = (h ^ c) * 1099511628211ull;
        return e;
    };
    ARK_HIP(digest(st.args.nodes, st.bvhStats.node_count * sizeof(GpuBvh8Node), out[0]));
    ARK_HIP(digest(st.args.tris, st.triRecords * sizeof(GpuTriangle), out[1]));
    const bool sun = st.sunArgs.sun_root >= 0;
    ARK_HIP(digest(sun ? st.sunArgs.sun_nodes : nullptr, st.sunBvhNodes * sizeof(GpuBvh8Node), out[2]));
    ARK_HIP(digest(sun ? st.sunArgs.sun_tris : nullptr, st.sunTriRecords * sizeof(GpuTriangle), out[3]));
    if (!sun) out[2] = out[3] = 0;
    return ARK_DDGI_OK;
}

int ark_ddgi_set_instances(ArkDdgiCtx* ctx, const ArkRTInstance* instances, uint32_t count)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    const auto t0 = std::chrono::steady_clock::now();
    if (const int rc = ark_ddgi_set_instances_async(ctx, instances, count, ctx->stream)) return rc;
    ARK_HIP(hipStreamSynchronize(ctx->stream));
    ctx->sceneStore->bvhStats.refit_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ctx->bvhStats = ctx->sceneStore->bvhStats;
    return ARK_DDGI_OK;
}

static uint32_t countSlabProbes(const ArkDdgiCtx* ctx, uint32_t first, uint32_t K)
{
    if (ctx->desc.shard_count <= 1) return K;
    return slabRankOf(static_cast<uint32_t>(ctx->X), static_cast<uint32_t>(ctx->Y), static_cast<uint32_t>(ctx->Z), static_cast<uint32_t>(ctx->slabZ0),
                      static_cast<uint32_t>(ctx->slabZ1), first, K);
}

static int updateImpl(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* p, void* hipStream, void* shadeWaitEvent, void* doneEvent, uint32_t shadeWaitSeq = 0);

// Fail-closed frame sequencing (VERDICT r03 "do this" #3): a k_seq_wait that gave up
// has set the context's timed-out word, so every path kernel that starts after it
// skips (frameAborted) and leaves atlases, surfels and offsets as they were (a launch
// already running when the wait gave up completes). The first context
// call that sees the host-mapped flag drains the device (the late producer ends by
// itself), clears both words, switches the context to event sequencing (which no
// queue order can stall) and reports ARK_DDGI_E_DEVICE; the calls after it run.
static int checkSequencing(ArkDdgiCtx* ctx)
{
    if (!ctx->hostAbort || __atomic_load_n(ctx->hostAbort, __ATOMIC_ACQUIRE) == 0u) return ARK_DDGI_OK;
    ARK_HIP(hipSetDevice(ctx->device));
    // the whole device (ADVICE r04 low asked for the context's own streams only): the
    // late producer may sit on a caller's stream (an exchange stream) whose end the
    // context recorded as a sequence word; once the context switches to events, nothing
    // else would order the next frame's shading after it
    ARK_HIP(hipDeviceSynchronize());
    ARK_HIP(hipMemset(ctx->seqWords.as<uint32_t>() + 64, 0, 4));
    __atomic_store_n(ctx->hostAbort, 0u, __ATOMIC_RELEASE);
    ctx->seqSync = false;
    ctx->pipeReady = false;
    ++ctx->seqTimeouts;
    return ctx->fail(ARK_DDGI_E_DEVICE,
                     "a frame-sequencing wait between the context's streams gave up after %u ms: every update kernel that started after it skipped "
                     "(its atlases, surfels and offsets left as they were); the context now orders its streams with events",
                     ctx->seqTimeoutMs);
}

int ark_ddgi_set_sequencing(ArkDdgiCtx* ctx, int device_sequence_words, uint32_t timeout_ms)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (timeout_ms > 3600u * 1000u) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "sequencing timeout %u ms above one hour", timeout_ms);
    ctx->seqSync = device_sequence_words != 0;
    if (timeout_ms) {
        ctx->seqTimeoutMs = timeout_ms;
        ctx->seqTimeoutTicks = ctx->wallClockKhz * timeout_ms;
    }
    return ARK_DDGI_OK;
}

int ark_ddgi_get_sequencing(const ArkDdgiCtx* ctx, int* out_device_sequence_words, uint32_t* out_timeout_ms, uint32_t* out_timeouts)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (out_device_sequence_words) *out_device_sequence_words = ctx->seqSync ? 1 : 0;
    if (out_timeout_ms) *out_timeout_ms = ctx->seqTimeoutMs;
    if (out_timeouts) *out_timeouts = ctx->seqTimeouts;
    return ARK_DDGI_OK;
}


int ark_ddgi_update(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* p, void* hipStream)
{
    return updateImpl(ctx, p, hipStream, nullptr, nullptr);
}

int ark_ddgi_update_overlapped(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* p, void* hipStream, void* shadeWaitEvent, void* doneEvent)
{
    return updateImpl(ctx, p, hipStream, shadeWaitEvent, doneEvent);
}

int ark_ddgi_update_exchanged(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* p, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    const uint32_t wait = ctx->pendingExchange;
    // without sequence words the exchange's end is an event (ark_ddgi_exchange_end)
    const int r = ctx->seqSync ? updateImpl(ctx, p, hipStream, nullptr, nullptr, wait)
                               : updateImpl(ctx, p, hipStream, wait ? ctx->evExchangeDone : nullptr, nullptr);
    if (r == ARK_DDGI_OK) ctx->pendingExchange = 0;
    return r;
}

int ark_ddgi_exchange_begin(ArkDdgiCtx* ctx, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    const hipStream_t x = streamOf(hipStream);
    if (const int r = checkSequencing(ctx)) return r;
    ARK_HIP(hipSetDevice(ctx->device));
    if (ctx->lastMainSeq) {
        uint32_t* w = ctx->seqWords.as<uint32_t>();
        ARK_HIP(launch_seq_wait(w + 32, ctx->lastMainSeq, w + 64, ctx->hostAbortDev, ctx->seqTimeoutTicks, x));
    } else {
        // the last update was not sequenced: everything enqueued on its stream so far
        ARK_HIP(hipEventRecord(ctx->evExchangeSrc, ctx->lastStream));
        ARK_HIP(hipStreamWaitEvent(x, ctx->evExchangeSrc, 0));
    }
    return ARK_DDGI_OK;
}

int ark_ddgi_exchange_end(ArkDdgiCtx* ctx, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ARK_HIP(hipSetDevice(ctx->device));
    const uint32_t n = ++ctx->exchSeq;
    if (ctx->seqSync) ARK_HIP(launch_seq_signal(ctx->seqWords.as<uint32_t>() + 96, n, streamOf(hipStream)));
    else ARK_HIP(hipEventRecord(ctx->evExchangeDone, streamOf(hipStream)));
    ctx->pendingExchange = n;
    return ARK_DDGI_OK;
}

static ArkDdgiWindowExchange windowExchangeInfo(const ArkDdgiCtx* ctx)
{
    ArkDdgiWindowExchange w {};
    w.struct_size = sizeof(w);
    w.first_probe = ctx->lastFirst;
    w.probe_updates = ctx->lastK;
    const uint32_t P = static_cast<uint32_t>(ctx->desc.shard_count), Zs = static_cast<uint32_t>(ctx->Z) / P;
    w.full_bands = ctx->lastK == static_cast<uint32_t>(ctx->N) ? 1u : 0u;
    for (uint32_t q = 0; q < P; ++q) {
        const uint32_t n = slabRankOf(static_cast<uint32_t>(ctx->X), static_cast<uint32_t>(ctx->Y), static_cast<uint32_t>(ctx->Z), q * Zs, (q + 1) * Zs, ctx->lastFirst,
                                      ctx->lastK);
        w.probes_per_rank = std::max(w.probes_per_rank, n);
        if (q == static_cast<uint32_t>(ctx->desc.shard_rank)) w.my_probes = n;
    }
    w.bytes_per_rank = w.full_bands ? 0u : static_cast<uint64_t>(w.probes_per_rank) * kWindowPacketBytes;
    return w;
}

int ark_ddgi_window_exchange_info(const ArkDdgiCtx* ctx, ArkDdgiWindowExchange* out)
{
    if (!ctx || !out) return ARK_DDGI_E_INVALID_ARGUMENT;
    *out = windowExchangeInfo(ctx);
    return ARK_DDGI_OK;
}

static int windowPack(ArkDdgiCtx* ctx, void* buf, uint64_t bytes, void* hipStream, bool unpack)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    const ArkDdgiWindowExchange w = windowExchangeInfo(ctx);
    if (w.full_bands) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "window exchange: the last window covered the grid (exchange the bands)");
    const uint64_t need = unpack ? w.bytes_per_rank * static_cast<uint64_t>(ctx->desc.shard_count) : w.bytes_per_rank;
    if (bytes != need) return ctx->fail(ARK_DDGI_E_SIZE_MISMATCH, "window exchange: %llu bytes, the window needs %llu", (unsigned long long)bytes, (unsigned long long)need);
    if (need && !buf) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "window exchange: null buffer");
    ARK_HIP(hipSetDevice(ctx->device));
    WindowExchangeArgs a {};
    a.X = ctx->X; a.Y = ctx->Y; a.Z = ctx->Z; a.N = ctx->N;
    a.first = ctx->lastFirst;
    a.K = ctx->lastK;
    a.Wi = ctx->Wi; a.Wv = ctx->Wv;
    a.slabDepth = static_cast<uint32_t>(ctx->Z / ctx->desc.shard_count);
    a.rank = static_cast<uint32_t>(ctx->desc.shard_rank);
    a.world = static_cast<uint32_t>(ctx->desc.shard_count);
    a.bytesPerRank = w.bytes_per_rank;
    a.irr = ctx->irr.as<uint16_t>();
    a.vis = ctx->vis.as<uint16_t>();
    a.buf = static_cast<uint8_t*>(buf);
    if (need) ARK_HIP(launch_window_pack(a, unpack, streamOf(hipStream)));
    return ARK_DDGI_OK;
}

int ark_ddgi_pack_window(ArkDdgiCtx* ctx, void* dst, uint64_t bytes, void* hipStream) { return windowPack(ctx, dst, bytes, hipStream, false); }

int ark_ddgi_unpack_window(ArkDdgiCtx* ctx, const void* src, uint64_t bytes, void* hipStream)
{
    return windowPack(ctx, const_cast<void*>(src), bytes, hipStream, true);
}

// The caller's stream s waits for the traversal stream's part of a pipelined frame
// (slot table, traversal, offsets): device-side sequencing, or an event.
static hipError_t tracedSync(ArkDdgiCtx* ctx, bool seq, uint32_t seqN, hipStream_t ts, hipStream_t s)
{
    if (seq) {
        uint32_t* w = ctx->seqWords.as<uint32_t>();
        hipError_t e = launch_seq_signal(w, seqN, ts);
        return e != hipSuccess ? e : launch_seq_wait(w, seqN, w + 64, ctx->hostAbortDev, ctx->seqTimeoutTicks, s);
    }
    hipError_t e = hipEventRecord(ctx->evTraced, ts);
    return e != hipSuccess ? e : hipStreamWaitEvent(s, ctx->evTraced, 0);
}

static int updateImpl(ArkDdgiCtx* ctx, const ArkDdgiFrameParams* p, void* hipStream, void* shadeWaitEvent, void* doneEvent, uint32_t shadeWaitSeq)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!p || p->struct_size != sizeof(ArkDdgiFrameParams)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkDdgiFrameParams");
    if (!ctx->hasScene) return ctx->fail(ARK_DDGI_E_NO_SCENE, "ark_ddgi_update before ark_ddgi_set_scene");
    const uint32_t N = static_cast<uint32_t>(ctx->N);
    const uint32_t K = std::min(p->probe_updates, N);
    const uint32_t R = p->rays_per_probe;
    if (K == 0 || R == 0 || K > static_cast<uint32_t>(ctx->Kmax) || R > static_cast<uint32_t>(ctx->Rmax))
        return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "probe_updates %u / rays_per_probe %u outside [1,%d] / [1,%d]", K, R, ctx->Kmax, ctx->Rmax);
    const hipStream_t s = streamOf(hipStream);
    if (const int r = checkSequencing(ctx)) return r;
    ARK_HIP(hipSetDevice(ctx->device));
    FrameArgs f {};
    f.abort_word = ctx->seqWords.as<uint32_t>() + 64;
    f.X = ctx->X; f.Y = ctx->Y; f.Z = ctx->Z;
    f.Wi = ctx->Wi; f.Hi = ctx->Hi; f.Wv = ctx->Wv; f.Hv = ctx->Hv;
    for (int k = 0; k < 3; ++k) {
        f.spacing[k] = ctx->desc.probe_spacing[k];
        f.origin[k] = ctx->desc.offset_to_first[k];
    }
    f.z_far = ctx->desc.z_far;
    f.frame = p->frame_index;
    f.first = p->first_probe_index % N;
    f.window = K;
    f.sharded = ctx->desc.shard_count > 1 ? 1 : 0;
    f.slab_z0 = ctx->slabZ0;
    f.slab_z1 = ctx->slabZ1;
    f.window_probes = countSlabProbes(ctx, f.first, K);
    f.R = R;
    f.Rmax = static_cast<uint32_t>(ctx->Rmax);
    f.window_rays = f.window_probes * R;
    f.hysteresis_irradiance = p->hysteresis_irradiance;
    f.hysteresis_visibility = p->hysteresis_visibility;
    f.visibility_sharpness = p->visibility_sharpness;
    f.ambient_amount = p->ambient_amount;
    f.environment_multiplier = p->environment_multiplier;
    f.delta_time = p->delta_time;
    f.update_offsets = p->update_offsets;
    f.irr = ctx->irr.as<uint16_t>();
    f.vis = ctx->vis.as<uint16_t>();
    f.offsets = ctx->offsets.as<float4>();
    const bool timing = ctx->timing;
    const bool count = ctx->counting;
    // Frames in flight: this frame's slot table, traversal and probe offsets read the
    // scene, the sample order and the probe offsets only, which nothing of the
    // previous frame's shadow rays, shading or atlas update writes (its offsets ran
    // before them). They may start before the previous frame is done when the sample
    // order is the same and no other writing context operation came in between.
    // Instrumented updates (per-kernel events, counters) run serially.
    const bool pipe = ctx->pipelining && ctx->pipeReady && !timing && !count && R == ctx->prevR;
    const uint32_t b = ctx->parity;
    const uint64_t Kmax = static_cast<uint64_t>(ctx->Kmax), Rmax = static_cast<uint64_t>(ctx->Rmax);
    f.slots = ctx->slots.as<GpuProbeSlot>() + b * Kmax;
    f.fib = ctx->fib.as<float4>() + b * Rmax;
    RoctxRange ddgiZone("DDGI");
    ARK_HIP(orderBegin(ctx, s));
    // finished background rebuilds installed (and refitted forward) on s, new ones started
    if (const int rc = sceneMaintenance(ctx, s)) return rc;
    if (ctx->sceneVersion != ctx->sceneStore->version) // another context refitted the shared scene or installed a BVH
        if (const int rc = refreshScene(ctx)) return rc;
    // lights changed since the last update: stored ahead of this frame's shadow rays and
    // shading on s (the traversal on the traversal stream reads no light)
    ARK_HIP(flushLights(ctx, s));
    if (ctx->orderR != R) {
        sampleTraversalOrder(R, ctx->orderHost);
        ARK_HIP(hipMemcpyAsync(ctx->order.ptr, ctx->orderHost.data(), R * 4, hipMemcpyHostToDevice, s));
        ctx->orderR = R;
    }
    f.order = ctx->order.as<uint32_t>();
    f.fib_order = ctx->fibOrder.as<float4>() + b * Rmax;
    f.hits = ctx->hits.as<GpuHit>() + b * Kmax * Rmax;
    f.surfels = ctx->surfels.as<uint16_t>();
    f.spill = ctx->spill.as<uint32_t>() + ctx->spillRegionWords; // region 1 (primary traversal)
    f.light_count = ctx->lightCount;
    f.refill_min = ctx->refillMin;
    f.sun_refill_min = ctx->sunRefillMin;
    // a half-occupancy window (below kPipeHalfRays) hands out 32 rays per partition-head
    // grab to the probe-ray and shadow-ray queues (K = 2048 windows 0.429 -> 0.420 ms;
    // the whole grid keeps 64: 4.13 vs 4.18 ms at 32, profiles/r02_m19)
    f.grab_chunk = (pipe && f.window_rays < kPipeHalfRays) ? std::min<uint32_t>(ctx->grabChunk, 32u) : ctx->grabChunk;
    f.ray_counter = ctx->rayCounter.as<uint32_t>() + b * kRayCounterWords;
    f.counters = ctx->counters.as<unsigned long long>();
    f.ray_steps = count ? ctx->raySteps.as<uint16_t>() : nullptr;
    // shading work set (ensureShadeWork): per-ray light bits | shadow-ray list
    {
        const ShadeWorkLayout l = shadeWorkLayout(ctx);
        char* w = static_cast<char*>(ctx->shadeWork.ptr);
        f.shadow_bits = reinterpret_cast<uint32_t*>(w + l.bits);
        f.shadow_rays = reinterpret_cast<ShadowRay*>(w + l.list);
    }
    f.shadow_count = f.ray_counter + kShadowCountWord;
    f.shadow_heads = f.ray_counter + kShadowHeadWord;
    // the sun's shadow rays in their own list (the first Kmax x Rmax entries of the
    // list area, the other lights' after them) for the light-space BVH
    if (ctx->scene.sun_root >= 0) {
        f.sun_rays = f.shadow_rays;
        f.shadow_rays += Kmax * Rmax;
        f.sun_count = f.ray_counter + kSunCountWord;
        f.sun_heads = f.ray_counter + kSunHeadWord;
    }
    // the slot table and the primary traversal: on traceStream after frame n - 2 (the
    // last user of buffer set b) when pipelined, else in line on the caller's stream
    const hipStream_t ts = pipe ? ctx->traceStream : s;
    uint32_t* seqTrace = ctx->seqWords.as<uint32_t>();
    uint32_t* seqMain = seqTrace + 32;
    uint32_t* seqTimedOut = seqTrace + 64;
    const bool seq = pipe && ctx->seqSync;
    const uint32_t seqN = seq ? ++ctx->frameSeq : 0u;
    if (pipe && ctx->setSeqValid[b]) ARK_HIP(launch_seq_wait(seqMain, ctx->setSeq[b], seqTimedOut, ctx->hostAbortDev, ctx->seqTimeoutTicks, ts));
    else if (pipe && ctx->frameDoneValid[b]) ARK_HIP(hipStreamWaitEvent(ts, ctx->evFrameDone[b], 0));
    // a serial previous frame wrote its offsets on the caller's stream
    if (pipe && !ctx->prevPipelined && ctx->frameDoneValid[b ^ 1u]) ARK_HIP(hipStreamWaitEvent(ts, ctx->evFrameDone[b ^ 1u], 0));
    // a refit or an installed rebuild enqueued since the last update (on any stream): the
    // traversal reads the BVH it writes
    if (ctx->refitPending) {
        if (ts != s) ARK_HIP(hipStreamWaitEvent(ts, ctx->evRefit, 0));
        ctx->refitPending = false;
    }
    if (count) ARK_HIP(hipMemsetAsync(ctx->counters.ptr, 0, ctx->counters.bytes, s));
    // (k_probe_slots zeroes f.ray_counter)
    if (timing) ARK_HIP(hipEventRecord(ctx->ev[0], s));
    f.slot_order = ctx->slotOrder.as<uint32_t>() + b * Kmax; // written by k_probe_slots
    ARK_HIP(launch_probe_slots(f, ts));
    if (f.window_probes > 0) {
        RoctxRange traceZone("Trace rays");
        const bool half = pipe && f.window_rays < kPipeHalfRays;
        ARK_HIP(launch_trace(ctx->scene, f, half ? ctx->pipeTraceBlocks : ctx->traceBlocks, count, ts));
        if (pipe) {
            // probeUpdateOffset (k_probe_offsets: from the hit records), so that the
            // next frame's slot table may follow on this stream. The rest of the frame
            // needs only the hit records, but waiting for the offsets too costs less
            // (7 us) than a second cross-stream wait for them at the end of the frame
            // (each wait ~11 us of queue latency, satisfied or not: profiles/r03_v)
            ARK_HIP(launch_probe_offsets(f, ts));
            ARK_HIP(tracedSync(ctx, seq, seqN, ts, s));
        }
        if (timing) ARK_HIP(hipEventRecord(ctx->ev[1], s));
        FrameArgs fs = f;
        fs.spill = ctx->spill.as<uint32_t>(); // region 0
        if (f.light_count > 0) {
            ARK_HIP(launch_shadow_gen(ctx->scene, fs, s));
            ARK_HIP(launch_trace_shadow(ctx->scene, fs, count ? ctx->shadowBlocks : shadowBlocksFor(ctx, f.window_rays), count, s));
        }
        if (timing) ARK_HIP(hipEventRecord(ctx->ev[5], s));
        // shading reads the previous frame's atlases at arbitrary probes: on a Z-slab
        // rank it waits here for the previous exchange (the traversal above did not)
        if (shadeWaitEvent) ARK_HIP(hipStreamWaitEvent(s, static_cast<hipEvent_t>(shadeWaitEvent), 0));
        if (shadeWaitSeq) ARK_HIP(launch_seq_wait(seqTrace + 96, shadeWaitSeq, seqTimedOut, ctx->hostAbortDev, ctx->seqTimeoutTicks, s));
        ARK_HIP(launch_shade(ctx->scene, fs, ctx->shadeBlocks, count, s));
        if (timing) ARK_HIP(hipEventRecord(ctx->ev[2], s));
        if (timing) ARK_HIP(hipEventRecord(ctx->ev[4], s));
        traceZone.end();
        // probeUpdateOffset (serial frames), probeUpdateIrradiance/Visibility + border
        // corners/edges, fused
        RoctxRange updateZone("Update probes");
        if (!pipe) ARK_HIP(launch_probe_offsets(fs, s));
        ARK_HIP(launch_probe_update(fs, s));
    } else {
        if (pipe) ARK_HIP(tracedSync(ctx, seq, seqN, ts, s));
        if (shadeWaitEvent) ARK_HIP(hipStreamWaitEvent(s, static_cast<hipEvent_t>(shadeWaitEvent), 0));
        if (shadeWaitSeq) ARK_HIP(launch_seq_wait(seqTrace + 96, shadeWaitSeq, seqTimedOut, ctx->hostAbortDev, ctx->seqTimeoutTicks, s));
        if (timing) {
            ARK_HIP(hipEventRecord(ctx->ev[1], s));
            ARK_HIP(hipEventRecord(ctx->ev[5], s));
            ARK_HIP(hipEventRecord(ctx->ev[2], s));
            ARK_HIP(hipEventRecord(ctx->ev[4], s));
        }
    }
    if (timing) ARK_HIP(hipEventRecord(ctx->ev[3], s));
    if (seq) {
        ARK_HIP(launch_seq_signal(seqMain, seqN, s));
        ctx->setSeq[b] = seqN;
        ctx->setSeqValid[b] = true;
    } else {
        ARK_HIP(hipEventRecord(ctx->evFrameDone[b], s));
        ctx->setSeqValid[b] = false;
    }
    ctx->frameDoneValid[b] = true;
    ctx->lastMainSeq = seq ? seqN : 0u;
    ctx->lastStream = s;
    if (doneEvent) ARK_HIP(hipEventRecord(static_cast<hipEvent_t>(doneEvent), s));
    ARK_HIP(orderEnd(ctx, s));
    ctx->parity = b ^ 1u;
    ctx->pipeReady = true;
    ctx->prevR = R;
    ctx->prevPipelined = pipe;
    ctx->lastParity = b;
    ctx->timingValid = timing;
    ctx->countersPending = count;
    ctx->lastRays = f.window_rays;
    ctx->lastProbes = f.window_probes;
    ctx->nextProbeIndex = (f.first + K) % N;
    ctx->lastFirst = f.first;
    ctx->lastK = K;
    return ARK_DDGI_OK;
}

int ark_ddgi_mark_external_write(ArkDdgiCtx* ctx)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->pipeReady = false; // the next update's traversal waits for this
    return ARK_DDGI_OK;
}

int ark_ddgi_synchronize(ArkDdgiCtx* ctx)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    return checkSequencing(ctx);
}

static int resourceInfo(const ArkDdgiCtx* ctx, int which, void** ptr, uint64_t* bytes)
{
    switch (which) {
    case ARK_DDGI_ATLAS_IRRADIANCE: *ptr = ctx->irr.ptr; *bytes = ctx->irr.bytes; return 0;
    case ARK_DDGI_ATLAS_VISIBILITY: *ptr = ctx->vis.ptr; *bytes = ctx->vis.bytes; return 0;
    case ARK_DDGI_SURFELS: *ptr = ctx->surfels.ptr; *bytes = ctx->surfels.bytes; return 0;
    case ARK_DDGI_PROBE_OFFSETS: *ptr = ctx->offsets.ptr; *bytes = ctx->offsets.bytes; return 0;
    case ARK_DDGI_DEBUG_HITS: *ptr = ctx->hits.as<GpuHit>() + static_cast<uint64_t>(ctx->lastParity) * ctx->Kmax * ctx->Rmax; *bytes = ctx->hits.bytes / 2; return 0;
    case ARK_DDGI_DEBUG_RAY_STEPS: *ptr = ctx->raySteps.ptr; *bytes = ctx->raySteps.bytes; return ctx->raySteps.ptr ? 0 : ARK_DDGI_E_INVALID_ARGUMENT;
    default: return ARK_DDGI_E_INVALID_ARGUMENT;
    }
}

int ark_ddgi_resource_size(const ArkDdgiCtx* ctx, int which, uint64_t* outBytes)
{
    if (!ctx || !outBytes) return ARK_DDGI_E_INVALID_ARGUMENT;
    void* p;
    return resourceInfo(ctx, which, &p, outBytes);
}

int ark_ddgi_read(ArkDdgiCtx* ctx, int which, void* dst, uint64_t bytes)
{
    if (!ctx || !dst) return ARK_DDGI_E_INVALID_ARGUMENT;
    void* p;
    uint64_t n;
    if (resourceInfo(ctx, which, &p, &n) != 0) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "unknown resource %d", which);
    if (bytes != n) return ctx->fail(ARK_DDGI_E_SIZE_MISMATCH, "resource %d is %llu bytes, got %llu", which, (unsigned long long)n, (unsigned long long)bytes);
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    ARK_HIP(hipMemcpy(dst, p, n, hipMemcpyDeviceToHost));
    return ARK_DDGI_OK;
}

int ark_ddgi_write(ArkDdgiCtx* ctx, int which, const void* src, uint64_t bytes)
{
    if (!ctx || !src) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->pipeReady = false; // the next update's traversal waits for this
    void* p;
    uint64_t n;
    if (resourceInfo(ctx, which, &p, &n) != 0) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "unknown resource %d", which);
    if (bytes != n) return ctx->fail(ARK_DDGI_E_SIZE_MISMATCH, "resource %d is %llu bytes, got %llu", which, (unsigned long long)n, (unsigned long long)bytes);
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    ARK_HIP(hipMemcpy(p, src, n, hipMemcpyHostToDevice));
    return ARK_DDGI_OK;
}

// --- history checkpoint ------------------------------------------------------
namespace {
struct StateHeader {
    char magic[8];           // "ARKDDGI1"
    int32_t grid[3];
    float spacing[3], origin[3];
    float zFar;
    int32_t clearMode, shardRank, shardCount;
    uint32_t nextProbeIndex; // the rolling window's next first probe (m_probeUpdateIdx, DDGINode.h:32)
    uint64_t irrBytes, visBytes, offBytes;
};
static_assert(sizeof(StateHeader) == 88, "state header layout");

StateHeader stateHeaderOf(const ArkDdgiCtx* ctx)
{
    StateHeader h {};
    std::memcpy(h.magic, "ARKDDGI1", 8);
    h.grid[0] = ctx->X;
    h.grid[1] = ctx->Y;
    h.grid[2] = ctx->Z;
    for (int k = 0; k < 3; ++k) {
        h.spacing[k] = ctx->desc.probe_spacing[k];
        h.origin[k] = ctx->desc.offset_to_first[k];
    }
    h.zFar = ctx->desc.z_far;
    h.clearMode = ctx->desc.clear_overflow_mode;
    h.shardRank = ctx->desc.shard_rank;
    h.shardCount = ctx->desc.shard_count;
    h.nextProbeIndex = ctx->nextProbeIndex;
    h.irrBytes = ctx->irr.bytes;
    h.visBytes = ctx->vis.bytes;
    h.offBytes = ctx->offsets.bytes;
    return h;
}
} // namespace

int ark_ddgi_state_size(const ArkDdgiCtx* ctx, uint64_t* outBytes)
{
    if (!ctx || !outBytes) return ARK_DDGI_E_INVALID_ARGUMENT;
    *outBytes = sizeof(StateHeader) + ctx->irr.bytes + ctx->vis.bytes + ctx->offsets.bytes;
    return ARK_DDGI_OK;
}

int ark_ddgi_save_state(ArkDdgiCtx* ctx, void* dst, uint64_t bytes)
{
    if (!ctx || !dst) return ARK_DDGI_E_INVALID_ARGUMENT;
    uint64_t need = 0;
    ark_ddgi_state_size(ctx, &need);
    if (bytes != need) return ctx->fail(ARK_DDGI_E_SIZE_MISMATCH, "state is %llu bytes, got %llu", (unsigned long long)need, (unsigned long long)bytes);
    const StateHeader h = stateHeaderOf(ctx);
    char* o = static_cast<char*>(dst);
    std::memcpy(o, &h, sizeof(h));
    o += sizeof(h);
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    ARK_HIP(hipMemcpy(o, ctx->irr.ptr, ctx->irr.bytes, hipMemcpyDeviceToHost));
    o += ctx->irr.bytes;
    ARK_HIP(hipMemcpy(o, ctx->vis.ptr, ctx->vis.bytes, hipMemcpyDeviceToHost));
    o += ctx->vis.bytes;
    ARK_HIP(hipMemcpy(o, ctx->offsets.ptr, ctx->offsets.bytes, hipMemcpyDeviceToHost));
    return ARK_DDGI_OK;
}

int ark_ddgi_load_state(ArkDdgiCtx* ctx, const void* src, uint64_t bytes)
{
    if (!ctx || !src) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->pipeReady = false; // the next update's traversal waits for this
    uint64_t need = 0;
    ark_ddgi_state_size(ctx, &need);
    if (bytes != need) return ctx->fail(ARK_DDGI_E_SIZE_MISMATCH, "state is %llu bytes, got %llu", (unsigned long long)need, (unsigned long long)bytes);
    StateHeader h;
    std::memcpy(&h, src, sizeof(h));
    StateHeader mine = stateHeaderOf(ctx);
    mine.nextProbeIndex = h.nextProbeIndex; // the window position is state, not geometry
    if (std::memcmp(&h, &mine, sizeof(h)) != 0 || h.nextProbeIndex >= static_cast<uint32_t>(ctx->N))
        return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "state blob is of another grid / zFar / clear mode / shard (or not a DDGI state)");
    const char* i = static_cast<const char*>(src) + sizeof(h);
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    ARK_HIP(hipMemcpy(ctx->irr.ptr, i, ctx->irr.bytes, hipMemcpyHostToDevice));
    i += ctx->irr.bytes;
    ARK_HIP(hipMemcpy(ctx->vis.ptr, i, ctx->vis.bytes, hipMemcpyHostToDevice));
    i += ctx->vis.bytes;
    ARK_HIP(hipMemcpy(ctx->offsets.ptr, i, ctx->offsets.bytes, hipMemcpyHostToDevice));
    ctx->nextProbeIndex = h.nextProbeIndex;
    return ARK_DDGI_OK;
}

int ark_ddgi_get_next_probe_index(const ArkDdgiCtx* ctx, uint32_t* out)
{
    if (!ctx || !out) return ARK_DDGI_E_INVALID_ARGUMENT;
    *out = ctx->nextProbeIndex;
    return ARK_DDGI_OK;
}

int ark_ddgi_get_device_views(ArkDdgiCtx* ctx, ArkDdgiDeviceViews* v)
{
    if (!ctx || !v) return ARK_DDGI_E_INVALID_ARGUMENT;
    std::memset(v, 0, sizeof(*v));
    v->irradiance_atlas = ctx->irr.ptr;
    v->irradiance_bytes = ctx->irr.bytes;
    v->irradiance_width = ctx->Wi;
    v->irradiance_height = ctx->Hi;
    v->visibility_atlas = ctx->vis.ptr;
    v->visibility_bytes = ctx->vis.bytes;
    v->visibility_width = ctx->Wv;
    v->visibility_height = ctx->Hv;
    v->probe_offsets = ctx->offsets.ptr;
    v->probe_offsets_bytes = ctx->offsets.bytes;
    // Z-slab = contiguous texel-row band of both atlases (tile row = z, ddgi/common.glsl:58-61)
    const uint64_t rowI = static_cast<uint64_t>(ctx->Wi) * 8, rowV = static_cast<uint64_t>(ctx->Wv) * 4;
    const int si = ARK_DDGI_IRRADIANCE_RES + 2, sv = ARK_DDGI_VISIBILITY_RES + 2;
    v->irradiance_slab_offset = static_cast<uint64_t>(ctx->slabZ0) * si * rowI;
    v->irradiance_slab_bytes = static_cast<uint64_t>(ctx->slabZ1 - ctx->slabZ0) * si * rowI;
    v->visibility_slab_offset = static_cast<uint64_t>(ctx->slabZ0) * sv * rowV;
    v->visibility_slab_bytes = static_cast<uint64_t>(ctx->slabZ1 - ctx->slabZ0) * sv * rowV;
    return ARK_DDGI_OK;
}

int ark_ddgi_reset_history(ArkDdgiCtx* ctx)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->pipeReady = false; // the next update's traversal waits for this
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    return clearHistory(ctx);
}

int ark_ddgi_set_counting(ArkDdgiCtx* ctx, int enabled)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->counting = enabled != 0;
    if (ctx->counting && !ctx->raySteps.ptr) {
        ARK_HIP(hipSetDevice(ctx->device));
        ARK_HIP(ctx->raySteps.alloc(static_cast<size_t>(ctx->Kmax) * ctx->Rmax * 2));
        ARK_HIP(hipMemset(ctx->raySteps.ptr, 0, ctx->raySteps.bytes));
    }
    return ARK_DDGI_OK;
}

int ark_ddgi_get_counters(ArkDdgiCtx* ctx, ArkDdgiCounters* out)
{
    if (!ctx || !out) return ARK_DDGI_E_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    out->rays = ctx->lastRays;
    out->probes = ctx->lastProbes;
    if (ctx->countersPending) {
        unsigned long long c[8];
        ARK_HIP(hipSetDevice(ctx->device));
        ARK_HIP(hipDeviceSynchronize());
        ARK_HIP(hipMemcpy(c, ctx->counters.ptr, sizeof(c), hipMemcpyDeviceToHost));
        out->primary_node_visits = c[0];
        out->primary_tri_tests = c[1];
        out->hits = c[2];
        out->shadow_rays = c[3];
        out->shadow_node_visits = c[4];
        out->shadow_tri_tests = c[5];
        out->front_hits = c[6];
        out->primary_wave_steps = c[7];
    }
    return ARK_DDGI_OK;
}

int ark_ddgi_set_timing(ArkDdgiCtx* ctx, int enabled)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    ctx->timing = enabled != 0;
    return ARK_DDGI_OK;
}

int ark_ddgi_get_last_timings(ArkDdgiCtx* ctx, float* out, int count)
{
    if (!ctx || !out || count <= 0) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!ctx->timingValid) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "timing not enabled for the last update");
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipEventSynchronize(ctx->ev[3]));
    float ms[5] = {};
    ARK_HIP(hipEventElapsedTime(&ms[0], ctx->ev[0], ctx->ev[3]));
    ARK_HIP(hipEventElapsedTime(&ms[1], ctx->ev[0], ctx->ev[1]));
    // shade = ev5 -> ev2; shadow = (ev1 -> ev5) + (ev2 -> ev4): whichever side of
    // shading the schedule put the shadow rays on (the other interval is ~0)
    float pre = 0.0f, post = 0.0f;
    ARK_HIP(hipEventElapsedTime(&ms[2], ctx->ev[5], ctx->ev[2]));
    ARK_HIP(hipEventElapsedTime(&ms[3], ctx->ev[4], ctx->ev[3]));
    ARK_HIP(hipEventElapsedTime(&pre, ctx->ev[1], ctx->ev[5]));
    ARK_HIP(hipEventElapsedTime(&post, ctx->ev[2], ctx->ev[4]));
    ms[4] = pre + post;
    for (int i = 0; i < count && i < 5; ++i) out[i] = ms[i];
    return ARK_DDGI_OK;
}

int ark_ddgi_get_bvh_stats(ArkDdgiCtx* ctx, ArkDdgiBvhStats* out)
{
    if (!ctx || !out) return ARK_DDGI_E_INVALID_ARGUMENT;
    *out = ctx->hasScene ? ctx->sceneStore->bvhStats : ctx->bvhStats; // the store's: installs and refits of any sharing context
    return ARK_DDGI_OK;
}

// AO / bent-normal bake (include/ark_ddgi.h; BakeAmbientOcclusionNode.cpp:15-131):
// raster -> barycentrics (+ covered-texel list) -> persistent AO rays, one stream.
int ark_ddgi_bake_ao(ArkDdgiCtx* ctx, const ArkBakeAoDesc* d, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!d || d->struct_size != sizeof(ArkBakeAoDesc)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkBakeAoDesc");
    if (!ctx->hasScene) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bake: no scene");
    if (d->instance_index >= ctx->sceneStore->instHost.size()) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bake: instance %u out of range", d->instance_index);
    if (d->width == 0 || d->height == 0 || d->width > 16384 || d->height > 16384 || d->sample_count == 0)
        return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bake: extent %ux%u / %u samples", d->width, d->height, d->sample_count);
    const ArkRTInstance& inst = ctx->sceneStore->instHost[d->instance_index];
    const ArkRTTriangleMesh& mesh = ctx->sceneStore->meshHost[inst.rt_mesh_index];
    const hipStream_t s = streamOf(hipStream);
    ARK_HIP(hipSetDevice(ctx->device));
    if (ctx->sceneVersion != ctx->sceneStore->version) // a sharing context refitted the scene or installed a deeper sun BVH
        if (const int rc = refreshScene(ctx)) return rc;
    ARK_HIP(orderBegin(ctx, s));
    const size_t texels = static_cast<size_t>(d->width) * d->height;
    const size_t outBytes = texels * (d->bent_normals ? 4 : 1);
    if (ctx->bakeTri.bytes < texels * 4) ARK_HIP(ctx->bakeTri.alloc(texels * 4));
    if (ctx->bakeBary.bytes < texels * 8) ARK_HIP(ctx->bakeBary.alloc(texels * 8));
    if (ctx->bakeOut.bytes < outBytes) ARK_HIP(ctx->bakeOut.alloc(outBytes));
    if (ctx->bakePixels.bytes < texels * 4) ARK_HIP(ctx->bakePixels.alloc(texels * 4));
    if (ctx->bakeCounters.bytes < 256) ARK_HIP(ctx->bakeCounters.alloc(256));
    ARK_HIP(hipMemsetAsync(ctx->bakeTri.ptr, 0, texels * 4, s)); // ClearValue::blackAtMaxDepth
    ARK_HIP(hipMemsetAsync(ctx->bakeCounters.ptr, 0, 256, s));
    BakeArgs b {};
    b.W = d->width;
    b.H = d->height;
    b.samples = d->sample_count;
    b.tri_count = inst.triangle_count;
    b.bent = d->bent_normals ? 1 : 0;
    b.first_index = static_cast<uint32_t>(mesh.first_index);
    b.first_vertex = static_cast<uint32_t>(mesh.first_vertex);
    b.indices = ctx->sceneStore->indices.as<uint32_t>();
    b.positions = ctx->sceneStore->positions.as<float>();
    b.vertices = ctx->sceneStore->vertices.as<float>();
    b.tri_idx = ctx->bakeTri.as<uint32_t>();
    b.bary = ctx->bakeBary.as<uint16_t>();
    b.out = ctx->bakeOut.as<uint8_t>();
    b.pixels = ctx->bakePixels.as<uint32_t>();
    b.counters = ctx->bakeCounters.as<uint32_t>();
    b.spill = ctx->spill.as<uint32_t>();
    if (b.tri_count > 0) ARK_HIP(launch_bake(ctx->scene, b, 0, 0, s));
    ARK_HIP(launch_bake(ctx->scene, b, 0, 1, s));
    // the persistent AO kernel uses the traversal spill area sized for shadowBlocks workgroups
    ARK_HIP(launch_bake(ctx->scene, b, ctx->shadowBlocks, 2, s));
    ARK_HIP(orderEnd(ctx, s));
    ctx->bakeW = d->width;
    ctx->bakeH = d->height;
    ctx->bakeBent = b.bent;
    return ARK_DDGI_OK;
}

int ark_ddgi_bake_read(ArkDdgiCtx* ctx, int which, void* dst, uint64_t bytes)
{
    if (!ctx || !dst) return ARK_DDGI_E_INVALID_ARGUMENT;
    const size_t texels = static_cast<size_t>(ctx->bakeW) * ctx->bakeH;
    const void* src = nullptr;
    size_t n = 0;
    switch (which) {
    case ARK_BAKE_TRIANGLE_INDEX: src = ctx->bakeTri.ptr; n = texels * 4; break;
    case ARK_BAKE_BARYCENTRICS: src = ctx->bakeBary.ptr; n = texels * 8; break;
    case ARK_BAKE_OUTPUT: src = ctx->bakeOut.ptr; n = texels * (ctx->bakeBent ? 4 : 1); break;
    default: return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bake_read: unknown resource %d", which);
    }
    if (texels == 0) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bake_read: no bake yet");
    if (bytes != n) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bake_read: %llu bytes, resource has %zu", static_cast<unsigned long long>(bytes), n);
    ARK_HIP(hipSetDevice(ctx->device));
    ARK_HIP(hipDeviceSynchronize());
    ARK_HIP(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
    return ARK_DDGI_OK;
}

int ark_ddgi_lighting_compose(ArkDdgiCtx* ctx, const ArkComposeDesc* desc, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!desc || desc->struct_size != sizeof(ArkComposeDesc)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkComposeDesc");
    if (!desc->out) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "lighting_compose: no output plane");
    if (static_cast<uint64_t>(desc->width) * desc->height >= (1ull << 32)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "lighting_compose: target too large");
    const hipStream_t s = streamOf(hipStream);
    ARK_HIP(hipSetDevice(ctx->device));
    // the DDGISamplingSet (DDGINode.cpp:45-66): grid constants + both atlases
    FrameArgs f {};
    f.X = ctx->X; f.Y = ctx->Y; f.Z = ctx->Z;
    f.Wi = ctx->Wi; f.Hi = ctx->Hi; f.Wv = ctx->Wv; f.Hv = ctx->Hv;
    for (int k = 0; k < 3; ++k) {
        f.spacing[k] = ctx->desc.probe_spacing[k];
        f.origin[k] = ctx->desc.offset_to_first[k];
    }
    f.irr = ctx->irr.as<uint16_t>();
    f.vis = ctx->vis.as<uint16_t>();
    ArkComposeDesc c = *desc;
    ARK_HIP(orderBegin(ctx, s));
    ARK_HIP(launch_lighting_compose(f, c, s));
    ARK_HIP(orderEnd(ctx, s));
    return ARK_DDGI_OK;
}

int ark_ddgi_rt_reflections(ArkDdgiCtx* ctx, const ArkReflectionsDesc* desc, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!desc || desc->struct_size != sizeof(ArkReflectionsDesc)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkReflectionsDesc");
    if (!ctx->hasScene) return ctx->fail(ARK_DDGI_E_NO_SCENE, "rt_reflections before ark_ddgi_set_scene");
    if (!desc->out_radiance || !desc->out_direction) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "rt_reflections: no output image");
    if (desc->blue_noise && (desc->noise_width == 0 || desc->noise_height == 0)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "rt_reflections: empty blue noise");
    if (static_cast<uint64_t>(desc->width) * desc->height >= (1ull << 32)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "rt_reflections: target too large");
    const hipStream_t s = streamOf(hipStream);
    ARK_HIP(hipSetDevice(ctx->device));
    int rc;
    // the scene first: a sharing context's deeper sun BVH may grow,
    // i.e. reallocate, the spill area that f.spill points into below
    if (ctx->sceneVersion != ctx->sceneStore->version) {
        if ((rc = refreshScene(ctx)) != 0) return rc;
    } else if ((rc = ensureSpill(ctx)) != 0) {
        return rc;
    }
    FrameArgs f {};
    f.X = ctx->X; f.Y = ctx->Y; f.Z = ctx->Z;
    f.Wi = ctx->Wi; f.Hi = ctx->Hi; f.Wv = ctx->Wv; f.Hv = ctx->Hv;
    for (int k = 0; k < 3; ++k) {
        f.spacing[k] = ctx->desc.probe_spacing[k];
        f.origin[k] = ctx->desc.offset_to_first[k];
    }
    f.irr = ctx->irr.as<uint16_t>();
    f.vis = ctx->vis.as<uint16_t>();
    f.z_far = ctx->desc.z_far;
    f.ambient_amount = desc->ambient_amount;
    f.environment_multiplier = desc->environment_multiplier;
    f.spill = ctx->spill.as<uint32_t>();
    // ray-list work set (ensureReflWork): rays, hit records, light bits, shadow rays, counters
    const uint64_t pixels = static_cast<uint64_t>(desc->width) * desc->height;
    if (pixels == 0) return ARK_DDGI_OK;
    if ((rc = ensureReflWork(ctx, pixels)) != 0) return rc;
    {
        char* w = static_cast<char*>(ctx->reflWork.ptr);
        auto take = [&](uint64_t bytes) {
            char* q = w;
            w += (bytes + 255) & ~static_cast<uint64_t>(255);
            return q;
        };
        f.ray_list = reinterpret_cast<const float4*>(take(pixels * 32));
        f.hits = reinterpret_cast<GpuHit*>(take(pixels * sizeof(GpuHit)));
        f.shadow_bits = reinterpret_cast<uint32_t*>(take(pixels * 4));
        f.ray_counter = reinterpret_cast<uint32_t*>(take((kRayCounterWords + kRayCounterStride) * 4));
        f.shadow_rays = reinterpret_cast<ShadowRay*>(take(pixels * ctx->lightCount * sizeof(ShadowRay)));
    }
    f.shadow_count = f.ray_counter + kShadowCountWord;
    f.shadow_heads = f.ray_counter + kShadowHeadWord;
    f.list_count = f.ray_counter + kRayCounterWords;
    f.light_count = ctx->lightCount;
    f.refill_min = ctx->refillMin;
    f.sun_refill_min = ctx->sunRefillMin;
    f.grab_chunk = ctx->grabChunk;
    f.counters = ctx->counters.as<unsigned long long>();
    ARK_HIP(orderBegin(ctx, s));
    ARK_HIP(flushLights(ctx, s));
    ARK_HIP(hipMemsetAsync(f.ray_counter, 0, (kRayCounterWords + kRayCounterStride) * 4, s));
    ARK_HIP(launch_rt_reflections(ctx->scene, f, *desc, ctx->traceBlocks, shadowBlocksFor(ctx, pixels), s));
    ARK_HIP(orderEnd(ctx, s));
    return ARK_DDGI_OK;
}

int ark_ddgi_probe_debug(ArkDdgiCtx* ctx, const ArkProbeDebugDesc* desc, void* hipStream)
{
    if (!ctx) return ARK_DDGI_E_INVALID_ARGUMENT;
    if (!desc || desc->struct_size != sizeof(ArkProbeDebugDesc)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "bad ArkProbeDebugDesc");
    if (desc->count && (!desc->probe_indices || !desc->directions || !desc->out)) return ctx->fail(ARK_DDGI_E_INVALID_ARGUMENT, "probe_debug: null plane");
    const hipStream_t s = streamOf(hipStream);
    ARK_HIP(hipSetDevice(ctx->device));
    FrameArgs f {};
    f.X = ctx->X; f.Y = ctx->Y; f.Z = ctx->Z;
    f.Wi = ctx->Wi; f.Hi = ctx->Hi; f.Wv = ctx->Wv; f.Hv = ctx->Hv;
    for (int k = 0; k < 3; ++k) {
        f.spacing[k] = ctx->desc.probe_spacing[k];
        f.origin[k] = ctx->desc.offset_to_first[k];
    }
    f.irr = ctx->irr.as<uint16_t>();
    f.vis = ctx->vis.as<uint16_t>();
    ARK_HIP(orderBegin(ctx, s));
    ARK_HIP(launch_probe_debug(f, *desc, s));
    ARK_HIP(orderEnd(ctx, s));
    return ARK_DDGI_OK;
}

} // extern "C"
