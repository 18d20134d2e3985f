#include "SlabExchange.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "core/Logging.h"

bool SlabBands::fromContext(ArkDdgiCtx* ctx, int rank, int world, SlabBands& out, std::string& error)
{
    ArkDdgiDeviceViews v {};
    if (ark_ddgi_get_device_views(ctx, &v) != ARK_DDGI_OK) {
        error = std::string("ark_ddgi_get_device_views: ") + ark_ddgi_last_error(ctx);
        return false;
    }
    // the context's own slab: equal bands (Z a multiple of P), band r at r * band
    if (world <= 0 || v.irradiance_slab_bytes == 0 || v.irradiance_slab_bytes * world != v.irradiance_bytes ||
        v.visibility_slab_bytes * world != v.visibility_bytes || v.irradiance_slab_offset != rank * v.irradiance_slab_bytes ||
        v.visibility_slab_offset != rank * v.visibility_slab_bytes) {
        error = "the context's Z-slab bands are not rank " + std::to_string(rank) + " of " + std::to_string(world) + " equal bands";
        return false;
    }
    out.irradiance = static_cast<uint8_t*>(v.irradiance_atlas);
    out.visibility = static_cast<uint8_t*>(v.visibility_atlas);
    out.irradianceBand = v.irradiance_slab_bytes;
    out.visibilityBand = v.visibility_slab_bytes;
    return true;
}

// --- RCCL ------------------------------------------------------------------------

bool RcclSlabExchange::createUniqueId(std::vector<uint8_t>& out)
{
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return false;
    out.assign(reinterpret_cast<const uint8_t*>(&id), reinterpret_cast<const uint8_t*>(&id) + sizeof(id));
    return true;
}

RcclSlabExchange::RcclSlabExchange(int device, int rank, int world, const void* uniqueId, const SlabBands& bands)
    : m_rank(rank), m_bands(bands)
{
    if (hipSetDevice(device) != hipSuccess) {
        m_error = "hipSetDevice failed";
        return;
    }
    ncclUniqueId id;
    std::memcpy(&id, uniqueId, sizeof(id));
    ncclComm_t comm = nullptr;
    if (ncclResult_t r = ncclCommInitRank(&comm, world, id, rank); r != ncclSuccess) {
        m_error = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        return;
    }
    m_comm = comm;
    hipStream_t s;
    hipEvent_t e;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        m_error = "side stream / event creation failed";
        return;
    }
    m_stream = s;
    m_done = e;
    m_ok = true;
}

RcclSlabExchange::~RcclSlabExchange()
{
    if (m_stream) (void)hipStreamSynchronize(static_cast<hipStream_t>(m_stream));
    if (m_comm) (void)ncclCommDestroy(static_cast<ncclComm_t>(m_comm));
    if (m_done) (void)hipEventDestroy(static_cast<hipEvent_t>(m_done));
    if (m_stream) (void)hipStreamDestroy(static_cast<hipStream_t>(m_stream));
}

void* RcclSlabExchange::exchange(int rank, void* updateDone)
{
    if (!m_ok || rank != m_rank) {
        ARKOSE_LOG(Error, "RcclSlabExchange: not usable (%s)", m_ok ? "wrong rank" : m_error.c_str());
        return nullptr;
    }
    const hipStream_t s = static_cast<hipStream_t>(m_stream);
    const ncclComm_t comm = static_cast<ncclComm_t>(m_comm);
    if (updateDone) (void)hipStreamWaitEvent(s, static_cast<hipEvent_t>(updateDone), 0);
    // in place: this rank's band already sits at recvbuff + rank * count
    ncclResult_t r = ncclGroupStart();
    if (r == ncclSuccess)
        r = ncclAllGather(m_bands.irradiance + m_rank * m_bands.irradianceBand, m_bands.irradiance, m_bands.irradianceBand, ncclUint8, comm, s);
    if (r == ncclSuccess)
        r = ncclAllGather(m_bands.visibility + m_rank * m_bands.visibilityBand, m_bands.visibility, m_bands.visibilityBand, ncclUint8, comm, s);
    const ncclResult_t g = ncclGroupEnd();
    if (r != ncclSuccess || g != ncclSuccess) {
        ARKOSE_LOG(Error, "RcclSlabExchange: all-gather failed: %s", ncclGetErrorString(r != ncclSuccess ? r : g));
        return nullptr;
    }
    (void)hipEventRecord(static_cast<hipEvent_t>(m_done), s);
    return m_done;
}

// --- device copies (one process, one GPU) ----------------------------------------

DeviceCopySlabExchange::DeviceCopySlabExchange(std::vector<SlabBands> ranks)
    : m_ranks(std::move(ranks)), m_ready(m_ranks.size(), nullptr)
{
    hipStream_t s;
    hipEvent_t e;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess || hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        ARKOSE_LOG(Fatal, "DeviceCopySlabExchange: side stream / event creation failed");
    m_stream = s;
    m_done = e;
}

DeviceCopySlabExchange::~DeviceCopySlabExchange()
{
    (void)hipStreamSynchronize(static_cast<hipStream_t>(m_stream));
    (void)hipEventDestroy(static_cast<hipEvent_t>(m_done));
    (void)hipStreamDestroy(static_cast<hipStream_t>(m_stream));
}

void* DeviceCopySlabExchange::exchange(int rank, void* updateDone)
{
    m_ready[rank] = updateDone;
    if (++m_arrived < static_cast<int>(m_ranks.size())) return m_done; // recorded when the last rank arrives
    m_arrived = 0;
    const hipStream_t s = static_cast<hipStream_t>(m_stream);
    for (void* e : m_ready)
        if (e) (void)hipStreamWaitEvent(s, static_cast<hipEvent_t>(e), 0);
    const size_t P = m_ranks.size();
    for (size_t src = 0; src < P; ++src)
        for (size_t dst = 0; dst < P; ++dst) {
            if (src == dst) continue;
            const SlabBands& a = m_ranks[src];
            const SlabBands& b = m_ranks[dst];
            (void)hipMemcpyAsync(b.irradiance + src * a.irradianceBand, a.irradiance + src * a.irradianceBand, a.irradianceBand, hipMemcpyDeviceToDevice, s);
            (void)hipMemcpyAsync(b.visibility + src * a.visibilityBand, a.visibility + src * a.visibilityBand, a.visibilityBand, hipMemcpyDeviceToDevice, s);
        }
    (void)hipEventRecord(static_cast<hipEvent_t>(m_done), s);
    return m_done;
}
