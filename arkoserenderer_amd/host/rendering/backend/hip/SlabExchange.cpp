#include "SlabExchange.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "core/Logging.h"

// --- failure detection -----------------------------------------------------------

ExchangeWatchdog::ExchangeWatchdog(double timeoutSeconds)
    : m_timeout(timeoutSeconds)
{
    if (m_timeout <= 0.0) {
        const char* e = std::getenv("ARK_EXCHANGE_TIMEOUT_S");
        m_timeout = e ? std::atof(e) : 0.0;
        if (m_timeout <= 0.0) m_timeout = 120.0;
    }
}

bool ExchangeWatchdog::wait(void* hipEvent, void* ncclComm, const char* what)
{
    const auto t0 = std::chrono::steady_clock::now();
    auto sleepFor = std::chrono::microseconds(10);
    for (;;) {
        const hipError_t q = hipEventQuery(static_cast<hipEvent_t>(hipEvent));
        if (q == hipSuccess) return true;
        if (q != hipErrorNotReady) {
            fail(ncclComm, std::string(what) + ": hipEventQuery: " + hipGetErrorString(q));
            return false;
        }
        if (ncclComm) {
            ncclResult_t async = ncclSuccess;
            const ncclResult_t r = ncclCommGetAsyncError(static_cast<ncclComm_t>(ncclComm), &async);
            if (r != ncclSuccess || (async != ncclSuccess && async != ncclInProgress)) {
                fail(ncclComm, std::string(what) + ": communicator error: " + ncclGetErrorString(r != ncclSuccess ? r : async));
                return false;
            }
        }
        const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (waited > m_timeout) {
            char buf[96];
            std::snprintf(buf, sizeof(buf), ": not complete after %.3f s (deadline %.3f s)", waited, m_timeout);
            fail(ncclComm, std::string(what) + buf);
            return false;
        }
        std::this_thread::sleep_for(sleepFor);
        // capped at 0.1 ms: a longer sleep overshoots the event by up to its own length
        sleepFor = std::min(sleepFor * 2, std::chrono::microseconds(100));
    }
}

void ExchangeWatchdog::fail(void* ncclComm, const std::string& why)
{
    if (m_onFailure) {
        m_onFailure(why);
        return;
    }
    abortAndExit(ncclComm, why);
}

void ExchangeWatchdog::abortAndExit(void* ncclComm, const std::string& why)
{
    // abort first: the communicator's pending operations are cancelled and peers
    // blocked on this rank see an error instead of waiting forever
    if (ncclComm) (void)ncclCommAbort(static_cast<ncclComm_t>(ncclComm));
    ARKOSE_LOG(Error, "Z-slab exchange failed, exiting: %s", why.c_str());
    std::fflush(stderr);
    std::fflush(stdout);
    std::_Exit(kExchangeFailureExitCode);
}

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
    out.ctx = ctx;
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

// A receive buffer of at least `bytes` (grown once the exchanges using it are done)
static bool ensureRecv(uint8_t*& buf, size_t& have, size_t bytes, hipStream_t s)
{
    if (have >= bytes) return true;
    if (buf) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(buf);
        buf = nullptr;
        have = 0;
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return false;
    buf = static_cast<uint8_t*>(p);
    have = bytes;
    return true;
}

RcclSlabExchange::RcclSlabExchange(int device, int rank, int world, const void* uniqueId, const SlabBands& bands, double timeoutSeconds)
    : m_rank(rank), m_bands(bands), m_world(world), m_watchdog(timeoutSeconds)
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
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        m_error = "side stream creation failed";
        return;
    }
    m_stream = s;
    for (void*& slot : m_done) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            m_error = "event creation failed";
            return;
        }
        slot = e;
    }
    m_ok = true;
}

RcclSlabExchange::~RcclSlabExchange()
{
    // bounded: a stuck exchange ends the process through the watchdog
    if (m_ok) (void)drain();
    if (m_stream) (void)hipStreamSynchronize(static_cast<hipStream_t>(m_stream));
    if (m_comm) (void)ncclCommDestroy(static_cast<ncclComm_t>(m_comm));
    if (m_recv) (void)hipFree(m_recv);
    for (void* e : m_done)
        if (e) (void)hipEventDestroy(static_cast<hipEvent_t>(e));
    if (m_stream) (void)hipStreamDestroy(static_cast<hipStream_t>(m_stream));
}

bool RcclSlabExchange::drain()
{
    if (!m_ok || m_frames == 0) return m_ok;
    return m_watchdog.wait(m_done[(m_frames - 1) % kRing], m_comm, "RcclSlabExchange drain");
}

void* RcclSlabExchange::exchange(int rank, void* updateDone)
{
    if (!m_ok || rank != m_rank) {
        ARKOSE_LOG(Error, "RcclSlabExchange: not usable (%s)", m_ok ? "wrong rank" : m_error.c_str());
        return nullptr;
    }
    const hipStream_t s = static_cast<hipStream_t>(m_stream);
    const ncclComm_t comm = static_cast<ncclComm_t>(m_comm);
    void* const slot = m_done[m_frames % kRing];
    // frame n - kRing's all-gather (the last record of this slot) must be complete
    if (m_frames >= kRing && !m_watchdog.wait(slot, m_comm, "RcclSlabExchange frame n-3")) return nullptr;
    if (updateDone) (void)hipStreamWaitEvent(s, static_cast<hipEvent_t>(updateDone), 0);
    ArkDdgiWindowExchange w {};
    if (!m_bands.ctx || ark_ddgi_window_exchange_info(m_bands.ctx, &w) != ARK_DDGI_OK) w.full_bands = 1;
    if (w.full_bands) {
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
    } else if (w.bytes_per_rank) {
        // the window's tiles only: pack, one all-gather of the packets, unpack
        const size_t n = w.bytes_per_rank;
        if (!ensureRecv(m_recv, m_recvBytes, n * m_world, s)) {
            ARKOSE_LOG(Error, "RcclSlabExchange: receive buffer of %zu bytes", n * m_world);
            return nullptr;
        }
        if (ark_ddgi_pack_window(m_bands.ctx, m_recv + m_rank * n, n, s) != ARK_DDGI_OK) {
            ARKOSE_LOG(Error, "RcclSlabExchange: ark_ddgi_pack_window: %s", ark_ddgi_last_error(m_bands.ctx));
            return nullptr;
        }
        if (const ncclResult_t r = ncclAllGather(m_recv + m_rank * n, m_recv, n, ncclUint8, comm, s); r != ncclSuccess) {
            ARKOSE_LOG(Error, "RcclSlabExchange: all-gather failed: %s", ncclGetErrorString(r));
            return nullptr;
        }
        if (ark_ddgi_unpack_window(m_bands.ctx, m_recv, n * m_world, s) != ARK_DDGI_OK) {
            ARKOSE_LOG(Error, "RcclSlabExchange: ark_ddgi_unpack_window: %s", ark_ddgi_last_error(m_bands.ctx));
            return nullptr;
        }
    }
    (void)hipEventRecord(static_cast<hipEvent_t>(slot), s);
    ++m_frames;
    return slot;
}

// --- device copies (one process, one GPU) ----------------------------------------

DeviceCopySlabExchange::DeviceCopySlabExchange(std::vector<SlabBands> ranks)
    : m_ranks(std::move(ranks)), m_ready(m_ranks.size(), nullptr), m_hasArrived(m_ranks.size(), false)
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
    if (m_recv) (void)hipFree(m_recv);
    (void)hipEventDestroy(static_cast<hipEvent_t>(m_done));
    (void)hipStreamDestroy(static_cast<hipStream_t>(m_stream));
}

bool DeviceCopySlabExchange::drain()
{
    return m_watchdog.wait(m_done, nullptr, "DeviceCopySlabExchange drain");
}

void* DeviceCopySlabExchange::exchange(int rank, void* updateDone)
{
    if (m_hasArrived[rank]) ARKOSE_LOG(Fatal, "DeviceCopySlabExchange: rank %d exchanged twice in one frame", rank);
    m_ready[rank] = updateDone;
    m_hasArrived[rank] = true;
    if (++m_arrived < static_cast<int>(m_ranks.size())) return m_done; // recorded when the last rank arrives
    m_arrived = 0;
    std::fill(m_hasArrived.begin(), m_hasArrived.end(), false);
    const hipStream_t s = static_cast<hipStream_t>(m_stream);
    for (void* e : m_ready)
        if (e) (void)hipStreamWaitEvent(s, static_cast<hipEvent_t>(e), 0);
    const size_t P = m_ranks.size();
    ArkDdgiWindowExchange w {};
    if (!m_ranks[0].ctx || ark_ddgi_window_exchange_info(m_ranks[0].ctx, &w) != ARK_DDGI_OK) w.full_bands = 1;
    if (!w.full_bands) {
        // the windowed exchange: every rank packs into its region, every rank unpacks
        const size_t n = w.bytes_per_rank;
        if (n && !ensureRecv(m_recv, m_recvBytes, n * P, s)) ARKOSE_LOG(Fatal, "DeviceCopySlabExchange: receive buffer of %zu bytes", n * P);
        for (size_t r = 0; n && r < P; ++r)
            if (ark_ddgi_pack_window(m_ranks[r].ctx, m_recv + r * n, n, s) != ARK_DDGI_OK)
                ARKOSE_LOG(Fatal, "DeviceCopySlabExchange: ark_ddgi_pack_window: %s", ark_ddgi_last_error(m_ranks[r].ctx));
        for (size_t r = 0; n && r < P; ++r)
            if (ark_ddgi_unpack_window(m_ranks[r].ctx, m_recv, n * P, s) != ARK_DDGI_OK)
                ARKOSE_LOG(Fatal, "DeviceCopySlabExchange: ark_ddgi_unpack_window: %s", ark_ddgi_last_error(m_ranks[r].ctx));
        (void)hipEventRecord(static_cast<hipEvent_t>(m_done), s);
        return m_done;
    }
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
