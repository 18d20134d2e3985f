// SlabExchange.h — the Z-slab ranks' atlas exchange.
//
// Rank r of P owns probe layers z in [r Z/P, (r+1) Z/P): a contiguous texel-row band
// of both atlases (tile row = probe z, ddgi/common.glsl:58-61). After each update
// every rank needs every band, because the next frame's indirect lookup samples the
// previous atlases at arbitrary hit points (probeSampling.glsl:64-163): the exchange
// is an in-place all-gather of the two bands. It runs on a side stream: the next
// frame's slot table and traversal do not read the atlases and go ahead; its shading
// waits for the event exchange() returns (ark_ddgi_update_overlapped).
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../../../../include/ark_ddgi.h"

// Band geometry of one context's atlases under P ranks.
struct SlabBands {
    ArkDdgiCtx* ctx { nullptr }; // the windowed exchange packs / unpacks through it
    uint8_t* irradiance { nullptr };
    uint8_t* visibility { nullptr };
    size_t irradianceBand { 0 };  // bytes of one rank's band
    size_t visibilityBand { 0 };
    // From the context of rank `rank` of `world` (ark_ddgi_get_device_views' slab
    // offsets); false (and `error` set) unless the bands are equal (Z a multiple of P).
    static bool fromContext(ArkDdgiCtx* ctx, int rank, int world, SlabBands& out, std::string& error);
};

class SlabExchange {
public:
    virtual ~SlabExchange() = default;
    // Enqueues this rank's share of the exchange of the update that `updateDone`
    // completes. Returns the event the next update's shading waits on.
    virtual void* exchange(int rank, void* updateDone) = 0;
    // false while the event exchange() returned to `rank` for the current frame is not
    // recorded yet: an update of the next frame must not be enqueued until it is
    virtual bool readyForNextUpdate(int rank) const { (void)rank; return true; }
    // Waits (bounded) until every exchange enqueued so far has completed.
    virtual bool drain() { return true; }
    virtual const char* name() const = 0;
};

// Failure detection of the exchange (ncclCommGetAsyncError polling in
// multi-GPU mode). A dead or stuck peer would otherwise hang every rank forever: the
// shading of the next frame waits on the all-gather's event on the device, and the
// host blocks at the next synchronisation. wait() polls the exchange's completion
// event and the communicator's asynchronous error until a deadline; on an error or
// at the deadline it calls the failure handler, whose default aborts the
// communicator (ncclCommAbort), logs an Error and ends the process with
// kExchangeFailureExitCode (the reference's ARKOSE_LOG(Fatal) -> exit convention,
// arkcore/core/Logging.h:87; no re-exec).
class ExchangeWatchdog {
public:
    static constexpr int kExchangeFailureExitCode = 14;
    // (what failed) -> the handler; after it returns, wait() returns false
    using FailureHandler = std::function<void(const std::string&)>;
    // timeout from ARK_EXCHANGE_TIMEOUT_S (seconds, default 120) unless given (> 0)
    explicit ExchangeWatchdog(double timeoutSeconds = 0.0);
    double timeoutSeconds() const { return m_timeout; }
    void setFailureHandler(FailureHandler h) { m_onFailure = std::move(h); }
    // true when `hipEvent` completed; polls ncclCommGetAsyncError(`ncclComm`) meanwhile
    // (null comm: event only). `what` names the wait in the log.
    bool wait(void* hipEvent, void* ncclComm, const char* what);
    // the default failure: ncclCommAbort (if a comm), an Error log, process exit
    [[noreturn]] static void abortAndExit(void* ncclComm, const std::string& why);

private:
    void fail(void* ncclComm, const std::string& why);
    double m_timeout;
    FailureHandler m_onFailure;
};

// One process per GPU: ncclAllGather (RCCL over xGMI) of each band in place, on a
// side stream of this rank's device. Both calls in one ncclGroup. When the update's
// window did not cover the grid (K < N: ark_ddgi_window_exchange_info), only the tiles
// it wrote travel: ark_ddgi_pack_window into this rank's region of a receive buffer,
// one ncclAllGather of the packets, ark_ddgi_unpack_window (ark_ddgi.h).
class RcclSlabExchange final : public SlabExchange {
public:
    // `uniqueId` = the 128-byte ncclUniqueId all ranks share (rank 0 creates it,
    // createUniqueId); the communicator is created here (ncclCommInitRank).
    RcclSlabExchange(int device, int rank, int world, const void* uniqueId, const SlabBands& bands, double timeoutSeconds = 0.0);
    ~RcclSlabExchange() override;
    bool ok() const { return m_ok; }
    const std::string& error() const { return m_error; }
    // Frame n's all-gather first waits (bounded, on the host) for frame n - kRing's:
    // the host runs at most kRing exchanges ahead of the device, and a peer that stops
    // answering ends the process at the deadline instead of hanging it. kRing = 3:
    // with 2, frame n - 2's exchange ends only after frame n - 2's update, and the host
    // enqueued frame n's traversal after the traversal stream had gone idle.
    void* exchange(int rank, void* updateDone) override;
    bool drain() override;
    const char* name() const override { return "rccl"; }
    ExchangeWatchdog& watchdog() { return m_watchdog; }
    // the side stream the all-gathers run on (hipStream_t) and the communicator
    void* stream() const { return m_stream; }
    void* comm() const { return m_comm; }
    static bool createUniqueId(std::vector<uint8_t>& out);

private:
    int m_rank;
    SlabBands m_bands;
    void* m_comm { nullptr };
    void* m_stream { nullptr };
    static constexpr uint32_t kRing = 3;
    void* m_done[kRing] {}; // completion of frame n in slot n % kRing
    uint64_t m_frames { 0 };
    int m_world { 1 };
    uint8_t* m_recv { nullptr }; // windowed exchange: world x bytes_per_rank
    size_t m_recvBytes { 0 };
    bool m_ok { false };
    std::string m_error;
    ExchangeWatchdog m_watchdog;
};

// P contexts in one process (the one-GPU test harness): the same band exchange as
// device-to-device copies on one side stream, issued when the last rank of a frame
// arrives, after every rank's update. Ranks must call exchange() once per frame, in
// any order, and start no update of the next frame before the last call.
class DeviceCopySlabExchange final : public SlabExchange {
public:
    explicit DeviceCopySlabExchange(std::vector<SlabBands> ranks);
    ~DeviceCopySlabExchange() override;
    void* exchange(int rank, void* updateDone) override;
    // a rank that already arrived at a frame the others have not finished may not
    // update again: its next shading would wait on the previous frame's record
    bool readyForNextUpdate(int rank) const override { return !m_hasArrived[rank]; }
    bool drain() override;
    const char* name() const override { return "device-copy"; }

private:
    std::vector<SlabBands> m_ranks;
    uint8_t* m_recv { nullptr }; // windowed exchange: every rank's packets
    size_t m_recvBytes { 0 };
    std::vector<void*> m_ready;
    std::vector<bool> m_hasArrived;
    int m_arrived { 0 };
    ExchangeWatchdog m_watchdog;
    void* m_stream { nullptr };
    void* m_done { nullptr };
};
