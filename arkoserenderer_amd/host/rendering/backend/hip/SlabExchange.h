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
#include <string>
#include <vector>

#include "../../../../../include/ark_ddgi.h"

// Band geometry of one context's atlases under P ranks.
struct SlabBands {
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
    virtual const char* name() const = 0;
};

// One process per GPU: ncclAllGather (RCCL over xGMI) of each band in place, on a
// side stream of this rank's device. Both calls in one ncclGroup.
class RcclSlabExchange final : public SlabExchange {
public:
    // `uniqueId` = the 128-byte ncclUniqueId all ranks share (rank 0 creates it,
    // createUniqueId); the communicator is created here (ncclCommInitRank).
    RcclSlabExchange(int device, int rank, int world, const void* uniqueId, const SlabBands& bands);
    ~RcclSlabExchange() override;
    bool ok() const { return m_ok; }
    const std::string& error() const { return m_error; }
    void* exchange(int rank, void* updateDone) override;
    const char* name() const override { return "rccl"; }
    static bool createUniqueId(std::vector<uint8_t>& out);

private:
    int m_rank;
    SlabBands m_bands;
    void* m_comm { nullptr };
    void* m_stream { nullptr };
    void* m_done { nullptr };
    bool m_ok { false };
    std::string m_error;
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
    const char* name() const override { return "device-copy"; }

private:
    std::vector<SlabBands> m_ranks;
    std::vector<void*> m_ready;
    int m_arrived { 0 };
    void* m_stream { nullptr };
    void* m_done { nullptr };
};
