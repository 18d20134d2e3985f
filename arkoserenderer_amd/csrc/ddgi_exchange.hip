// ddgi_exchange.hip — the windowed Z-slab exchange's pack and unpack (SURVEY §8e option
// (a); VERDICT r05 "do this" #2). With a rolling window (K < N, DDGINode.cpp:138-140) a
// rank's update writes only the tiles of its window probes, so instead of the whole row
// band it contributes one packet per updated probe: the probe's irradiance tile (10 x 10
// RGBA16F texels incl. its border, 800 B) and visibility tile (18 x 18 RG16F, 1,296 B),
// 2,096 B. Every rank knows every rank's packet order without any index exchange: the
// window (first, K) is the same on all ranks, and a probe's slot among its slab's window
// probes is slabRankOf (the closed form k_probe_slots uses). The packets of all ranks
// are all-gathered (equal counts: padded to the largest slab share), then each rank
// writes the other slabs' packets into their tiles.
//
//   k_window_pack    one wave per window position: a probe of this rank's slab copies its
//                    two tiles (524 dwords) into its packet slot
//   k_window_unpack  one wave per window position: a probe of another rank's slab copies
//                    its packet from that rank's region into its tiles
// HBM-bound copies (2 x 2,096 B per probe moved), coalesced 4-byte lanes over each tile
// row; the atlases keep their layout (DDGINode.cpp:262-281).
#include <hip/hip_runtime.h>

#include "ddgi_kernels.h"

namespace ark {
namespace dev {

template<bool kUnpack>
__global__ void __launch_bounds__(64) k_window_pack(WindowExchangeArgs a)
{
    const uint32_t i = blockIdx.x; // window position
    const uint32_t p = (a.first + i) % a.N;
    const uint32_t x = p % a.X, z = (p % (a.X * a.Z)) / a.X, y = p / (a.X * a.Z);
    const uint32_t owner = z / a.slabDepth;
    if (kUnpack ? owner == a.rank : owner != a.rank) return;
    const uint32_t z0 = owner * a.slabDepth;
    const uint32_t slot = slabRankOf(a.X, a.Y, a.Z, z0, z0 + a.slabDepth, a.first, i);
    uint32_t* pkt = reinterpret_cast<uint32_t*>(a.buf + (kUnpack ? owner * a.bytesPerRank : 0ull) + static_cast<uint64_t>(slot) * kWindowPacketBytes);
    constexpr uint32_t ti = ARK_DDGI_IRRADIANCE_RES + 2 * ARK_DDGI_ATLAS_PADDING, tv = ARK_DDGI_VISIBILITY_RES + 2 * ARK_DDGI_ATLAS_PADDING;
    constexpr uint32_t irrWords = kIrrTileTexels * 2u, visWords = kVisTileTexels;
    const uint32_t col = x + y * a.X;
    uint32_t* irr = reinterpret_cast<uint32_t*>(a.irr);
    uint32_t* vis = reinterpret_cast<uint32_t*>(a.vis);
    // irradiance: 10 rows of 20 dwords (8-B texels); visibility: 18 rows of 18 dwords
    for (uint32_t w = threadIdx.x; w < irrWords + visWords; w += 64u) {
        uint64_t at;
        if (w < irrWords) {
            const uint32_t r = w / (2u * ti), c = w % (2u * ti);
            at = (static_cast<uint64_t>(z * ti + r) * a.Wi + col * ti) * 2u + c;
            if (kUnpack) irr[at] = pkt[w];
            else pkt[w] = irr[at];
        } else {
            const uint32_t v = w - irrWords, r = v / tv, c = v % tv;
            at = static_cast<uint64_t>(z * tv + r) * a.Wv + col * tv + c;
            if (kUnpack) vis[at] = pkt[w];
            else pkt[w] = vis[at];
        }
    }
}

} // namespace dev

hipError_t launch_window_pack(const WindowExchangeArgs& a, bool unpack, hipStream_t s)
{
    if (a.K == 0) return hipSuccess;
    if (unpack) hipLaunchKernelGGL(dev::k_window_pack<true>, dim3(a.K), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(dev::k_window_pack<false>, dim3(a.K), dim3(64), 0, s, a);
    return hipGetLastError();
}

} // namespace ark
