// Exhaustive CPU check of the closed-form window -> slot and slot -> traversal-queue
// maps that k_probe_slots evaluates per thread (ddgi_kernels.h: slabRankOf,
// slotQueuePos) against the plain construction: slots = the window's probes (slab
// probes only when sharded) in window order, queue = a stable bucket sort of the slots
// by their x-z block. Small grids, every window start and size, every Z-slab split.
#include "ddgi_kernels.h"

#include <algorithm>
#include <cstdio>
#include <vector>

using namespace ark;

int main()
{
    long bad = 0, n = 0;
    for (uint32_t X : { 1u, 3u, 4u, 5u, 8u })
        for (uint32_t Y : { 1u, 2u, 3u })
            for (uint32_t Z : { 1u, 2u, 3u, 4u, 6u })
                for (uint32_t P : { 1u, 2u, 3u, 6u }) {
                    if (Z % P) continue;
                    const uint32_t N = X * Y * Z;
                    for (uint32_t r = 0; r < P; ++r) {
                        const bool sharded = P > 1;
                        const uint32_t z0 = r * (Z / P), z1 = z0 + Z / P;
                        const uint32_t zlo = sharded ? z0 : 0u, zhi = sharded ? z1 : Z, zext = std::max(1u, zhi - zlo);
                        for (uint32_t first = 0; first < N; first += (N > 40 ? 3u : 1u))
                            for (uint32_t K = 1; K <= N; ++K) {
                                std::vector<uint32_t> probe, pos;
                                for (uint32_t s = 0; s < K; ++s) {
                                    const uint32_t p = (first + s) % N, z = (p % (X * Z)) / X;
                                    if (sharded && !(z >= z0 && z < z1)) continue;
                                    probe.push_back(p);
                                    pos.push_back(s);
                                }
                                std::vector<uint32_t> queue;
                                for (uint32_t b = 0; b < 8; ++b)
                                    for (uint32_t j = 0; j < probe.size(); ++j) {
                                        const uint32_t x = probe[j] % X, z = (probe[j] % (X * Z)) / X;
                                        const uint32_t bb = zext >= 2 ? x * 4 / X + 4 * std::min(1u, (z - zlo) * 2 / zext) : x * 8 / X;
                                        if (bb == b) queue.push_back(j);
                                    }
                                if (sharded && slabRankOf(X, Y, Z, z0, z1, first, K) != probe.size()) bad++;
                                for (uint32_t j = 0; j < probe.size(); ++j) {
                                    const uint32_t slot = sharded ? slabRankOf(X, Y, Z, z0, z1, first, pos[j]) : pos[j];
                                    const uint32_t q = slotQueuePos(X, Y, Z, zlo, zext, first, K, pos[j], probe[j]);
                                    if (slot != j || q >= queue.size() || queue[q] != j) bad++;
                                    n++;
                                }
                            }
                    }
                }
    std::printf("checked %ld slots, %ld wrong\n", n, bad);
    if (bad == 0) std::printf("OK\n");
    return bad != 0;
}
