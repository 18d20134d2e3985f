// Cost of one select among FMAs on gfx950 (tools/probe): per unit of 8
// instructions, 7 independent v_fma_f32 and one select written as v_cndmask_b32_e32
// (reads VCC), v_cndmask_b32_e64 with an SGPR-pair mask, or v_bitop3_b32 with a lane
// mask in a VGPR; 4 and 6 waves per SIMD. Cycles per unit per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP16(X) X X X X X X X X X X X X X X X X
#define F7 "v_fma_f32 %0, %8, %9, %10\n v_fma_f32 %1, %8, %9, %10\n v_fma_f32 %2, %8, %9, %10\n v_fma_f32 %3, %8, %9, %10\n " \
           "v_fma_f32 %4, %8, %9, %10\n v_fma_f32 %5, %8, %9, %10\n v_fma_f32 %6, %8, %9, %10\n"
#define BODY(name, pre, sel)                                                                                    \
    __global__ void __launch_bounds__(384) name(uint32_t* out, int iters, uint32_t s0, uint32_t s1, uint32_t s2) \
    {                                                                                                           \
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;                                \
        const uint32_t x = s0 + threadIdx.x * 0u, y = s1, z = s2 + (threadIdx.x & 1u);                          \
        for (int i = 0; i < iters; ++i) {                                                                       \
            asm volatile(pre REP16(F7 sel) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(x), "v"(y), "v"(z) : "vcc", "s40", "s41");                                        \
        }                                                                                                       \
        out[blockIdx.x * 384 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                           \
    }
BODY(k_f8, "", "v_fma_f32 %7, %8, %9, %10\n")
BODY(k_cnd_vcc, "v_cmp_gt_u32 vcc, %10, %9\n", "v_cndmask_b32_e32 %7, %8, %9, vcc\n")
BODY(k_cnd_sgpr, "v_cmp_gt_u32 s[40:41], %10, %9\n", "v_cndmask_b32_e64 %7, %8, %9, s[40:41]\n")
BODY(k_bitop3, "", "v_bitop3_b32 %7, %10, %8, %9 bitop3:0xca\n")
BODY(k_cmp_cnd_vcc, "", "v_cmp_gt_u32 vcc, %10, %9\n v_cndmask_b32_e32 %7, %8, %9, vcc\n")
BODY(k_cmp_cnd_sgpr, "", "v_cmp_gt_u32 s[40:41], %10, %9\n v_cndmask_b32_e64 %7, %8, %9, s[40:41]\n")
BODY(k_addc_vcc, "v_cmp_gt_u32 vcc, %10, %9\n", "v_addc_co_u32 %7, s[40:41], %8, %9, vcc\n")

typedef void (*K)(uint32_t*, int, uint32_t, uint32_t, uint32_t);
int main()
{
    int dev = 0, clk = 0, cus = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int iters = 4000;
    uint32_t* out;
    (void)hipMalloc(&out, cus * 8 * 384 * 4);
    struct { const char* name; K k; } ks[] = { { "8 fma", k_f8 }, { "7 fma + cndmask vcc", k_cnd_vcc }, { "7 fma + cndmask sgpr", k_cnd_sgpr },
                                               { "7 fma + bitop3", k_bitop3 }, { "7 fma + cmp vcc + cndmask vcc", k_cmp_cnd_vcc },
                                               { "7 fma + cmp sgpr + cndmask sgpr", k_cmp_cnd_sgpr }, { "7 fma + addc (vcc in)", k_addc_vcc } };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int wps : { 4, 6 }) {
        // blocks of 384 threads = 6 waves: wps waves per SIMD -> cus * 4 * wps / 6 blocks
        const int blocks = cus * 4 * wps / 6;
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(384), 0, 0, out, 20, 0x3f800001u, 2u, 3u);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(384), 0, 0, out, iters, 0x3f800001u, 2u, 3u);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double units = static_cast<double>(blocks) * 6 / (cus * 4) * iters * 16;
            std::printf("%d waves/SIMD  %-34s %8.3f ms  %.2f cycles/unit/SIMD\n", wps, k.name, ms, ms * 1e-3 * clk * 1e3 / units);
        }
    }
    (void)hipFree(out);
    return 0;
}
