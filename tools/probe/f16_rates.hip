// Packed-fp16 issue cost with subnormal operands and directed rounding on gfx950
// (tools/probe; DESIGN.md §9, the packed-fp16 BVH8 child test): every SIMD runs 4
// waves, each executing ITER x 128 independent instructions of one form from
// constant operands; cycles per instruction per SIMD = elapsed x clock / count.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP16(X) X X X X X X X X X X X X X X X X
// 8 independent results per unit from the constant operands %8, %9, %10
#define UNIT(op) \
    op " %0, %8, %9, %10\n " op " %1, %8, %9, %10\n " op " %2, %8, %9, %10\n " op " %3, %8, %9, %10\n " \
    op " %4, %8, %9, %10\n " op " %5, %8, %9, %10\n " op " %6, %8, %9, %10\n " op " %7, %8, %9, %10\n"
#define BODY(name, ins, MODE)                                                                                    \
    __global__ void __launch_bounds__(256) name(uint32_t* out, int iters, uint32_t s0, uint32_t s1, uint32_t s2)  \
    {                                                                                                            \
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;                                 \
        const uint32_t x = s0 + threadIdx.x * 0u, y = s1, z = s2;                                                \
        asm volatile(MODE);                                                                                      \
        for (int i = 0; i < iters; ++i) {                                                                        \
            asm volatile(REP16(ins) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(x), "v"(y), "v"(z));                                                              \
        }                                                                                                        \
        asm volatile("s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 0");                                          \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                            \
    }

#define RNE "s_nop 0"
#define RDN "s_setreg_imm32_b32 hwreg(HW_REG_MODE, 0, 4), 0xa\n s_nop 1"
BODY(k_pk_fma, UNIT("v_pk_fma_f16"), RNE)
BODY(k_pk_fma_rd, UNIT("v_pk_fma_f16"), RDN)
BODY(k_fma_f32, UNIT("v_fma_f32"), RNE)
BODY(k_fma_f32_rd, UNIT("v_fma_f32"), RDN)
BODY(k_pk_max3, UNIT("v_pk_maximum3_f16"), RNE)
BODY(k_pk_min3_rd, UNIT("v_pk_minimum3_f16"), RDN)

typedef void (*K)(uint32_t*, int, uint32_t, uint32_t, uint32_t);
int main()
{
    int dev = 0, clk = 0, cus = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int wavesPerSimd = 4, blocks = cus * wavesPerSimd;
    const int iters = 4000;
    uint32_t* out;
    hipMalloc(&out, blocks * 256 * 4);
    // operands: fp16 pairs (hi | lo) / fp32 bit patterns
    const uint32_t h_norm = 0x3c013c02u, h_A = 0x50005000u /* 32 */, h_B = 0x3c003c00u;
    const uint32_t h_sub = 0x00ff0003u /* subnormals 255 / 3 x 2^-24 */, h_Abig = 0x70007000u /* 8192 */;
    const uint32_t f_norm = 0x3f800001u, f_A = 0x42000000u, f_sub = 0x00000fffu;
    struct { const char* name; K k; uint32_t s0, s1, s2; } ks[] = {
        { "pk_fma_f16 normal", k_pk_fma, h_norm, h_A, h_B },
        { "pk_fma_f16 subnormal q", k_pk_fma, h_sub, h_Abig, h_B },
        { "pk_fma_f16 subnormal result", k_pk_fma, h_sub, h_B, 0u },
        { "pk_fma_f16 normal, round down", k_pk_fma_rd, h_norm, h_A, h_B },
        { "pk_fma_f16 subnormal q, round down", k_pk_fma_rd, h_sub, h_Abig, h_B },
        { "fma_f32 normal", k_fma_f32, f_norm, f_A, f_norm },
        { "fma_f32 subnormal", k_fma_f32, f_sub, f_A, 0u },
        { "fma_f32 normal, round down", k_fma_f32_rd, f_norm, f_A, f_norm },
        { "pk_maximum3_f16 normal", k_pk_max3, h_norm, h_A, h_B },
        { "pk_maximum3_f16 subnormal", k_pk_max3, h_sub, h_sub, h_B },
        { "pk_minimum3_f16 round down", k_pk_min3_rd, h_norm, h_A, h_B },
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 20, k.s0, k.s1, k.s2);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters, k.s0, k.s1, k.s2);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double perSimd = static_cast<double>(wavesPerSimd) * iters * 128;
        std::printf("%-36s %8.3f ms  %.2f cycles/instr/SIMD\n", k.name, ms, ms * 1e-3 * clk * 1e3 / perSimd);
    }
    hipFree(out);
    return 0;
}
