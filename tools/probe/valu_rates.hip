// VALU issue cost per instruction form on gfx950 (tools/probe; DESIGN.md §3 node-test
// budget): every SIMD runs W waves, each executing ITER x 16 independent instructions of
// one form; cycles per instruction per SIMD = elapsed x clock / (instructions per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define REP16(X) X X X X X X X X X X X X X X X X
#define BODY(name, ins)                                                                          \
    __global__ void __launch_bounds__(256) name(float* out, int iters)                           \
    {                                                                                            \
        float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5; \
        float a6 = a0 + 6, a7 = a0 + 7, b = 1.0001f, c = 0.5f;                                   \
        for (int i = 0; i < iters; ++i) {                                                        \
            asm volatile(REP16(ins) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c)); \
        }                                                                                        \
        out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;             \
    }

// 16 instructions per REP16 unit would be 8x16; use 2 instrs per unit -> 32 per iteration? keep simple:
// each unit below = 8 independent instructions (one per accumulator)
BODY(k_fma_f32, "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n")
BODY(k_pk_fma_f16, "v_pk_fma_f16 %0, %0, %8, %9\n v_pk_fma_f16 %1, %1, %8, %9\n v_pk_fma_f16 %2, %2, %8, %9\n v_pk_fma_f16 %3, %3, %8, %9\n v_pk_fma_f16 %4, %4, %8, %9\n v_pk_fma_f16 %5, %5, %8, %9\n v_pk_fma_f16 %6, %6, %8, %9\n v_pk_fma_f16 %7, %7, %8, %9\n")
BODY(k_pk_max3_f16, "v_pk_maximum3_f16 %0, %0, %8, %9\n v_pk_maximum3_f16 %1, %1, %8, %9\n v_pk_maximum3_f16 %2, %2, %8, %9\n v_pk_maximum3_f16 %3, %3, %8, %9\n v_pk_maximum3_f16 %4, %4, %8, %9\n v_pk_maximum3_f16 %5, %5, %8, %9\n v_pk_maximum3_f16 %6, %6, %8, %9\n v_pk_maximum3_f16 %7, %7, %8, %9\n")
BODY(k_pk_max_f16, "v_pk_max_f16 %0, %0, %8\n v_pk_max_f16 %1, %1, %8\n v_pk_max_f16 %2, %2, %8\n v_pk_max_f16 %3, %3, %8\n v_pk_max_f16 %4, %4, %8\n v_pk_max_f16 %5, %5, %8\n v_pk_max_f16 %6, %6, %8\n v_pk_max_f16 %7, %7, %8\n")
BODY(k_max3_f32, "v_max3_f32 %0, %0, %8, %9\n v_max3_f32 %1, %1, %8, %9\n v_max3_f32 %2, %2, %8, %9\n v_max3_f32 %3, %3, %8, %9\n v_max3_f32 %4, %4, %8, %9\n v_max3_f32 %5, %5, %8, %9\n v_max3_f32 %6, %6, %8, %9\n v_max3_f32 %7, %7, %8, %9\n")
BODY(k_perm, "v_perm_b32 %0, %0, %8, %9\n v_perm_b32 %1, %1, %8, %9\n v_perm_b32 %2, %2, %8, %9\n v_perm_b32 %3, %3, %8, %9\n v_perm_b32 %4, %4, %8, %9\n v_perm_b32 %5, %5, %8, %9\n v_perm_b32 %6, %6, %8, %9\n v_perm_b32 %7, %7, %8, %9\n")
BODY(k_cvt_ubyte, "v_cvt_f32_ubyte1 %0, %0\n v_cvt_f32_ubyte1 %1, %1\n v_cvt_f32_ubyte1 %2, %2\n v_cvt_f32_ubyte1 %3, %3\n v_cvt_f32_ubyte1 %4, %4\n v_cvt_f32_ubyte1 %5, %5\n v_cvt_f32_ubyte1 %6, %6\n v_cvt_f32_ubyte1 %7, %7\n")
BODY(k_dot2_f32_f16, "v_dot2_f32_f16 %0, %0, %8, %9\n v_dot2_f32_f16 %1, %1, %8, %9\n v_dot2_f32_f16 %2, %2, %8, %9\n v_dot2_f32_f16 %3, %3, %8, %9\n v_dot2_f32_f16 %4, %4, %8, %9\n v_dot2_f32_f16 %5, %5, %8, %9\n v_dot2_f32_f16 %6, %6, %8, %9\n v_dot2_f32_f16 %7, %7, %8, %9\n")
BODY(k_cmp_addc, "v_cmp_le_f32 vcc, %0, %8\n v_addc_co_u32 %0, vcc, %0, %0, vcc\n v_cmp_le_f32 vcc, %1, %8\n v_addc_co_u32 %1, vcc, %1, %1, vcc\n v_cmp_le_f32 vcc, %2, %8\n v_addc_co_u32 %2, vcc, %2, %2, vcc\n v_cmp_le_f32 vcc, %3, %8\n v_addc_co_u32 %3, vcc, %3, %3, vcc\n")
BODY(k_cmp_sdwa, "v_cmp_le_f16_sdwa vcc, %0, %8 src0_sel:WORD_1 src1_sel:WORD_1\n v_addc_co_u32 %0, vcc, %0, %0, vcc\n v_cmp_le_f16_sdwa vcc, %1, %8 src0_sel:WORD_1 src1_sel:WORD_1\n v_addc_co_u32 %1, vcc, %1, %1, vcc\n v_cmp_le_f16_sdwa vcc, %2, %8 src0_sel:WORD_1 src1_sel:WORD_1\n v_addc_co_u32 %2, vcc, %2, %2, vcc\n v_cmp_le_f16_sdwa vcc, %3, %8 src0_sel:WORD_1 src1_sel:WORD_1\n v_addc_co_u32 %3, vcc, %3, %3, vcc\n")

typedef void (*K)(float*, int);
int main()
{
    int dev = 0, clk = 0, cus = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int wavesPerSimd = 4, blocks = cus * wavesPerSimd; // 256 threads = 4 waves = 1 per SIMD per block
    const int iters = 20000;
    float* out;
    hipMalloc(&out, blocks * 256 * 4);
    struct { const char* name; K k; int ins; } ks[] = {
        { "v_fma_f32", k_fma_f32, 128 }, { "v_pk_fma_f16", k_pk_fma_f16, 128 }, { "v_pk_maximum3_f16", k_pk_max3_f16, 128 },
        { "v_pk_max_f16", k_pk_max_f16, 128 }, { "v_max3_f32", k_max3_f32, 128 }, { "v_perm_b32", k_perm, 128 },
        { "v_cvt_f32_ubyte1", k_cvt_ubyte, 128 }, { "v_dot2_f32_f16", k_dot2_f32_f16, 128 },
        { "v_cmp_le_f32+v_addc", k_cmp_addc, 128 }, { "v_cmp_le_f16_sdwa+v_addc", k_cmp_sdwa, 128 } };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 100);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        // instructions per SIMD: waves per SIMD x iters x ins
        const double perSimd = static_cast<double>(wavesPerSimd) * iters * k.ins;
        const double cyc = ms * 1e-3 * clk * 1e3 / perSimd;
        std::printf("%-26s %8.3f ms  %.2f cycles/instr/SIMD (clock %d MHz, %d CUs)\n", k.name, ms, cyc, clk / 1000, cus);
    }
    hipFree(out);
    return 0;
}
