// VALU issue cost per instruction on gfx950 (third table: fp16-operand FMA mixes, conversions, alignbit) (tools/probe; DESIGN.md §3 traversal
// budget): every SIMD runs 4 waves, each executing ITER x 128 instructions of one
// form, 8 independent destinations written from constant operands; cycles per
// instruction per SIMD = elapsed x clock / count.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP16(X) X X X X X X X X X X X X X X X X
#define U8(op, args) \
    op " %0, " args "\n " op " %1, " args "\n " op " %2, " args "\n " op " %3, " args "\n " \
    op " %4, " args "\n " op " %5, " args "\n " op " %6, " args "\n " op " %7, " args "\n"
#define A3 "%8, %9, %10"
#define A2 "%8, %9"
#define A1 "%8"
#define BODY(name, ins)                                                                                         \
    __global__ void __launch_bounds__(256) name(uint32_t* out, int iters, uint32_t s0, uint32_t s1, uint32_t s2) \
    {                                                                                                           \
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;                                \
        const uint32_t x = s0 + threadIdx.x * 0u, y = s1, z = s2;                                               \
        for (int i = 0; i < iters; ++i) {                                                                       \
            asm volatile(REP16(ins) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(x), "v"(y), "v"(z) : "vcc", "s40", "s41");                                                     \
        }                                                                                                       \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                           \
    }
// packed-f32 forms: 64-bit destinations, 8 instructions per unit over 4 pairs
#define BODY64(name, op, args)                                                                                  \
    __global__ void __launch_bounds__(256) name(uint32_t* out, int iters, uint32_t s0, uint32_t s1, uint32_t s2) \
    {                                                                                                           \
        uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;                                                                \
        const uint64_t x = s0 | (static_cast<uint64_t>(s0) << 32), y = s1 | (static_cast<uint64_t>(s1) << 32),  \
                       z = s2 | (static_cast<uint64_t>(s2) << 32);                                              \
        for (int i = 0; i < iters; ++i) {                                                                       \
            asm volatile(REP16(op " %0, " args "\n " op " %1, " args "\n " op " %2, " args "\n " op " %3, " args "\n " \
                               op " %0, " args "\n " op " %1, " args "\n " op " %2, " args "\n " op " %3, " args "\n") \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(x), "v"(y), "v"(z));                  \
        }                                                                                                       \
        out[blockIdx.x * 256 + threadIdx.x] = static_cast<uint32_t>(a0 ^ a1 ^ a2 ^ a3);                         \
    }

BODY(k_fma, U8("v_fma_f32", A3))
BODY(k_fma_mix_lo, U8("v_fma_mix_f32", "%8, %9, %10 op_sel_hi:[1,0,0]"))
BODY(k_fma_mix_hi, U8("v_fma_mix_f32", "%8, %9, %10 op_sel:[1,0,0] op_sel_hi:[1,0,0]"))
BODY(k_cvt_f16, U8("v_cvt_f32_f16", A1))
BODY(k_cvt_ub0, U8("v_cvt_f32_ubyte0", A1))
BODY(k_cvt_ub3, U8("v_cvt_f32_ubyte3", A1))
BODY(k_alignbit, U8("v_alignbit_b32", "%8, %9, 31"))
BODY(k_sub_sgpr, "s_mov_b32 s40, 0x3f800000\n" U8("v_sub_f32", "%8, s40"))
BODY(k_max3, U8("v_max3_f32", A3))
BODY(k_cmp_e32, U8("v_cmp_le_f32 vcc, %8, %9\n v_mov_b32", A1))
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
    const uint32_t f1 = 0x3f800001u, f2 = 0x40000000u, f3 = 0x3f000000u;
    struct { const char* name; K k; } ks[] = {
        { "k_fma", k_fma },
        { "k_fma_mix_lo", k_fma_mix_lo },
        { "k_fma_mix_hi", k_fma_mix_hi },
        { "k_cvt_f16", k_cvt_f16 },
        { "k_cvt_ub0", k_cvt_ub0 },
        { "k_cvt_ub3", k_cvt_ub3 },
        { "k_alignbit", k_alignbit },
        { "k_sub_sgpr", k_sub_sgpr },
        { "k_max3", k_max3 },
        { "k_cmp_e32", k_cmp_e32 },
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 20, f1, f2, f3);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters, f1, f2, f3);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double perSimd = static_cast<double>(wavesPerSimd) * iters * 128;
        std::printf("%-30s %8.3f ms  %.2f cycles/instr/SIMD\n", k.name, ms, ms * 1e-3 * clk * 1e3 / perSimd);
    }
    (void)hipFree(out);
    return 0;
}
