// VALU issue cost per instruction on gfx950 (tools/probe; DESIGN.md §3 traversal
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
                         : "v"(x), "v"(y), "v"(z) : "vcc");                                                     \
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
BODY(k_fmac, U8("v_fmac_f32", A2))
BODY(k_add, U8("v_add_f32", A2))
BODY(k_mul, U8("v_mul_f32", A2))
BODY(k_sub, U8("v_sub_f32", A2))
BODY(k_max, U8("v_max_f32", A2))
BODY(k_min, U8("v_min_f32", A2))
BODY(k_max3, U8("v_max3_f32", A3))
BODY(k_min3, U8("v_min3_f32", A3))
BODY(k_med3, U8("v_med3_f32", A3))
BODY(k_fma_mix, U8("v_fma_mix_f32", A3))
BODY(k_ldexp, U8("v_ldexp_f32", A2))
BODY(k_cvt_ub, U8("v_cvt_f32_ubyte1", A1))
BODY(k_cvt_f16, U8("v_cvt_f32_f16", A1))
BODY(k_cvt_u32, U8("v_cvt_f32_u32", A1))
BODY(k_rcp, U8("v_rcp_f32", A1))
BODY(k_addu, U8("v_add_u32", A2))
BODY(k_subu, U8("v_sub_u32", A2))
BODY(k_add3, U8("v_add3_u32", A3))
BODY(k_and, U8("v_and_b32", A2))
BODY(k_or3, U8("v_or3_b32", A3))
BODY(k_lshl, U8("v_lshlrev_b32", A2))
BODY(k_lshl_or, U8("v_lshl_or_b32", A3))
BODY(k_bfe, U8("v_bfe_u32", A3))
BODY(k_perm, U8("v_perm_b32", A3))
BODY(k_mov, U8("v_mov_b32", A1))
BODY(k_cnd, U8("v_cndmask_b32", "%8, %9, vcc"))
BODY(k_cmp, U8("v_cmp_le_f32 vcc, %8, %9\n v_mov_b32", A1))
BODY(k_addc, U8("v_addc_co_u32", "vcc, %8, %9, vcc"))
BODY(k_mad24, U8("v_mad_u32_u24", A3))
BODY(k_mullo, U8("v_mul_lo_u32", A2))
BODY(k_bcnt, U8("v_bcnt_u32_b32", A2))
BODY(k_ffbl, U8("v_ffbl_b32", A1))
BODY(k_mbcnt, U8("v_mbcnt_lo_u32_b32", A2))
BODY(k_pk_fma_f16, U8("v_pk_fma_f16", A3))
BODY(k_dot2, U8("v_dot2_f32_f16", A3))
BODY64(k_pk_fma_f32, "v_pk_fma_f32", "%4, %5, %6")
BODY64(k_pk_mul_f32, "v_pk_mul_f32", "%4, %5")
BODY64(k_pk_add_f32, "v_pk_add_f32", "%4, %5")
BODY64(k_lshl_add64, "v_lshl_add_u64", "%4, 4, %5")

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
        { "v_fma_f32", k_fma }, { "v_fmac_f32", k_fmac }, { "v_add_f32", k_add }, { "v_mul_f32", k_mul }, { "v_sub_f32", k_sub },
        { "v_max_f32", k_max }, { "v_min_f32", k_min }, { "v_max3_f32", k_max3 }, { "v_min3_f32", k_min3 }, { "v_med3_f32", k_med3 },
        { "v_fma_mix_f32", k_fma_mix }, { "v_ldexp_f32", k_ldexp }, { "v_cvt_f32_ubyte1", k_cvt_ub }, { "v_cvt_f32_f16", k_cvt_f16 },
        { "v_cvt_f32_u32", k_cvt_u32 }, { "v_rcp_f32", k_rcp }, { "v_add_u32", k_addu }, { "v_sub_u32", k_subu }, { "v_add3_u32", k_add3 },
        { "v_and_b32", k_and }, { "v_or3_b32", k_or3 }, { "v_lshlrev_b32", k_lshl }, { "v_lshl_or_b32", k_lshl_or }, { "v_bfe_u32", k_bfe },
        { "v_perm_b32", k_perm }, { "v_mov_b32", k_mov }, { "v_cndmask_b32", k_cnd }, { "v_cmp_le_f32+v_mov (pair)", k_cmp },
        { "v_addc_co_u32", k_addc }, { "v_mad_u32_u24", k_mad24 }, { "v_mul_lo_u32", k_mullo }, { "v_bcnt_u32_b32", k_bcnt },
        { "v_ffbl_b32", k_ffbl }, { "v_mbcnt_lo_u32_b32", k_mbcnt }, { "v_pk_fma_f16", k_pk_fma_f16 }, { "v_dot2_f32_f16", k_dot2 },
        { "v_pk_fma_f32", k_pk_fma_f32 }, { "v_pk_mul_f32", k_pk_mul_f32 }, { "v_pk_add_f32", k_pk_add_f32 }, { "v_lshl_add_u64", k_lshl_add64 },
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
