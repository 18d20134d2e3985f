// VALU issue cost with distinct source registers on gfx950 (tools/probe):
// 8 results per unit, each from three different source VGPRs of eight (VGPR banks =
// index mod 4), so operand reads are not served by one cached register; 4 waves per
// SIMD; cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP16(X) X X X X X X X X X X X X X X X X
// dst %0..%7, sources %8..%15
#define T3(op) op " %0, %8, %9, %10\n " op " %1, %9, %10, %11\n " op " %2, %10, %11, %12\n " op " %3, %11, %12, %13\n " \
               op " %4, %12, %13, %14\n " op " %5, %13, %14, %15\n " op " %6, %14, %15, %8\n " op " %7, %15, %8, %9\n"
#define T2(op) op " %0, %8, %9\n " op " %1, %9, %10\n " op " %2, %10, %11\n " op " %3, %11, %12\n " \
               op " %4, %12, %13\n " op " %5, %13, %14\n " op " %6, %14, %15\n " op " %7, %15, %8\n"
#define T1(op) op " %0, %8\n " op " %1, %9\n " op " %2, %10\n " op " %3, %11\n " op " %4, %12\n " op " %5, %13\n " op " %6, %14\n " op " %7, %15\n"
#define TC(op) op " %0, %8, %9, vcc\n " op " %1, %9, %10, vcc\n " op " %2, %10, %11, vcc\n " op " %3, %11, %12, vcc\n " \
               op " %4, %12, %13, vcc\n " op " %5, %13, %14, vcc\n " op " %6, %14, %15, vcc\n " op " %7, %15, %8, vcc\n"
// fmac: accumulate into the destination (its own read), sources rotating
#define TA(op) op " %0, %8, %9\n " op " %1, %9, %10\n " op " %2, %10, %11\n " op " %3, %11, %12\n " \
               op " %4, %12, %13\n " op " %5, %13, %14\n " op " %6, %14, %15\n " op " %7, %15, %8\n"
#define BODY(name, ins)                                                                                         \
    __global__ void __launch_bounds__(256) name(uint32_t* out, int iters, uint32_t s0)                          \
    {                                                                                                           \
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;                                \
        uint32_t b[8];                                                                                          \
        for (int k = 0; k < 8; ++k) b[k] = s0 + (threadIdx.x & 3u) * 0x100u + k * 0x10000u;                     \
        asm volatile("v_cmp_gt_u32 vcc, %0, %1" : : "v"(b[0]), "v"(b[1]) : "vcc");                            \
        for (int i = 0; i < iters; ++i) {                                                                       \
            asm volatile(REP16(ins) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]) : "vcc"); \
        }                                                                                                       \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                           \
    }
BODY(k_fma, T3("v_fma_f32"))
BODY(k_fmac, TA("v_fmac_f32"))
BODY(k_mul, T2("v_mul_f32"))
BODY(k_add, T2("v_add_f32"))
BODY(k_sub, T2("v_sub_f32"))
BODY(k_max3, T3("v_max3_f32"))
BODY(k_max, T2("v_max_f32"))
BODY(k_cvt, T1("v_cvt_f32_ubyte2"))
BODY(k_cnd, TC("v_cndmask_b32"))
BODY(k_and, T2("v_and_b32"))
BODY(k_addu, T2("v_add_u32"))
#define TB(op) op " %0, %8, %9, %10 bitop3:0xca\n " op " %1, %9, %10, %11 bitop3:0xca\n " op " %2, %10, %11, %12 bitop3:0xca\n " op " %3, %11, %12, %13 bitop3:0xca\n " op " %4, %12, %13, %14 bitop3:0xca\n " op " %5, %13, %14, %15 bitop3:0xca\n " op " %6, %14, %15, %8 bitop3:0xca\n " op " %7, %15, %8, %9 bitop3:0xca\n"
BODY(k_bitop3, TB("v_bitop3_b32"))
BODY(k_mov, T1("v_mov_b32"))
BODY(k_lshr, T2("v_lshrrev_b32"))
BODY(k_lshl, T2("v_lshlrev_b32"))

typedef void (*K)(uint32_t*, int, uint32_t);
int main()
{
    int dev = 0, clk = 0, cus = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int wavesPerSimd = 4, blocks = cus * wavesPerSimd;
    const int iters = 4000;
    uint32_t* out;
    (void)hipMalloc(&out, blocks * 256 * 4);
    struct { const char* name; K k; } ks[] = {
        { "v_fma_f32", k_fma }, { "v_fmac_f32", k_fmac }, { "v_mul_f32", k_mul }, { "v_add_f32", k_add }, { "v_sub_f32", k_sub },
        { "v_max3_f32", k_max3 }, { "v_max_f32", k_max }, { "v_cvt_f32_ubyte2", k_cvt }, { "v_cndmask_b32 (vcc)", k_cnd },
        { "v_and_b32", k_and }, { "v_add_u32", k_addu }, { "v_bitop3_b32", k_bitop3 }, { "v_mov_b32", k_mov },
        { "v_lshrrev_b32", k_lshr }, { "v_lshlrev_b32", k_lshl } };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 20, 0x3f800000u);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, iters, 0x3f800000u);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double perSimd = static_cast<double>(wavesPerSimd) * iters * 128;
        std::printf("%-24s %8.3f ms  %.2f cycles/instr/SIMD\n", k.name, ms, ms * 1e-3 * clk * 1e3 / perSimd);
    }
    (void)hipFree(out);
    return 0;
}
