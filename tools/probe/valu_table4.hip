// VALU issue cost per instruction on gfx950 (fourth table: accumulating and dependent
// forms; tools/probe). Every SIMD runs 4 waves, each executing
// ITER x 128 instructions of one form over 8 destinations; cycles per instruction per
// SIMD = elapsed x clock / count. The earlier tables wrote each destination from the
// same constant operands (no dependence between instructions); here the destination
// is also a source (the accumulator of a sum), or the previous instruction's result is.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define REP16(X) X X X X X X X X X X X X X X X X
// one line per destination %0..%7; L(i) expands the operand text for destination i
#define U8L(L) L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7)
#define BODY(name, ins)                                                                                         \
    __global__ void __launch_bounds__(256) name(uint32_t* out, int iters, uint32_t s0, uint32_t s1, uint32_t s2) \
    {                                                                                                           \
        uint32_t a0 = s0, a1 = s1, a2 = s2, a3 = s0, a4 = s1, a5 = s2, a6 = s0, a7 = s1;                        \
        const uint32_t x = s0 + threadIdx.x * 0u, y = s1, z = s2;                                               \
        for (int i = 0; i < iters; ++i) {                                                                       \
            asm volatile("s_mov_b64 s[40:41], exec\n" REP16(ins)                                               \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)        \
                         : "v"(x), "v"(y), "v"(z) : "vcc", "s40", "s41");                                       \
        }                                                                                                       \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                           \
    }
#define STR_(x) #x
#define STR(x) STR_(x)
// independent: d = op(x, y[, z])
#define L_FMA(i) "v_fma_f32 %" STR(i) ", %8, %9, %10\n "
#define L_ADD(i) "v_add_f32 %" STR(i) ", %8, %9\n "
// accumulating: d = op(x, y, d)
#define L_FMA_ACC(i) "v_fma_f32 %" STR(i) ", %8, %9, %" STR(i) "\n "
#define L_FMAC(i) "v_fmac_f32 %" STR(i) ", %8, %9\n "
#define L_ADD_ACC(i) "v_add_f32 %" STR(i) ", %" STR(i) ", %8\n "
#define L_MUL_ACC(i) "v_mul_f32 %" STR(i) ", %" STR(i) ", %8\n "
// reads the previous instruction's destination (a dependent chain through all 8)
#define L_FMA_CHAIN0 "v_fma_f32 %0, %7, %9, %10\n v_fma_f32 %1, %0, %9, %10\n v_fma_f32 %2, %1, %9, %10\n v_fma_f32 %3, %2, %9, %10\n "
#define L_FMA_CHAIN1 "v_fma_f32 %4, %3, %9, %10\n v_fma_f32 %5, %4, %9, %10\n v_fma_f32 %6, %5, %9, %10\n v_fma_f32 %7, %6, %9, %10\n "
// reads the destination written two instructions before (pairs independent)
#define L_FMA_PAIR "v_fma_f32 %0, %6, %9, %10\n v_fma_f32 %1, %7, %9, %10\n v_fma_f32 %2, %0, %9, %10\n v_fma_f32 %3, %1, %9, %10\n " \
                   "v_fma_f32 %4, %2, %9, %10\n v_fma_f32 %5, %3, %9, %10\n v_fma_f32 %6, %4, %9, %10\n v_fma_f32 %7, %5, %9, %10\n "
#define L_CND_SGPR(i) "v_cndmask_b32 %" STR(i) ", %8, %9, s[40:41]\n "
#define L_MAX_ACC(i) "v_max_f32 %" STR(i) ", %" STR(i) ", %8\n "

BODY(k_fma, U8L(L_FMA))
BODY(k_add, U8L(L_ADD))
BODY(k_fma_acc, U8L(L_FMA_ACC))
BODY(k_fmac, U8L(L_FMAC))
BODY(k_add_acc, U8L(L_ADD_ACC))
BODY(k_mul_acc, U8L(L_MUL_ACC))
BODY(k_fma_chain, L_FMA_CHAIN0 L_FMA_CHAIN1)
BODY(k_fma_pair, L_FMA_PAIR)
BODY(k_cnd_sgpr, U8L(L_CND_SGPR))
BODY(k_max_acc, U8L(L_MAX_ACC))
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
    // operands near 1 so that accumulations stay finite
    const uint32_t f1 = 0x3f800001u, f2 = 0x3f7fffffu, f3 = 0x00000000u;
    struct { const char* name; K k; } ks[] = {
        { "fma d, x, y, z", k_fma },
        { "add d, x, y", k_add },
        { "fma d, x, y, d", k_fma_acc },
        { "fmac d, x, y", k_fmac },
        { "add d, d, x", k_add_acc },
        { "mul d, d, x", k_mul_acc },
        { "fma chain (prev result)", k_fma_chain },
        { "fma pairs (result 2 back)", k_fma_pair },
        { "cndmask d, x, y, sgpr", k_cnd_sgpr },
        { "max d, d, x", k_max_acc },
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
