// debug_kernels.hip — device evaluation of ark_fmath.h for the parity tests.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/ark_ddgi.h"
#include "../../include/ark_ddgi_debug.h"
#include "ark_fmath.h"

namespace {

__host__ __device__ inline float evalOp(int op, float x, float y)
{
    switch (op) {
    case 0: return ark::sinf_(x);
    case 1: return ark::cosf_(x);
    case 2: return ark::acosf_(x);
    case 3: return ark::atan2f_(x, y);
    case 4: return ark::log2f_(x);
    case 5: return ark::exp2f_(x);
    case 6: return ark::powf_(x, y);
    case 8: return ark::powf_pos_(x, y);
    default: return x;
    }
}

__global__ void k_fmath(int op, const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ out, uint64_t n)
{
    uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
    if (i >= n) return;
    if (op == 7) {
        float v = x[i];
        out[i] = (v != v) ? v : static_cast<float>(static_cast<_Float16>(v));
        return;
    }
    out[i] = evalOp(op, x[i], y ? y[i] : 0.0f);
}

} // namespace

extern "C" int ark_ddgi_debug_fmath(int device, int op, const float* x, const float* y, float* out, uint64_t n)
{
    if (!x || !out || n == 0) return -1;
    if (hipSetDevice(device) != hipSuccess) return -5;
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    size_t bytes = n * sizeof(float);
    if (hipMalloc(&dx, bytes) != hipSuccess || hipMalloc(&dy, bytes) != hipSuccess || hipMalloc(&dout, bytes) != hipSuccess) return -4;
    if (hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice) != hipSuccess) return -5;
    if (y && hipMemcpy(dy, y, bytes, hipMemcpyHostToDevice) != hipSuccess) return -5;
    hipLaunchKernelGGL(k_fmath, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, 0, op, dx, y ? dy : nullptr, dout, n);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(dy);
    (void)hipFree(dout);
    return e == hipSuccess ? 0 : -5;
}

extern "C" int ark_ddgi_debug_fmath_host(int op, const float* x, const float* y, float* out, uint64_t n)
{
    if (!x || !out) return -1;
    for (uint64_t i = 0; i < n; ++i) {
        if (op == 7) {
            float v = x[i];
            out[i] = (v != v) ? v : static_cast<float>(static_cast<_Float16>(v));
        } else {
            out[i] = evalOp(op, x[i], y ? y[i] : 0.0f);
        }
    }
    return 0;
}

extern "C" int ark_ddgi_debug_struct_sizes(uint32_t* out, int n)
{
    const uint32_t sizes[] = { sizeof(ArkDdgiDesc), sizeof(ArkRTVertex), sizeof(ArkRTTriangleMesh), sizeof(ArkShaderMaterial), sizeof(ArkTexture),
                               sizeof(ArkRTInstance), sizeof(ArkDirectionalLight), sizeof(ArkSpotLight), sizeof(ArkDdgiScene), sizeof(ArkDdgiFrameParams),
                               sizeof(ArkDdgiCounters), sizeof(ArkDdgiDeviceViews), sizeof(ArkDdgiBvhStats), sizeof(ArkBakeAoDesc), sizeof(ArkComposeDesc), sizeof(ArkProbeDebugDesc), sizeof(ArkReflectionsDesc) };
    int m = static_cast<int>(sizeof(sizes) / sizeof(sizes[0]));
    for (int i = 0; i < n && i < m; ++i) out[i] = sizes[i];
    return m < n ? m : n;
}
