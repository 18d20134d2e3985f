// Checks that a 16-B global load from an 8-B-aligned (not 16-B-aligned) address
// returns the right bytes on this device (used to decide whether the DDGI atlas
// gather may fetch two adjacent RGBA16F texels with one load).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(const uint32_t* base, uint4* out)
{
    const uint32_t i = threadIdx.x;
    const uint4* p = reinterpret_cast<const uint4*>(base + 2 + 2 * i); // 8-B aligned, 16-B misaligned
    out[i] = *p;
}

int main()
{
    const int n = 64;
    uint32_t h[2 * n + 8];
    for (int i = 0; i < 2 * n + 8; ++i) h[i] = 0x1000u + i;
    uint32_t* d;
    uint4* o;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess || hipMalloc(&o, n * sizeof(uint4)) != hipSuccess) return 2;
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(n), 0, 0, d, o);
    uint4 r[n];
    hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t* e = h + 2 + 2 * i;
        if (r[i].x != e[0] || r[i].y != e[1] || r[i].z != e[2] || r[i].w != e[3]) bad++;
    }
    std::printf("unaligned 16B loads: %s (%d/%d wrong)\n", bad ? "WRONG" : "ok", bad, n);
    return bad ? 1 : 0;
}
