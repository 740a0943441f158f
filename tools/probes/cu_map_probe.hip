// cu_map_probe.hip -- which physical XCC / SE / CU does logical CU i of a
// hipExtStreamCreateWithCUMask mask land on?  One single-CU stream per i, one
// 64-thread workgroup reading HW_REG_XCC_ID and HW_REG_HW_ID.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

__global__ void where(uint32_t *out, int i) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (threadIdx.x == 0) { out[16 * i + 2 * blockIdx.x] = xcc; out[16 * i + 2 * blockIdx.x + 1] = hw; }
}

int main() {
    int n = 0;
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t *d;
    (void)hipMalloc(&d, 16 * n * sizeof(uint32_t));
    std::vector<uint32_t> h(16 * n);
    for (int i = 0; i < n; ++i) {
        std::vector<uint32_t> mask((n + 31) / 32, 0u);
        mask[i / 32] = 1u << (i % 32);
        hipStream_t s;
        if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) { printf("mask %d failed\n", i); return 1; }
        hipLaunchKernelGGL(where, dim3(8), dim3(64), 0, s, d, i);
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
    (void)hipMemcpy(h.data(), d, 16 * n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    printf("logical: 8 workgroups as xcc/se/sh/cu\n");
    for (int i = 0; i < n; ++i) {
        printf("%3d", i);
        for (int b = 0; b < 8; ++b) {
            uint32_t hw = h[16 * i + 2 * b + 1];
            printf("  %u/%u/%u/%u", h[16 * i + 2 * b] & 0xf, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15);
        }
        printf("\n");
    }
    return 0;
}
