// isa_probe2.hip -- gfx950 VALU issue costs of instruction MIXES (distance between dependent
// instructions), SDWA forms, and rotate alternatives.  8 waves/SIMD, 2000 iterations.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define V8(M) M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#define V4(M) M(a0) M(a1) M(a2) M(a3)
#define ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
#define ALIGN2(x) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b));
#define SDWAX(x) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(x) : "v"(b));
#define SDWAX2(x) asm volatile("v_xor_b32_sdwa %0, %1, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(x) : "v"(b));
#define SDWAADD(x) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(x) : "v"(b));
#define LSHL(x) asm volatile("v_lshlrev_b32 %0, 7, %0" : "+v"(x));
#define OR(x) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define DEP3(x) ADD(x) XOR(x) ALIGN(x)

#define KERNEL(NAME, BODY, PER)                                                                        \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk) {          \
        uint32_t b = threadIdx.x * 7 + 1;                                                             \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
                 a6 = a0 + 6, a7 = a0 + 7;                                                            \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();            \
        for (int i = 0; i < iters; ++i) { BODY }                                                      \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();            \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                  \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }              \
    }                                                                                                 \
    static const int per_##NAME = PER;

KERNEL(mix_dist8, V8(ADD) V8(XOR) V8(ALIGN) V8(ADD) V8(XOR) V8(ALIGN), 48)
KERNEL(mix_dist4, V4(ADD) V4(XOR) V4(ALIGN) V4(ADD) V4(XOR) V4(ALIGN) V4(ADD) V4(XOR) V4(ALIGN), 36)
KERNEL(mix_dep, V8(DEP3) V8(DEP3), 48)
KERNEL(addxor_dist8, V8(ADD) V8(XOR) V8(ADD) V8(XOR), 32)
KERNEL(align_2src, V8(ALIGN2) V8(ALIGN2) V8(ALIGN2) V8(ALIGN2), 32)
KERNEL(align_dist4, V4(ALIGN) V4(ALIGN) V4(ALIGN) V4(ALIGN) V4(ALIGN) V4(ALIGN) V4(ALIGN) V4(ALIGN), 32)
KERNEL(add_dist4, V4(ADD) V4(ADD) V4(ADD) V4(ADD) V4(ADD) V4(ADD) V4(ADD) V4(ADD), 32)
KERNEL(add_dist1, ADD(a0) ADD(a0) ADD(a0) ADD(a0) ADD(a0) ADD(a0) ADD(a0) ADD(a0), 8)
KERNEL(sdwa_xor, V8(SDWAX) V8(SDWAX2) V8(SDWAX) V8(SDWAX2), 32)
KERNEL(sdwa_add, V8(SDWAADD) V8(SDWAADD) V8(SDWAADD) V8(SDWAADD), 32)
KERNEL(shift_or, V8(LSHL) V8(OR) V8(LSHL) V8(OR), 32)

int main() {
    uint32_t *out;
    uint64_t *clk, hclk[2];
    const int grid = 8192, iters = 2000;
    hipMalloc(&out, grid * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
#define RUN(NAME)                                                                                       \
    {                                                                                                   \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk);                     \
        hipDeviceSynchronize();                                                                         \
        hipEventRecord(a);                                                                              \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk);                     \
        hipEventRecord(b);                                                                              \
        hipEventSynchronize(b);                                                                         \
        float ms;                                                                                       \
        hipEventElapsedTime(&ms, a, b);                                                                 \
        hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);                                                \
        double ghz = (double)hclk[0] / ((double)hclk[1] / 100e6) / 1e9;                                 \
        double winstr = (double)grid * 4 * iters * per_##NAME;                                          \
        double cpi = 1.0 / (winstr / 1024 / (ms * 1e-3 * ghz * 1e9));                                   \
        printf("%-14s %7.3f ms  clk %.2f GHz  cycles/wave-instr/SIMD %.2f\n", #NAME, ms, ghz, cpi);     \
    }
    RUN(mix_dist8) RUN(mix_dist4) RUN(mix_dep) RUN(addxor_dist8) RUN(align_2src) RUN(align_dist4) RUN(add_dist4)
    RUN(add_dist1) RUN(sdwa_xor) RUN(sdwa_add) RUN(shift_or)
    return 0;
}
