// isa_probe.hip -- issue cost of single VALU instruction types on gfx950 (wave64),
// 8 independent dependency chains per lane, full occupancy.  Reports wave-instructions
// per SIMD per shader cycle (clock from s_memtime / s_memrealtime inside the kernel).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(x));
#define ALIGNB(x) asm volatile("v_alignbyte_b32 %0, %0, %0, 2" : "+v"(x));
#define PERM(x) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(x) : "v"(b));
#define XAD(x) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x) : "v"(b));
#define ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(b));
#define LSHLOR(x) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(x) : "v"(b));
#define LSHR(x) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(x));
#define BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(x) : "v"(b));
#define PKADD16(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(b));
#define ADDE64(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
#define XORE64(x) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
#define MIX(x) asm volatile("v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n v_alignbit_b32 %0, %0, %0, 7" : "+v"(x) : "v"(b));

#define KERNEL(NAME, OP, PER)                                                                          \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk) {          \
        uint32_t b = threadIdx.x * 7 + 1;                                                             \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,     \
                 a6 = a0 + 6, a7 = a0 + 7;                                                            \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();            \
        for (int i = 0; i < iters; ++i) { R8(OP) R8(OP) R8(OP) R8(OP) }                               \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();            \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                  \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }              \
    }                                                                                                 \
    static const int per_##NAME = PER;

KERNEL(add, ADD, 32)
KERNEL(xor, XOR, 32)
KERNEL(align, ALIGN, 32)
KERNEL(alignbyte, ALIGNB, 32)
KERNEL(perm, PERM, 32)
KERNEL(xad, XAD, 32)
KERNEL(add3, ADD3, 32)
KERNEL(lshlor, LSHLOR, 32)
KERNEL(lshr, LSHR, 32)
KERNEL(bitop3, BITOP3, 32)
KERNEL(pkadd16, PKADD16, 32)
KERNEL(adde64, ADDE64, 32)
KERNEL(xore64, XORE64, 32)
KERNEL(mix, MIX, 96)

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
        printf("%-10s %7.3f ms  clk %.2f GHz  wave-instr/SIMD/cycle %.3f  (cycles/instr %.2f)\n", #NAME, ms, ghz, \
               winstr / 1024 / (ms * 1e-3 * ghz * 1e9), 1.0 / (winstr / 1024 / (ms * 1e-3 * ghz * 1e9)));  \
    }
    RUN(add) RUN(xor) RUN(align) RUN(alignbyte) RUN(perm) RUN(xad) RUN(add3) RUN(lshlor) RUN(lshr) RUN(bitop3)
    RUN(pkadd16) RUN(adde64) RUN(xore64) RUN(mix)
    return 0;
}
