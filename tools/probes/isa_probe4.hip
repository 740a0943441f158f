// isa_probe4.hip -- gfx950: issue cost of VALU ops with an SGPR or literal source, v_mov from an SGPR,
// and 3-source ops (the ChaCha block's non-QR instructions).  8 independent chains, 8 waves/SIMD, cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define A8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
#define OPS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), \
            "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7])
// operand numbering: a[i] = %i, b[i] = %(8+i), s = %16
#define S_(x) #x
#define S(x) S_(x)
#define BI_0 8
#define BI_1 9
#define BI_2 10
#define BI_3 11
#define BI_4 12
#define BI_5 13
#define BI_6 14
#define BI_7 15
#define PV_0 7
#define PV_1 0
#define PV_2 1
#define PV_3 2
#define PV_4 3
#define PV_5 4
#define PV_6 5
#define PV_7 6
#define ADD_DIST(i) "v_add_u32 %" S(i) ", %" S(BI_##i) ", %" S(i) "\n"
#define ADD_SGPR(i) "v_add_u32 %" S(i) ", %16, %" S(i) "\n"
#define ADD_LIT(i) "v_add_u32 %" S(i) ", 0x61707865, %" S(i) "\n"
#define XOR_SGPR(i) "v_xor_b32 %" S(i) ", %16, %" S(i) "\n"
#define MOV_SGPR(i) "v_mov_b32 %" S(i) ", %16\n"
#define MOV_DIST(i) "v_mov_b32 %" S(i) ", %" S(BI_##i) "\n"
#define ADD3_DIST(i) "v_add3_u32 %" S(i) ", %" S(BI_##i) ", %" S(i) ", %" S(PV_##i) "\n"
#define XAD_SGPR(i) "v_xad_u32 %" S(i) ", %" S(i) ", %16, %" S(BI_##i) "\n"
#define XAD_DIST(i) "v_xad_u32 %" S(i) ", %" S(i) ", %" S(PV_##i) ", %" S(BI_##i) "\n"
#define ADD_SGPR_E64(i) "v_add_u32_e64 %" S(i) ", %" S(i) ", %16\n"
#define ADD_E64(i) "v_add_u32_e64 %" S(i) ", %" S(i) ", %" S(BI_##i) "\n"
#define KERNEL(NAME, BODY, PER)                                                                         \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk, uint32_t s) { \
        uint32_t a[8], b[8];                                                                           \
        for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * (i + 3); b[i] = threadIdx.x ^ (i * 77); }  \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();             \
        for (int it = 0; it < iters; ++it) asm volatile(A8(BODY) A8(BODY) : OPS : "s"(s));             \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();             \
        uint32_t x = 0;                                                                                \
        for (int i = 0; i < 8; ++i) x += a[i] ^ b[i];                                                  \
        out[blockIdx.x * 256 + threadIdx.x] = x;                                                       \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }               \
    }                                                                                                  \
    static const int per_##NAME = PER;

KERNEL(add_dist, ADD_DIST, 16)
KERNEL(add_sgpr, ADD_SGPR, 16)
KERNEL(add_lit, ADD_LIT, 16)
KERNEL(xor_sgpr, XOR_SGPR, 16)
KERNEL(mov_sgpr, MOV_SGPR, 16)
KERNEL(mov_dist, MOV_DIST, 16)
KERNEL(add3_dist, ADD3_DIST, 16)
KERNEL(xad_sgpr, XAD_SGPR, 16)
KERNEL(xad_dist, XAD_DIST, 16)
KERNEL(add_sgpr_e64, ADD_SGPR_E64, 16)
KERNEL(add_e64, ADD_E64, 16)

int main() {
    uint32_t *out;
    uint64_t *clk, h[2];
    const int grid = 8192, iters = 4000;
    hipMalloc(&out, grid * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
#define RUN(NAME)                                                                                       \
    {                                                                                                   \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk, 5u);                 \
        hipDeviceSynchronize();                                                                         \
        hipEventRecord(e0);                                                                             \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk, 5u);                 \
        hipEventRecord(e1);                                                                             \
        hipEventSynchronize(e1);                                                                        \
        float ms;                                                                                       \
        hipEventElapsedTime(&ms, e0, e1);                                                               \
        hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);                                                   \
        double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;                                       \
        double wi = (double)grid * 4 * iters * per_##NAME;                                              \
        printf("%-22s %7.3f ms clk %.2f GHz cycles/wave-instr/SIMD %.2f\n", #NAME, ms, ghz,             \
               (ms * 1e-3 * ghz * 1e9) / (wi / 1024));                                                  \
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN(add_dist) RUN(add_sgpr) RUN(add_lit) RUN(xor_sgpr) RUN(mov_sgpr) RUN(mov_dist) RUN(add3_dist) RUN(xad_sgpr) RUN(xad_dist) RUN(add_sgpr_e64) RUN(add_e64)
    }
    return 0;
}
