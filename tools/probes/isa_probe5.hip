// isa_probe5.hip -- gfx950: issue cost of the candidate ways to do ChaCha20's 16- and 8-bit rotates.
// isa_probe3 measured v_add_u32 / v_xor_b32 at ~2.3 cycles per wave-instruction per SIMD and the
// v_alignbit_b32 rotate at ~4.1 (profiles/r01_isa_probe3.log).  Here: v_perm_b32 (byte permute,
// selector in a VGPR), v_alignbyte_b32, SDWA forms of v_xor_b32 / v_mov_b32 (word selects: a
// rotate by 16 fused into the xor as two half-word xors into a fresh register), and the chacha
// step "a += b; d ^= a; d = rotl(d, 16)" written both ways.  8 independent chains per wave,
// 8 waves/SIMD, cycles per wave-instruction per SIMD from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define A8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
#define OPS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), \
            "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]), \
            "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]), "+v"(t[4]), "+v"(t[5]), "+v"(t[6]), "+v"(t[7])
// operand numbering: a[i] = %i, b[i] = %(8+i), t[i] = %(16+i), selector VGPR = %24
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
#define TI_0 16
#define TI_1 17
#define TI_2 18
#define TI_3 19
#define TI_4 20
#define TI_5 21
#define TI_6 22
#define TI_7 23
#define ALIGN16(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %" S(i) ", 16\n"
#define PERM(i) "v_perm_b32 %" S(i) ", %" S(i) ", %" S(i) ", %24\n"
#define ALIGNBYTE(i) "v_alignbyte_b32 %" S(i) ", %" S(i) ", %" S(i) ", 2\n"
#define XOR_SDWA(i) "v_xor_b32_sdwa %" S(i) ", %" S(i) ", %" S(BI_##i) " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n"
#define MOV_SDWA(i) "v_mov_b32_sdwa %" S(i) ", %" S(BI_##i) " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n"
#define XOR(i) "v_xor_b32 %" S(i) ", %" S(BI_##i) ", %" S(i) "\n"
// step with a plain xor + rotate: a += b; d ^= a; d = rotl(d, 16)   (a = b[i], b = t[i], d = a[i])
#define STEP_ALIGN(i) "v_add_u32 %" S(BI_##i) ", %" S(TI_##i) ", %" S(BI_##i) "\n" \
                      "v_xor_b32 %" S(i) ", %" S(BI_##i) ", %" S(i) "\n" ALIGN16(i)
// the same step with the rotate fused into two half-word xors: n.lo = d.hi ^ a.hi, n.hi = d.lo ^ a.lo,
// written into t (the step after would read t as d); then the roles swap back with a plain add into a
// (keeps the chain's register set fixed for the probe: 4 instructions, 3 of them the step's)
#define STEP_SDWA(i) "v_add_u32 %" S(BI_##i) ", %" S(TI_##i) ", %" S(BI_##i) "\n" \
    "v_xor_b32_sdwa %" S(TI_##i) ", %" S(i) ", %" S(BI_##i) " dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n" \
    "v_xor_b32_sdwa %" S(TI_##i) ", %" S(i) ", %" S(BI_##i) " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n" \
    "v_add_u32 %" S(i) ", %" S(TI_##i) ", %" S(i) "\n"
#define STEP_PERM(i) "v_add_u32 %" S(BI_##i) ", %" S(TI_##i) ", %" S(BI_##i) "\n" \
                     "v_xor_b32 %" S(i) ", %" S(BI_##i) ", %" S(i) "\n" PERM(i)

#define KERNEL(NAME, BODY, PER)                                                                         \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk, uint32_t sel) { \
        uint32_t a[8], b[8], t[8];                                                                     \
        uint32_t vs = sel + (threadIdx.x >> 10);                                                       \
        for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * (i + 3); b[i] = threadIdx.x ^ (i * 77); t[i] = i; } \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();             \
        for (int it = 0; it < iters; ++it) asm volatile(A8(BODY) A8(BODY) : OPS : "v"(vs));           \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();             \
        uint32_t x = 0;                                                                                \
        for (int i = 0; i < 8; ++i) x += a[i] ^ b[i] ^ t[i];                                           \
        out[blockIdx.x * 256 + threadIdx.x] = x;                                                       \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }               \
    }                                                                                                  \
    static const int per_##NAME = PER;

KERNEL(xor_plain, XOR, 16)
KERNEL(align16, ALIGN16, 16)
KERNEL(perm_vsel, PERM, 16)
KERNEL(alignbyte, ALIGNBYTE, 16)
KERNEL(xor_sdwa, XOR_SDWA, 16)
KERNEL(mov_sdwa, MOV_SDWA, 16)
KERNEL(step_align, STEP_ALIGN, 48)
KERNEL(step_sdwa, STEP_SDWA, 64)
KERNEL(step_perm, STEP_PERM, 48)

int main() {
    uint32_t *out;
    uint64_t *clk, h[2];
    const int grid = 8192, iters = 4000;
    (void)hipMalloc(&out, grid * 256 * 4);
    (void)hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
#define RUN(NAME)                                                                                       \
    {                                                                                                   \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk, 0x01000302u);        \
        (void)hipDeviceSynchronize();                                                                   \
        (void)hipEventRecord(e0);                                                                       \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk, 0x01000302u);        \
        (void)hipEventRecord(e1);                                                                       \
        (void)hipEventSynchronize(e1);                                                                  \
        float ms;                                                                                       \
        (void)hipEventElapsedTime(&ms, e0, e1);                                                         \
        (void)hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);                                             \
        double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;                                       \
        double wi = (double)grid * 4 * iters * per_##NAME;                                              \
        printf("%-12s %7.3f ms clk %.2f GHz cycles/wave-instr/SIMD %.2f\n", #NAME, ms, ghz,             \
               (ms * 1e-3 * ghz * 1e9) / (wi / 1024));                                                  \
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN(xor_plain) RUN(align16) RUN(perm_vsel) RUN(alignbyte) RUN(xor_sdwa) RUN(mov_sdwa) RUN(step_align)
        RUN(step_sdwa) RUN(step_perm)
    }
    return 0;
}
