// mix_probe.hip -- gfx950: why does a grouped add/xor/alignbit mix reach ~3.1 cycles per
// wave-instruction (isa_probe2 mix_dist8) while ChaCha20 with the same grouping stays at ~3.9?
// Bridges the two one operand pattern at a time: 8 chains a0..a7, runs of 8 same-type ops.
//   A: add a_i,b        xor a_i,b        align a_i   (isa_probe2 mix_dist8)
//   B: add a_i,a_{i+1}  xor a_i,b        align a_i
//   C: add a_i,b        xor a_i,a_{i+1}  align a_i
//   D: add a_i,a_{i+1}  xor a_i,a_{i+1}  align a_i
//   E: add a_i,c_i      xor a_i,c_i      align a_i    (c_i distinct, never written)
//   F: as D with the align run split: 4 aligns, 8 adds, 4 aligns, 8 xors
//   G: ChaCha column QRs of 2 blocks in lockstep (4 QRs x 2 blocks = 8 chains per step)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/mix_probe tools/probes/mix_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define S_(x) #x
#define S(x) S_(x)
#define NX(i) NX_##i
#define NX_0 1
#define NX_1 2
#define NX_2 3
#define NX_3 4
#define NX_4 5
#define NX_5 6
#define NX_6 7
#define NX_7 0
// operands: a[i] = %i (0..7), b = %8, c[i] = %(9+i)
#define ADDB(i) "v_add_u32 %" S(i) ", %8, %" S(i) "\n"
#define XORB(i) "v_xor_b32 %" S(i) ", %8, %" S(i) "\n"
#define ADDN(i) "v_add_u32 %" S(i) ", %" S(NX(i)) ", %" S(i) "\n"
#define XORN(i) "v_xor_b32 %" S(i) ", %" S(NX(i)) ", %" S(i) "\n"
#define ADDC(i) "v_add_u32 %" S(i) ", %" S(CI(i)) ", %" S(i) "\n"
#define XORC(i) "v_xor_b32 %" S(i) ", %" S(CI(i)) ", %" S(i) "\n"
#define CI(i) CI_##i
#define CI_0 9
#define CI_1 10
#define CI_2 11
#define CI_3 12
#define CI_4 13
#define CI_5 14
#define CI_6 15
#define CI_7 16
#define ALN(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %" S(i) ", 7\n"
#define R8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
#define R4a(M) M(0) M(1) M(2) M(3)
#define R4b(M) M(4) M(5) M(6) M(7)

#define BODY_A R8(ADDB) R8(XORB) R8(ALN)
#define BODY_B R8(ADDN) R8(XORB) R8(ALN)
#define BODY_C R8(ADDB) R8(XORN) R8(ALN)
#define BODY_D R8(ADDN) R8(XORN) R8(ALN)
#define BODY_E R8(ADDC) R8(XORC) R8(ALN)
#define BODY_F R4a(ALN) R8(ADDN) R4b(ALN) R8(XORN)

#define OPS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
#define INS "v"(b), "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7])

#define KERNEL(NAME, BODY)                                                                              \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk) {          \
        uint32_t a[8], c[8], b = threadIdx.x * 7 + 1;                                                  \
        for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * (i + 3); c[i] = threadIdx.x ^ (i * 77); }  \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();             \
        for (int it = 0; it < iters; ++it) asm volatile(BODY BODY : OPS : INS);                        \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();             \
        uint32_t x = 0;                                                                                \
        for (int i = 0; i < 8; ++i) x += a[i];                                                         \
        out[blockIdx.x * 256 + threadIdx.x] = x;                                                       \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }               \
    }

KERNEL(A, BODY_A)
KERNEL(B, BODY_B)
KERNEL(C, BODY_C)
KERNEL(D, BODY_D)
KERNEL(E, BODY_E)
KERNEL(F, BODY_F)

// G: column QR of ChaCha for 2 blocks (x: 16 words each) in lockstep; 96 ops per loop body x2.
#define ROTL(v, c) __builtin_rotateleft32((v), (c))
__global__ __launch_bounds__(256) void k_G(int iters, uint32_t *out, uint64_t *clk) {
    uint32_t x[32];
    for (int i = 0; i < 32; ++i) x[i] = threadIdx.x * (i + 3) + blockIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#define Q(a, b, c, d)                                                                    \
    for (int k = 0; k < 8; ++k) { x[a[k]] += x[b[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[d[k]] ^= x[a[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[d[k]] = ROTL(x[d[k]], 16); }                         \
    for (int k = 0; k < 8; ++k) { x[c[k]] += x[d[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[b[k]] ^= x[c[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[b[k]] = ROTL(x[b[k]], 12); }                         \
    for (int k = 0; k < 8; ++k) { x[a[k]] += x[b[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[d[k]] ^= x[a[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[d[k]] = ROTL(x[d[k]], 8); }                          \
    for (int k = 0; k < 8; ++k) { x[c[k]] += x[d[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[b[k]] ^= x[c[k]]; }                                  \
    for (int k = 0; k < 8; ++k) { x[b[k]] = ROTL(x[b[k]], 7); }
            {
                const int A[8] = {0, 1, 2, 3, 16, 17, 18, 19}, B[8] = {4, 5, 6, 7, 20, 21, 22, 23},
                          C[8] = {8, 9, 10, 11, 24, 25, 26, 27}, D[8] = {12, 13, 14, 15, 28, 29, 30, 31};
#pragma unroll
                for (int z = 0; z < 1; ++z) { Q(A, B, C, D) }
            }
            {
                const int A[8] = {0, 1, 2, 3, 16, 17, 18, 19}, B[8] = {5, 6, 7, 4, 21, 22, 23, 20},
                          C[8] = {10, 11, 8, 9, 26, 27, 24, 25}, D[8] = {15, 12, 13, 14, 31, 28, 29, 30};
#pragma unroll
                for (int z = 0; z < 1; ++z) { Q(A, B, C, D) }
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
    for (int i = 0; i < 32; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

int main() {
    uint32_t *out;
    uint64_t *clk, hclk[2];
    const int iters = 1000;
    hipMalloc(&out, 16384 * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t ea, eb;
    hipEventCreate(&ea);
    hipEventCreate(&eb);
    auto run = [&](const char *name, auto kern, int grid, double per) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        hipDeviceSynchronize();
        hipEventRecord(ea);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        hipEventRecord(eb);
        hipEventSynchronize(eb);
        float ms;
        hipEventElapsedTime(&ms, ea, eb);
        hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
        double ghz = (double)hclk[0] / ((double)hclk[1] / 100e6) / 1e9;
        double winstr = (double)grid * 4 * iters * per;   // wave-instructions (4 waves per block)
        double per_ns = winstr / 1024 / (ms * 1e6);      // wave-instr per ns per SIMD
        printf("%-3s grid %5d %8.3f ms clk %.2f GHz  cycles/wave-instr/SIMD %.2f  wave-instr/ns/SIMD %.3f\n",
               name, grid, ms, ghz, ghz / per_ns, per_ns);
    };
    for (int grid : {1024, 2048, 8192}) {
        run("A", k_A, grid, 48);
        run("B", k_B, grid, 48);
        run("C", k_C, grid, 48);
        run("D", k_D, grid, 48);
        run("E", k_E, grid, 48);
        run("F", k_F, grid, 48);
        run("G", k_G, grid / 4, 2.0 * 2 * 96 * 1.0);
    }
    return 0;
}
