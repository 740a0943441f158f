// mix_probe2.hip -- follow-up to mix_probe.hip: chain count (8/16/32 chains of the D pattern:
// add a_i,a_{i+1}; xor a_i,a_{i+1}; alignbit a_i) against ChaCha QRs of 1/2/4 blocks in lockstep
// (compiler-scheduled), at one resident batch of 8 waves/SIMD and at two batches.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/mix_probe2 tools/probes/mix_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ROTL(v, c) __builtin_rotateleft32((v), (c))
// D pattern in C with an asm barrier per group so the compiler keeps the grouping
template <int NC, bool CHROT = false>
__global__ __launch_bounds__(256) void k_D(int iters, uint32_t *out, uint64_t *clk) {
    uint32_t a[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) a[i] = threadIdx.x * (i + 3) + blockIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int rep = 0; rep < 256 / (3 * NC) + 1; ++rep) {
#pragma unroll
            for (int i = 0; i < NC; ++i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) % NC]));
#pragma unroll
            for (int i = 0; i < NC; ++i) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) % NC]));
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                if (!CHROT) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(a[i]));
                else if ((rep & 3) == 0) asm volatile("v_alignbit_b32 %0, %0, %0, 16" : "+v"(a[i]));
                else if ((rep & 3) == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 20" : "+v"(a[i]));
                else if ((rep & 3) == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 24" : "+v"(a[i]));
                else asm volatile("v_alignbit_b32 %0, %0, %0, 25" : "+v"(a[i]));
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) s += a[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

// ChaCha double rounds on NB blocks per lane, lockstep across the NB*4 QRs of a half-round
template <int NB, bool R7 = false>
__global__ __launch_bounds__(256) void k_G(int iters, uint32_t *out, uint64_t *clk) {
    uint32_t x[NB][16];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) x[b][i] = threadIdx.x * (i + 3 + b) + blockIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int h = 0; h < 4 / NB + 0; ++h) {
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                int A[4], B[4], C[4], D[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    A[q] = q; B[q] = 4 + (half ? (q + 1) & 3 : q); C[q] = 8 + (half ? (q + 2) & 3 : q);
                    D[q] = 12 + (half ? (q + 3) & 3 : q);
                }
#define STEP(dst, src, op)                                                   \
    _Pragma("unroll") for (int b = 0; b < NB; ++b) _Pragma("unroll") for (int q = 0; q < 4; ++q) { op; }
                STEP(0, 0, x[b][A[q]] += x[b][B[q]])
                STEP(0, 0, x[b][D[q]] ^= x[b][A[q]])
                STEP(0, 0, x[b][D[q]] = ROTL(x[b][D[q]], R7 ? 7 : 16))
                STEP(0, 0, x[b][C[q]] += x[b][D[q]])
                STEP(0, 0, x[b][B[q]] ^= x[b][C[q]])
                STEP(0, 0, x[b][B[q]] = ROTL(x[b][B[q]], R7 ? 7 : 12))
                STEP(0, 0, x[b][A[q]] += x[b][B[q]])
                STEP(0, 0, x[b][D[q]] ^= x[b][A[q]])
                STEP(0, 0, x[b][D[q]] = ROTL(x[b][D[q]], R7 ? 7 : 8))
                STEP(0, 0, x[b][C[q]] += x[b][D[q]])
                STEP(0, 0, x[b][B[q]] ^= x[b][C[q]])
                STEP(0, 0, x[b][B[q]] = ROTL(x[b][B[q]], 7))
            }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) s += x[b][i];
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
        double winstr = (double)grid * 4 * iters * per;
        double per_ns = winstr / 1024 / (ms * 1e6);
        printf("%-6s grid %5d %8.3f ms clk %.2f GHz  cyc/instr %.2f  instr/ns/SIMD %.3f  instr/clk %.3f\n", name, grid,
               ms, ghz, ghz / per_ns, per_ns, per_ns / ghz);
    };
    for (int grid : {2048, 4096}) {
        run("D8", k_D<8>, grid, 3.0 * 8 * (256 / 24 + 1));
        run("D16", k_D<16>, grid, 3.0 * 16 * (256 / 48 + 1));
        run("D32", k_D<32>, grid, 3.0 * 32 * (256 / 96 + 1));
        run("G1", k_G<1>, grid, 4.0 * 2 * 12 * 4 * 1);
        run("G2", k_G<2>, grid, 2.0 * 2 * 12 * 4 * 2);
        run("G4", k_G<4>, grid, 1.0 * 2 * 12 * 4 * 4);
        run("D8rot", k_D<8, true>, grid, 3.0 * 8 * (256 / 24 + 1));
        run("G2r7", k_G<2, true>, grid, 2.0 * 2 * 12 * 4 * 2);
        run("G1r7", k_G<1, true>, grid, 4.0 * 2 * 12 * 4 * 1);
    }
    return 0;
}
