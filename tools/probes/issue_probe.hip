// issue_probe.hip -- why does the D8 mix (profiles/r01_mix_probe2.log: 3.44 cycles per wave
// instruction) issue faster than ChaCha20 QRs grouped the same way (~4.0)?  Every variant is
// inline asm, one instruction per statement, 8 independent chains, 8 waves/SIMD:
//   D8        ring a[i] += a[i+1]; a[i] ^= a[i+1]; a[i] = rot(a[i])   (mix_probe2's D8)
//   TWOSET    a[i] += b[i]; b[i] ^= a[i]; b[i] = rot(b[i])            (two register sets)
//   QR8       8 ChaCha quarter rounds in lockstep (a += b; d ^= a; d = rot d; c += d; ...)
//   QR8_LSHR  QR8 with every rotate replaced by a (fast) v_lshrrev_b32: the no-rotate bound
//   QR8_ROTLAST  QR8 with the 4 rotate groups of each QR moved behind one another (same count)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/issue_probe tools/probes/issue_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ADD(x, y) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "v"(y))
#define XOR(x, y) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(y))
#define ROT(x, s) asm volatile("v_alignbit_b32 %0, %0, %0, " #s : "+v"(x))
#define LSR(x, s) asm volatile("v_lshrrev_b32 %0, " #s ", %0" : "+v"(x))

enum { kD8 = 0, kTwoSet = 1, kQR8 = 2, kQR8Lshr = 3, kQR8RotLast = 4 };

template <int V>
__global__ __launch_bounds__(256) void probe(int iters, uint32_t *out, uint64_t *clk) {
    uint32_t a[8], b[8], c[8], d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * (i + 3) + blockIdx.x;
        b[i] = threadIdx.x ^ (i * 77);
        c[i] = threadIdx.x + i * 1234567u;
        d[i] = blockIdx.x * (i + 5);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int rep = 0; rep < 4; ++rep) {
            if constexpr (V == kD8) {  // 8 x 3 x 3 = 72 ... repeated 4 x per rep -> 96 per rep
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) ADD(a[i], a[(i + 1) & 7]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) XOR(a[i], a[(i + 1) & 7]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) ROT(a[i], 25);
                }
            } else if constexpr (V == kTwoSet) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) ADD(a[i], b[i]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) XOR(b[i], a[i]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) ROT(b[i], 25);
                }
            } else if constexpr (V == kQR8 || V == kQR8Lshr) {
#define R_(x, s) do { if constexpr (V == kQR8) ROT(x, s); else LSR(x, s); } while (0)
#pragma unroll
                for (int i = 0; i < 8; ++i) ADD(a[i], b[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) XOR(d[i], a[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) R_(d[i], 16);
#pragma unroll
                for (int i = 0; i < 8; ++i) ADD(c[i], d[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) XOR(b[i], c[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) R_(b[i], 20);
#pragma unroll
                for (int i = 0; i < 8; ++i) ADD(a[i], b[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) XOR(d[i], a[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) R_(d[i], 24);
#pragma unroll
                for (int i = 0; i < 8; ++i) ADD(c[i], d[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) XOR(b[i], c[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) R_(b[i], 25);
#undef R_
            } else {  // kQR8RotLast: the first QR half with 4 of the 8 chains' rotates deferred
                // a += b; d ^= a for chains 0..7, then the 8 rotates split 4 + 4 around c += d of
                // the chains already rotated: the same 96 instructions, fast ops in runs of 12
#pragma unroll
                for (int i = 0; i < 8; ++i) ADD(a[i], b[i]);
#pragma unroll
                for (int i = 0; i < 8; ++i) XOR(d[i], a[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) ROT(d[i], 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) ADD(c[i], d[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ROT(d[i], 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) XOR(b[i], c[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ADD(c[i], d[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) ROT(b[i], 20);
#pragma unroll
                for (int i = 4; i < 8; ++i) XOR(b[i], c[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) ADD(a[i], b[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ROT(b[i], 20);
#pragma unroll
                for (int i = 0; i < 4; ++i) XOR(d[i], a[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ADD(a[i], b[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) ROT(d[i], 24);
#pragma unroll
                for (int i = 4; i < 8; ++i) XOR(d[i], a[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) ADD(c[i], d[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ROT(d[i], 24);
#pragma unroll
                for (int i = 0; i < 4; ++i) XOR(b[i], c[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ADD(c[i], d[i]);
#pragma unroll
                for (int i = 0; i < 4; ++i) ROT(b[i], 25);
#pragma unroll
                for (int i = 4; i < 8; ++i) XOR(b[i], c[i]);
#pragma unroll
                for (int i = 4; i < 8; ++i) ROT(b[i], 25);
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] ^ b[i] ^ c[i] ^ d[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

int main() {
    uint32_t *out;
    uint64_t *clk, hclk[2];
    const int iters = 2000;
    hipMalloc(&out, 16384 * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t ea, eb;
    hipEventCreate(&ea);
    hipEventCreate(&eb);
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    auto run = [&](const char *name, auto kern, int grid, double per_iter) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        hipDeviceSynchronize();
        hipEventRecord(ea);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        hipEventRecord(eb);
        hipEventSynchronize(eb);
        float ms;
        hipEventElapsedTime(&ms, ea, eb);
        hipMemcpy(hclk, clk, 16, hipMemcpyDeviceToHost);
        const double ghz = (double)hclk[0] / ((double)hclk[1] / 100e6) / 1e9;
        const double winstr = (double)grid * 4 * iters * per_iter;        // wave instructions
        const double per_ns = winstr / (4.0 * n_cu) / (ms * 1e6);           // per SIMD per ns
        printf("%-12s grid %5d %8.3f ms clk %.2f GHz  cycles/wave-instr/SIMD %.2f\n", name, grid, ms, ghz,
               ghz / per_ns);
    };
    const int grid = 8 * n_cu;  // 8 waves per SIMD (256-thread workgroups, 4 waves each)
    for (int pass = 0; pass < 2; ++pass) {
        run("D8", probe<kD8>, grid, 4.0 * 4 * 24);
        run("TWOSET", probe<kTwoSet>, grid, 4.0 * 4 * 24);
        run("QR8", probe<kQR8>, grid, 4.0 * 96);
        run("QR8_LSHR", probe<kQR8Lshr>, grid, 4.0 * 96);
        run("QR8_ROTLAST", probe<kQR8RotLast>, grid, 4.0 * 96);
    }
    return 0;
}
