// chacha_full_probe.hip -- gfx950: whole ChaCha20 mask job (init, 20 rounds, feed-forward, XOR
// "abcd", accumulate) in one asm block; 1 vs 2 blocks per lane, lockstep vs staggered QR order.
// Checked against a plain C version of the same job.
// Build: python3 tools/probes/gen_chacha_asm.py full > tools/probes/chacha_full_gen.h &&
//        hipcc --offload-arch=gfx950 -O3 -o tools/probes/chacha_full_probe tools/probes/chacha_full_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "chacha_full_gen.h"

#define ROTL(v, c) __builtin_rotateleft32((v), (c))
#define QR(a, b, c, d) a += b; d ^= a; d = ROTL(d, 16); c += d; b ^= c; b = ROTL(b, 12); a += b; d ^= a; d = ROTL(d, 8); c += d; b ^= c; b = ROTL(b, 7);

#define CLOB1 "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47"
#define CLOB2 CLOB1, "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63"
#define ACC [a0] "+v"(acc[0]), [a1] "+v"(acc[1]), [a2] "+v"(acc[2]), [a3] "+v"(acc[3]), [a4] "+v"(acc[4]), \
    [a5] "+v"(acc[5]), [a6] "+v"(acc[6]), [a7] "+v"(acc[7]), [a8] "+v"(acc[8]), [a9] "+v"(acc[9]),           \
    [a10] "+v"(acc[10]), [a11] "+v"(acc[11]), [a12] "+v"(acc[12]), [a13] "+v"(acc[13]), [a14] "+v"(acc[14]), \
    [a15] "+v"(acc[15])
#define KEYS [k0] "s"(k[0]), [k1] "s"(k[1]), [k2] "s"(k[2]), [k3] "s"(k[3]), [k4] "s"(k[4]), [k5] "s"(k[5]), \
    [k6] "s"(k[6]), [k7] "s"(k[7])

__device__ __forceinline__ void cblock(const uint32_t (&k)[8], uint32_t ctr, uint32_t (&acc)[16]) {
    uint32_t x[16] = {0x61707865u, 0x3320646Eu, 0x79622D32u, 0x6B206574u, k[0], k[1], k[2], k[3],
                      k[4], k[5], k[6], k[7], ctr, 0, 0, 0};
    uint32_t in[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) in[i] = x[i];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]); QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]); QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] += (x[i] + in[i]) ^ 0x64636261u;
}

// V: 0 = C (2 blocks per iteration), 1 = asm NB1 lockstep (x2), 2 = asm NB1 stagger (x2),
//    3 = asm NB2 lockstep, 4 = asm NB2 stagger
template <int V>
__global__ __launch_bounds__(256) void probe(int iters, uint32_t *out, uint64_t *clk) {
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    const uint32_t c0 = (blockIdx.x * 256 + threadIdx.x) * 2;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        uint32_t k[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) k[i] = 0x9e3779b9u * (it + 1) * (i + 1) + i;
        if constexpr (V == 0) {
            cblock(k, c0, acc);
            cblock(k, c0 + 1, acc);
        } else if constexpr (V == 1 || V == 2) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const uint32_t cb = c0 + b;
                if constexpr (V == 1)
                    asm volatile(CHACHA_FULL_NB1_LOCKSTEP : ACC : KEYS, [ctr] "v"(cb) : CLOB1);
                else
                    asm volatile(CHACHA_FULL_NB1_STAGGER : ACC : KEYS, [ctr] "v"(cb) : CLOB1);
                (void)cb;
            }
        } else if constexpr (V == 3) {
            asm volatile(CHACHA_FULL_NB2_LOCKSTEP : ACC : KEYS, [ctr] "v"(c0) : CLOB2);
        } else {
            asm volatile(CHACHA_FULL_NB2_STAGGER : ACC : KEYS, [ctr] "v"(c0) : CLOB2);
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s = s * 31 + acc[i];
    out[c0 / 2] = s;
    if (c0 == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

static uint32_t h[1 << 21];
static uint32_t hsum(const uint32_t *d, size_t n) {
    (void)hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
    uint32_t s = 0;
    for (size_t i = 0; i < n; ++i) s = s * 1000003u + h[i];
    return s;
}

int main() {
    uint32_t *out;
    uint64_t *clk, hc[2];
    const int grid = 8192, iters = 32;
    const size_t n = (size_t)grid * 256;
    (void)hipMalloc(&out, n * 4);
    (void)hipMalloc(&clk, 16);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    uint32_t ref = 0;
    const char *names[] = {"C compiler", "asm NB1 lockstep", "asm NB1 stagger", "asm NB2 lockstep", "asm NB2 stagger"};
    auto run = [&](auto kern, int v) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        (void)hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost);
        double ghz = (double)hc[0] / ((double)hc[1] / 100e6) / 1e9;
        uint32_t hh = hsum(out, n);
        if (v == 0) ref = hh;
        double words = (double)n * iters * 2 * 16;
        printf("%-18s %.3f ms  %6.1f Gw/s  clk %.2f GHz  %s\n", names[v], ms, words / ms / 1e6, ghz,
               hh == ref ? "match" : "MISMATCH");
    };
    for (int rep = 0; rep < 2; ++rep) {
        run(probe<0>, 0);
        run(probe<1>, 1);
        run(probe<2>, 2);
        run(probe<3>, 3);
        run(probe<4>, 4);
    }
    return 0;
}
