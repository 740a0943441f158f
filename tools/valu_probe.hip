// valu_probe.hip -- microbenchmark: ChaCha20 block throughput on gfx950 VALU.
// Variants: blocks interleaved per lane (ILP 4 vs 8), rotate form, occupancy.
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_probe valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ROTL(v, c) __builtin_rotateleft32((v), (c))
#define QR(a, b, c, d) a += b; d ^= a; d = ROTL(d, 16); c += d; b ^= c; b = ROTL(b, 12); a += b; d ^= a; d = ROTL(d, 8); c += d; b ^= c; b = ROTL(b, 7);

template <int NB>
__device__ __forceinline__ void blocks(uint32_t k, uint32_t ctr, uint32_t (&acc)[16]) {
    uint32_t x[NB][16];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[b][i] = k * (i + 1) + b;
        x[b][12] = ctr + b;
    }
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            QR(x[b][0], x[b][4], x[b][8], x[b][12]); QR(x[b][1], x[b][5], x[b][9], x[b][13]);
            QR(x[b][2], x[b][6], x[b][10], x[b][14]); QR(x[b][3], x[b][7], x[b][11], x[b][15]);
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            QR(x[b][0], x[b][5], x[b][10], x[b][15]); QR(x[b][1], x[b][6], x[b][11], x[b][12]);
            QR(x[b][2], x[b][7], x[b][8], x[b][13]); QR(x[b][3], x[b][4], x[b][9], x[b][14]);
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += x[b][i] ^ 0x64636261u;
}

template <int NB, int WPS>
__global__ __launch_bounds__(256, WPS) void probe(int iters, uint32_t *out) {
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    const uint32_t ctr = blockIdx.x * 256 + threadIdx.x;
    for (int it = 0; it < iters; it += NB) blocks<NB>(0x9e3779b9u * (it + 1), ctr, acc);
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s ^= acc[i];
    out[ctr] = s;
}

// pure independent-op probe: 8 chains of add/xor/alignbit
template <int CH>
__global__ __launch_bounds__(256) void indep(int iters, uint32_t *out) {
    uint32_t v[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = threadIdx.x * (i + 3);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) { v[i] += 0x1234567u; v[i] ^= it; v[i] = ROTL(v[i], 7); }
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) s += v[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    uint32_t *out;
    hipMalloc(&out, 256 * 1024 * 64 * 4);
    const int iters = 64;
    for (int grid : {2048, 4096, 8192}) {
        double words = (double)grid * 256 * iters * 16;
        float t1 = timeit([&] { hipLaunchKernelGGL((probe<1, 1>), dim3(grid), dim3(256), 0, 0, iters, out); });
        float t2 = timeit([&] { hipLaunchKernelGGL((probe<2, 1>), dim3(grid), dim3(256), 0, 0, iters, out); });
        float t1o = timeit([&] { hipLaunchKernelGGL((probe<1, 2>), dim3(grid), dim3(256), 0, 0, iters, out); });
        float t2o = timeit([&] { hipLaunchKernelGGL((probe<2, 2>), dim3(grid), dim3(256), 0, 0, iters, out); });
        printf("grid %5d  NB1 %.3f ms %.1f Gw/s | NB2 %.3f ms %.1f Gw/s | NB1,w2 %.3f ms %.1f | NB2,w2 %.3f ms %.1f\n", grid,
               t1, words / t1 / 1e6, t2, words / t2 / 1e6, t1o, words / t1o / 1e6, t2o, words / t2o / 1e6);
    }
    for (int grid : {4096, 16384}) {
        const int it2 = 4096;
        double ops = (double)grid * 256 * it2 * 8 * 3;
        float t = timeit([&] { hipLaunchKernelGGL((indep<8>), dim3(grid), dim3(256), 0, 0, it2, out); });
        double wave_instr = ops / 64;
        printf("indep8 grid %d: %.3f ms  %.2f Tops/s  wave-instr per SIMD-cycle @2.4GHz: %.3f\n", grid, t, ops / t / 1e9,
               wave_instr / (t * 1e-3) / 1024 / 2.4e9);
        float t4 = timeit([&] { hipLaunchKernelGGL((indep<2>), dim3(grid), dim3(256), 0, 0, it2, out); });
        double ops2 = (double)grid * 256 * it2 * 2 * 3;
        printf("indep2 grid %d: %.3f ms  %.2f Tops/s  wave-instr per SIMD-cycle @2.4GHz: %.3f\n", grid, t4, ops2 / t4 / 1e9,
               ops2 / 64 / (t4 * 1e-3) / 1024 / 2.4e9);
    }
    hipFree(out);
    return 0;
}
