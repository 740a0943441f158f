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

// grouped schedule: the 4 independent QRs advance in lock-step, one op type per
// group of 4, sched_barrier between groups so the compiler keeps the pattern.
#define SB __builtin_amdgcn_sched_barrier(0);
#define G4(OPA, OPB, OPC, OPD) OPA; OPB; OPC; OPD; SB
#define RQ4(a0,b0,c0,d0, a1,b1,c1,d1, a2,b2,c2,d2, a3,b3,c3,d3) \
    G4(a0 += b0, a1 += b1, a2 += b2, a3 += b3) G4(d0 ^= a0, d1 ^= a1, d2 ^= a2, d3 ^= a3) \
    G4(d0 = ROTL(d0,16), d1 = ROTL(d1,16), d2 = ROTL(d2,16), d3 = ROTL(d3,16)) \
    G4(c0 += d0, c1 += d1, c2 += d2, c3 += d3) G4(b0 ^= c0, b1 ^= c1, b2 ^= c2, b3 ^= c3) \
    G4(b0 = ROTL(b0,12), b1 = ROTL(b1,12), b2 = ROTL(b2,12), b3 = ROTL(b3,12)) \
    G4(a0 += b0, a1 += b1, a2 += b2, a3 += b3) G4(d0 ^= a0, d1 ^= a1, d2 ^= a2, d3 ^= a3) \
    G4(d0 = ROTL(d0,8), d1 = ROTL(d1,8), d2 = ROTL(d2,8), d3 = ROTL(d3,8)) \
    G4(c0 += d0, c1 += d1, c2 += d2, c3 += d3) G4(b0 ^= c0, b1 ^= c1, b2 ^= c2, b3 ^= c3) \
    G4(b0 = ROTL(b0,7), b1 = ROTL(b1,7), b2 = ROTL(b2,7), b3 = ROTL(b3,7))

__device__ __forceinline__ void block_grouped(uint32_t k, uint32_t ctr, uint32_t (&acc)[16]) {
    uint32_t x0,x1,x2,x3,x4,x5,x6,x7,x8,x9,x10,x11,x12,x13,x14,x15;
    x0=k;x1=k*2;x2=k*3;x3=k*4;x4=k*5;x5=k*6;x6=k*7;x7=k*8;x8=k*9;x9=k*10;x10=k*11;x11=k*12;x12=ctr;x13=k*14;x14=k*15;x15=k*16;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        RQ4(x0,x4,x8,x12, x1,x5,x9,x13, x2,x6,x10,x14, x3,x7,x11,x15)
        RQ4(x0,x5,x10,x15, x1,x6,x11,x12, x2,x7,x8,x13, x3,x4,x9,x14)
    }
    acc[0]+=x0^0x64636261u; acc[1]+=x1^0x64636261u; acc[2]+=x2^0x64636261u; acc[3]+=x3^0x64636261u;
    acc[4]+=x4^0x64636261u; acc[5]+=x5^0x64636261u; acc[6]+=x6^0x64636261u; acc[7]+=x7^0x64636261u;
    acc[8]+=x8^0x64636261u; acc[9]+=x9^0x64636261u; acc[10]+=x10^0x64636261u; acc[11]+=x11^0x64636261u;
    acc[12]+=x12^0x64636261u; acc[13]+=x13^0x64636261u; acc[14]+=x14^0x64636261u; acc[15]+=x15^0x64636261u;
}

__global__ __launch_bounds__(256) void probe_grouped(int iters, uint32_t *out) {
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    const uint32_t ctr = blockIdx.x * 256 + threadIdx.x;
    for (int it = 0; it < iters; ++it) block_grouped(0x9e3779b9u * (it + 1), ctr, acc);
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s ^= acc[i];
    out[ctr] = s;
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
        float tg = timeit([&] { hipLaunchKernelGGL(probe_grouped, dim3(grid), dim3(256), 0, 0, iters, out); });
        printf("grid %5d  grouped %.3f ms %.1f Gw/s\n", grid, tg, words / tg / 1e6);
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
