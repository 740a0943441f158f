// c2_native_probe.hip -- the c2 round (N=128, L=16384, K=128) enqueued from C++ through the C ABI,
// no Python in the loop: separates host submission cost from GPU time.  Prints the per-round time of
// 500 back-to-back rounds (HIP events) and, with a 200-us spin kernel queued first so the host runs
// ahead, the GPU-side cost per round with submission hidden.
// Build: hipcc --offload-arch=gfx950 -O3 -I include -o tools/probes/c2_native_probe tools/probes/c2_native_probe.hip \
//          -L flamingo_amd/lib -lflamingo_hip -Wl,-rpath,'$ORIGIN/../flamingo_amd/lib'
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "flamingo_hip.h"

__global__ void spin(long long cycles) {
    long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
}

int main() {
    const int N = 128, K = 128;
    const size_t L = 16384;
    flm_ctx *ctx = nullptr;
    if (flm_init(&ctx, 0)) { printf("init failed\n"); return 1; }
    uint32_t *rows, *out;
    uint8_t *seeds;
    int8_t *signs;
    (void)hipMalloc(&rows, (size_t)N * L * 4);
    (void)hipMalloc(&out, L * 4);
    (void)hipMalloc(&seeds, K * 32);
    (void)hipMalloc(&signs, K);
    std::vector<uint8_t> hs(K * 32);
    std::vector<int8_t> hg(K);
    for (int i = 0; i < K * 32; ++i) hs[i] = (uint8_t)(i * 131 + 7);
    for (int i = 0; i < K; ++i) hg[i] = (i & 1) ? -1 : 1;
    (void)hipMemcpy(seeds, hs.data(), hs.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(signs, hg.data(), hg.size(), hipMemcpyHostToDevice);
    (void)hipMemset(rows, 1, (size_t)N * L * 4);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto round = [&] {
        return flm_aggregate_unmask_dev(ctx, rows, L, N, seeds, signs, K, L, 0, L, 0, out, s);
    };
    for (int i = 0; i < 20; ++i) round();
    (void)hipStreamSynchronize(s);
    for (int rep = 0; rep < 3; ++rep) {
        const int n = 500;
        auto h0 = std::chrono::steady_clock::now();
        (void)hipEventRecord(a, s);
        for (int i = 0; i < n; ++i) round();
        (void)hipEventRecord(b, s);
        auto h1 = std::chrono::steady_clock::now();
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        double host_us = std::chrono::duration<double, std::micro>(h1 - h0).count() / n;
        // host runs ahead of a long spin: the events then time GPU work only
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 2400LL * 4000);
        (void)hipEventRecord(a, s);
        for (int i = 0; i < n; ++i) round();
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms2;
        (void)hipEventElapsedTime(&ms2, a, b);
        printf("back-to-back %.2f us/round (host submit %.2f us/round) | queued behind spin %.2f us/round\n",
               ms * 1e3 / n, host_us, ms2 * 1e3 / n);
    }
    flm_free(ctx);
    return 0;
}
