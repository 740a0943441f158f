// h2d_probe.hip -- host->device copy rate on the GPU box: 1024 x 4 MiB rows from pinned memory,
// one stream vs several (several SDMA engines), one large copy, and pinned-allocation flags.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    const size_t row = 4u << 20, n = 1024, total = row * n;
    void *d;
    CK(hipMalloc(&d, total));
    struct Flag { const char *name; unsigned f; } flags[] = {{"default", hipHostMallocDefault},
                                                             {"numa_user", hipHostMallocNumaUser},
                                                             {"noncoherent", hipHostMallocNonCoherent}};
    for (auto fl : flags) {
        void *h = nullptr;
        if (hipHostMalloc(&h, total, fl.f) != hipSuccess) { printf("%s: alloc failed\n", fl.name); continue; }
        memset(h, 1, total);
        for (int ns : {1, 2, 4, 8}) {
            std::vector<hipStream_t> st(ns);
            for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            double best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipDeviceSynchronize());
                auto t0 = std::chrono::steady_clock::now();
                for (size_t i = 0; i < n; ++i)
                    CK(hipMemcpyAsync((char *)d + i * row, (char *)h + i * row, row, hipMemcpyHostToDevice, st[i % ns]));
                CK(hipDeviceSynchronize());
                double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                best = s < best ? s : best;
            }
            printf("%-12s rows x %d streams: %.1f ms  %.1f GB/s\n", fl.name, ns, best * 1e3, total / best / 1e9);
            for (auto &s : st) CK(hipStreamDestroy(s));
        }
        double best = 1e9;
        for (int rep = 0; rep < 3; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            CK(hipMemcpy(d, h, total, hipMemcpyHostToDevice));
            double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            best = s < best ? s : best;
        }
        printf("%-12s one 4 GiB copy: %.1f ms  %.1f GB/s\n", fl.name, best * 1e3, total / best / 1e9);
        CK(hipHostFree(h));
    }
    return 0;
}
