// rect_probe.hip -- hipMemcpy2DAsync between pageable host memory and the GPU at 4 MiB .. 512 MiB
// (one row, and 16 rows at a device pitch wider than the host rows): round-trip time, bytes exact
// after the trip, and -- run under AMD_LOG_LEVEL=4 -- whether the runtime ever pins the pageable
// buffer for it (it logs "Using Pinned resource" when it does; the rect path logs "Unpinned ... rect
// path" and stages through its own buffers).  The linear hipMemcpyAsync of the same buffers is
// timed beside it.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include <sys/mman.h>

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_us(F f, int n) {
    f();
    std::vector<double> t;
    for (int i = 0; i < n; ++i) {
        const double t0 = now_us();
        f();
        t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[n / 2];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (size_t mib : {4, 16, 64, 256, 512}) {
        const size_t n = mib << 20;
        // page-aligned anonymous mappings, as numpy's large arrays are
        auto *src = static_cast<uint8_t *>(mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
        auto *dst = static_cast<uint8_t *>(mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
        if (src == MAP_FAILED || dst == MAP_FAILED) return 1;
        for (size_t i = 0; i < n; ++i) src[i] = (uint8_t)(i * 2654435761u >> 13);
        void *d = nullptr;
        if (hipMalloc(&d, n + (n >> 2)) != hipSuccess) return 1;
        const int reps = mib >= 256 ? 5 : 15;
        fprintf(stdout, "== %zu MiB rect 1 row\n", mib);
        fflush(stdout);
        const double t_rect = median_us([&] {
            (void)hipMemcpy2DAsync(d, n, src, n, n, 1, hipMemcpyHostToDevice, s);
            (void)hipMemcpy2DAsync(dst, n, d, n, n, 1, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
        }, reps);
        const bool ok1 = std::memcmp(src, dst, n) == 0;
        std::memset(dst, 0, n);
        // 16 host rows packed, device rows at 1.25x the width
        const size_t w = n / 16, dp = w + (w >> 2);
        fprintf(stdout, "== %zu MiB rect 16 rows\n", mib);
        fflush(stdout);
        const double t_rows = median_us([&] {
            (void)hipMemcpy2DAsync(d, dp, src, w, w, 16, hipMemcpyHostToDevice, s);
            (void)hipMemcpy2DAsync(dst, w, d, dp, w, 16, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
        }, reps);
        const bool ok2 = std::memcmp(src, dst, n) == 0;
        fprintf(stdout, "== %zu MiB linear\n", mib);
        fflush(stdout);
        const double t_lin = median_us([&] {
            (void)hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, s);
            (void)hipMemcpyAsync(dst, d, n, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
        }, reps);
        printf("%4zu MiB  rect 1 row %9.1f us (%s, %5.1f GB/s)  rect 16 rows %9.1f us (%s)  linear %9.1f us\n", mib,
               t_rect, ok1 ? "exact" : "MISMATCH", 2.0 * n / t_rect / 1e3, t_rows, ok2 ? "exact" : "MISMATCH", t_lin);
        fflush(stdout);
        (void)hipFree(d);
        munmap(src, n);
        munmap(dst, n);
        if (!ok1 || !ok2) return 2;
    }
    return 0;
}
