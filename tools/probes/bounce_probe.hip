// bounce_probe.hip -- the cost of moving 4 MiB between pageable host memory and the GPU three ways:
// (a) hipMemcpyAsync straight from/to the pageable buffer (the HIP runtime stages or pins it itself),
// (b) std::memcpy into / out of a pinned bounce buffer + DMA, for hipHostMalloc's default (coherent)
//     and hipHostMallocNonCoherent allocations, (c) the CPU copies alone, so the DMA share is visible.
// Median of 50 round trips (H2D of one buffer + D2H of another), microseconds.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class F>
static double median_us(F f, int n = 50) {
    for (int i = 0; i < 5; ++i) f();
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
    const size_t n = 4u << 20;
    std::vector<uint8_t> src(n, 1), dst(n, 0);
    void *d = nullptr;
    (void)hipMalloc(&d, n);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    void *pin_def = nullptr, *pin_nc = nullptr;
    (void)hipHostMalloc(&pin_def, 2 * n, hipHostMallocDefault);
    (void)hipHostMalloc(&pin_nc, 2 * n, hipHostMallocNonCoherent);
    auto *pd = static_cast<uint8_t *>(pin_def), *pn = static_cast<uint8_t *>(pin_nc);

    printf("(a) pageable hipMemcpyAsync H2D + D2H:      %8.1f us\n", median_us([&] {
        (void)hipMemcpyAsync(d, src.data(), n, hipMemcpyHostToDevice, s);
        (void)hipMemcpyAsync(dst.data(), d, n, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }));
    for (int v = 0; v < 2; ++v) {
        uint8_t *b = v ? pn : pd;
        const char *name = v ? "non-coherent" : "default";
        printf("(b) bounce %-12s memcpy+DMA H2D + D2H:  %8.1f us\n", name, median_us([&] {
            std::memcpy(b, src.data(), n);
            (void)hipMemcpyAsync(d, b, n, hipMemcpyHostToDevice, s);
            (void)hipMemcpyAsync(b + n, d, n, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            std::memcpy(dst.data(), b + n, n);
        }));
        printf("(c) memcpy into %-12s:                %8.1f us\n", name, median_us([&] { std::memcpy(b, src.data(), n); }));
        printf("(c) memcpy out of %-12s:              %8.1f us\n", name, median_us([&] { std::memcpy(dst.data(), b + n, n); }));
        printf("(c) DMA alone %-12s H2D + D2H:         %8.1f us\n", name, median_us([&] {
            (void)hipMemcpyAsync(d, b, n, hipMemcpyHostToDevice, s);
            (void)hipMemcpyAsync(b + n, d, n, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
        }));
    }
    printf("(c) memcpy pageable -> pageable:             %8.1f us\n", median_us([&] { std::memcpy(dst.data(), src.data(), n); }));
    // (d) the runtime's rect path from/to the pageable buffer (one row): staged by the runtime, never pinned
    printf("(d) pageable hipMemcpy2DAsync 1 row H2D+D2H: %8.1f us\n", median_us([&] {
        (void)hipMemcpy2DAsync(d, n, src.data(), n, n, 1, hipMemcpyHostToDevice, s);
        (void)hipMemcpy2DAsync(dst.data(), n, d, n, n, 1, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
    }));
    // (e) 1 MiB pieces: memcpy piece i+1 while piece i's DMA runs (H2D), D2H pieces copied out as they land
    const size_t pc = 1u << 20;
    std::vector<hipEvent_t> ev(n / pc);
    for (auto &e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    for (int v = 0; v < 2; ++v) {
        uint8_t *b = v ? pn : pd;
        printf("(e) bounce %-12s pipelined 1 MiB pieces: %8.1f us\n", v ? "non-coherent" : "default", median_us([&] {
            for (size_t o = 0; o < n; o += pc) {
                std::memcpy(b + o, src.data() + o, pc);
                (void)hipMemcpyAsync(static_cast<uint8_t *>(d) + o, b + o, pc, hipMemcpyHostToDevice, s);
            }
            for (size_t o = 0, i = 0; o < n; o += pc, ++i) {
                (void)hipMemcpyAsync(b + n + o, static_cast<uint8_t *>(d) + o, pc, hipMemcpyDeviceToHost, s);
                (void)hipEventRecord(ev[i], s);
            }
            for (size_t o = 0, i = 0; o < n; o += pc, ++i) {
                (void)hipEventSynchronize(ev[i]);
                std::memcpy(dst.data() + o, b + n + o, pc);
            }
        }));
    }
    return 0;
}
