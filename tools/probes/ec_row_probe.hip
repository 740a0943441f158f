// ec_row_probe.hip -- the row-sliced P-256 field layer (flamingo_amd/csrc/flm_fe_row.h) on gfx950:
// bit-exactness and lone-wave latency against the per-lane product-scanning multiply.
//   ec_row_probe check IN OUT   IN: n x 2 x 8 LE words (a, b); OUT per element: mul, add, sub,
//                               canon(mul), chain of 64 muls, canon(chain), is_zero flags (a - a, a)
//   ec_row_probe time           dependent multiply chains: row layout (4 elements per wave) and
//                               per-lane layout (64 per wave) over 1 .. 9600 waves
// Driven by tools/probes/ec_row_probe.py (inputs, checks against Python integers, the log).
// Build: hipcc --offload-arch=gfx950 -O3 -I flamingo_amd/csrc -o tools/probes/ec_row_probe tools/probes/ec_row_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "flm_fe_row.h"

using namespace flm;

// ------------------------------------------------------------ per-lane reference (Montgomery)
struct Fe {
    uint32_t v[8];
};
__device__ constexpr uint32_t kP[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};

__device__ __forceinline__ void mad1(uint64_t &A, uint32_t &hA, uint32_t a0, uint32_t b0) {
    uint64_t cA;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
        "v_addc_co_u32_e64 %1, %2, 0, %1, %2"
        : "+v"(A), "+v"(hA), "=&s"(cA)
        : "v"(a0), "v"(b0));
}

__device__ __forceinline__ Fe lane_mul(const Fe &a, const Fe &b) {
    uint32_t t[16];
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        uint64_t A = carry;
        uint32_t hA = 0;
        const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
#pragma unroll
        for (int q = 0; q < hi - lo + 1; ++q) mad1(A, hA, a.v[lo + q], b.v[k - lo - q]);
        t[k] = (uint32_t)A;
        carry = (A >> 32) | ((uint64_t)hA << 32);
    }
    t[15] = (uint32_t)carry;
    uint32_t m[8];
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int64_t s = (int64_t)t[i] + c;
        if (i >= 3 && i - 3 < 8) s += m[i - 3];
        if (i >= 6 && i - 6 < 8) s += m[i - 6];
        if (i >= 7 && i - 7 < 8) s -= m[i - 7];
        if (i >= 8 && i - 8 < 8) s += m[i - 8];
        if (i < 8) m[i] = (uint32_t)s; else t[i - 8] = (uint32_t)s;
        c = s >> 32;
    }
    uint32_t d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(t[i], kP[i], br, &br);
    const bool take = c || !br;
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = take ? d[i] : t[i];
    return r;
}

// ------------------------------------------------------------ kernels
// element e = blockIdx.x * 4 + (lane >> 4); its limbs in lanes r < 8 of the row
__global__ __launch_bounds__(64) void row_check(const uint32_t *in, uint32_t *out, int n) {
    const row::Ctx K = row::make_ctx();
    const int lane = threadIdx.x, r = lane & 15;
    const int e = blockIdx.x * 4 + (lane >> 4);
    const bool ok = e < n;
    const uint32_t a = ok && r < 8 ? in[(size_t)e * 16 + r] : 0u;
    const uint32_t b = ok && r < 8 ? in[(size_t)e * 16 + 8 + r] : 0u;
    const uint32_t m = row::mul(a, b, K);
    const uint32_t s = row::add(a, b, K);
    const uint32_t d = row::sub(a, b, K);
    const uint32_t mc = row::canon(m, K);
    uint32_t z = a;
#pragma unroll 1
    for (int i = 0; i < 64; ++i) z = row::mul(z, b, K);
    const uint32_t zc = row::canon(z, K);
    const bool z0 = row::is_zero(row::sub(a, a, K), K), z1 = row::is_zero(a, K);
    if (ok && r < 8) {
        uint32_t *o = out + (size_t)e * 48;
        o[r] = m;
        o[8 + r] = s;
        o[16 + r] = d;
        o[24 + r] = mc;
        o[32 + r] = z;
        o[40 + r] = zc;
    }
    if (ok && r == 8) out[(size_t)n * 48 + e] = (z0 ? 1u : 0u) | (z1 ? 2u : 0u);
}

__global__ __launch_bounds__(64) void row_chain(uint32_t *x, int reps) {
    const row::Ctx K = row::make_ctx();
    const int lane = threadIdx.x, r = lane & 15;
    uint32_t a = r < 8 ? x[blockIdx.x * 64 + lane] : 0u, b = r < 8 ? (a ^ 0x9e3779b9u) : 0u;
#pragma unroll 1
    for (int i = 0; i < reps; ++i) a = row::mul(a, b, K);
    x[blockIdx.x * 64 + lane] = a;
}

__global__ __launch_bounds__(64) void row_add_chain(uint32_t *x, int reps) {
    const row::Ctx K = row::make_ctx();
    const int lane = threadIdx.x, r = lane & 15;
    uint32_t a = r < 8 ? x[blockIdx.x * 64 + lane] : 0u, b = r < 8 ? (a ^ 0x9e3779b9u) : 0u;
#pragma unroll 1
    for (int i = 0; i < reps; ++i) a = row::sub(row::add(a, b, K), a, K);
    x[blockIdx.x * 64 + lane] = a;
}

__global__ __launch_bounds__(64) void lane_chain(Fe *x, int reps) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    Fe a = x[i], b = a;
    b.v[0] ^= 0x9e3779b9u;
    b.v[7] &= 0x7fffffffu;
    a.v[7] &= 0x7fffffffu;
#pragma unroll 1
    for (int r = 0; r < reps; ++r) a = lane_mul(a, b);
    x[i] = a;
}

#define CK(e)                                                                   \
    do {                                                                        \
        hipError_t er = (e);                                                    \
        if (er != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(er)); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main(int argc, char **argv) {
    if (argc >= 4 && std::string(argv[1]) == "check") {
        FILE *f = fopen(argv[2], "rb");
        if (!f) return 2;
        std::vector<uint32_t> h;
        uint32_t w;
        while (fread(&w, 4, 1, f) == 1) h.push_back(w);
        fclose(f);
        const int n = (int)(h.size() / 16);
        uint32_t *din, *dout;
        CK(hipMalloc(&din, h.size() * 4));
        CK(hipMalloc(&dout, ((size_t)n * 49) * 4));
        CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(row_check, dim3((n + 3) / 4), dim3(64), 0, 0, din, dout, n);
        CK(hipGetLastError());
        std::vector<uint32_t> o((size_t)n * 49);
        CK(hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost));
        FILE *g = fopen(argv[3], "wb");
        fwrite(o.data(), 4, o.size(), g);
        fclose(g);
        printf("check: %d elements\n", n);
        return 0;
    }
    // timing: a dependent chain of `reps` multiplies per element
    const int reps = 2000, maxw = 9600;
    uint32_t *x;
    CK(hipMalloc(&x, (size_t)maxw * 64 * 32));
    std::vector<uint32_t> h((size_t)maxw * 64 * 8);
    uint64_t z = 88172645463325252ull;
    for (auto &v : h) {
        z ^= z << 13; z ^= z >> 7; z ^= z << 17;
        v = (uint32_t)z;
    }
    CK(hipMemcpy(x, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    printf("waves  row_mul_ns  row_addsub_ns  lane_mul_ns   (per dependent operation, %d reps)\n", reps);
    for (int waves : {1, 64, 256, 600, 1024, 2400, 4800, 9600}) {
        const float tr = timeit([&] { hipLaunchKernelGGL(row_chain, dim3(waves), dim3(64), 0, 0, x, reps); });
        const float ta = timeit([&] { hipLaunchKernelGGL(row_add_chain, dim3(waves), dim3(64), 0, 0, x, reps); });
        const float tl = waves <= 2400
                             ? timeit([&] { hipLaunchKernelGGL(lane_chain, dim3(waves), dim3(64), 0, 0, (Fe *)x, reps); })
                             : 0.f;
        printf("%5d  %10.1f  %13.1f  %11.1f\n", waves, tr * 1e6 / reps, ta * 1e6 / reps / 2, tl * 1e6 / reps);
        fflush(stdout);
    }
    CK(hipGetLastError());
    return 0;
}
