// ec_probe.hip -- P-256 field-multiply variants on gfx950: single-wave latency and full-chip throughput.
// V0: CIOS with 64-bit C arithmetic (first kernel version)
// V1: product scanning, 96-bit column accumulator via __builtin_addc, one-pass special-form Montgomery reduction
// V3: V1 with the mad's own carry-out (inline asm v_mad_u64_u32 + v_addc) for the column sums
// Build: hipcc --offload-arch=gfx950 -O3 -o ec_probe ec_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

struct Fe { uint32_t v[8]; };
__device__ constexpr uint32_t kP[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};

__device__ __forceinline__ void reduce_once(Fe &r, const uint32_t (&t)[8], uint32_t t8) {
    uint32_t d[8];
    uint64_t b = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t x = (uint64_t)t[i] - kP[i] - b;
        d[i] = (uint32_t)x;
        b = x >> 63;
    }
    bool take = t8 || !b;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = take ? d[i] : t[i];
}

__device__ __forceinline__ Fe mont_special(uint32_t (&t)[16]) {
    uint32_t m[8];
    int64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        int64_t s = (int64_t)t[i] + carry;
        if (i >= 3 && i - 3 < 8) s += m[i - 3];
        if (i >= 6 && i - 6 < 8) s += m[i - 6];
        if (i >= 7 && i - 7 < 8) s -= m[i - 7];
        if (i >= 8 && i - 8 < 8) s += m[i - 8];
        if (i < 8) m[i] = (uint32_t)s; else t[i - 8] = (uint32_t)s;
        carry = s >> 32;
    }
    Fe r;
    uint32_t tt[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) tt[i] = t[i];
    reduce_once(r, tt, (uint32_t)carry);
    return r;
}

template <int V> __device__ __forceinline__ Fe fe_mul(const Fe &a, const Fe &b);

template <> __device__ __forceinline__ Fe fe_mul<0>(const Fe &a, const Fe &b) {
    uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t t8 = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c = (uint64_t)a.v[j] * b.v[i] + t[j] + (c >> 32);
            t[j] = (uint32_t)c;
        }
        uint64_t s = (uint64_t)t8 + (c >> 32);
        uint32_t hi0 = (uint32_t)s, hi1 = (uint32_t)(s >> 32);
        uint32_t m = t[0];
        c = (uint64_t)m * kP[0] + t[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            c = (uint64_t)m * kP[j] + t[j] + (c >> 32);
            t[j - 1] = (uint32_t)c;
        }
        s = (uint64_t)hi0 + (c >> 32);
        t[7] = (uint32_t)s;
        t8 = hi1 + (uint32_t)(s >> 32);
    }
    Fe r;
    reduce_once(r, t, t8);
    return r;
}

template <> __device__ __forceinline__ Fe fe_mul<1>(const Fe &a, const Fe &b) {
    uint32_t t[16];
    uint32_t c0 = 0, c1 = 0, c2 = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int j = k - i;
            if (j < 0 || j > 7) continue;
            uint64_t p = (uint64_t)a.v[i] * b.v[j];
            unsigned cy;
            c0 = __builtin_addc(c0, (uint32_t)p, 0u, &cy);
            c1 = __builtin_addc(c1, (uint32_t)(p >> 32), cy, &cy);
            c2 += cy;
        }
        t[k] = c0; c0 = c1; c1 = c2; c2 = 0;
    }
    t[15] = c0;
    return mont_special(t);
}

__device__ __forceinline__ void mad_acc(uint64_t &acc, uint32_t &hi, uint32_t a, uint32_t b) {
    uint64_t n, c, d;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(n), "=s"(c) : "v"(a), "v"(b), "v"(acc));
    asm("v_addc_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(hi), "=s"(d) : "v"(hi), "s"(c));
    acc = n;
}

template <> __device__ __forceinline__ Fe fe_mul<3>(const Fe &a, const Fe &b) {
    uint32_t t[16];
    uint64_t acc = 0;
    uint32_t hi = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int j = k - i;
            if (j < 0 || j > 7) continue;
            mad_acc(acc, hi, a.v[i], b.v[j]);
        }
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
        hi = 0;
    }
    t[15] = (uint32_t)acc;
    return mont_special(t);
}

// acc + t in one instruction (v_mad_u64_u32 t*1 + acc), two's complement so acc may be "negative"
__device__ __forceinline__ uint64_t add32(uint64_t acc, uint32_t t) {
    uint64_t r, c;
    asm("v_mad_u64_u32 %0, %1, %2, 1, %3" : "=v"(r), "=s"(c) : "v"(t), "v"(acc));
    return r;
}

// Montgomery reduction for p (quotient digit = low limb), column-signed accumulation, mads for the adds
__device__ __forceinline__ Fe mont_special_mad(uint32_t (&t)[16]) {
    uint32_t m[8];
    uint64_t s = t[0];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i > 0) s = add32(s, t[i]);
        if (i >= 3 && i - 3 < 8) s = add32(s, m[i - 3]);
        if (i >= 6 && i - 6 < 8) s = add32(s, m[i - 6]);
        if (i >= 8 && i - 8 < 8) s = add32(s, m[i - 8]);
        if (i >= 7 && i - 7 < 8) s -= m[i - 7];
        if (i < 8) m[i] = (uint32_t)s; else t[i - 8] = (uint32_t)s;
        s = (uint64_t)((int64_t)s >> 32);
    }
    Fe r;
    uint32_t tt[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) tt[i] = t[i];
    reduce_once(r, tt, (uint32_t)s);
    return r;
}

template <> __device__ __forceinline__ Fe fe_mul<4>(const Fe &a, const Fe &b) {
    uint32_t t[16];
    uint64_t acc = 0;
    uint32_t hi = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int j = k - i;
            if (j < 0 || j > 7) continue;
            mad_acc(acc, hi, a.v[i], b.v[j]);
        }
        t[k] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
        hi = 0;
    }
    t[15] = (uint32_t)acc;
    return mont_special_mad(t);
}

// squaring: 28 cross products doubled + 8 squares
template <> __device__ __forceinline__ Fe fe_mul<5>(const Fe &a, const Fe &) {
    uint32_t t[16];
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        uint64_t x = 0;
        uint32_t xh = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int j = k - i;
            if (j <= i || j > 7) continue;
            mad_acc(x, xh, a.v[i], a.v[j]);
        }
        xh = (xh << 1) | (uint32_t)(x >> 63);
        x <<= 1;
        uint64_t n = x + c;
        xh += (n < x);
        x = n;
        if ((k & 1) == 0) mad_acc(x, xh, a.v[k / 2], a.v[k / 2]);
        t[k] = (uint32_t)x;
        c = (x >> 32) | ((uint64_t)xh << 32);
    }
    t[15] = (uint32_t)c;
    return mont_special_mad(t);
}

// two independent accumulator chains per column (even / odd i) so the mad -> addc SGPR-carry
// hazard slots can be filled by the other chain instead of s_nop
template <> __device__ __forceinline__ Fe fe_mul<6>(const Fe &a, const Fe &b) {
    uint32_t t[16];
    uint64_t carry = 0;   // carry into this column (< 2^37)
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        uint64_t A = carry, B = 0;
        uint32_t ha = 0, hb = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int j = k - i;
            if (j < 0 || j > 7) continue;
            if (i & 1) mad_acc(B, hb, a.v[i], b.v[j]);
            else mad_acc(A, ha, a.v[i], b.v[j]);
        }
        uint64_t s = A + B;
        uint32_t h = ha + hb + (s < A);
        t[k] = (uint32_t)s;
        carry = (s >> 32) | ((uint64_t)h << 32);
    }
    t[15] = (uint32_t)carry;
    return mont_special(t);
}

// two products into two accumulators in ONE asm block: each carry is read one instruction
// after it is written, and no compiler s_nop pads between asm statements
__device__ __forceinline__ void mad_acc2(uint64_t &A, uint32_t &hA, uint64_t &B, uint32_t &hB, uint32_t a0,
                                         uint32_t b0, uint32_t a1, uint32_t b1) {
    uint64_t cA, cB;
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\t"
        "v_mad_u64_u32 %1, %5, %8, %9, %1\n\t"
        "v_addc_co_u32_e64 %2, %4, 0, %2, %4\n\t"
        "v_addc_co_u32_e64 %3, %5, 0, %3, %5"
        : "+v"(A), "+v"(B), "+v"(hA), "+v"(hB), "=&s"(cA), "=&s"(cB)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}

// single chain, mad and addc back to back in one block (tests whether a wait state is needed)
__device__ __forceinline__ void mad_acc1(uint64_t &A, uint32_t &hA, uint32_t a0, uint32_t b0) {
    uint64_t cA;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
        "v_addc_co_u32_e64 %1, %2, 0, %1, %2"
        : "+v"(A), "+v"(hA), "=&s"(cA)
        : "v"(a0), "v"(b0));
}

template <int PAIRED>
__device__ __forceinline__ void product_cols(const Fe &a, const Fe &b, uint32_t (&t)[16]) {
    uint64_t carry = 0;
#pragma unroll
    for (int k = 0; k < 15; ++k) {
        uint64_t A = carry, B = 0;
        uint32_t hA = 0, hB = 0;
        int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
        int n = hi - lo + 1;
        if (PAIRED) {
#pragma unroll
            for (int q = 0; q + 1 < n; q += 2)
                mad_acc2(A, hA, B, hB, a.v[lo + q], b.v[k - lo - q], a.v[lo + q + 1], b.v[k - lo - q - 1]);
            if (n & 1) mad_acc1(A, hA, a.v[hi], b.v[k - hi]);
            uint64_t s = A + B;
            uint32_t h = hA + hB + (s < A);
            t[k] = (uint32_t)s;
            carry = (s >> 32) | ((uint64_t)h << 32);
        } else {
#pragma unroll
            for (int q = 0; q < n; ++q) mad_acc1(A, hA, a.v[lo + q], b.v[k - lo - q]);
            t[k] = (uint32_t)A;
            carry = (A >> 32) | ((uint64_t)hA << 32);
        }
    }
    t[15] = (uint32_t)carry;
}

template <> __device__ __forceinline__ Fe fe_mul<7>(const Fe &a, const Fe &b) {
    uint32_t t[16];
    product_cols<1>(a, b, t);
    return mont_special(t);
}

template <> __device__ __forceinline__ Fe fe_mul<8>(const Fe &a, const Fe &b) {
    uint32_t t[16];
    product_cols<0>(a, b, t);
    return mont_special(t);
}

template <int V>
__global__ __launch_bounds__(64) void mul_chain(Fe *x, const Fe *y, int reps) {
    int i = blockIdx.x * 64 + threadIdx.x;
    Fe a = x[i], b = y[i];
#pragma unroll 1
    for (int r = 0; r < reps; ++r) a = fe_mul<V>(a, b);
    x[i] = a;
}

__global__ __launch_bounds__(64) void mad_chain(uint64_t *x, int reps) {
    int i = blockIdx.x * 64 + threadIdx.x;
    uint64_t a = x[i];
    uint32_t b = (uint32_t)a | 1u, c = (uint32_t)(a >> 7);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a) : "v"(b), "v"(c) : "s0", "s1");
    }
    x[i] = a;
}

__global__ __launch_bounds__(64) void mad_indep(uint64_t *x, int reps) {
    int i = blockIdx.x * 64 + threadIdx.x;
    uint64_t a0 = x[i], a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    uint32_t b = (uint32_t)a0 | 1u, c = (uint32_t)(a0 >> 7);
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a0) : "v"(b), "v"(c) : "s0", "s1");
            asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a1) : "v"(b), "v"(c) : "s0", "s1");
            asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a2) : "v"(b), "v"(c) : "s0", "s1");
            asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a3) : "v"(b), "v"(c) : "s0", "s1");
        }
    }
    x[i] = a0 ^ a1 ^ a2 ^ a3;
}

__global__ __launch_bounds__(64) void add_chain(uint32_t *x, int reps) {
    int i = blockIdx.x * 64 + threadIdx.x;
    uint32_t a = x[i], b = a * 3;
#pragma unroll 1
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int k = 0; k < 16; ++k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
    }
    x[i] = a;
}

__global__ void check_variants(const Fe *x, const Fe *y, int *bad) {
    int i = blockIdx.x * 64 + threadIdx.x;
    Fe a = x[i], b = y[i];
    // bring inputs below p first
    a = fe_mul<0>(a, a);
    b = fe_mul<0>(b, a);
    Fe r0 = fe_mul<0>(a, b), r1 = fe_mul<1>(a, b), r3 = fe_mul<3>(a, b), r4 = fe_mul<4>(a, b), r6 = fe_mul<6>(a, b), r7 = fe_mul<7>(a, b),
       r8 = fe_mul<8>(a, b);
    Fe s0 = fe_mul<0>(a, a), s5 = fe_mul<5>(a, a);
    int e = 0;
    for (int k = 0; k < 8; ++k) e |= (r0.v[k] != r1.v[k]) | (r0.v[k] != r3.v[k]) << 1 | (r0.v[k] != r4.v[k]) << 2 |
                                     (s0.v[k] != s5.v[k]) << 3 | (r0.v[k] != r6.v[k]) << 4 |
                                     (r0.v[k] != r7.v[k]) << 5 | (r0.v[k] != r8.v[k]) << 6;
    if (e) atomicOr(bad, e);
}

#define CK(e) do { hipError_t er = (e); if (er != hipSuccess) { printf("%s\n", hipGetErrorString(er)); return 1; } } while (0)

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    const int maxblk = 16384;
    Fe *x, *y;
    CK(hipMalloc(&x, sizeof(Fe) * 64 * maxblk));
    CK(hipMalloc(&y, sizeof(Fe) * 64 * maxblk));
    CK(hipMemset(x, 0x11, sizeof(Fe) * 64 * maxblk));
    CK(hipMemset(y, 0x37, sizeof(Fe) * 64 * maxblk));
    {
        // random-ish inputs for the check
        uint32_t *h = (uint32_t *)malloc(sizeof(Fe) * 64 * 1024 * 2);
        uint64_t z = 88172645463325252ull;
        for (int i = 0; i < 64 * 1024 * 16; ++i) { z ^= z << 13; z ^= z >> 7; z ^= z << 17; h[i] = (uint32_t)z; }
        for (int i = 0; i < 64; ++i) for (int k = 0; k < 8; ++k) h[i * 8 + k] = (i & 1) ? 0xffffffffu : h[i * 8 + k];
        CK(hipMemcpy(x, h, sizeof(Fe) * 64 * 1024, hipMemcpyHostToDevice));
        CK(hipMemcpy(y, h + 64 * 1024 * 8, sizeof(Fe) * 64 * 1024, hipMemcpyHostToDevice));
        int *bad; CK(hipMalloc(&bad, 4)); CK(hipMemset(bad, 0, 4));
        hipLaunchKernelGGL(check_variants, dim3(1024), dim3(64), 0, 0, x, y, bad);
        int hb = -1; CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
        printf("variant check mismatch mask: %d (0 = all variants agree)\n", hb);
        free(h);
    }
    int reps = 2000;
    for (int blk : {1, 256, 1024, 4096, 16384}) {
        float t0 = timeit([&] { hipLaunchKernelGGL(mul_chain<0>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t1 = timeit([&] { hipLaunchKernelGGL(mul_chain<1>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t3 = timeit([&] { hipLaunchKernelGGL(mul_chain<3>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t4 = timeit([&] { hipLaunchKernelGGL(mul_chain<4>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t5 = timeit([&] { hipLaunchKernelGGL(mul_chain<5>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t6 = timeit([&] { hipLaunchKernelGGL(mul_chain<6>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t7 = timeit([&] { hipLaunchKernelGGL(mul_chain<7>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        float t8 = timeit([&] { hipLaunchKernelGGL(mul_chain<8>, dim3(blk), dim3(64), 0, 0, x, y, reps); });
        double n = (double)blk * 64 * reps;
        printf("fe_mul waves %5d  V0 %7.1f ns/mul/wave %8.1f Gmul/s | V1 %7.1f ns %8.1f Gmul/s | V3 %7.1f ns %8.1f Gmul/s"
               " | V4 %7.1f ns %8.1f Gmul/s | sqr5 %7.1f ns %8.1f Gsqr/s | V6 %7.1f ns %8.1f Gmul/s | V7 %7.1f ns %8.1f | V8 %7.1f ns %8.1f\n",
               blk, t0 * 1e6 / reps, n / t0 / 1e6, t1 * 1e6 / reps, n / t1 / 1e6, t3 * 1e6 / reps, n / t3 / 1e6,
               t4 * 1e6 / reps, n / t4 / 1e6, t5 * 1e6 / reps, n / t5 / 1e6, t6 * 1e6 / reps, n / t6 / 1e6, t7 * 1e6 / reps, n / t7 / 1e6,
               t8 * 1e6 / reps, n / t8 / 1e6);
    }
    int r2 = 20000;
    for (int blk : {1, 1024, 16384}) {
        float tm = timeit([&] { hipLaunchKernelGGL(mad_chain, dim3(blk), dim3(64), 0, 0, (uint64_t *)x, r2); });
        float ti = timeit([&] { hipLaunchKernelGGL(mad_indep, dim3(blk), dim3(64), 0, 0, (uint64_t *)x, r2); });
        float ta = timeit([&] { hipLaunchKernelGGL(add_chain, dim3(blk), dim3(64), 0, 0, (uint32_t *)x, r2); });
        double ops = (double)r2 * 16;
        printf("waves %5d  dependent mad_u64 %.2f ns/op/wave  independent mad %.2f ns/op/wave  dependent add %.2f ns/op/wave\n",
               blk, tm * 1e6 / ops, ti * 1e6 / ops, ta * 1e6 / ops);
    }
    return 0;
}
