// pack_probe.hip -- gfx950: is v_pack_b32_f16 with op_sel:[1,0] (lo = src0.hi, hi = src1.lo) a
// bit-exact 32-bit rotate by 16 for all 2^32 inputs (no fp16 denormal flush, no NaN quieting),
// and what does it cost next to v_alignbit_b32 (4 cycles) in the ChaCha add/xor/rotate mix?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define A8(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7)
#define OPS "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), \
            "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7])
// operand numbering: a[i] = %i, b[i] = %(8+i), s = %16
#define S_(x) #x
#define S(x) S_(x)
#define BI_0 8
#define BI_1 9
#define BI_2 10
#define BI_3 11
#define BI_4 12
#define BI_5 13
#define BI_6 14
#define BI_7 15
#define PV_0 7
#define PV_1 0
#define PV_2 1
#define PV_3 2
#define PV_4 3
#define PV_5 4
#define PV_6 5
#define PV_7 6
#define ADD_FRESH(i) "v_add_u32 %" S(i) ", %" S(PV_##i) ", %" S(i) "\n"
#define XOR_FRESH(i) "v_xor_b32 %" S(i) ", %" S(PV_##i) ", %" S(i) "\n"
#define ALIGN16(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %" S(i) ", 16\n"
#define ALIGN20(i) "v_alignbit_b32 %" S(i) ", %" S(i) ", %" S(i) ", 20\n"
#define PACK16(i) "v_pack_b32_f16 %" S(i) ", %" S(i) ", %" S(i) " op_sel:[1,0]\n"
#define ADD_DIST(i) "v_add_u32 %" S(i) ", %" S(BI_##i) ", %" S(i) "\n"
#define QR_ALIGN(i) ADD_FRESH(i) XOR_FRESH(i) ALIGN16(i) ADD_FRESH(i) XOR_FRESH(i) ALIGN20(i)
#define QR_PACK(i) ADD_FRESH(i) XOR_FRESH(i) PACK16(i) ADD_FRESH(i) XOR_FRESH(i) ALIGN20(i)
#define KERNEL(NAME, BODY, PER)                                                                         \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk, uint32_t s) { \
        uint32_t a[8], b[8];                                                                           \
        for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * (i + 3); b[i] = threadIdx.x ^ (i * 77); }  \
        uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();             \
        for (int it = 0; it < iters; ++it) asm volatile(A8(BODY) A8(BODY) : OPS : "s"(s));             \
        uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();             \
        uint32_t x = 0;                                                                                \
        for (int i = 0; i < 8; ++i) x += a[i] ^ b[i];                                                  \
        out[blockIdx.x * 256 + threadIdx.x] = x;                                                       \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }               \
    }                                                                                                  \
    static const int per_##NAME = PER;

KERNEL(add_dist, ADD_DIST, 16)
KERNEL(align16, ALIGN16, 16)
KERNEL(pack16, PACK16, 16)
KERNEL(mix_align, QR_ALIGN, 96)
KERNEL(mix_pack, QR_PACK, 96)

// all 2^32 inputs: pack(x) == rotl(x, 16)?
__global__ void k_check(unsigned long long *bad, unsigned *first) {
    unsigned long long nbad = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    for (unsigned long long v = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; v < (1ull << 32); v += stride) {
        const uint32_t x = (uint32_t)v;
        uint32_t r;
        asm volatile("v_pack_b32_f16 %0, %1, %1 op_sel:[1,0]" : "=v"(r) : "v"(x));
        if (r != ((x << 16) | (x >> 16))) {
            ++nbad;
            atomicMin(first, x);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main() {
    uint32_t *out;
    uint64_t *clk, h[2];
    const int grid = 8192, iters = 4000;
    hipMalloc(&out, grid * 256 * 4);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
#define RUN(NAME)                                                                                       \
    {                                                                                                   \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk, 5u);                 \
        hipDeviceSynchronize();                                                                         \
        hipEventRecord(e0);                                                                             \
        hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk, 5u);                 \
        hipEventRecord(e1);                                                                             \
        hipEventSynchronize(e1);                                                                        \
        float ms;                                                                                       \
        hipEventElapsedTime(&ms, e0, e1);                                                               \
        hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);                                                   \
        double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;                                       \
        double wi = (double)grid * 4 * iters * per_##NAME;                                              \
        printf("%-22s %7.3f ms clk %.2f GHz cycles/wave-instr/SIMD %.2f\n", #NAME, ms, ghz,             \
               (ms * 1e-3 * ghz * 1e9) / (wi / 1024));                                                  \
    }
    {
        unsigned long long *bad;
        unsigned *first;
        hipMalloc(&bad, 8);
        hipMalloc(&first, 4);
        hipMemset(bad, 0, 8);
        hipMemset(first, 0xff, 4);
        hipLaunchKernelGGL(k_check, dim3(8192), dim3(256), 0, 0, bad, first);
        unsigned long long hb = 0;
        unsigned hf = 0;
        hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
        printf("pack_rot16_check mismatches %llu of 2^32 (first 0x%08x)\n", hb, hb ? hf : 0u);
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN(add_dist) RUN(align16) RUN(pack16) RUN(mix_align) RUN(mix_pack)
    }
    return 0;
}
