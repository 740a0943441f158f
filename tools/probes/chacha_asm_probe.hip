// chacha_asm_probe.hip -- gfx950: ChaCha20 block throughput with hand-scheduled inline asm,
// pinned VGPRs (bank-aware vs naive) and issue order (lockstep vs staggered QRs), against the
// compiler's own code.  Each variant's output is checked against the compiler version.
// Build: python3 tools/probes/gen_chacha_asm.py > tools/probes/chacha_asm_gen.h &&
//        hipcc --offload-arch=gfx950 -O3 -o tools/probes/chacha_asm_probe tools/probes/chacha_asm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "chacha_asm_gen.h"

#define ROTL(v, c) __builtin_rotateleft32((v), (c))
#define QR(a, b, c, d) a += b; d ^= a; d = ROTL(d, 16); c += d; b ^= c; b = ROTL(b, 12); a += b; d ^= a; d = ROTL(d, 8); c += d; b ^= c; b = ROTL(b, 7);

#define R10(X) X X X X X X X X X X
#define CLOB1 "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47"
#define CLOB2 CLOB1, "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63"

// phys reg of word i for the banked / naive plan (must match gen_chacha_asm.py)
#define MOVIN(p, o) "v_mov_b32 v" #p ", %" #o "\n"
#define MOVOUT(p, o) "v_mov_b32 %" #o ", v" #p "\n"
#define B_IN(b) MOVIN(32,0) MOVIN(33,1) MOVIN(34,2) MOVIN(35,3) MOVIN(37,4) MOVIN(38,5) MOVIN(39,6) MOVIN(36,7) \
                MOVIN(42,8) MOVIN(43,9) MOVIN(40,10) MOVIN(41,11) MOVIN(47,12) MOVIN(44,13) MOVIN(45,14) MOVIN(46,15)
#define B_OUT MOVOUT(32,0) MOVOUT(33,1) MOVOUT(34,2) MOVOUT(35,3) MOVOUT(37,4) MOVOUT(38,5) MOVOUT(39,6) MOVOUT(36,7) \
              MOVOUT(42,8) MOVOUT(43,9) MOVOUT(40,10) MOVOUT(41,11) MOVOUT(47,12) MOVOUT(44,13) MOVOUT(45,14) MOVOUT(46,15)
#define N_IN MOVIN(32,0) MOVIN(33,1) MOVIN(34,2) MOVIN(35,3) MOVIN(36,4) MOVIN(37,5) MOVIN(38,6) MOVIN(39,7) \
             MOVIN(40,8) MOVIN(41,9) MOVIN(42,10) MOVIN(43,11) MOVIN(44,12) MOVIN(45,13) MOVIN(46,14) MOVIN(47,15)
#define N_OUT MOVOUT(32,0) MOVOUT(33,1) MOVOUT(34,2) MOVOUT(35,3) MOVOUT(36,4) MOVOUT(37,5) MOVOUT(38,6) MOVOUT(39,7) \
              MOVOUT(40,8) MOVOUT(41,9) MOVOUT(42,10) MOVOUT(43,11) MOVOUT(44,12) MOVOUT(45,13) MOVOUT(46,14) MOVOUT(47,15)
#define OPS16(x) "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), \
                 "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])

__device__ __forceinline__ void init(uint32_t (&x)[16], uint32_t k, uint32_t ctr) {
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = k * (i + 1);
    x[12] = ctr;
}

enum { V_C = 0, V_BL, V_BS, V_NL, V_NS, V_SH, V_LO, V_PE };
#define CLOBT CLOB1, "v48", "v49", "v50", "v51"
#define SELS [rot16] "s"(0x01000302u), [rot8] "s"(0x02010003u)

template <int V>
__device__ __forceinline__ void rounds(uint32_t (&x)[16]) {
    if constexpr (V == V_C) {
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]); QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
            QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]); QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
        }
    } else if constexpr (V == V_BL) {
        asm volatile(B_IN(0) R10(CHACHA_DR_BANKED_LOCKSTEP_NB1) B_OUT : OPS16(x) :: CLOB1);
    } else if constexpr (V == V_BS) {
        asm volatile(B_IN(0) R10(CHACHA_DR_BANKED_STAGGER_NB1) B_OUT : OPS16(x) :: CLOB1);
    } else if constexpr (V == V_NL) {
        asm volatile(N_IN R10(CHACHA_DR_NAIVE_LOCKSTEP_NB1) N_OUT : OPS16(x) :: CLOB1);
    } else if constexpr (V == V_NS) {
        asm volatile(N_IN R10(CHACHA_DR_NAIVE_STAGGER_NB1) N_OUT : OPS16(x) :: CLOB1);
    } else if constexpr (V == V_SH) {
        asm volatile(N_IN R10(CHACHA_DR_NAIVE_LOCKSTEP_SHIFTS) N_OUT : OPS16(x) :: CLOBT);
    } else if constexpr (V == V_LO) {
        asm volatile(N_IN R10(CHACHA_DR_NAIVE_LOCKSTEP_LSHLOR) N_OUT : OPS16(x) :: CLOBT);
    } else {
        asm volatile(N_IN R10(CHACHA_DR_NAIVE_LOCKSTEP_PERM) N_OUT : OPS16(x) : SELS : CLOBT);
    }
}

template <int V>
__global__ __launch_bounds__(256) void probe(int iters, uint32_t *out, uint64_t *clk) {
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    const uint32_t ctr = blockIdx.x * 256 + threadIdx.x;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        uint32_t x[16];
        init(x, 0x9e3779b9u * (it + 1), ctr);
        rounds<V>(x);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += x[i] ^ 0x64636261u;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s = s * 31 + acc[i];
    out[ctr] = s;
    if (ctr == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

static uint32_t hsum(const uint32_t *d, size_t n) {
    static uint32_t h[1 << 21];
    hipMemcpy(h, d, n * 4, hipMemcpyDeviceToHost);
    uint32_t s = 0;
    for (size_t i = 0; i < n; ++i) s = s * 1000003u + h[i];
    return s;
}

int main() {
    uint32_t *out;
    uint64_t *clk, hc[2];
    const int grid = 8192, iters = 64;
    const size_t n = (size_t)grid * 256;
    hipMalloc(&out, n * 4);
    hipMalloc(&clk, 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    uint32_t ref = 0;
    const char *names[] = {"compiler", "asm banked lockstep", "asm banked stagger", "asm naive lockstep", "asm naive stagger", "asm rot=3 shifts", "asm rot=lshr+lshl_or", "asm rot16/8=perm"};
    auto run = [&](auto kern, int v) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        hipDeviceSynchronize();
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, iters, out, clk);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        ms /= 5;
        hipMemcpy(hc, clk, 16, hipMemcpyDeviceToHost);
        double ghz = (double)hc[0] / ((double)hc[1] / 100e6) / 1e9;
        uint32_t h = hsum(out, n);
        if (v == 0) ref = h;
        double words = (double)n * iters * 16;
        printf("%-22s %.3f ms  %6.1f Gw/s  clk %.2f GHz  %s\n", names[v], ms, words / ms / 1e6, ghz,
               h == ref ? "match" : "MISMATCH");
    };
    for (int rep = 0; rep < 2; ++rep) {
        run(probe<V_C>, 0);
        run(probe<V_BL>, 1);
        run(probe<V_BS>, 2);
        run(probe<V_NL>, 3);
        run(probe<V_NS>, 4);
        run(probe<V_SH>, 5);
        run(probe<V_LO>, 6);
        run(probe<V_PE>, 7);
    }
    return 0;
}
