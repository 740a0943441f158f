// qr8_probe.hip -- issue-rate probe for ChaCha quarter-round instruction patterns on gfx950.
//
// Each lane runs ITER double rounds of one pattern on its own registers (no memory in the loop),
// 1024-thread workgroups, GRID workgroups; time per launch from hipEvents -> VALU instructions per
// cycle per SIMD (at the clock rocprof would show; here we report ns and instr/ns/SIMD).
//   P0  FLM_QR4 as in items_kernel: 4 adds, 4 xors, 4 rotates, s_nop 1 after each of the first three
//       rotates and s_nop 2 after the fourth (one block per lane, 16 state registers)
//   P1  two blocks per lane, pipelined: block B's adds fill block A's rotate gaps and vice versa,
//       no s_nop (32 state registers)
//   P2  P1 with s_nop 0 after every rotate
//   P3  two blocks per lane as two QR4 streams back to back (the production gaps)
// Output words are folded into one store per lane so nothing is dead.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define A_(a, b) "v_add_u32 %[" #a "], %[" #b "], %[" #a "]\n\t"
#define X_(a, b) "v_xor_b32 %[" #a "], %[" #b "], %[" #a "]\n\t"
#define R_(a, s) "v_alignbit_b32 %[" #a "], %[" #a "], %[" #a "], " #s "\n\t"
#define N1 "s_nop 1\n\t"
#define N2 "s_nop 2\n\t"
#define N0 "s_nop 0\n\t"

// production QR4 step: a += b; d ^= a; d = rot(d)
#define STEP4(p, a, b, d, s)                                                                        \
    A_(p##a##0, p##b##0) A_(p##a##1, p##b##1) A_(p##a##2, p##b##2) A_(p##a##3, p##b##3)              \
    X_(p##d##0, p##a##0) X_(p##d##1, p##a##1) X_(p##d##2, p##a##2) X_(p##d##3, p##a##3)              \
    R_(p##d##0, s) N1 R_(p##d##1, s) N1 R_(p##d##2, s) N1 R_(p##d##3, s) N2
#define HALF4(p) STEP4(p, a, b, d, 16) STEP4(p, c, d, b, 20) STEP4(p, a, b, d, 24) STEP4(p, c, d, b, 25)

// pipelined two-block step pieces
#define ADDX(p, a, b, d) A_(p##a##0, p##b##0) A_(p##a##1, p##b##1) A_(p##a##2, p##b##2) A_(p##a##3, p##b##3) \
    X_(p##d##0, p##a##0) X_(p##d##1, p##a##1) X_(p##d##2, p##a##2) X_(p##d##3, p##a##3)
// rotates of block P's d interleaved with the adds of block Q (Q: a += b), G = gap after each pair
#define RIA(P, d, s, Q, a, b, G) R_(P##d##0, s) A_(Q##a##0, Q##b##0) G R_(P##d##1, s) A_(Q##a##1, Q##b##1) G \
    R_(P##d##2, s) A_(Q##a##2, Q##b##2) G R_(P##d##3, s) A_(Q##a##3, Q##b##3) G
#define XONLY(p, a, d) X_(p##d##0, p##a##0) X_(p##d##1, p##a##1) X_(p##d##2, p##a##2) X_(p##d##3, p##a##3)

#define OPS16(p) [p##a0] "+v"(p##a0), [p##b0] "+v"(p##b0), [p##c0] "+v"(p##c0), [p##d0] "+v"(p##d0),    \
                 [p##a1] "+v"(p##a1), [p##b1] "+v"(p##b1), [p##c1] "+v"(p##c1), [p##d1] "+v"(p##d1),    \
                 [p##a2] "+v"(p##a2), [p##b2] "+v"(p##b2), [p##c2] "+v"(p##c2), [p##d2] "+v"(p##d2),    \
                 [p##a3] "+v"(p##a3), [p##b3] "+v"(p##b3), [p##c3] "+v"(p##c3), [p##d3] "+v"(p##d3)

#define DECL(p, seed) uint32_t p##a0 = seed, p##b0 = seed * 3, p##c0 = seed * 5, p##d0 = seed * 7, \
    p##a1 = seed + 1, p##b1 = seed + 2, p##c1 = seed + 3, p##d1 = seed + 4, p##a2 = seed ^ 5, p##b2 = seed ^ 6, \
    p##c2 = seed ^ 7, p##d2 = seed ^ 8, p##a3 = seed * 9, p##b3 = seed * 11, p##c3 = seed * 13, p##d3 = seed * 15
#define FOLD(p) (p##a0 ^ p##b0 ^ p##c0 ^ p##d0 ^ p##a1 ^ p##b1 ^ p##c1 ^ p##d1 ^ p##a2 ^ p##b2 ^ p##c2 ^ \
                 p##d2 ^ p##a3 ^ p##b3 ^ p##c3 ^ p##d3)

template <int P>
__global__ __launch_bounds__(1024, 4) void probe(uint32_t *out, int iter) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    DECL(u, t);
    DECL(v, t + 0x9e3779b9u);
    for (int i = 0; i < iter; ++i) {
        if constexpr (P == 0) {
            // one block: a column half round then a diagonal (register roles rotate; the pattern is what counts)
            asm volatile(HALF4(u) : OPS16(u));
            asm volatile(HALF4(u) : OPS16(u));
        } else if constexpr (P == 3) {
            asm volatile(HALF4(u) : OPS16(u));
            asm volatile(HALF4(v) : OPS16(v));
            asm volatile(HALF4(u) : OPS16(u));
            asm volatile(HALF4(v) : OPS16(v));
        } else {
            // one half round of both blocks, pipelined: steps (a,b,d,16) (c,d,b,20) (a,b,d,24) (c,d,b,25)
            // u's rotates carry v's adds of the same step; v's rotates carry u's adds of the next step
#define G_ (P == 2 ? N0 : "")
#define PIPE                                                                                          \
    ADDX(u, a, b, d) RIA(u, d, 16, v, a, b, "") XONLY(v, a, d)                                          \
    RIA(v, d, 16, u, c, d, "") XONLY(u, c, b) RIA(u, b, 20, v, c, d, "") XONLY(v, c, b)              \
    RIA(v, b, 20, u, a, b, "") XONLY(u, a, d) RIA(u, d, 24, v, a, b, "") XONLY(v, a, d)              \
    RIA(v, d, 24, u, c, d, "") XONLY(u, c, b) RIA(u, b, 25, v, c, d, "") XONLY(v, c, b)              \
    R_(vb0, 25) R_(vb1, 25) R_(vb2, 25) R_(vb3, 25)
#define PIPE_G                                                                                        \
    ADDX(u, a, b, d) RIA(u, d, 16, v, a, b, N0) XONLY(v, a, d)                                          \
    RIA(v, d, 16, u, c, d, N0) XONLY(u, c, b) RIA(u, b, 20, v, c, d, N0) XONLY(v, c, b)              \
    RIA(v, b, 20, u, a, b, N0) XONLY(u, a, d) RIA(u, d, 24, v, a, b, N0) XONLY(v, a, d)              \
    RIA(v, d, 24, u, c, d, N0) XONLY(u, c, b) RIA(u, b, 25, v, c, d, N0) XONLY(v, c, b)              \
    R_(vb0, 25) N1 R_(vb1, 25) N1 R_(vb2, 25) N1 R_(vb3, 25) N2
            if constexpr (P == 1) {
                asm volatile(PIPE : OPS16(u), OPS16(v));
                asm volatile(PIPE : OPS16(u), OPS16(v));
            } else {
                asm volatile(PIPE_G : OPS16(u), OPS16(v));
                asm volatile(PIPE_G : OPS16(u), OPS16(v));
            }
        }
    }
    out[t] = FOLD(u) ^ FOLD(v);
}

template <int P>
double run(int grid, int iter, uint32_t *d) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(probe<P>, dim3(grid), dim3(1024), 0, 0, d, iter);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(probe<P>, dim3(grid), dim3(1024), 0, 0, d, iter);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char **argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 2048;
    const int iter = argc > 2 ? atoi(argv[2]) : 200;
    uint32_t *d;
    hipMalloc(&d, (size_t)grid * 1024 * 4);
    // VALU instructions per lane per iteration (s_nop excluded): P0 2 x 48; P1/P2/P3 4 x 48
    const double waves = (double)grid * 16, simds = 256.0 * 4;
    for (int rep = 0; rep < 2; ++rep) {
        const double t0 = run<0>(grid, iter, d), t1 = run<1>(grid, iter, d), t2 = run<2>(grid, iter, d),
                     t3 = run<3>(grid, iter, d);
        const double i0 = waves * iter * 96, i1 = waves * iter * 192;
        printf("grid %d iter %d: P0 %.3f ms %.3f instr/ns/SIMD | P1 %.3f ms %.3f | P2 %.3f ms %.3f | P3 %.3f ms %.3f\n",
               grid, iter, t0, i0 / (t0 * 1e6) / simds, t1, i1 / (t1 * 1e6) / simds, t2, i1 / (t2 * 1e6) / simds, t3,
               i1 / (t3 * 1e6) / simds);
    }
    hipFree(d);
    return 0;
}
