// chacha_sdwa_probe.hip -- gfx950: ChaCha20 block throughput with the production quarter-round form
// (items_kernel's FLM_QR4: four QRs in lockstep, v_alignbit_b32 rotates, s_nop gaps) against a form
// whose 16-bit rotate is fused into the xor before it as two SDWA half-word xors into a fresh
// register (n.lo = d.hi ^ a.hi, n.hi = d.lo ^ a.lo), and optionally v_perm_b32 for the 8-bit rotate.
// Every lane makes `blocks` blocks of one key; the outputs of both forms are compared word for word
// and block 0 is checked against a host ChaCha20.  Prints ms and G words/s per form, 3 rounds.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define ROTL(v, c) (((v) << (c)) | ((v) >> (32 - (c))))
static void qr_host(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
    a += b; d ^= a; d = ROTL(d, 16);
    c += d; b ^= c; b = ROTL(b, 12);
    a += b; d ^= a; d = ROTL(d, 8);
    c += d; b ^= c; b = ROTL(b, 7);
}

#define S_A(a, b) "v_add_u32 %[" #a "], %[" #b "], %[" #a "]\n\t"
#define S_X(a, b) "v_xor_b32 %[" #a "], %[" #b "], %[" #a "]\n\t"
#define S_R(a, s) "v_alignbit_b32 %[" #a "], %[" #a "], %[" #a "], " #s "\n\t"
#define S_P(a) "v_perm_b32 %[" #a "], %[" #a "], %[" #a "], %[sel]\n\t"
// production step (flm_kernels.hip FLM_S_STEP with its default gaps)
#define STEP(a, b, c, d, s)                                                                       \
    S_A(a##0, b##0) S_A(a##1, b##1) S_A(a##2, b##2) S_A(a##3, b##3)                                   \
    S_X(d##0, a##0) S_X(d##1, a##1) S_X(d##2, a##2) S_X(d##3, a##3)                                   \
    S_R(d##0, s) "s_nop 1\n\t" S_R(d##1, s) "s_nop 1\n\t" S_R(d##2, s) "s_nop 1\n\t" S_R(d##3, s) "s_nop 2\n\t"
#define QR4_BASE(A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3)                    \
    asm volatile(STEP(a, b, c, d, 16) STEP(c, d, a, b, 20) STEP(a, b, c, d, 24) STEP(c, d, a, b, 25)      \
                 : [a0] "+v"(A0), [b0] "+v"(B0), [c0] "+v"(C0), [d0] "+v"(D0), [a1] "+v"(A1),           \
                   [b1] "+v"(B1), [c1] "+v"(C1), [d1] "+v"(D1), [a2] "+v"(A2), [b2] "+v"(B2),           \
                   [c2] "+v"(C2), [d2] "+v"(D2), [a3] "+v"(A3), [b3] "+v"(B3), [c3] "+v"(C3),           \
                   [d3] "+v"(D3))

// fused form: step 1's xor + rotate-16 as two SDWA xors into n (n becomes d); step 3 works on n
#define X16(n, d, a)                                                                                         \
    "v_xor_b32_sdwa %[" #n "], %[" #d "], %[" #a "] dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_1\n\t" \
    "v_xor_b32_sdwa %[" #n "], %[" #d "], %[" #a "] dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_0\n\t"
#define STEP1_SDWA                                                                                           \
    S_A(a0, b0) S_A(a1, b1) S_A(a2, b2) S_A(a3, b3) X16(n0, d0, a0) X16(n1, d1, a1) X16(n2, d2, a2) X16(n3, d3, a3) "s_nop 1\n\t"
#define STEP2(PERM8)                                                                                         \
    S_A(c0, n0) S_A(c1, n1) S_A(c2, n2) S_A(c3, n3) S_X(b0, c0) S_X(b1, c1) S_X(b2, c2) S_X(b3, c3)                \
    S_R(b0, 20) "s_nop 1\n\t" S_R(b1, 20) "s_nop 1\n\t" S_R(b2, 20) "s_nop 1\n\t" S_R(b3, 20) "s_nop 2\n\t"
#define STEP3_ALIGN                                                                                          \
    S_A(a0, b0) S_A(a1, b1) S_A(a2, b2) S_A(a3, b3) S_X(n0, a0) S_X(n1, a1) S_X(n2, a2) S_X(n3, a3)                \
    S_R(n0, 24) "s_nop 1\n\t" S_R(n1, 24) "s_nop 1\n\t" S_R(n2, 24) "s_nop 1\n\t" S_R(n3, 24) "s_nop 2\n\t"
#define STEP3_PERM                                                                                           \
    S_A(a0, b0) S_A(a1, b1) S_A(a2, b2) S_A(a3, b3) S_X(n0, a0) S_X(n1, a1) S_X(n2, a2) S_X(n3, a3)                \
    S_P(n0) "s_nop 1\n\t" S_P(n1) "s_nop 1\n\t" S_P(n2) "s_nop 1\n\t" S_P(n3) "s_nop 2\n\t"
#define STEP4                                                                                                \
    S_A(c0, n0) S_A(c1, n1) S_A(c2, n2) S_A(c3, n3) S_X(b0, c0) S_X(b1, c1) S_X(b2, c2) S_X(b3, c3)                \
    S_R(b0, 25) "s_nop 1\n\t" S_R(b1, 25) "s_nop 1\n\t" S_R(b2, 25) "s_nop 1\n\t" S_R(b3, 25) "s_nop 2\n\t"
#define QR4_FUSED(STEP3, A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3)                     \
    {                                                                                                        \
        uint32_t n0_, n1_, n2_, n3_;                                                                         \
        asm volatile(STEP1_SDWA STEP2(0) STEP3 STEP4                                                         \
                     : [a0] "+v"(A0), [b0] "+v"(B0), [c0] "+v"(C0), [a1] "+v"(A1), [b1] "+v"(B1),            \
                       [c1] "+v"(C1), [a2] "+v"(A2), [b2] "+v"(B2), [c2] "+v"(C2), [a3] "+v"(A3),            \
                       [b3] "+v"(B3), [c3] "+v"(C3), [n0] "=&v"(n0_), [n1] "=&v"(n1_), [n2] "=&v"(n2_),      \
                       [n3] "=&v"(n3_)                                                                       \
                     : [d0] "v"(D0), [d1] "v"(D1), [d2] "v"(D2), [d3] "v"(D3), [sel] "v"(sel));              \
        D0 = n0_; D1 = n1_; D2 = n2_; D3 = n3_;                                                              \
    }

template <int FORM>  // 0 production, 1 SDWA rot16, 2 SDWA rot16 + v_perm rot8
__global__ __launch_bounds__(256) void k_chacha(const uint32_t *key, int blocks, uint32_t *out, uint32_t sel_in) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t k0 = key[0], k1 = key[1], k2 = key[2], k3 = key[3], k4 = key[4], k5 = key[5], k6 = key[6],
                   k7 = key[7];
    uint32_t sel = sel_in + (threadIdx.x >> 16);  // a VGPR (perm selector 0x02010003: rotl 8)
    uint32_t acc[16];
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    for (int bi = 0; bi < blocks; ++bi) {
        const uint32_t ctr = lane * (uint32_t)blocks + (uint32_t)bi;
        uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
        uint32_t x4 = k0, x5 = k1, x6 = k2, x7 = k3, x8 = k4, x9 = k5, x10 = k6, x11 = k7;
        uint32_t x12 = ctr, x13 = 0, x14 = 0, x15 = 0;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if constexpr (FORM == 0) {
                QR4_BASE(x0, x4, x8, x12, x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15);
                QR4_BASE(x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
            } else if constexpr (FORM == 1) {
                QR4_FUSED(STEP3_ALIGN, x0, x4, x8, x12, x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15);
                QR4_FUSED(STEP3_ALIGN, x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
            } else {
                QR4_FUSED(STEP3_PERM, x0, x4, x8, x12, x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15);
                QR4_FUSED(STEP3_PERM, x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
            }
        }
        const uint32_t w[16] = {x0 + 0x61707865u, x1 + 0x3320646eu, x2 + 0x79622d32u, x3 + 0x6b206574u,
                                x4 + k0, x5 + k1, x6 + k2, x7 + k3, x8 + k4, x9 + k5, x10 + k6, x11 + k7,
                                x12 + ctr, x13, x14, x15};
        if (bi == 0)
            for (int i = 0; i < 16; ++i) out[(size_t)lane * 32 + i] = w[i];
        for (int i = 0; i < 16; ++i) acc[i] += w[i];
    }
    for (int i = 0; i < 16; ++i) out[(size_t)lane * 32 + 16 + i] = acc[i];
}

int main() {
    const int grid = 8192, threads = 256, blocks = 64;
    const size_t lanes = (size_t)grid * threads;
    uint32_t hkey[8];
    for (int i = 0; i < 8; ++i) hkey[i] = 0x01234567u * (i + 1) ^ 0x9e3779b9u;
    uint32_t *key, *out[3];
    (void)hipMalloc(&key, 32);
    (void)hipMemcpy(key, hkey, 32, hipMemcpyHostToDevice);
    for (int f = 0; f < 3; ++f) (void)hipMalloc(&out[f], lanes * 32 * 4);
    const uint32_t sel = 0x02010003u;  // v_perm_b32 selector: bytes [2,1,0,3] of the source = rotl 8
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](int f) {
        if (f == 0) hipLaunchKernelGGL(k_chacha<0>, dim3(grid), dim3(threads), 0, 0, key, blocks, out[0], sel);
        if (f == 1) hipLaunchKernelGGL(k_chacha<1>, dim3(grid), dim3(threads), 0, 0, key, blocks, out[1], sel);
        if (f == 2) hipLaunchKernelGGL(k_chacha<2>, dim3(grid), dim3(threads), 0, 0, key, blocks, out[2], sel);
    };
    const double words = (double)lanes * blocks * 16;
    for (int rep = 0; rep < 3; ++rep)
        for (int f = 0; f < 3; ++f) {
            run(f);
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            run(f);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("form %d (%s): %.3f ms  %.1f G words/s\n", f,
                   f == 0 ? "production alignbit" : f == 1 ? "SDWA rot16" : "SDWA rot16 + perm rot8", ms,
                   words / (ms * 1e-3) / 1e9);
        }
    // correctness: all forms equal, block 0 of lane 0..3 against the host
    static uint32_t h[3][4096 * 32];
    for (int f = 0; f < 3; ++f) (void)hipMemcpy(h[f], out[f], sizeof h[f], hipMemcpyDeviceToHost);
    bool same = memcmp(h[0], h[1], sizeof h[0]) == 0 && memcmp(h[0], h[2], sizeof h[0]) == 0;
    bool host_ok = true;
    for (uint32_t lane = 0; lane < 4; ++lane) {
        uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, hkey[0], hkey[1], hkey[2], hkey[3],
                          hkey[4], hkey[5], hkey[6], hkey[7], lane * (uint32_t)blocks, 0, 0, 0};
        uint32_t in[16];
        memcpy(in, x, sizeof in);
        for (int r = 0; r < 10; ++r) {
            qr_host(x[0], x[4], x[8], x[12]); qr_host(x[1], x[5], x[9], x[13]);
            qr_host(x[2], x[6], x[10], x[14]); qr_host(x[3], x[7], x[11], x[15]);
            qr_host(x[0], x[5], x[10], x[15]); qr_host(x[1], x[6], x[11], x[12]);
            qr_host(x[2], x[7], x[8], x[13]); qr_host(x[3], x[4], x[9], x[14]);
        }
        for (int i = 0; i < 16; ++i) host_ok &= h[0][lane * 32 + i] == x[i] + in[i];
    }
    printf("forms identical: %s; block 0 matches host ChaCha20: %s\n", same ? "yes" : "NO", host_ok ? "yes" : "NO");
    return same && host_ok ? 0 : 1;
}
