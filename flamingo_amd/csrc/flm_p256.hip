// flm_p256.hip -- P-256 batch kernels for Flamingo's seed recovery (gfx950).
//
// The server recovers every dropped pair's seed from the committee's threshold
// ElGamal decryption shares (SA_ServiceAgent.py:542-585):
//     point_i = c1_i - sum_j lambda_j * share_{j,i}          (share = sk_j * c0_i)
//     seed_i  = SHA-256(x(point_i) || y(point_i))            (32-byte big endian)
// and the clients/committee do single scalar multiplications (ECDH :256-263,
// ElGamal :434-447, decryption shares :397-400).  All of it is 256-bit modular
// arithmetic on independent points -- one lane per (term, pair) scalar
// multiplication (or four cooperating waves per 64 of them, exchanging field
// elements through LDS), a few lanes per pair for the combine -- so this is
// VALU integer work: no MFMA.  A small batch is one latency chain, bound by the
// quarter-rate v_mad_u64_u32 on its critical path.
//
// Field: p = 2^256 - 2^224 + 2^192 + 2^96 - 1, eight 32-bit limbs little
// endian, Montgomery form with R = 2^256 (-p^-1 mod 2^32 = 1, so the CIOS
// quotient digit is the low limb itself).  Points: Jacobian (X, Y, Z), Z = 0
// is the point at infinity; curve a = -3.
// Wire format (host <-> device): points are 64 bytes x||y, each a 32-byte
// big-endian integer (SEC1 uncompressed without the 0x04 prefix; the same
// bytes the reference hashes at :584-585); scalars are 32-byte big endian.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "flm_fe_row.h"
#include "flm_internal.h"

namespace flm {
namespace {

struct Fe {
    uint32_t v[8];
};
template <class E>
struct JacT {
    E X, Y, Z;
};
using Jac = JacT<Fe>;

__device__ constexpr uint32_t kP[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};
__device__ constexpr uint32_t kOne[8] = {0x00000001u, 0x00000000u, 0x00000000u, 0xffffffffu,
                                         0xffffffffu, 0xffffffffu, 0xfffffffeu, 0x00000000u};  // R mod p
__device__ constexpr uint32_t kR2[8] = {0x00000003u, 0x00000000u, 0xffffffffu, 0xfffffffbu,
                                        0xfffffffeu, 0xffffffffu, 0xfffffffdu, 0x00000004u};  // R^2 mod p
__device__ constexpr uint32_t kBm[8] = {0x29c4bddfu, 0xd89cdf62u, 0x78843090u, 0xacf005cdu,
                                        0xf7212ed6u, 0xe5a220abu, 0x04874834u, 0xdc30061du};  // b*R mod p

__device__ __forceinline__ Fe fe_const(const uint32_t (&c)[8]) {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = c[i];
    return r;
}

__device__ __forceinline__ bool fe_is_zero(const Fe &a) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.v[i];
    return o == 0;
}

__device__ __forceinline__ bool fe_eq(const Fe &a, const Fe &b) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
    return o == 0;
}

// a < p for a canonical (non-Montgomery) input
__device__ __forceinline__ bool fe_lt_p(const Fe &a) {
    uint64_t b = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint64_t d = (uint64_t)a.v[i] - kP[i] - b;
        b = d >> 63;
    }
    return b != 0;
}

// Carry chains go through __builtin_addc / __builtin_subc, which lower to v_add_co / v_addc_co
// (v_sub_co / v_subb_co) with the carry in VCC: 8 instructions per 256-bit add.  The earlier
// 64-bit C form compiled to 64-bit shift-adds plus register moves: fe_add 95 VALU -> 28, fe_sub
// 75 -> 24 (gfx950 ISA count); a lone wave of the EC chain issues one VALU per ~8 cycles, so the
// instruction count is its latency.
// r = (t8:t) - p if that does not borrow (or t8 set), else t; requires t < 2p
__device__ __forceinline__ void fe_reduce_once(Fe &r, const uint32_t (&t)[8], uint32_t t8) {
    uint32_t d[8], b = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(t[i], kP[i], b, &b);
    const bool take = t8 || !b;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = take ? d[i] : t[i];
}

__device__ __forceinline__ Fe fe_add(const Fe &a, const Fe &b) {
    uint32_t s[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    Fe r;
    fe_reduce_once(r, s, c);
    return r;
}

__device__ __forceinline__ Fe fe_sub(const Fe &a, const Fe &b) {
    uint32_t d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
    // borrow -> add p back (mask instead of branch)
    const uint32_t m = 0u - br;
    Fe r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = __builtin_addc(d[i], kP[i] & m, c, &c);
    return r;
}

// Montgomery reduction of a 512-bit product t by p = 2^256 - 2^224 + 2^192 + 2^96 - 1 in one
// signed column pass: the quotient digit m_i is the running limb i itself (-p^-1 = 1 mod
// 2^32) and adding m_i*p touches limbs i (-m, clears it), i+3 (+m), i+6 (+m), i+7 (-m), i+8 (+m).
__device__ __forceinline__ Fe mont_reduce(uint32_t (&t)[16]) {
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
    uint32_t r8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r8[i] = t[i];
    Fe r;
    fe_reduce_once(r, r8, (uint32_t)carry);
    return r;
}

// A whole product column in ONE asm statement: NP mad/addc pairs, acc (64-bit) += a[q]*b[q]
// with every carry-out of the 64-bit accumulator counted in hi (v_mad_u64_u32's own carry-out
// feeds one v_addc).  The compiler pads each inline-asm boundary with s_nop (it cannot see
// through asm): one statement per product pair measured 543 ns per single-wave multiply,
// against 669 ns with mad and addc in separate statements and 860 ns for a plain 64-bit C CIOS
// (tools/probes/ec_probe.hip); one statement per column drops most of the remaining pads.
#define FLM_MC(n) "v_mad_u64_u32 %[acc], %[c], %[a" #n "], %[b" #n "], %[acc]\n\t" \
                  "v_addc_co_u32_e64 %[hi], %[c], 0, %[hi], %[c]\n\t"
// first product of a column whose carry counter starts at zero: hi = carry, written fresh (no
// zeroing move before the statement)
#define FLM_MC_H "v_mad_u64_u32 %[acc], %[c], %[a0], %[b0], %[acc]\n\t" \
                 "v_addc_co_u32_e64 %[hi], %[c], 0, 0, %[c]\n\t"
// first product of a column whose accumulator starts at zero: acc = a*b (cannot carry), hi = 0
#define FLM_MC_Z "v_mad_u64_u32 %[acc], %[c], %[a0], %[b0], 0\n\t" \
                 "v_mov_b32 %[hi], 0\n\t"
#define FLM_R1
#define FLM_R2 FLM_R1 FLM_MC(1)
#define FLM_R3 FLM_R2 FLM_MC(2)
#define FLM_R4 FLM_R3 FLM_MC(3)
#define FLM_R5 FLM_R4 FLM_MC(4)
#define FLM_R6 FLM_R5 FLM_MC(5)
#define FLM_R7 FLM_R6 FLM_MC(6)
#define FLM_R8 FLM_R7 FLM_MC(7)
#define FLM_MI(n) [a##n] "v"(a[n]), [b##n] "v"(b[n])
#define FLM_I1 FLM_MI(0)
#define FLM_I2 FLM_I1, FLM_MI(1)
#define FLM_I3 FLM_I2, FLM_MI(2)
#define FLM_I4 FLM_I3, FLM_MI(3)
#define FLM_I5 FLM_I4, FLM_MI(4)
#define FLM_I6 FLM_I5, FLM_MI(5)
#define FLM_I7 FLM_I6, FLM_MI(6)
#define FLM_I8 FLM_I7, FLM_MI(7)
// acc/hi are early-clobber: later products read inputs after the first mad/addc wrote them,
// so no input may share their registers (the compiler otherwise reuses one holding the same
// value, e.g. a zero limb of the constant 1 against hi's initial 0)
#define FLM_MOUT0 [acc] "+&v"(acc), [hi] "+&v"(hi), [c] "=&s"(c)
#define FLM_MOUT1 [acc] "+&v"(acc), [hi] "=&v"(hi), [c] "=&s"(c)
#define FLM_MOUT2 [acc] "=&v"(acc), [hi] "=&v"(hi), [c] "=&s"(c)
#define FLM_MCASE(N)                                                                \
    if constexpr (NP == N) {                                                        \
        if constexpr (MODE == 0) asm(FLM_MC(0) FLM_R##N : FLM_MOUT0 : FLM_I##N);    \
        else if constexpr (MODE == 1) asm(FLM_MC_H FLM_R##N : FLM_MOUT1 : FLM_I##N); \
        else asm(FLM_MC_Z FLM_R##N : FLM_MOUT2 : FLM_I##N);                          \
    }
// MODE 0: acc and hi carry in; 1: acc carries in, hi starts at zero; 2: both start at zero
// (modes 1/2 write the fresh words in the statement instead of zeroing registers before it:
// the per-column moves were ~45 of fe_mul's VALU instructions)
template <int NP, int MODE = 0>
__device__ __forceinline__ void mad_col(uint64_t &acc, uint32_t &hi, const uint32_t (&a)[NP], const uint32_t (&b)[NP]) {
    uint64_t c;
    FLM_MCASE(1) FLM_MCASE(2) FLM_MCASE(3) FLM_MCASE(4) FLM_MCASE(5) FLM_MCASE(6) FLM_MCASE(7) FLM_MCASE(8)
}
#undef FLM_MCASE
#undef FLM_MC
#undef FLM_MC_H
#undef FLM_MC_Z
#undef FLM_MI
#undef FLM_MOUT0
#undef FLM_MOUT1
#undef FLM_MOUT2

// column K of a*b (products a_i b_{K-i}) into acc/hi
template <int K>
__device__ __forceinline__ void mul_col(uint64_t &acc, uint32_t &hi, const Fe &a, const Fe &b) {
    constexpr int lo = K < 8 ? 0 : K - 7, top = K < 8 ? K : 7, n = top - lo + 1;
    uint32_t av[n], bv[n];
#pragma unroll
    for (int q = 0; q < n; ++q) {
        av[q] = a.v[lo + q];
        bv[q] = b.v[K - lo - q];
    }
    mad_col<n, K == 0 ? 2 : 1>(acc, hi, av, bv);  // hi (and at K = 0 acc) start at zero
}

// column K of the doubled cross products of a^2 (a_i a_j, i < j, i + j = K)
template <int K>
__device__ __forceinline__ void sqr_col(uint64_t &x, uint32_t &xh, const Fe &a) {
    constexpr int lo = K < 8 ? 0 : K - 7, top = K >= 1 ? (K - 1) / 2 : -1, n = top - lo + 1;
    if constexpr (n > 0) {
        uint32_t av[n], bv[n];
#pragma unroll
        for (int q = 0; q < n; ++q) {
            av[q] = a.v[lo + q];
            bv[q] = a.v[K - lo - q];
        }
        mad_col<n, 2>(x, xh, av, bv);  // x and xh start at zero
    } else {
        x = 0;
        xh = 0;
    }
}

template <int K>
__device__ __forceinline__ void mul_cols(uint64_t &acc, uint32_t &hi, uint32_t (&t)[16], const Fe &a, const Fe &b) {
    if constexpr (K < 15) {
        mul_col<K>(acc, hi, a, b);
        t[K] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)hi << 32);
        mul_cols<K + 1>(acc, hi, t, a, b);
    }
}

// Montgomery product a*b*R^-1 mod p: product scanning with a 96-bit column accumulator
__device__ __forceinline__ Fe fe_mul(const Fe &a, const Fe &b) {
    uint32_t t[16];
    uint64_t acc;  // written by column 0
    uint32_t hi;
    mul_cols<0>(acc, hi, t, a, b);
    t[15] = (uint32_t)acc;
    return mont_reduce(t);
}

template <int K>
__device__ __forceinline__ void sqr_cols(uint64_t &c, uint32_t (&t)[16], const Fe &a) {
    if constexpr (K < 15) {
        uint64_t x;
        uint32_t xh;
        sqr_col<K>(x, xh, a);
        xh = (xh << 1) | (uint32_t)(x >> 63);
        x <<= 1;
        uint64_t n = x + c;
        xh += (n < x);
        x = n;
        if constexpr ((K & 1) == 0) {
            const uint32_t av[1] = {a.v[K / 2]};
            mad_col<1>(x, xh, av, av);
        }
        t[K] = (uint32_t)x;
        c = (x >> 32) | ((uint64_t)xh << 32);
        sqr_cols<K + 1>(c, t, a);
    }
}

// a^2 R^-1: 28 cross products summed once and doubled, plus 8 squares (36 mads instead of 64)
__device__ __forceinline__ Fe fe_sqr(const Fe &a) {
    uint32_t t[16];
    uint64_t c = 0;
    sqr_cols<0>(c, t, a);
    t[15] = (uint32_t)c;
    return mont_reduce(t);
}

__device__ __forceinline__ Fe fe_neg(const Fe &a) {
    Fe z = {};
    return fe_sub(z, a);
}

__device__ __forceinline__ Fe to_mont(const Fe &a) { return fe_mul(a, fe_const(kR2)); }
__device__ __forceinline__ Fe from_mont(const Fe &a) {
    Fe one = {};
    one.v[0] = 1;
    return fe_mul(a, one);
}

// ec_finish inverts by binary GCD (fe_inv_bingcd below), not Fermat's a^(p-2) (round 3)

// ---- inversion by binary GCD (ec_finish_kernel's one-lane chain)
// Pornin, "Optimized Binary GCD for Modular Inversion" (eprint 2020/972), Algorithm 2, with
// k - 1 = 30 inner steps per outer step so the update factors fit int32: 18 outer steps, i.e.
// 540 >= 2 * 256 - 1 inner steps, the algorithm's bound (tools/bingcd_model.py runs exactly this
// schedule in Python: it matches Fermat on 20k random and edge inputs, the worst needing all 18).
// An outer step runs 30 binary-GCD steps on 64-bit approximations of a and b (the low 30 bits
// exact, above them the top 34 bits of the longer one's window), then applies the 2 x 2 update
// matrix to the 256-bit a, b and to the Bezout coefficients u, v mod p (with a Montgomery
// division by 2^30; -p^-1 = 1 mod 2^30, so the quotient digit is the low 30 bits).  No
// data-dependent branches, so a wave's lanes never diverge.  ~25k VALU instructions against
// Fermat's ~73k (266 squarings, 11 multiplications).
__device__ constexpr uint32_t kR3[8] = {0x0000000au, 0xfffffffdu, 0xfffffff7u, 0xffffffedu,
                                        0xfffffffcu, 0x00000005u, 0x00000001u, 0x00000018u};  // R^3 mod p

// r (9 limbs, two's complement) = a * f for a unsigned 256-bit and f signed 32-bit
__device__ __forceinline__ void bg_mul_s32(uint32_t (&r)[9], const uint32_t (&a)[8], int32_t f) {
    const uint32_t F = (uint32_t)f;
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        c = (uint64_t)a[i] * F + (c >> 32);
        r[i] = (uint32_t)c;
    }
    r[8] = (uint32_t)(c >> 32);
    // f < 0: F = f + 2^32, so a * f = a * F - a * 2^32
    const uint32_t m = f < 0 ? 0xffffffffu : 0u;
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i + 1] = __builtin_subc(r[i + 1], a[i] & m, br, &br);
}

// r = (a * f + b * g) >> 30 (arithmetic; exact for the matrix's products), 9 limbs
__device__ __forceinline__ void bg_lin(uint32_t (&r)[9], const uint32_t (&a)[8], int32_t f, const uint32_t (&b)[8],
                                       int32_t g) {
    uint32_t x[9], y[9], c = 0;
    bg_mul_s32(x, a, f);
    bg_mul_s32(y, b, g);
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = __builtin_addc(x[i], y[i], c, &c);
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = __builtin_amdgcn_alignbit(x[i + 1], x[i], 30);
    r[8] = (uint32_t)((int32_t)x[8] >> 30);
}

// (u * f + v * g) / 2^30 mod p, into [0, p): the sum plus q p with q its low 30 bits is divisible
// by 2^30; |u f + v g| <= p 2^30 (|f| + |g| <= 2^30), so the quotient lies in [-p, 2p]
__device__ __forceinline__ void bg_lin_modp(uint32_t (&r)[8], const uint32_t (&u)[8], int32_t f,
                                            const uint32_t (&v)[8], int32_t g) {
    uint32_t x[9], y[9], c = 0;
    bg_mul_s32(x, u, f);
    bg_mul_s32(y, v, g);
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = __builtin_addc(x[i], y[i], c, &c);
    const uint32_t q = x[0] & 0x3fffffffu;
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        m = (uint64_t)kP[i] * q + (m >> 32);
        y[i] = (uint32_t)m;
    }
    y[8] = (uint32_t)(m >> 32);
    c = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = __builtin_addc(x[i], y[i], c, &c);
    uint32_t w[9];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = __builtin_amdgcn_alignbit(x[i + 1], x[i], 30);
    w[8] = (uint32_t)((int32_t)x[8] >> 30);
    // [-p, 0) -> + p
    const uint32_t neg = (int32_t)w[8] < 0 ? 0xffffffffu : 0u;
    c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = __builtin_addc(w[i], kP[i] & neg, c, &c);
    w[8] = __builtin_addc(w[8], 0u, c, &c);  // the sign word wraps to 0 when p was added
    // [p, 2p] -> - p
    uint32_t d[8], br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(w[i], kP[i], br, &br);
    const bool take = w[8] != 0 || !br;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = take ? d[i] : w[i];
}

// x^-1 mod p for 0 < x < p (plain integers: the caller's Montgomery form is just an integer here)
__device__ Fe fe_inv_bingcd(const Fe &x) {
    uint32_t a[8], b[8], u[8], v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = x.v[i];
        b[i] = kP[i];
        u[i] = i == 0 ? 1u : 0u;
        v[i] = 0u;
    }
#pragma unroll 1
    for (int it = 0; it < 18; ++it) {
        // n = max(bitlen(a), bitlen(b), 64): the approximations take bits [n - 64, n) and the low 30
        uint32_t top = a[0] | b[0];
        int t = 0;
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            const uint32_t ck = a[k] | b[k];
            if (ck) {
                t = k;
                top = ck;
            }
        }
        const int bl = 32 * t + 32 - (int)__clz(top);  // b >= 1 throughout
        const int sh = (bl > 64 ? bl : 64) - 64;
        const int q = sh >> 5, r = sh & 31;            // q <= 6
        uint32_t a0 = a[0], a1 = a[1], a2 = a[2], b0 = b[0], b1 = b[1], b2 = b[2];
#pragma unroll
        for (int k = 1; k <= 6; ++k) {
            if (q == k) {
                a0 = a[k]; a1 = a[k + 1]; a2 = k + 2 < 8 ? a[(k + 2) & 7] : 0u;
                b0 = b[k]; b1 = b[k + 1]; b2 = k + 2 < 8 ? b[(k + 2) & 7] : 0u;
            }
        }
        uint64_t ab = ((uint64_t)__builtin_amdgcn_alignbit(a2, a1, r) << 32) |
                      ((__builtin_amdgcn_alignbit(a1, a0, r) & 0xc0000000u) | (a[0] & 0x3fffffffu));
        uint64_t bb = ((uint64_t)__builtin_amdgcn_alignbit(b2, b1, r) << 32) |
                      ((__builtin_amdgcn_alignbit(b1, b0, r) & 0xc0000000u) | (b[0] & 0x3fffffffu));
        int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll
        for (int j = 0; j < 30; ++j) {
            const bool odd = (uint32_t)ab & 1u;
            const bool sw = odd && ab < bb;
            const uint64_t xa = sw ? bb : ab, xb = sw ? ab : bb;
            const int32_t xf0 = sw ? f1 : f0, xg0 = sw ? g1 : g0, xf1 = sw ? f0 : f1, xg1 = sw ? g0 : g1;
            ab = (xa - (odd ? xb : 0ull)) >> 1;
            bb = xb;
            f0 = xf0 - (odd ? xf1 : 0);
            g0 = xg0 - (odd ? xg1 : 0);
            f1 = xf1 * 2;
            g1 = xg1 * 2;
        }
        uint32_t na[9], nb[9];
        bg_lin(na, a, f0, b, g0);
        bg_lin(nb, a, f1, b, g1);
        // a negative result: negate it and its row of the matrix
        const bool nga = (int32_t)na[8] < 0, ngb = (int32_t)nb[8] < 0;
        {
            const uint32_t ma = nga ? 0xffffffffu : 0u, mb = ngb ? 0xffffffffu : 0u;
            uint32_t ca = nga ? 1u : 0u, cb = ngb ? 1u : 0u;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                a[i] = __builtin_addc(na[i] ^ ma, 0u, ca, &ca);
                b[i] = __builtin_addc(nb[i] ^ mb, 0u, cb, &cb);
            }
        }
        if (nga) { f0 = -f0; g0 = -g0; }
        if (ngb) { f1 = -f1; g1 = -g1; }
        uint32_t nu[8], nv[8];
        bg_lin_modp(nu, u, f0, v, g0);
        bg_lin_modp(nv, u, f1, v, g1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            u[i] = nu[i];
            v[i] = nv[i];
        }
    }
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = v[i];  // b = 1 = v x (mod p)
    return r;
}

// -------------------------------------------------------------- points (a = -3)
__device__ __forceinline__ Jac jac_inf() {
    Jac r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.X.v[i] = r.Y.v[i] = r.Z.v[i] = 0;
    r.X = fe_const(kOne);
    r.Y = fe_const(kOne);
    return r;
}

// dbl-2001-b
__device__ __forceinline__ Jac jac_dbl(const Jac &P) {
    Fe delta = fe_sqr(P.Z);
    Fe gamma = fe_sqr(P.Y);
    Fe beta = fe_mul(P.X, gamma);
    Fe t = fe_mul(fe_sub(P.X, delta), fe_add(P.X, delta));
    Fe alpha = fe_add(fe_add(t, t), t);
    Fe beta2 = fe_add(beta, beta);
    Fe beta4 = fe_add(beta2, beta2);
    Fe beta8 = fe_add(beta4, beta4);
    Jac R;
    R.X = fe_sub(fe_sqr(alpha), beta8);
    Fe yz = fe_add(P.Y, P.Z);
    R.Z = fe_sub(fe_sub(fe_sqr(yz), gamma), delta);
    Fe g2 = fe_sqr(gamma);
    Fe g4 = fe_add(g2, g2);
    Fe g8 = fe_add(g4, g4);
    g8 = fe_add(g8, g8);
    R.Y = fe_sub(fe_mul(alpha, fe_sub(beta4, R.X)), g8);
    return R;
}

// add-2007-bl with the exceptional cases (P == Q, P == -Q, infinity) handled
__device__ __forceinline__ Jac jac_add(const Jac &P, const Jac &Q) {
    if (fe_is_zero(P.Z)) return Q;
    if (fe_is_zero(Q.Z)) return P;
    Fe z1z1 = fe_sqr(P.Z);
    Fe z2z2 = fe_sqr(Q.Z);
    Fe u1 = fe_mul(P.X, z2z2);
    Fe u2 = fe_mul(Q.X, z1z1);
    Fe s1 = fe_mul(fe_mul(P.Y, Q.Z), z2z2);
    Fe s2 = fe_mul(fe_mul(Q.Y, P.Z), z1z1);
    Fe h = fe_sub(u2, u1);
    Fe r = fe_sub(s2, s1);
    if (fe_is_zero(h)) {
        if (fe_is_zero(r)) return jac_dbl(P);
        return jac_inf();
    }
    r = fe_add(r, r);
    Fe h2 = fe_add(h, h);
    Fe i = fe_sqr(h2);
    Fe j = fe_mul(h, i);
    Fe v = fe_mul(u1, i);
    Jac R;
    R.X = fe_sub(fe_sub(fe_sqr(r), j), fe_add(v, v));
    Fe s1j = fe_mul(s1, j);
    R.Y = fe_sub(fe_mul(r, fe_sub(v, R.X)), fe_add(s1j, s1j));
    Fe zz = fe_add(P.Z, Q.Z);
    R.Z = fe_mul(fe_sub(fe_sub(fe_sqr(zz), z1z1), z2z2), h);
    return R;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 32-byte big endian -> limbs
__device__ __forceinline__ Fe load_be(const uint8_t *p) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 a = q[0], b = q[1];
    uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    Fe r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = bswap32(w[7 - k]);
    return r;
}

__device__ __forceinline__ void store_be(uint8_t *p, const Fe &a) {
    uint4 *q = reinterpret_cast<uint4 *>(p);
    q[0] = make_uint4(bswap32(a.v[7]), bswap32(a.v[6]), bswap32(a.v[5]), bswap32(a.v[4]));
    q[1] = make_uint4(bswap32(a.v[3]), bswap32(a.v[2]), bswap32(a.v[1]), bswap32(a.v[0]));
}

// Load an affine wire point; false if a coordinate is >= p or the point is off the curve.
__device__ __forceinline__ bool load_point(const uint8_t *p, Jac &out) {
    Fe x = load_be(p), y = load_be(p + 32);
    bool ok = fe_lt_p(x) && fe_lt_p(y);
    x = to_mont(x);
    y = to_mont(y);
    // y^2 == x^3 - 3x + b
    Fe rhs = fe_mul(fe_sqr(x), x);
    Fe x3 = fe_add(fe_add(x, x), x);
    rhs = fe_add(fe_sub(rhs, x3), fe_const(kBm));
    ok = ok && fe_eq(fe_sqr(y), rhs);
    out.X = x;
    out.Y = y;
    out.Z = fe_const(kOne);
    return ok;
}

// ------------------------------------------------------------------ SHA-256
__device__ constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

__device__ void sha256_block(uint32_t (&h)[8], const uint32_t (&m)[16]) {
    uint32_t w[64];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = m[t];
#pragma unroll
    for (int t = 16; t < 64; ++t) {
        uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
        uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = hh + S1 + ch + kK[t] + w[t];
        uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        hh = g;
        g = f;
        f = e;
        e = d + t1;
        d = c;
        c = b;
        b = a;
        a = t1 + t2;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
    h[5] += f;
    h[6] += g;
    h[7] += hh;
}

// SHA-256 of the 64-byte big-endian x||y; digest written as 32 bytes
__device__ void sha256_point(const Fe &x, const Fe &y, uint8_t *out) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint32_t m[16];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        m[t] = x.v[7 - t];
        m[8 + t] = y.v[7 - t];
    }
    sha256_block(h, m);
#pragma unroll
    for (int t = 0; t < 16; ++t) m[t] = 0;
    m[0] = 0x80000000u;
    m[15] = 512;
    sha256_block(h, m);
    uint4 *q = reinterpret_cast<uint4 *>(out);
    q[0] = make_uint4(bswap32(h[0]), bswap32(h[1]), bswap32(h[2]), bswap32(h[3]));
    q[1] = make_uint4(bswap32(h[4]), bswap32(h[5]), bswap32(h[6]), bswap32(h[7]));
}

// ------------------------------------------------------------------ kernels
constexpr int kEcThreads = 64;

__device__ __forceinline__ void store_jac(uint32_t *jac, size_t plane_stride, const Jac &R) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        jac[(size_t)k * plane_stride] = R.X.v[k];
        jac[(size_t)(8 + k) * plane_stride] = R.Y.v[k];
        jac[(size_t)(16 + k) * plane_stride] = R.Z.v[k];
    }
}

__device__ __forceinline__ Jac load_jac(const uint32_t *jac, size_t plane_stride) {
    Jac R;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        R.X.v[k] = jac[(size_t)k * plane_stride];
        R.Y.v[k] = jac[(size_t)(8 + k) * plane_stride];
        R.Z.v[k] = jac[(size_t)(16 + k) * plane_stride];
    }
    return R;
}

// Width-5 NAF of a 256-bit scalar (32-byte big endian) into d[0..kNafLen), least significant
// digit first: digits are 0 or odd in [-15, 15] and every non-zero digit is followed by at
// least four zeros, so a scalar multiplication costs ~256/6 additions instead of 64 (4-bit
// windows).  A ninth limb absorbs k + 15 for scalars near 2^256.
constexpr int kNafLen = 258;

__device__ __forceinline__ void wnaf5(const uint8_t *k_be, int8_t (&d)[kNafLen]) {
    uint32_t k[9];
    {
        const Fe f = load_be(k_be);
#pragma unroll
        for (int i = 0; i < 8; ++i) k[i] = f.v[i];
        k[8] = 0;
    }
#pragma unroll 1
    for (int i = 0; i < kNafLen; ++i) {
        int v = 0;
        if (k[0] & 1u) {
            v = (int)(k[0] & 31u);
            if (v >= 16) v -= 32;
            // k -= v  (v odd, |v| <= 15)
            uint64_t c;
            if (v > 0) {
                c = (uint64_t)k[0] - (uint32_t)v;
                k[0] = (uint32_t)c;
#pragma unroll
                for (int l = 1; l < 9; ++l) {
                    c = (uint64_t)k[l] - (c >> 63);
                    k[l] = (uint32_t)c;
                }
            } else {
                c = (uint64_t)k[0] + (uint32_t)(-v);
                k[0] = (uint32_t)c;
#pragma unroll
                for (int l = 1; l < 9; ++l) {
                    c = (uint64_t)k[l] + (c >> 32);
                    k[l] = (uint32_t)c;
                }
            }
        }
        d[i] = (int8_t)v;
#pragma unroll
        for (int l = 0; l < 8; ++l) k[l] = (k[l] >> 1) | (k[l + 1] << 31);
        k[8] >>= 1;
    }
}

// Scalar multiplication scalar * point for T x D (term, element) pairs, flattened to one lane
// per pair g = j*D + i (1-D grid; the workgroup size is a launch parameter).
// points: [T][D][64] wire bytes; scalars: [T][32] (one per term) or [T][D][32] when
// per_element; jac out: SoA planes [T][24][D].
// wNAF (w = 5) with a table of the odd multiples P, 3P, ..., 15P: ~256 doublings and ~43
// additions from the most significant digit (was: fixed 4-bit windows, 252 + 63 + 13 table).
// The combine's scalars are one per term, so a wave's digits (and branches) are uniform.
template <int TPB, int WPE>
__global__ __launch_bounds__(TPB, WPE) void ec_mul_kernel(const uint8_t *__restrict__ points,
                                                     const uint8_t *__restrict__ scalars, int per_element, int T,
                                                     int D, uint32_t *__restrict__ jac,
                                                     uint32_t *__restrict__ flags) {
    // Latency-bound (one wave's issue chain sets the time): when the unmask runs beside it on
    // another stream (flamingo_amd/reconstruct.py), let these waves issue first; the
    // throughput-bound unmask waves fill the remaining slots.
    __builtin_amdgcn_s_setprio(3);
    const size_t g = (size_t)blockIdx.x * TPB + threadIdx.x;
    if (g >= (size_t)T * D) return;
    const int j = (int)(g / D);
    const int i = (int)(g - (size_t)j * D);
    const size_t e = g;
    Jac P;
    bool ok = load_point(points + e * 64, P);
    if (!ok) atomicOr(&flags[i], 2u);
    int8_t dig[kNafLen];
    wnaf5(scalars + (per_element ? e : (size_t)j) * 32, dig);

    Jac tab[8];  // tab[t] = (2t+1) P
    tab[0] = P;
    const Jac P2 = jac_dbl(P);
#pragma unroll 1
    for (int t = 1; t < 8; ++t) tab[t] = jac_add(tab[t - 1], P2);

    Jac acc = jac_inf();
    bool started = false;
#pragma unroll 1
    for (int w = kNafLen - 1; w >= 0; --w) {
        if (started) acc = jac_dbl(acc);
        const int v = dig[w];
        if (v) {
            Jac Q = tab[(v < 0 ? -v : v) >> 1];
            if (v < 0) Q.Y = fe_neg(Q.Y);
            acc = started ? jac_add(acc, Q) : Q;
            started = true;
        }
    }
    if (!ok) acc = jac_inf();
    store_jac(jac + (size_t)j * 24 * D + i, (size_t)D, acc);
}

// ------------------------------------------------ Straus: NT terms per lane
// The combine's sum_j lambda_j share_{j,i} with NT consecutive terms per lane sharing ONE chain
// of doublings (Straus / Shamir's trick): ~256 doublings + NT x ~43 additions + NT tables per lane
// instead of NT x (256 + 43 + 8) -- 35 % less work at NT = 2, for a longer chain per lane.  Worth it
// where the combine is throughput-bound (ServerReconstruction's 32 EC CUs).  Output: the per-lane
// partial sums as SoA planes [ceil(T/NT)][24][D] for ec_finish_kernel.  Off-curve points count as
// infinity and set flag bit 1, as in ec_mul_kernel.
template <int NT>
__global__ __launch_bounds__(kEcThreads) void ec_mul_straus_kernel(const uint8_t *__restrict__ points,
                                                                  const uint8_t *__restrict__ scalars, int T, int D,
                                                                  uint32_t *__restrict__ jac,
                                                                  uint32_t *__restrict__ flags) {
    __builtin_amdgcn_s_setprio(3);
    const int Tg = (T + NT - 1) / NT;
    const size_t g = (size_t)blockIdx.x * kEcThreads + threadIdx.x;
    if (g >= (size_t)Tg * D) return;
    const int jg = (int)(g / D);
    const int i = (int)(g - (size_t)jg * D);
    int8_t dig[NT][kNafLen];
    Jac tab[NT][8];
#pragma unroll 1
    for (int u = 0; u < NT; ++u) {
        const int j = jg * NT + u;
        Jac P = jac_inf();
        if (j < T) {
            if (!load_point(points + ((size_t)j * D + i) * 64, P)) {
                atomicOr(&flags[i], 2u);
                P = jac_inf();
            }
            wnaf5(scalars + (size_t)j * 32, dig[u]);
        } else {
#pragma unroll 1
            for (int k = 0; k < kNafLen; ++k) dig[u][k] = 0;
        }
        tab[u][0] = P;
        const Jac P2 = jac_dbl(P);
#pragma unroll 1
        for (int t = 1; t < 8; ++t) tab[u][t] = jac_add(tab[u][t - 1], P2);
    }
    Jac acc = jac_inf();
#pragma unroll 1
    for (int w = kNafLen - 1; w >= 0; --w) {
        acc = jac_dbl(acc);  // doubling infinity keeps Z = 0
#pragma unroll
        for (int u = 0; u < NT; ++u) {
            const int v = dig[u][w];
            if (v) {
                Jac Q = tab[u][(v < 0 ? -v : v) >> 1];
                if (v < 0) Q.Y = fe_neg(Q.Y);
                acc = jac_add(acc, Q);
            }
        }
    }
    store_jac(jac + (size_t)jg * 24 * D + i, (size_t)D, acc);
}

// ------------------------------------------------ cooperative scalar multiplication
// The same product as ec_mul_kernel, with FOUR waves (on the CU's four SIMDs) per 64 scalar
// multiplications: lane l of every wave works on item g = blockIdx.x * 64 + l, and the field
// multiplications of each point doubling are spread over the waves, exchanging field elements
// through LDS between three barriers:
//   L1  w0: delta = Z^2          w1: gamma = Y^2          w2: s = (Y+Z)^2
//   L2  w0: t = (X-delta)(X+delta), 3t   w1: beta = X gamma, 4 beta, 8 beta   w2: 8 gamma^2
//       w3: Z3 = s - gamma - delta
//   L3  w0: X3 = (3t)^2 - 8 beta, Y3 = 3t (4 beta - X3) - 8 gamma^2
// so a doubling costs 4 multiplications of latency instead of 8 (dbl-2001-b, a = -3).  Additions
// (~43 per scalar) run on wave 0 with the table of odd multiples in LDS.  A scalar multiplication is
// one lane's latency chain (~2,850 field multiplications), so where the batch leaves most SIMDs
// idle -- seed recovery on the whole chip, one rank's share of the pairs on G GPUs, the agents'
// ECDH/ElGamal batches -- this halves it; where the batch already fills its CUs (the CU-split
// reconstruction) the per-lane kernel issues fewer instructions.  Exceptional cases as jac_add.
constexpr int kCoopWaves = 4;
constexpr int kCoopSlots = 11;
// The cooperative kernels carry W = Z^4 (modified Jacobian, coop_dbl_w / coop_add_w below).

// lane-major slots: a lane's 8 words are 32 contiguous bytes, moved with two 16-byte LDS ops
// (0.5-1 % faster than word-major single-dword ops, profiles/r02_ab_coop_b128.log)
__device__ __forceinline__ void xput(uint32_t *slot, const Fe &a, int lane) {
    uint4 *q = reinterpret_cast<uint4 *>(slot + lane * 8);
    q[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    q[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
__device__ __forceinline__ Fe xget(const uint32_t *slot, int lane) {
    const uint4 *q = reinterpret_cast<const uint4 *>(slot + lane * 8);
    const uint4 x = q[0], y = q[1];
    Fe a;
    a.v[0] = x.x; a.v[1] = x.y; a.v[2] = x.z; a.v[3] = x.w;
    a.v[4] = y.x; a.v[5] = y.y; a.v[6] = y.z; a.v[7] = y.w;
    return a;
}


// ---- modified Jacobian (X, Y, Z, W = Z^4) for the cooperative kernels 
// Carrying W takes the doubling's a Z^4 term off the critical path: alpha = 3 (X^2 - W) needs one
// squaring, so alpha^2 lands one level earlier and a doubling is 3 multiplications of latency and
// two barriers instead of 4 and three.  Same outputs as dbl-2001-b (X3, Y3, Z3 are identical), so
// the Jacobian result and everything after it are bit-identical.
//
// The formulas are written once over a field policy F: LaneField (one element per lane, the
// Montgomery limbs of flm_p256.hip, exchange slots of 512 words) for ec_mul_coop_kernel, and
// RowField (one element per 16-lane row, flm_fe_row.h, slots of 64 words) for ec_mul_row_kernel.
template <class E>
struct JacWT {
    E X, Y, Z, W;
};
using JacW = JacWT<Fe>;

struct LaneField {
    using E = Fe;
    static constexpr int kSlot = 512;       // words per exchange slot: 64 lanes x 8 limbs
    static constexpr int kCoord = 8 * 64;   // words per coordinate of a table entry
    static constexpr int kEntry = 24 * 64;  // words per table entry (X, Y, Z)
    __device__ __forceinline__ E mul(const E &a, const E &b) const { return fe_mul(a, b); }
    __device__ __forceinline__ E sqr(const E &a) const { return fe_sqr(a); }
    __device__ __forceinline__ E add(const E &a, const E &b) const { return fe_add(a, b); }
    __device__ __forceinline__ E sub(const E &a, const E &b) const { return fe_sub(a, b); }
    __device__ __forceinline__ E neg(const E &a) const { return fe_neg(a); }
    __device__ __forceinline__ bool is_zero(const E &a) const { return fe_is_zero(a); }
    __device__ __forceinline__ void put(uint32_t *slot, const E &a, int lane) const { xput(slot, a, lane); }
    __device__ __forceinline__ E get(const uint32_t *slot, int lane) const { return xget(slot, lane); }
    __device__ __forceinline__ JacT<E> inf() const { return jac_inf(); }
    __device__ __forceinline__ JacT<E> dbl(const JacT<E> &P) const { return jac_dbl(P); }
};

struct RowField {
    using E = uint32_t;
    static constexpr int kSlot = 64;  // one word per lane: 4 elements x 16 lanes
    static constexpr int kCoord = 64;
    static constexpr int kEntry = 3 * 64;
    row::Ctx K;
    __device__ __forceinline__ E mul(E a, E b) const { return row::mul(a, b, K); }
    __device__ __forceinline__ E sqr(E a) const { return row::sqr(a, K); }
    __device__ __forceinline__ E add(E a, E b) const { return row::add(a, b, K); }
    __device__ __forceinline__ E sub(E a, E b) const { return row::sub(a, b, K); }
    __device__ __forceinline__ E neg(E a) const { return row::neg(a, K); }
    __device__ __forceinline__ bool is_zero(E a) const { return row::is_zero(a, K); }
    __device__ __forceinline__ void put(uint32_t *slot, E a, int lane) const { slot[lane] = a; }
    __device__ __forceinline__ E get(const uint32_t *slot, int lane) const { return slot[lane]; }
    __device__ __forceinline__ E one() const { return (threadIdx.x & 15) == 0 ? 1u : 0u; }
    __device__ __forceinline__ JacT<E> inf() const {  // (1, 1, 0), normal form
        JacT<E> r;
        r.X = r.Y = one();
        r.Z = 0u;
        return r;
    }
    // dbl-2001-b, as jac_dbl (the rare acc == Q path of an addition)
    __device__ JacT<E> dbl(const JacT<E> &P) const {
        const E delta = sqr(P.Z), gamma = sqr(P.Y), beta = mul(P.X, gamma);
        const E t = mul(sub(P.X, delta), add(P.X, delta));
        const E alpha = add(add(t, t), t);
        const E beta4 = add(add(beta, beta), add(beta, beta));
        JacT<E> R;
        R.X = sub(sqr(alpha), add(beta4, beta4));
        R.Z = sub(sub(sqr(add(P.Y, P.Z)), gamma), delta);
        const E g2 = sqr(gamma), g4 = add(g2, g2), g8 = add(g4, g4);
        R.Y = sub(mul(alpha, sub(beta4, R.X)), g8);
        return R;
    }
};

//   before barrier 1  w0: XX = X^2, alpha = 3 (XX - W), alpha^2
//                     w1: beta = X Y^2 -> 4 beta (slot 0), 8 beta (slot 1)
//                     w2: gamma^2 -> 8 gamma^2 (slot 2)            w3: Z3 = 2 Y Z
//   between barriers  w0: X3 = alpha^2 - 8 beta, Y3 = alpha (4 beta - X3) - 8 gamma^2 (slots 6, 7)
//                     w2: W3 = 16 gamma^2 W (slot 9)                w3: Z3 (slot 8)
// Slots 0..2 are read by w0 before barrier 2; the results (6..9) are written only between the two
// barriers, so the next operation's writes before its first barrier (slots 0..2 for a doubling,
// A/B = 0/1 for an addition) never land on a slot another wave is still reading.
template <class F>
__device__ __forceinline__ void coop_dbl_w(JacWT<typename F::E> &acc, int w, int lane, uint32_t *S, const F &f) {
    using E = typename F::E;
    constexpr int Q = F::kSlot;
    E alpha, a2, g8, z3;
    if (w == 0) {
        const E t = f.sub(f.sqr(acc.X), acc.W);
        alpha = f.add(f.add(t, t), t);
        a2 = f.sqr(alpha);
    } else if (w == 1) {
        const E beta = f.mul(acc.X, f.sqr(acc.Y));
        const E b2 = f.add(beta, beta);
        const E b4 = f.add(b2, b2);
        f.put(S + 0 * Q, b4, lane);
        f.put(S + 1 * Q, f.add(b4, b4), lane);
    } else if (w == 2) {
        E g = f.sqr(f.sqr(acc.Y));
        g = f.add(g, g);
        g = f.add(g, g);
        g8 = f.add(g, g);
        f.put(S + 2 * Q, g8, lane);
    } else {
        const E yz = f.mul(acc.Y, acc.Z);
        z3 = f.add(yz, yz);
    }
    __syncthreads();
    if (w == 0) {
        const E x3 = f.sub(a2, f.get(S + 1 * Q, lane));
        f.put(S + 6 * Q, x3, lane);
        f.put(S + 7 * Q, f.sub(f.mul(alpha, f.sub(f.get(S + 0 * Q, lane), x3)), f.get(S + 2 * Q, lane)), lane);
    } else if (w == 2) {
        f.put(S + 9 * Q, f.mul(f.add(g8, g8), acc.W), lane);
    } else if (w == 3) {
        f.put(S + 8 * Q, z3, lane);
    }
    __syncthreads();
    acc.X = f.get(S + 6 * Q, lane);
    acc.Y = f.get(S + 7 * Q, lane);
    acc.Z = f.get(S + 8 * Q, lane);
    acc.W = f.get(S + 9 * Q, lane);
}

// coop_add with W carried: the same six levels; w3, idle after L3, squares its Z3 twice (L4, L5)
// into slot H, and L6 picks W for the exceptional cases (Q or a doubling: two squarings of the new
// Z on that rare path; infinity: 0; acc: its own W).  Result slots D, E, F and K (W).
template <class F>
__device__ __forceinline__ void coop_add_w(JacWT<typename F::E> &acc, bool sel, int tab_idx, bool neg, int w, int lane,
                                           uint32_t *S, const uint32_t *tab, const F &f) {
    using E = typename F::E;
    constexpr int Q_ = F::kSlot;
    const uint32_t *q = tab + (size_t)tab_idx * F::kEntry;
    JacT<E> Q;
    Q.X = f.get(q, lane);
    Q.Y = f.get(q + F::kCoord, lane);
    Q.Z = f.get(q + 2 * F::kCoord, lane);
    if (neg) Q.Y = f.neg(Q.Y);
    uint32_t *A = S, *B = S + Q_, *C = S + 2 * Q_, *Dd = S + 3 * Q_, *Ee = S + 4 * Q_, *Fs = S + 5 * Q_,
             *G = S + 6 * Q_, *H = S + 7 * Q_, *I = S + 8 * Q_, *J = S + 9 * Q_, *K = S + 10 * Q_;
    E z1z1, z2z2, zz, s2a, s1a, u1, u2, s2, s1, h, i, j, v, x3, y3a, z3;
    // L1
    if (w == 0) {
        z1z1 = f.sqr(acc.Z);
        f.put(A, z1z1, lane);
    } else if (w == 1) {
        z2z2 = f.sqr(Q.Z);
        f.put(B, z2z2, lane);
    } else if (w == 2) {
        zz = f.sqr(f.add(acc.Z, Q.Z));
    } else {
        s1a = f.mul(acc.Y, Q.Z);
    }
    __syncthreads();
    // L2
    if (w == 0) {
        f.put(Dd, f.mul(Q.X, z1z1), lane);  // u2
    } else if (w == 1) {
        u1 = f.mul(acc.X, z2z2);
        f.put(Ee, u1, lane);
    } else if (w == 2) {
        z1z1 = f.get(A, lane);
        z2z2 = f.get(B, lane);
        f.put(Fs, f.sub(f.sub(zz, z1z1), z2z2), lane);  // Z3'
        s2a = f.mul(Q.Y, acc.Z);
    } else {
        z2z2 = f.get(B, lane);
        f.put(G, f.mul(s1a, z2z2), lane);  // s1
    }
    __syncthreads();
    // L3
    if (w == 0) {
        u2 = f.get(Dd, lane);
        u1 = f.get(Ee, lane);
        h = f.sub(u2, u1);
        const E h2 = f.add(h, h);
        i = f.sqr(h2);
        f.put(H, i, lane);
    } else if (w == 2) {
        s2 = f.mul(s2a, z1z1);
    } else if (w == 3) {
        u2 = f.get(Dd, lane);
        u1 = f.get(Ee, lane);
        z3 = f.mul(f.get(Fs, lane), f.sub(u2, u1));  // Z3 = Z3' h
        f.put(I, z3, lane);
    }
    __syncthreads();
    // L4
    if (w == 0) {
        j = f.mul(h, i);
        f.put(J, j, lane);
    } else if (w == 1) {
        i = f.get(H, lane);
        v = f.mul(u1, i);
        f.put(K, v, lane);
        f.put(Dd, f.add(v, v), lane);
    } else if (w == 2) {
        s1 = f.get(G, lane);
        E r = f.sub(s2, s1);
        r = f.add(r, r);
        f.put(A, r, lane);
        f.put(B, f.sqr(r), lane);
    } else {
        z3 = f.sqr(z3);
    }
    __syncthreads();
    // L5
    E r;
    if (w == 0) {
        v = f.get(K, lane);
        r = f.get(A, lane);
        const E rr = f.get(B, lane);
        x3 = f.sub(f.sub(rr, j), f.get(Dd, lane));
        y3a = f.mul(r, f.sub(v, x3));
    } else if (w == 1) {
        s1 = f.get(G, lane);
        j = f.get(J, lane);
        const E s1j = f.mul(s1, j);
        f.put(C, f.add(s1j, s1j), lane);
    } else if (w == 3) {
        f.put(H, f.sqr(z3), lane);  // W3 = Z3^4 (H's i was read at L4)
    }
    __syncthreads();
    // L6
    if (w == 0) {
        JacWT<E> R;
        R.X = x3;
        R.Y = f.sub(y3a, f.get(C, lane));
        R.Z = f.get(I, lane);
        R.W = f.get(H, lane);
        if (f.is_zero(acc.Z)) {
            R.X = Q.X; R.Y = Q.Y; R.Z = Q.Z;
            R.W = f.sqr(f.sqr(Q.Z));
        } else if (f.is_zero(Q.Z)) {
            R = acc;
        } else if (f.is_zero(h)) {
            JacT<E> a;
            a.X = acc.X; a.Y = acc.Y; a.Z = acc.Z;
            const JacT<E> d = f.is_zero(r) ? f.dbl(a) : f.inf();  // acc == Q / acc == -Q (rare: one lane)
            R.X = d.X; R.Y = d.Y; R.Z = d.Z;
            R.W = f.sqr(f.sqr(d.Z));
        }
        if (!sel) R = acc;
        f.put(Dd, R.X, lane);
        f.put(Ee, R.Y, lane);
        f.put(Fs, R.Z, lane);
        f.put(K, R.W, lane);
    }
    __syncthreads();
    acc.X = f.get(Dd, lane);
    acc.Y = f.get(Ee, lane);
    acc.Z = f.get(Fs, lane);
    acc.W = f.get(K, lane);
}


__global__ __launch_bounds__(64 * kCoopWaves) void ec_mul_coop_kernel(const uint8_t *__restrict__ points,
                                                                   const uint8_t *__restrict__ scalars,
                                                                   int per_element, int T, int D,
                                                                   uint32_t *__restrict__ jac,
                                                                   uint32_t *__restrict__ flags) {
    // latency-bound like ec_mul_kernel: beside the unmask on another stream (the unpartitioned
    // overlap, every rank of a sharded reconstruction) these waves issue first
    __builtin_amdgcn_s_setprio(3);
    __shared__ __attribute__((aligned(16))) uint32_t S[kCoopSlots * 8 * 64];  // exchange slots, 512 words each
    __shared__ __attribute__((aligned(16))) uint32_t tab[9 * 24 * 64];  // (2t+1) P, t = 0..7, + a spare row
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t g = (size_t)blockIdx.x * 64 + lane;
    const bool valid = g < (size_t)T * D;
    const int j = valid ? (int)(g / D) : 0;
    const int i = valid ? (int)(g - (size_t)j * D) : 0;
    // every wave loads the point and recodes the scalar itself (no exchange needed for either)
    Jac P = jac_inf();
    bool ok = true;
    int8_t dig[kNafLen];
    if (valid) {
        ok = load_point(points + g * 64, P);
        if (!ok) P = jac_inf();
        wnaf5(scalars + (per_element ? g : (size_t)j) * 32, dig);
    } else {
#pragma unroll 1
        for (int k = 0; k < kNafLen; ++k) dig[k] = 0;
    }
    if (w == 0 && valid && !ok) atomicOr(&flags[i], 2u);
    // table of odd multiples (2k+1) P (X, Y, Z only: an addend's W is needed on the rare path only)
    JacW PW;
    PW.X = P.X; PW.Y = P.Y; PW.Z = P.Z;
    PW.W = fe_sqr(fe_sqr(P.Z));
    JacW P2 = PW;
    coop_dbl_w(P2, w, lane, S, LaneField{});
    if (w == 0) {
        xput(tab, P.X, lane);
        xput(tab + 8 * 64, P.Y, lane);
        xput(tab + 16 * 64, P.Z, lane);
        xput(tab + 24 * 64, P2.X, lane);
        xput(tab + 32 * 64, P2.Y, lane);
        xput(tab + 40 * 64, P2.Z, lane);
    }
    __syncthreads();
    JacW t = PW;
#pragma unroll 1
    for (int k = 1; k < 8; ++k) {
        coop_add_w(t, true, 1, false, w, lane, S, tab, LaneField{});
        if (w == 0) {
            uint32_t *q = tab + (size_t)(k == 1 ? 8 : k) * 24 * 64;
            xput(q, t.X, lane);
            xput(q + 8 * 64, t.Y, lane);
            xput(q + 16 * 64, t.Z, lane);
        }
        __syncthreads();
    }
    if (w == 0) {
        const uint32_t *q = tab + (size_t)8 * 24 * 64;
        xput(tab + 24 * 64, xget(q, lane), lane);
        xput(tab + 32 * 64, xget(q + 8 * 64, lane), lane);
        xput(tab + 40 * 64, xget(q + 16 * 64, lane), lane);
    }
    __syncthreads();
    JacW accw;
    {
        const Jac inf = jac_inf();
        accw.X = inf.X; accw.Y = inf.Y; accw.Z = inf.Z;
        accw.W = inf.Z;  // 0
    }
    // the next digit is read from scratch before the doubling, so its latency hides under it (read
    // after the doubling, every step waited for the scratch load: tools/probes/ec_row_split.py)
    int v_next = dig[kNafLen - 1];
#pragma unroll 1
    for (int k = kNafLen - 1; k >= 0; --k) {
        const int v = v_next;
        if (k > 0) v_next = dig[k - 1];
        coop_dbl_w(accw, w, lane, S, LaneField{});
        if (__any(v != 0)) coop_add_w(accw, v != 0, (v < 0 ? -v : v) >> 1, v < 0, w, lane, S, tab, LaneField{});
    }
    if (w == 0 && valid) {
        Jac acc;
        acc.X = accw.X; acc.Y = accw.Y; acc.Z = accw.Z;
        if (!ok) acc = jac_inf();
        store_jac(jac + (size_t)j * 24 * D + i, (size_t)D, acc);
    }
}

// The cooperative kernel with every field element spread over a 16-lane row (flm_fe_row.h): a
// workgroup is the same four waves (formula roles w0..w3 as coop_dbl_w / coop_add_w), each wave
// holding four scalar multiplications, one per row.  A row multiplication is ~93 instructions per
// lane against ~258 for the per-lane Montgomery one, so each level of the formulas is that much
// shorter; in exchange the batch takes 16x the lanes.  For batches that leave most SIMDs idle --
// one G = 8 rank's share of the c5 pairs (ceil(962/8) x 20 products), the agents' ECDH batches --
// that is the trade to make (tools/ec_row_model.py).  Values stay in normal
// form inside; the result is converted to the Montgomery Jacobian planes ec_finish_kernel reads.
__device__ constexpr uint32_t kBn[8] = {0x27d2604bu, 0x3bce3c3eu, 0xcc53b0f6u, 0x651d06b0u,
                                        0x769886bcu, 0xb3ebbd55u, 0xaa3a93e7u, 0x5ac635d8u};  // b

__global__ __launch_bounds__(64 * kCoopWaves) void ec_mul_row_kernel(const uint8_t *__restrict__ points,
                                                                  const uint8_t *__restrict__ scalars,
                                                                  int per_element, int T, int D,
                                                                  uint32_t *__restrict__ jac,
                                                                  uint32_t *__restrict__ flags) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ uint32_t S[kCoopSlots * 64];   // exchange slots, one word per lane
    __shared__ uint32_t tab[9 * 3 * 64];      // (2t+1) P, t = 0..7, + a spare entry
    const int lane = threadIdx.x & 63, r = lane & 15;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    RowField f;
    f.K = row::make_ctx();
    const size_t g = (size_t)blockIdx.x * 4 + (lane >> 4);
    const bool valid = g < (size_t)T * D;
    const int j = valid ? (int)(g / D) : 0;
    const int i = valid ? (int)(g - (size_t)j * D) : 0;
    // the point: lane r < 8 holds limb r of x and of y (the wire is big endian)
    uint32_t x = 0, y = 0;
    if (valid && r < 8) {
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(points + g * 64);
        x = __builtin_bswap32(pw[7 - r]);
        y = __builtin_bswap32(pw[15 - r]);
    }
    // x, y < p and y^2 == x^3 - 3x + b (every lane runs every row operation: no divergence around
    // the carry loops' wave-wide votes)
    const uint32_t rhs = f.add(f.sub(f.mul(f.sqr(x), x), f.add(f.add(x, x), x)), r < 8 ? kBn[r & 7] : 0u);
    const bool in_x = row::row_all8(row::canon(x, f.K) == x, f.K);
    const bool in_y = row::row_all8(row::canon(y, f.K) == y, f.K);
    const bool on_c = row::row_all8(row::canon(f.sqr(y), f.K) == row::canon(rhs, f.K), f.K);
    const bool ok = in_x && in_y && on_c;
    if (w == 0 && valid && !ok && r == 0) atomicOr(&flags[i], 2u);
    JacWT<uint32_t> PW;
    PW.X = ok ? x : f.one();
    PW.Y = ok ? y : f.one();
    PW.Z = ok ? f.one() : 0u;
    PW.W = PW.Z;  // Z^4 of Z = 1 or 0
    int8_t dig[kNafLen];
    if (valid) {
        wnaf5(scalars + (per_element ? g : (size_t)j) * 32, dig);
    } else {
#pragma unroll 1
        for (int k = 0; k < kNafLen; ++k) dig[k] = 0;
    }
    // table of odd multiples (2k+1) P: 2P into entry 1 as the addend, then entry k = entry k-1 + 2P
    JacWT<uint32_t> P2 = PW;
    coop_dbl_w(P2, w, lane, S, f);
    if (w == 0) {
        tab[0 * 64 + lane] = PW.X;
        tab[1 * 64 + lane] = PW.Y;
        tab[2 * 64 + lane] = PW.Z;
        tab[3 * 64 + lane] = P2.X;
        tab[4 * 64 + lane] = P2.Y;
        tab[5 * 64 + lane] = P2.Z;
    }
    __syncthreads();
    JacWT<uint32_t> t = PW;
#pragma unroll 1
    for (int k = 1; k < 8; ++k) {
        coop_add_w(t, true, 1, false, w, lane, S, tab, f);
        if (w == 0) {
            uint32_t *q = tab + (size_t)(k == 1 ? 8 : k) * 3 * 64;
            q[lane] = t.X;
            q[64 + lane] = t.Y;
            q[128 + lane] = t.Z;
        }
        __syncthreads();
    }
    if (w == 0) {
        const uint32_t *q = tab + (size_t)8 * 3 * 64;
        tab[3 * 64 + lane] = q[lane];
        tab[4 * 64 + lane] = q[64 + lane];
        tab[5 * 64 + lane] = q[128 + lane];
    }
    __syncthreads();
    JacWT<uint32_t> acc;
    acc.X = acc.Y = f.one();
    acc.Z = acc.W = 0u;
    int v_next = dig[kNafLen - 1];  // read one step ahead, as ec_mul_coop_kernel
#pragma unroll 1
    for (int k = kNafLen - 1; k >= 0; --k) {
        const int v = v_next;
        if (k > 0) v_next = dig[k - 1];
        coop_dbl_w(acc, w, lane, S, f);
        if (__any(v != 0)) coop_add_w(acc, v != 0, (v < 0 ? -v : v) >> 1, v < 0, w, lane, S, tab, f);
    }
    if (w == 0) {
        // to the Montgomery form of ec_finish_kernel (x R mod p; R mod p = kOne as a normal value),
        // canonical; an invalid point went in as infinity (1, 1, 0) and comes out as (R, R, 0)
        const uint32_t rm = r < 8 ? kOne[r & 7] : 0u;
        const uint32_t X = row::canon(f.mul(acc.X, rm), f.K);
        const uint32_t Y = row::canon(f.mul(acc.Y, rm), f.K);
        const uint32_t Z = row::canon(f.mul(acc.Z, rm), f.K);
        if (valid && r < 8) {
            uint32_t *o = jac + (size_t)j * 24 * D + i;
            o[(size_t)r * D] = X;
            o[(size_t)(8 + r) * D] = Y;
            o[(size_t)(16 + r) * D] = Z;
        }
    }
}

// Per element i: acc = base_i (c1, or infinity when base == nullptr) + sign * sum_j R_{j,i};
// write the affine wire point and optionally SHA-256(x||y).
// flags bit 0: base off-curve, bit 1: an input share was off-curve (ec_mul), bit 2: result at infinity.
// kFinishLanes lanes per element split the T terms (lane q adds j = q, q + kFinishLanes, ...), then
// log2(kFinishLanes) LDS tree levels add the partials.  At T = 20: 8 lanes make it 3 + 3 sequential
// additions (lane 0 adds c1 first), 4 lanes 5 + 2 (round 3: 8).
// Lane 0 of each element then inverts Z and hashes (the inversion is one lane's chain either way).
constexpr int kFinishLanes = 8;
static_assert(kFinishLanes >= 1 && (kFinishLanes & (kFinishLanes - 1)) == 0 && kFinishLanes <= 64,
              "kFinishLanes: a power of two dividing the workgroup");
__global__ __launch_bounds__(kEcThreads) void ec_finish_kernel(const uint8_t *__restrict__ base,
                                                               const uint32_t *__restrict__ jac, int T, int D,
                                                               int negate, uint8_t *__restrict__ points_out,
                                                               uint8_t *__restrict__ digests_out,
                                                               uint32_t *__restrict__ flags) {
    __builtin_amdgcn_s_setprio(3);
    __shared__ uint32_t part[kEcThreads * 24];
    const int q = threadIdx.x % kFinishLanes;
    const int i = blockIdx.x * (kEcThreads / kFinishLanes) + threadIdx.x / kFinishLanes;
    const bool valid = i < D;
    uint32_t fl = 0;
    Jac acc = jac_inf();
    if (valid && q == 0 && base) {
        if (!load_point(base + (size_t)i * 64, acc)) {
            fl |= 1u;
            acc = jac_inf();
        }
    }
    if (valid) {
#pragma unroll 1
        for (int j = q; j < T; j += kFinishLanes) {
            Jac R = load_jac(jac + (size_t)j * 24 * D + i, (size_t)D);
            if (negate) R.Y = fe_neg(R.Y);
            acc = jac_add(acc, R);
        }
    }
    // tree over the element's 4 lanes (adjacent threads): level 1 lanes 0,2 add lanes 1,3;
    // level 2 lane 0 adds lane 2
    uint32_t *mine = part + threadIdx.x * 24;
#pragma unroll 1
    for (int step = 1; step < kFinishLanes; step *= 2) {
        store_jac(mine, 1, acc);
        __syncthreads();
        if (valid && (q % (2 * step)) == 0) acc = jac_add(acc, load_jac(mine + step * 24, 1));
        __syncthreads();
    }
    if (!valid || q != 0) return;
    Fe x = {}, y = {};
    if (fe_is_zero(acc.Z)) {
        fl |= 4u;
    } else {
        // acc.Z is Z R mod p as an integer: (Z R)^-1 R^3 R^-1 = Z^-1 R, the Montgomery form of Z^-1
        Fe zi = fe_mul(fe_inv_bingcd(acc.Z), fe_const(kR3));
        Fe zi2 = fe_sqr(zi);
        x = from_mont(fe_mul(acc.X, zi2));
        y = from_mont(fe_mul(acc.Y, fe_mul(zi2, zi)));
    }
    if (points_out) {
        store_be(points_out + (size_t)i * 64, x);
        store_be(points_out + (size_t)i * 64 + 32, y);
    }
    if (digests_out) sha256_point(x, y, digests_out + (size_t)i * 32);
    if (fl) atomicOr(&flags[i], fl);
}

// ------------------------------------------------- scalar field (mod n)
// Shamir recovery of the self-mask seeds (SA_ServiceAgent.py:506-526):
//     m_i = sum_j lambda_j * y_{j,i} mod n,   seed_i = m_i.to_bytes(32, 'big')
// with n the P-256 group order (the reference's `prime`, ecchash.n).  Generic
// CIOS Montgomery (n has no special form); T multiplications per lane.
__device__ constexpr uint32_t kN[8] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                                       0xffffffffu, 0xffffffffu, 0x00000000u, 0xffffffffu};
__device__ constexpr uint32_t kR2N[8] = {0xbe79eea2u, 0x83244c95u, 0x49bd6fa6u, 0x4699799cu,
                                         0x2b6bec59u, 0x2845b239u, 0xf3d95620u, 0x66e12d94u};  // R^2 mod n
constexpr uint32_t kN0 = 0xee00bc4fu;                                                             // -n^-1 mod 2^32

__device__ __forceinline__ void sc_reduce_once(Fe &r, const uint32_t (&t)[8], uint32_t t8) {
    uint32_t d[8], b = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(t[i], kN[i], b, &b);
    const bool take = t8 || !b;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = take ? d[i] : t[i];
}

__device__ __forceinline__ Fe sc_mul(const Fe &a, const Fe &b) {
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
        uint32_t m = t[0] * kN0;
        c = (uint64_t)m * kN[0] + t[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            c = (uint64_t)m * kN[j] + t[j] + (c >> 32);
            t[j - 1] = (uint32_t)c;
        }
        s = (uint64_t)hi0 + (c >> 32);
        t[7] = (uint32_t)s;
        t8 = hi1 + (uint32_t)(s >> 32);
    }
    Fe r;
    sc_reduce_once(r, t, t8);
    return r;
}

__device__ __forceinline__ Fe sc_add(const Fe &a, const Fe &b) {
    uint32_t s[8], c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    Fe r;
    sc_reduce_once(r, s, c);
    return r;
}

// shares: [T][M][32] big endian; lambdas: [T][32]; out: [M][32] big endian
__global__ __launch_bounds__(kEcThreads) void shamir_combine_kernel(const uint8_t *__restrict__ shares,
                                                                    const uint8_t *__restrict__ lambdas, int T,
                                                                    int M, uint8_t *__restrict__ out) {
    const int i = blockIdx.x * kEcThreads + threadIdx.x;
    if (i >= M) return;
    Fe acc = {};
    const Fe r2 = fe_const(kR2N);
#pragma unroll 1
    for (int j = 0; j < T; ++j) {
        Fe y = load_be(shares + ((size_t)j * M + i) * 32);
        Fe z = {};
        y = sc_add(y, z);                                   // y < 2^256 < 2n: one subtraction makes y < n
        Fe lm = sc_mul(load_be(lambdas + (size_t)j * 32), r2);   // lambda * R mod n
        acc = sc_add(acc, sc_mul(lm, y));                   // lambda * y mod n
    }
    store_be(out + (size_t)i * 32, acc);
}

// ------------------------------------------------------------- hash to curve
// The client's pairwise seed group element (SA_ClientAgent.py:275-286): h_ijt, a decimal string
// below 2^16, goes through util/crypto/ecchash.hash_str_to_curve(msg, count=2, modulus=n, degree=1,
// blen=48, XMDExpander(DST, sha256, 128)) (:277-283):
//   uniform = expand_message_xmd(msg, DST, 96)                                   (:90-133)
//   u_k     = OS2IP(uniform[48k : 48k + 48]) mod n      (the client passes n, not p: :285)  (:50-61)
//   Q_k     = map_to_curve(u_k)                                                   (:233-275)
//   H       = Q_0 + Q_1                                                           (:282)
// One lane per message, Montgomery field of the scalar-multiplication kernels.  map_to_curve is the
// reference's own simplified-SWU variant with Z = -10: tv1 = (100 u^4 - 10 u^2)^-1 (0 -> 0, the x1 =
// b/30 branch), x1 = -b/a (1 + tv1), x2 = -10 u^2 x1, y = the first square root of g(x1) else of g(x2).
// Square roots are a^((p+1)/4) (p = 3 mod 4): the root the host restatement (flamingo_amd/crypto.py)
// takes first for libnum's sqrtmod -- the one convention that stays "parity unpinned" (DESIGN.md).
// The sgn0 step (:271-272) flips y only when exactly one of u, y is zero.  The whole table of the
// protocol's 2^16 inputs is one launch (flm_hash_to_curve_decimal).
constexpr int kH2cMaxMsg = 64;
__device__ constexpr uint32_t kAm[8] = {0xfffffffcu, 0xffffffffu, 0xffffffffu, 0x00000003u,
                                        0x00000000u, 0x00000000u, 0x00000004u, 0xfffffffcu};  // a R (a = -3)
__device__ constexpr uint32_t kC1m[8] = {0x6341949fu, 0x9d899fcbu, 0x7d816585u, 0x8efaac9au,
                                         0xa7b5ba47u, 0xa1e0b58eu, 0x01826d67u, 0xf4100209u};  // (-b/a) R
__device__ constexpr uint32_t kC2m[8] = {0xf0535ba9u, 0x5c8dc32du, 0x8c8cf08du, 0xc17f77a9u,
                                         0x43f892a0u, 0x7696788eu, 0x99c03e24u, 0x98680033u};  // (b/30) R
__device__ constexpr uint32_t k10m[8] = {0x0000000au, 0x00000000u, 0x00000000u, 0xfffffff6u,
                                         0xffffffffu, 0xffffffffu, 0xfffffff5u, 0x00000009u};  // 10 R
__device__ constexpr uint32_t k100m[8] = {0x00000064u, 0x00000000u, 0x00000000u, 0xffffff9cu,
                                          0xffffffffu, 0xffffffffu, 0xffffff9bu, 0x00000063u};  // 100 R
__device__ constexpr uint32_t kNeg10m[8] = {0xfffffff5u, 0xffffffffu, 0xffffffffu, 0x0000000au,
                                            0x00000000u, 0x00000000u, 0x0000000bu, 0xfffffff5u};  // -10 R
__device__ constexpr uint32_t kNc[7] = {0x039cdaafu, 0x0c46353du, 0x58e8617bu, 0x43190552u,
                                        0x00000000u, 0x00000000u, 0xffffffffu};  // 2^256 - n (< 2^224)
// ecchash.test_dst("P256_XMD:SHA-256_SSWU_RO_") || I2OSP(44, 1): DST_prime of :104
__device__ constexpr uint8_t kDstPrime[45] = {'Q', 'U', 'U', 'X', '-', 'V', '0', '1', '-', 'C', 'S', '0', '2', '-', 'w',
                                              'i', 't', 'h', '-', 'P', '2', '5', '6', '_', 'X', 'M', 'D', ':', 'S', 'H',
                                              'A', '-', '2', '5', '6', '_', 'S', 'S', 'W', 'U', '_', 'R', 'O', '_', 44};

// SHA-256 fed byte by byte (the messages are short and their layout depends on the message length)
struct Sha256 {
    uint32_t h[8];
    uint32_t w[16];
    uint32_t n;      // bytes in w
    uint32_t total;  // bytes hashed
};

__device__ __forceinline__ void sha_init(Sha256 &s) {
    const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab,
                            0x5be0cd19};
#pragma unroll
    for (int i = 0; i < 8; ++i) s.h[i] = iv[i];
#pragma unroll
    for (int i = 0; i < 16; ++i) s.w[i] = 0;
    s.n = 0;
    s.total = 0;
}

__device__ void sha_put(Sha256 &s, uint32_t b) {
    s.w[s.n >> 2] |= (b & 0xffu) << (24 - 8 * (s.n & 3));
    ++s.total;
    if (++s.n == 64) {
        sha256_block(s.h, s.w);
#pragma unroll
        for (int i = 0; i < 16; ++i) s.w[i] = 0;
        s.n = 0;
    }
}

__device__ void sha_put_dst(Sha256 &s) {
#pragma unroll 1
    for (int i = 0; i < 45; ++i) sha_put(s, kDstPrime[i]);
}

// the digest as 8 big-endian words (word k = bytes 4k..4k+3)
__device__ void sha_final(Sha256 &s, uint32_t (&out)[8]) {
    const uint64_t bits = (uint64_t)s.total * 8;
    sha_put(s, 0x80);
#pragma unroll 1
    while (s.n != 56) sha_put(s, 0);
#pragma unroll 1
    for (int i = 7; i >= 0; --i) sha_put(s, (uint32_t)(bits >> (8 * i)));
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = s.h[i];
}

// 384-bit big-endian words u[0..11] mod n: fold t = lo + hi (2^256 mod n) until t < 2^256 (at most
// 7 folds for any 384-bit input: the high part shrinks by >= 31 bits a fold), then one subtraction
__device__ Fe mod_n_384(const uint32_t *u) {
    uint32_t t[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) t[i] = u[11 - i];
#pragma unroll 1
    for (int it = 0; it < 7; ++it) {
        uint32_t hi[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            hi[i] = t[8 + i];
            t[8 + i] = 0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint64_t c = 0;
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                c = (uint64_t)hi[i] * kNc[j] + t[i + j] + (c >> 32);
                t[i + j] = (uint32_t)c;
            }
            c >>= 32;
#pragma unroll
            for (int k = i + 7; k < 12; ++k) {
                c += t[k];
                t[k] = (uint32_t)c;
                c >>= 32;
            }
        }
    }
    uint32_t d[8], b = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(t[i], kN[i], b, &b);
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = b ? t[i] : d[i];  // no borrow: t >= n
    return r;
}

// Montgomery-form inverse by binary GCD (ec_finish_kernel's: ~25k VALU instructions against Fermat's
// ~73k): (a R)^-1 R^3 R^-1 = a^-1 R; 0 -> 0, as the reference's tv1 branch needs
__device__ __forceinline__ Fe fe_inv_mont(const Fe &a) {
    if (fe_is_zero(a)) return a;
    return fe_mul(fe_inv_bingcd(a), fe_const(kR3));
}

__device__ __forceinline__ Fe fe_sqr_n(Fe a, int n) {
#pragma unroll 1
    for (int i = 0; i < n; ++i) a = fe_sqr(a);
    return a;
}

// a^((p+1)/4), (p+1)/4 = (2^32 - 1) 2^222 + 2^190 + 2^94: 253 squarings, 7 multiplications
__device__ Fe fe_sqrt_cand(const Fe &a) {
    const Fe x2 = fe_mul(fe_sqr(a), a);
    const Fe x4 = fe_mul(fe_sqr_n(x2, 2), x2);
    const Fe x8 = fe_mul(fe_sqr_n(x4, 4), x4);
    const Fe x16 = fe_mul(fe_sqr_n(x8, 8), x8);
    const Fe x32 = fe_mul(fe_sqr_n(x16, 16), x16);
    Fe r = fe_mul(fe_sqr_n(x32, 32), a);
    r = fe_mul(fe_sqr_n(r, 96), a);
    return fe_sqr_n(r, 94);
}

// map_to_curve (ecchash.py:233-275) of u (canonical, < n < p), affine Montgomery (x, y); bad = neither
// g(x1) nor g(x2) had a root (cannot happen for this map; flagged rather than assumed)
__device__ void h2c_map(const Fe &u_plain, Fe &x, Fe &y, bool &bad) {
    const Fe u = to_mont(u_plain);
    const Fe u2 = fe_sqr(u);
    const Fe u4 = fe_sqr(u2);
    const Fe den = fe_sub(fe_mul(fe_const(k100m), u4), fe_mul(fe_const(k10m), u2));
    const Fe tv1 = fe_inv_mont(den);                              // 0 -> 0 (the :247-248 branch)
    Fe x1 = fe_mul(fe_const(kC1m), fe_add(fe_const(kOne), tv1));
    if (fe_is_zero(tv1)) x1 = fe_const(kC2m);
    const Fe gx1 = fe_add(fe_mul(x1, fe_add(fe_sqr(x1), fe_const(kAm))), fe_const(kBm));
    const Fe x2 = fe_mul(fe_const(kNeg10m), fe_mul(u2, x1));
    const Fe gx2 = fe_add(fe_mul(x2, fe_add(fe_sqr(x2), fe_const(kAm))), fe_const(kBm));
    const Fe y1 = fe_sqrt_cand(gx1);
    const bool sq1 = fe_eq(fe_sqr(y1), gx1);
    const Fe y2 = fe_sqrt_cand(gx2);
    bad = !sq1 && !fe_eq(fe_sqr(y2), gx2);
    x = sq1 ? x1 : x2;
    y = sq1 ? y1 : y2;
    if (fe_is_zero(u_plain) != fe_is_zero(y)) y = fe_neg(y);    // sgn0(u) != sgn0(y), :271-272
}

// msgs: n x kH2cMaxMsg bytes (message i in its first lens[i] bytes), or NULL for the decimal
// strings of v0 + i (str(h_ijt), SA_ClientAgent.py:280).  out: n x 64 wire bytes (infinity: zeros,
// flags bit 2); flags bit 3: no square root (not expected).
// Two adjacent lanes per message: both expand it (9 SHA-256 compressions, cheap next to the field
// work), lane 2m maps u_0 and lane 2m+1 maps u_1 -- the two map_to_curve calls are independent, so
// the chain a lane runs is one inversion + two square roots instead of two of each -- then the odd
// lane hands its point to the even one (a lane swap, no LDS), which adds, inverts and stores.
__global__ __launch_bounds__(kEcThreads) void hash_to_curve_kernel(const uint8_t *__restrict__ msgs,
                                                                   const uint32_t *__restrict__ lens, uint32_t v0,
                                                                   int n, uint8_t *__restrict__ out,
                                                                   uint32_t *__restrict__ flags) {
    const int t = blockIdx.x * kEcThreads + threadIdx.x;
    const int i = t >> 1, half = t & 1;
    const bool valid = i < n;  // both lanes of a pair stay to the swap: no early return
    uint8_t msg[kH2cMaxMsg];
    int m = 0;
    if (valid && msgs) {
        m = (int)lens[i];
#pragma unroll 1
        for (int k = 0; k < m; ++k) msg[k] = msgs[(size_t)i * kH2cMaxMsg + k];
    } else if (valid) {
        uint32_t v = v0 + (uint32_t)i;
        uint8_t dig[10];
        int nd = 0;
#pragma unroll 1
        do {
            dig[nd++] = (uint8_t)('0' + v % 10);
            v /= 10;
        } while (v);
#pragma unroll 1
        for (int k = 0; k < nd; ++k) msg[k] = dig[nd - 1 - k];
        m = nd;
    }
    // b_0 = H(Z_pad || msg || I2OSP(96, 2) || I2OSP(0, 1) || DST_prime)   (:113-114)
    Sha256 s;
    sha_init(s);
    sha256_block(s.h, s.w);  // Z_pad: one all-zero block (s.w is zero)
    s.total = 64;
#pragma unroll 1
    for (int k = 0; k < m; ++k) sha_put(s, msg[k]);
    sha_put(s, 0);
    sha_put(s, 96);
    sha_put(s, 0);
    sha_put_dst(s);
    uint32_t b0[8], bi[8], uni[24];
    sha_final(s, b0);
    // b_1 = H(b_0 || 1 || DST_prime), b_i = H((b_0 ^ b_{i-1}) || i || DST_prime)   (:115-117)
#pragma unroll
    for (int k = 0; k < 8; ++k) bi[k] = 0;
#pragma unroll 1
    for (int blk = 1; blk <= 3; ++blk) {
        sha_init(s);
#pragma unroll 1
        for (int k = 0; k < 32; ++k) sha_put(s, (b0[k >> 2] ^ bi[k >> 2]) >> (24 - 8 * (k & 3)));
        sha_put(s, (uint32_t)blk);
        sha_put_dst(s);
        sha_final(s, bi);
#pragma unroll
        for (int k = 0; k < 8; ++k) uni[(blk - 1) * 8 + k] = bi[k];
    }
    Fe x, y;
    bool bad;
    h2c_map(mod_n_384(half ? uni + 12 : uni), x, y, bad);   // Q_half = map_to_curve(u_half)
    Fe x1, y1;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x1.v[k] = (uint32_t)__shfl_xor((int)x.v[k], 1);
        y1.v[k] = (uint32_t)__shfl_xor((int)y.v[k], 1);
    }
    const bool bad1 = __shfl_xor((int)bad, 1) != 0;
    if (!valid || half) return;
    Jac Q0, Q1;
    Q0.X = x;
    Q0.Y = y;
    Q0.Z = fe_const(kOne);
    Q1.X = x1;
    Q1.Y = y1;
    Q1.Z = fe_const(kOne);
    const Jac R = jac_add(Q0, Q1);                                 // Q0 + Q1 (:282), P == +-Q handled
    uint32_t fl = (bad || bad1) ? 8u : 0u;
    Fe ax = {}, ay = {};
    if (fe_is_zero(R.Z)) {
        fl |= 4u;
    } else {
        const Fe zi = fe_inv_mont(R.Z);
        const Fe zi2 = fe_sqr(zi);
        ax = from_mont(fe_mul(R.X, zi2));
        ay = from_mont(fe_mul(R.Y, fe_mul(zi2, zi)));
    }
    store_be(out + (size_t)i * 64, ax);
    store_be(out + (size_t)i * 64 + 32, ay);
    flags[i] = fl;
}

}  // namespace

template <int TPB, int WPE>
static void launch_ec_mul_t(const uint8_t *d_points, const uint8_t *d_scalars, int per_element, int T, int D,
                            uint32_t *d_jac, uint32_t *d_flags, hipStream_t stream, unsigned lds_pad) {
    const size_t n = (size_t)T * D;
    hipLaunchKernelGGL((ec_mul_kernel<TPB, WPE>), dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), lds_pad, stream,
                       d_points, d_scalars, per_element, T, D, d_jac, d_flags);
}

// threads: lanes per workgroup (64/128/256); waves: register budget, as minimum waves per SIMD
// (2: no cap, 172 VGPRs; 4: 128 VGPRs; 8: 64 VGPRs, both with spills)
int ec_mul_groups(int T, int terms) { return terms > 1 ? (T + terms - 1) / terms : T; }

hipError_t launch_ec_mul(const uint8_t *d_points, const uint8_t *d_scalars, int per_element, int T, int D,
                         uint32_t *d_jac, uint32_t *d_flags, hipStream_t stream, int threads, int waves, int coop,
                         int terms, unsigned lds_pad) {
    if (T <= 0 || D <= 0) return hipSuccess;
    if (terms > 1 && !per_element) {
        const size_t n = (size_t)ec_mul_groups(T, terms) * D;
        const dim3 grid((unsigned)((n + kEcThreads - 1) / kEcThreads));
        if (terms == 2)
            hipLaunchKernelGGL(ec_mul_straus_kernel<2>, grid, dim3(kEcThreads), lds_pad, stream, d_points, d_scalars, T, D,
                               d_jac, d_flags);
        else if (terms == 4)
            hipLaunchKernelGGL(ec_mul_straus_kernel<4>, grid, dim3(kEcThreads), lds_pad, stream, d_points, d_scalars, T, D,
                               d_jac, d_flags);
        else
            return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (coop == 2) {  // one element per 16-lane row: four scalar multiplications per workgroup
        const size_t n = (size_t)T * D;
        hipLaunchKernelGGL(ec_mul_row_kernel, dim3((unsigned)((n + 3) / 4)), dim3(64 * kCoopWaves), 0, stream,
                           d_points, d_scalars, per_element, T, D, d_jac, d_flags);
        return hipGetLastError();
    }
    if (coop) {
        const size_t n = (size_t)T * D;
        hipLaunchKernelGGL(ec_mul_coop_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64 * kCoopWaves), 0, stream,
                           d_points, d_scalars, per_element, T, D, d_jac, d_flags);
        return hipGetLastError();
    }
#define FLM_EC(TPB)                                                                                          \
    switch (waves) {                                                                                         \
        case 4: launch_ec_mul_t<TPB, 4>(d_points, d_scalars, per_element, T, D, d_jac, d_flags, stream, lds_pad); break; \
        case 8: launch_ec_mul_t<TPB, 8>(d_points, d_scalars, per_element, T, D, d_jac, d_flags, stream, lds_pad); break; \
        default: launch_ec_mul_t<TPB, 1>(d_points, d_scalars, per_element, T, D, d_jac, d_flags, stream, lds_pad); break; \
    }
    switch (threads) {
        case 64: FLM_EC(64) break;
        case 128: FLM_EC(128) break;
        default: FLM_EC(256) break;
    }
#undef FLM_EC
    return hipGetLastError();
}

hipError_t launch_shamir_combine(const uint8_t *d_shares, const uint8_t *d_lambdas, int T, int M, uint8_t *d_out,
                                 hipStream_t stream) {
    if (M <= 0) return hipSuccess;
    dim3 grid((M + kEcThreads - 1) / kEcThreads);
    hipLaunchKernelGGL(shamir_combine_kernel, grid, dim3(kEcThreads), 0, stream, d_shares, d_lambdas, T, M, d_out);
    return hipGetLastError();
}

hipError_t launch_ec_finish(const uint8_t *d_base, const uint32_t *d_jac, int T, int D, int negate,
                            uint8_t *d_points_out, uint8_t *d_digests_out, uint32_t *d_flags, hipStream_t stream) {
    if (D <= 0) return hipSuccess;
    constexpr int per_group = kEcThreads / kFinishLanes;
    dim3 grid((D + per_group - 1) / per_group);
    hipLaunchKernelGGL(ec_finish_kernel, grid, dim3(kEcThreads), 0, stream, d_base, d_jac, T, D, negate,
                       d_points_out, d_digests_out, d_flags);
    return hipGetLastError();
}

hipError_t launch_hash_to_curve(const uint8_t *d_msgs, const uint32_t *d_lens, uint32_t v0, int n, uint8_t *d_out,
                                uint32_t *d_flags, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const size_t lanes = 2 * (size_t)n;  // two lanes per message
    hipLaunchKernelGGL(hash_to_curve_kernel, dim3((unsigned)((lanes + kEcThreads - 1) / kEcThreads)), dim3(kEcThreads),
                       0, stream, d_msgs, d_lens, v0, n, d_out, d_flags);
    return hipGetLastError();
}

}  // namespace flm
