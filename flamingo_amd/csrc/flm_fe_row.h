// flm_fe_row.h -- P-256 field arithmetic with one element spread over a 16-lane DPP row (gfx950).
//
// The seed recovery of one G = 8 rank (SA_ServiceAgent.py:542-585 over ceil(D/8) pairs) is a few
// hundred waves on 1,024 SIMDs: a latency chain, and a lone wave issues one VALU instruction per
// ~8 cycles, so its time is the instruction count on the critical path.  The
// per-lane field multiplication of flm_p256.hip is ~258 instructions on one lane.  Here one field
// element occupies a DPP row: lane r = lane & 15 holds 32-bit limb r (little endian) for r < 8 and
// 0 for r >= 8, so a multiplication is ~90 instructions per lane:
//   * product scanning, one column per lane: lane t accumulates sum_i a_i b_(t-i) with a_i broadcast
//     from lane i (DPP row_newbcast:i) and b shifted by i lanes (row_shr:i, zero from below) -- 8
//     v_mad_u64_u32 with their carries, every column of the 512-bit product at once;
//   * the columns (96 bits each) become 16 saturated limbs by carry passes along the row;
//   * NIST's fast reduction for p = 2^256 - 2^224 + 2^192 + 2^96 - 1: limb r of the result is
//     c_r + sum_k A[r][k] c_(8+k), A a fixed 8x8 matrix of -1..3 (each c_(8+k) broadcast once, two
//     multiply-adds per k: the lane's own coefficient A + 1 >= 0, and the row-uniform sum it biases);
//   * signed carry passes along the row, the carry out of limb 7 folded back as
//     t 2^256 = t (2^224 - 2^192 - 2^96 + 1) (mod p), until no limb carries.
// Values are kept lazily in [0, 2^256) (possibly >= p); canon() gives the representative < p.
// The carry passes loop until no lane of the wave carries (wave-uniform branch after each pass): one
// pass for almost every input, up to ~10 for adversarial ones (tools/ec_row_model.py runs the same
// loops).
// Normal form (no Montgomery factor): the reduction is the parallel NIST fold, not the sequential
// Montgomery digit chain.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace flm {
namespace row {

// gfx9 DPP controls: row_shr:n = 0x110 + n, row_newbcast:n = 0x150 + n (gfx90a and later).
// bound_ctrl set: a lane whose source is outside its row reads 0, so no "old" value (and no
// zeroing move before each DPP instruction) is needed.
template <int N>
__device__ __forceinline__ uint32_t bcast(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + N, 0xf, 0xf, true);
}
template <int N>
__device__ __forceinline__ uint32_t shr(uint32_t x) {  // lane r gets lane r - N of its row, 0 for r < N
    if constexpr (N == 0) return x;
    else return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x110 + N, 0xf, 0xf, true);
}

// NIST fold coefficients A[r][k] (limb r of the result takes A[r][k] * c_(8+k); tools/ec_row_model.py)
__device__ constexpr int8_t kFold[8][8] = {
    {1, 1, 0, -1, -1, -1, -1, 0}, {0, 1, 1, 0, -1, -1, -1, -1}, {0, 0, 1, 1, 0, -1, -1, -1},
    {-1, -1, 0, 2, 2, 1, 0, -1}, {0, -1, -1, 0, 2, 2, 1, 0},   {0, 0, -1, -1, 0, 2, 2, 1},
    {-1, -1, 0, 0, 0, 1, 3, 2},  {1, 0, -1, -1, -1, -1, 0, 3}};
__device__ constexpr uint32_t kPl[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};

// Per-lane constants, built once per kernel (kept in VGPRs).
struct Ctx {
    uint32_t a1[8];    // A[r][k] + 1 (0..4) for r < 8, else 0: the fold adds sum_k a1 c_(8+k) - sum_k c_(8+k)
    uint32_t one8;     // 1 for r < 8, else 0 (the weight of that row-uniform sum)
    int32_t fco;       // the top carry's weight at limb r: +1 (r = 0, 7), -1 (r = 3, 6), else 0
    uint32_t lo8;      // ~0 for r < 8, else 0
    uint32_t plimb;    // limb r of p (0 for r >= 8)
    uint32_t rbit;     // lane & ~15: this row's first bit in a wave-wide ballot
};

__device__ __forceinline__ Ctx make_ctx() {
    Ctx c;
    const int lane = (int)(threadIdx.x & 63), r = lane & 15;
    const bool low = r < 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) c.a1[k] = low ? (uint32_t)(kFold[r & 7][k] + 1) : 0u;
    c.one8 = low ? 1u : 0u;
    c.fco = !low ? 0 : (r == 0 || r == 7) ? 1 : (r == 3 || r == 6) ? -1 : 0;
    c.lo8 = low ? ~0u : 0u;
    c.plimb = low ? kPl[r] : 0u;
    c.rbit = (uint32_t)(lane & ~15);
    return c;
}

// Signed carry passes: v (lanes r < 8: a signed 64-bit limb value, lanes >= 8: 0) -> the limbs of a
// value congruent mod p in [0, 2^256).  The carry out of limb r moves to limb r + 1; limb 7's is
// folded back at limbs 0, 3, 6, 7.  Every caller's input carries somewhere (a product fold, a
// limb-wise add or subtract), so the first pass runs unconditionally and the wave-wide vote comes
// after it: one branch for almost every input.
__device__ __forceinline__ uint32_t snorm(int64_t v, const Ctx &K) {
    int32_t c = (int32_t)(v >> 32);
    uint32_t lo = (uint32_t)v;
#pragma unroll 1
    do {
        const int32_t t = (int32_t)bcast<7>((uint32_t)c);
        const int32_t cin = (int32_t)(shr<1>((uint32_t)c) & K.lo8);
        v = (int64_t)(uint64_t)lo + (int64_t)(cin + t * K.fco);
        c = (int32_t)(v >> 32);
        lo = (uint32_t)v;
    } while (__any(c != 0));
    return lo;
}

// acc (64-bit) += a * b, carry out of the 64 bits counted in hi: one asm statement (v_mad_u64_u32's
// own carry-out feeds one v_addc), as the per-lane product columns of flm_p256.hip.
__device__ __forceinline__ void mad_carry(uint64_t &acc, uint32_t &hi, uint32_t a, uint32_t b) {
    uint64_t c;
    asm("v_mad_u64_u32 %[acc], %[c], %[a], %[b], %[acc]\n\t"
        "v_addc_co_u32_e64 %[hi], %[c], 0, %[hi], %[c]"
        : [acc] "+&v"(acc), [hi] "+&v"(hi), [c] "=&s"(c)
        : [a] "v"(a), [b] "v"(b));
}

template <int I>
__device__ __forceinline__ void prod_step(uint64_t &acc, uint32_t &hi, uint32_t a, uint32_t b) {
    if constexpr (I < 8) {
        mad_carry(acc, hi, bcast<I>(a), shr<I>(b));
        prod_step<I + 1>(acc, hi, a, b);
    }
}

// a * b mod p (lazy, < 2^256).  a, b < 2^256 in the row layout.
__device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b, const Ctx &K) {
    // column t = sum_i a_i b_(t-i) in lane t: 64-bit accumulator + carry count (column < 2^67)
    uint64_t acc = (uint64_t)bcast<0>(a) * b;
    uint32_t hi = 0;
    prod_step<1>(acc, hi, a, b);
    // columns -> 16 saturated limbs: limb t = lo(col t) + hi32(col t-1) + hi(col t-2) + carries
    uint64_t s = (uint64_t)(uint32_t)acc + shr<1>((uint32_t)(acc >> 32)) + shr<2>(hi);
    uint32_t c = (uint32_t)(s >> 32), lo = (uint32_t)s;
#pragma unroll 1
    do {  // the three-term sums carry in some lane of every product: first pass unconditional
        s = (uint64_t)lo + shr<1>(c);
        c = (uint32_t)(s >> 32);
        lo = (uint32_t)s;
    } while (__any(c != 0));
    // NIST fold: limb r = c_r + sum_k A[r][k] c_(8+k) = c_r + sum_k (A[r][k] + 1) c_(8+k) - sum_k c_(8+k),
    // the coefficients made non-negative so every term is one v_mad_u64_u32 (lanes >= 8 stay 0)
    uint64_t pos = (uint64_t)(lo & K.lo8), hsum = 0;
#define FLM_ROW_FOLD(k)                               \
    {                                                 \
        const uint32_t h = bcast<8 + k>(lo);          \
        pos += (uint64_t)h * K.a1[k];                 \
        hsum += (uint64_t)h * K.one8;                 \
    }
    FLM_ROW_FOLD(0) FLM_ROW_FOLD(1) FLM_ROW_FOLD(2) FLM_ROW_FOLD(3)
    FLM_ROW_FOLD(4) FLM_ROW_FOLD(5) FLM_ROW_FOLD(6) FLM_ROW_FOLD(7)
#undef FLM_ROW_FOLD
    return snorm((int64_t)(pos - hsum), K);
}

__device__ __forceinline__ uint32_t sqr(uint32_t a, const Ctx &K) { return mul(a, a, K); }

__device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b, const Ctx &K) {
    return snorm((int64_t)(uint64_t)a + b, K);
}

__device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b, const Ctx &K) {
    return snorm((int64_t)(uint64_t)a - (int64_t)(uint64_t)b, K);
}

__device__ __forceinline__ uint32_t neg(uint32_t a, const Ctx &K) { return sub(0u, a, K); }

// this row's bits of a wave-wide ballot of `pred`, as a per-lane bool: true when pred holds in
// every lane r < 8 of the row
__device__ __forceinline__ bool row_all8(bool pred, const Ctx &K) {
    const uint64_t m = __ballot(pred);
    return ((uint32_t)(m >> K.rbit) & 0xffu) == 0xffu;
}

// a == 0 mod p for a lazy value (a < 2^256 < 2p: a is 0 or p)
__device__ __forceinline__ bool is_zero(uint32_t a, const Ctx &K) {
    return row_all8(a == 0u, K) || row_all8(a == K.plimb, K);
}

// the representative < p: subtract p once when a >= p (a < 2^256 < 2p).  a - p with the borrows
// passed along the row; the borrows out of limb 7, summed, are the sign of a - p.
__device__ __forceinline__ uint32_t canon(uint32_t a, const Ctx &K) {
    int64_t d = (int64_t)(uint64_t)a - (int64_t)(uint64_t)K.plimb;
    int32_t c = (int32_t)(d >> 32), top = 0;
    uint32_t lo = (uint32_t)d;
#pragma unroll 1
    do {
        top += (int32_t)bcast<7>((uint32_t)c);
        d = (int64_t)(uint64_t)lo + (int32_t)(shr<1>((uint32_t)c) & K.lo8);
        c = (int32_t)(d >> 32);
        lo = (uint32_t)d;
    } while (__any(c != 0));
    return top == 0 ? lo : a;
}

}  // namespace row
}  // namespace flm
