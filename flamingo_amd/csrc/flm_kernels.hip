// flm_kernels.hip -- gfx950 (CDNA4) kernels for Flamingo's mask-and-aggregate path.
//
// Reference behaviour (paths relative to the reference root):
//   PRG(seed)[l] = LE32(ChaCha20_DJB(seed, nonce 0^8) word l) ^ 0x64636261
//     -- ChaCha20.new(key=seed, nonce=param.nonce).encrypt(param.fixed_key*L)
//        + np.frombuffer(..,'uint32'): agent/flamingo/SA_ServiceAgent.py:533-536,
//        596-603; agent/flamingo/SA_ClientAgent.py:248-250, 296-298.
//   partial sum        S = sum_i y_i          SA_ServiceAgent.py:346-350
//   self-mask unmask   M = -sum_i PRG(m_i)    SA_ServiceAgent.py:529-536
//   dropout-pair unmask C = sum sigma PRG(s)  SA_ServiceAgent.py:587-603
//   final              out = S + C + M        SA_ServiceAgent.py:538-540, 605
//   client masking     y = x + PRG(m) +- PRG(s_ij)   SA_ClientAgent.py:304-324
//
// Design (MI355X-first):
//   * Integer elementwise work: VALU only, no MFMA.  ChaCha20 is ~59 VALU ops
//     per output word, so regenerating masks is VALU-bound; summing rows is
//     HBM-bound.  One kernel does both so the two overlap inside every wave.
//   * A wave owns a 1024-slot sub-tile.  Masks are generated in "block layout"
//     (lane t computes ChaCha block t: slots 16t..16t+15) and never written to
//     HBM; rows are streamed in "coalesced layout" (lane t loads 16 B at
//     slot 4t + 256j, j = 0..3: every load instruction is 1 KiB contiguous).
//     The two layouts meet once per work item, through LDS.
//   * Signs fold into the XOR constant: -(ks ^ C) = (ks ^ ~C) + 1 mod 2^32, so
//     every seed costs one v_xad_u32 per word and the "+1" per negative seed
//     is added once per slot as a bias (count kept on the device).
//   * Everything of ChaCha's first double round that does not depend on the
//     block counter is computed once per seed (SeedRec), not per block.
//   * 1024-thread workgroups: 16 waves split an item's rows/seeds, partial
//     sums are combined through LDS; tiles shared by several items are
//     combined with u32 atomics (exact: integer adds commute).
#include "flm_internal.h"

namespace flm {

#define FLM_ROTL(v, c) __builtin_rotateleft32((v), (c))
#define FLM_QR(a, b, c, d)                       \
    a += b; d ^= a; d = FLM_ROTL(d, 16);          \
    c += d; b ^= c; b = FLM_ROTL(b, 12);          \
    a += b; d ^= a; d = FLM_ROTL(d, 8);           \
    c += d; b ^= c; b = FLM_ROTL(b, 7);

// Rounds 2..10 as ONE inline-asm statement per half round: the four quarter rounds in lockstep
// (each of the QR's 12 steps issues for all four QRs back to back: 4 adds, 4 xors, 4 rotates,
// ...), and an s_nop after every rotate.  gfx950 issues v_add_u32 / v_xor_b32 in about 2 cycles
// and the v_alignbit_b32 rotate in about 4 (profiles/r01_isa_probe3.log); a wave that issues a
// rotate right behind another rotate, or right before the add that reads it, holds up the SIMD
// for the other waves.  Measured on the c4 mask-only launch (tools/ab/ab_variants.sh,
// profiles/r02_ab_nops.log; 1024 seeds x 2^20 slots, 8 waves/SIMD):
//   one asm statement per instruction (round 1: the compiler then pads each statement boundary
//   where the next reads what the previous wrote with an s_nop 0, i.e. after every group of 4)  1.426 ms
//   one statement, no s_nop                                                                      1.60
//   one statement, s_nop 0 after every group of 4                                                1.394
//   one statement, s_nop 0 after every rotate (and after every group)                            1.297
//   one statement, s_nop 1 after each of the first three rotates, s_nop 2 after the fourth,
//   nothing between the adds and xors (FLM_GAP_* defaults below)                                 1.176
// Gaps between simple ops cost time; gaps after rotates buy it.
#define FLM_GAP_A1 ""  // between the 2nd and 3rd add of a step
#define FLM_GAP_AX ""  // adds -> xors
#define FLM_GAP_X1 ""  // between the 2nd and 3rd xor
#define FLM_GAP_XR ""  // xors -> rotates
#define FLM_GAP_R0 "s_nop 1\n\t"  // after the 1st rotate
#define FLM_GAP_R1 "s_nop 1\n\t"  // after the 2nd rotate
#define FLM_GAP_R2 "s_nop 1\n\t"  // after the 3rd rotate
#define FLM_GAP_RA "s_nop 2\n\t"  // after the 4th rotate, before the adds that read them
#define FLM_S_A(a, b) "v_add_u32 %[" #a "], %[" #b "], %[" #a "]\n\t"
#define FLM_S_X(a, b) "v_xor_b32 %[" #a "], %[" #b "], %[" #a "]\n\t"
#define FLM_S_R(a, s) "v_alignbit_b32 %[" #a "], %[" #a "], %[" #a "], " #s "\n\t"  // rotl(a, 32 - s)
// one QR step for QRs 0..3: a += b; d ^= a; d = rotl(d, 32 - s)
#define FLM_S_STEP(a, b, c, d, s)                                                                       \
    FLM_S_A(a##0, b##0) FLM_S_A(a##1, b##1) FLM_GAP_A1 FLM_S_A(a##2, b##2) FLM_S_A(a##3, b##3) FLM_GAP_AX \
    FLM_S_X(d##0, a##0) FLM_S_X(d##1, a##1) FLM_GAP_X1 FLM_S_X(d##2, a##2) FLM_S_X(d##3, a##3) FLM_GAP_XR \
    FLM_S_R(d##0, s) FLM_GAP_R0 FLM_S_R(d##1, s) FLM_GAP_R1 FLM_S_R(d##2, s) FLM_GAP_R2 FLM_S_R(d##3, s)  \
    FLM_GAP_RA
// QR(a_i, b_i, c_i, d_i) for i = 0..3: steps (a,b,d,16) (c,d,b,12) (a,b,d,8) (c,d,b,7)
#define FLM_QR4(A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3)                   \
    asm volatile(FLM_S_STEP(a, b, c, d, 16) FLM_S_STEP(c, d, a, b, 20) FLM_S_STEP(a, b, c, d, 24)  \
                 FLM_S_STEP(c, d, a, b, 25)                                                     \
                 : [a0] "+v"(A0), [b0] "+v"(B0), [c0] "+v"(C0), [d0] "+v"(D0), [a1] "+v"(A1),   \
                   [b1] "+v"(B1), [c1] "+v"(C1), [d1] "+v"(D1), [a2] "+v"(A2), [b2] "+v"(B2),   \
                   [c2] "+v"(C2), [d2] "+v"(D2), [a3] "+v"(A3), [b3] "+v"(B3), [c3] "+v"(C3),   \
                   [d3] "+v"(D3))

// ------------------------------------------------------------------ seeds
// One thread per seed builds its SeedRec from the raw 32 seed bytes and sign.
// Workgroup p writes its count of negative / invalid signs to meta[2+2p],
// meta[3+2p] and meta[0] = number of workgroups, so no zeroing pass is needed.
// zero_out/zero_n: when the round's plan adds into its output with atomics, the same
// launch zero-fills it (grid-stride, 16-B stores) -- one submission fewer than a memset.
__global__ __launch_bounds__(256) void seed_schedule_kernel(const uint8_t *__restrict__ seeds,
                                                            const int8_t *__restrict__ signs, int K,
                                                            SeedRec *__restrict__ recs,
                                                            uint32_t *__restrict__ meta,
                                                            uint32_t *__restrict__ zero_out, uint64_t zero_n) {
    if (zero_out) {
        const uint64_t quads = zero_n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
        for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < quads; q += stride)
            reinterpret_cast<uint4 *>(zero_out)[q] = make_uint4(0u, 0u, 0u, 0u);
        const uint64_t t = 4 * quads + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (t < zero_n) zero_out[t] = 0u;
    }
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t neg = 0, bad = 0;
    if (k < K) {
        const uint8_t *p = seeds + 32 * (size_t)k;
        uint32_t key[8];
        if (((uintptr_t)seeds & 15) == 0) {
            const uint4 a = reinterpret_cast<const uint4 *>(p)[0], b = reinterpret_cast<const uint4 *>(p)[1];
            key[0] = a.x; key[1] = a.y; key[2] = a.z; key[3] = a.w;
            key[4] = b.x; key[5] = b.y; key[6] = b.z; key[7] = b.w;
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                key[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
                         ((uint32_t)p[4 * i + 3] << 24);
        }
        const int sg = signs[k];
        neg = (sg < 0);
        bad = (sg != 1 && sg != -1);
        SeedRec r;
#pragma unroll
        for (int i = 0; i < 8; ++i) r.k[i] = key[i];
        r.xorc = sg < 0 ? ~kAbcd : kAbcd;
        r.a0 = kSigma0 + key[0];
        uint32_t x1 = kSigma1, x5 = key[1], x9 = key[5], x13 = 0u;
        uint32_t x2 = kSigma2, x6 = key[2], x10 = key[6], x14 = 0u;
        uint32_t x3 = kSigma3, x7 = key[3], x11 = key[7], x15 = 0u;
        FLM_QR(x1, x5, x9, x13);
        FLM_QR(x2, x6, x10, x14);
        FLM_QR(x3, x7, x11, x15);
        r.col1[0] = x1; r.col1[1] = x5; r.col1[2] = x9; r.col1[3] = x13;
        r.col2[0] = x2; r.col2[1] = x6; r.col2[2] = x10; r.col2[3] = x14;
        r.col3[0] = x3; r.col3[1] = x7; r.col3[2] = x11; r.col3[3] = x15;
#pragma unroll
        for (int i = 0; i < 10; ++i) r.pad[i] = 0;
        recs[k] = r;
    }
    // workgroup totals (64-lane ballots, then 4 waves through LDS)
    __shared__ uint32_t s_cnt[2][4];
    const unsigned long long bn = __ballot(neg != 0), bb = __ballot(bad != 0);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_cnt[0][w] = __popcll(bn); s_cnt[1][w] = __popcll(bb); }
    __syncthreads();
    if (threadIdx.x == 0) {
        meta[2 + 2 * blockIdx.x] = s_cnt[0][0] + s_cnt[0][1] + s_cnt[0][2] + s_cnt[0][3];
        meta[3 + 2 * blockIdx.x] = s_cnt[1][0] + s_cnt[1][1] + s_cnt[1][2] + s_cnt[1][3];
        if (blockIdx.x == 0) meta[0] = gridDim.x;
    }
}

// Total negative signs of the current seed table (sum of the per-workgroup counts).
__device__ __forceinline__ uint32_t meta_nneg(const uint32_t *__restrict__ meta) {
    const uint32_t parts = meta[0];
    uint32_t n = 0;
    for (uint32_t p = 0; p < parts; ++p) n += meta[2 + 2 * p];
    return n;
}

// -------------------------------------------------------------- ChaCha core
// m[i] += ChaCha20_block(seed, ctr)[i] ^ xorc for the 16 words of block `ctr`.
// `rec` is wave-uniform (scalar loads); `ctr` is per lane.
__device__ __forceinline__ void chacha_mask_add(const SeedRec *__restrict__ rec, uint32_t ctr,
                                                uint32_t (&m)[16]) {
    const uint32_t k0 = rec->k[0], k1 = rec->k[1], k2 = rec->k[2], k3 = rec->k[3];
    const uint32_t k4 = rec->k[4], k5 = rec->k[5], k6 = rec->k[6], k7 = rec->k[7];
    const uint32_t xc = rec->xorc;
    uint32_t x0, x1, x2, x3, x4, x5, x6, x7, x8, x9, x10, x11, x12, x13, x14, x15;
    // round 1, column QR(0,4,8,12): a = sigma0 + k0 precomputed
    x0 = rec->a0;
    x12 = FLM_ROTL(ctr ^ x0, 16);
    x8 = k4 + x12;
    x4 = FLM_ROTL(k0 ^ x8, 12);
    x0 += x4;
    x12 = FLM_ROTL(x12 ^ x0, 8);
    x8 += x12;
    x4 = FLM_ROTL(x4 ^ x8, 7);
    // round 1, columns 1..3: counter independent
    x1 = rec->col1[0]; x5 = rec->col1[1]; x9 = rec->col1[2]; x13 = rec->col1[3];
    x2 = rec->col2[0]; x6 = rec->col2[1]; x10 = rec->col2[2]; x14 = rec->col2[3];
    x3 = rec->col3[0]; x7 = rec->col3[1]; x11 = rec->col3[2]; x15 = rec->col3[3];
    // round 1, diagonals
    // the whole diagonal round in lockstep, like rounds 2..10: 0.8 % faster than the compiler's order
    // with the first steps of QR(1,6,11,12) and QR(2,7,8,13) hoisted into SeedRec
    // (profiles/r02_ab_round1.log)
    FLM_QR4(x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
    // rounds 2..10
#pragma unroll
    for (int r = 0; r < 9; ++r) {
        FLM_QR4(x0, x4, x8, x12, x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15);
        FLM_QR4(x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
    }
    // feed-forward (input words 13..15 are zero), fold "abcd"/sign, accumulate
    m[0] += (x0 + kSigma0) ^ xc;
    m[1] += (x1 + kSigma1) ^ xc;
    m[2] += (x2 + kSigma2) ^ xc;
    m[3] += (x3 + kSigma3) ^ xc;
    m[4] += (x4 + k0) ^ xc;
    m[5] += (x5 + k1) ^ xc;
    m[6] += (x6 + k2) ^ xc;
    m[7] += (x7 + k3) ^ xc;
    m[8] += (x8 + k4) ^ xc;
    m[9] += (x9 + k5) ^ xc;
    m[10] += (x10 + k6) ^ xc;
    m[11] += (x11 + k7) ^ xc;
    m[12] += (x12 + ctr) ^ xc;
    m[13] += x13 ^ xc;
    m[14] += x14 ^ xc;
    m[15] += x15 ^ xc;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Load the wave's 4 KiB of one row in coalesced layout through a buffer
// descriptor whose range ends at the tile's last valid quad: quads past it
// (tail tile) come back as zero from the hardware range check, no branches.
// BL = block layout: lane t loads its own 64 B (slots 16t..16t+15), the layout
// the ChaCha block is generated in; otherwise coalesced layout (slot 4t + 256j).
// AUX = buffer cache-policy bits (0 default, 2 = nt: streamed once, MI355X_MICROARCH.md nt-weights).
template <bool BL, int AUX = 0>
__device__ __forceinline__ void load_row(const uint32_t *base, uint32_t bytes, int lane, u32x4 (&v)[4]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(base), 0,
                                                                        (int)bytes, 0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, BL ? 64 * lane + 16 * j : 16 * lane + 1024 * j, 0, AUX));
}

// Sum the Cw chunk partials of every sub-tile from LDS and write the tile.
template <int S>
__device__ __forceinline__ void reduce_out(const u32x4 *__restrict__ lds, uint32_t *__restrict__ out,
                                           uint64_t base, int valid, uint32_t bias, bool atomic) {
    constexpr int Cw = kWavesPerGroup / S;
    if (!atomic) {
        for (int q = threadIdx.x; q < S * 256; q += kThreads) {
            const int s = q >> 8, p = q & 255;
            u32x4 acc = u32x4(bias);
#pragma unroll
            for (int c = 0; c < Cw; ++c) acc = acc + lds[(s + S * c) * 256 + p];
            const int slot = s * kWaveSlots + 4 * p;
            uint32_t *dst = out + base + slot;
            if (slot + 3 < valid) {
                *reinterpret_cast<u32x4 *>(dst) = acc;
            } else {
                if (slot + 0 < valid) dst[0] = acc.x;
                if (slot + 1 < valid) dst[1] = acc.y;
                if (slot + 2 < valid) dst[2] = acc.z;
            }
        }
    } else {
        const uint32_t *l32 = reinterpret_cast<const uint32_t *>(lds);
        for (int d = threadIdx.x; d < S * kWaveSlots; d += kThreads) {
            const int s = d >> 10, o = d & 1023;
            uint32_t acc = bias;
#pragma unroll
            for (int c = 0; c < Cw; ++c) acc += l32[(s + S * c) * 1024 + o];
            const int slot = s * kWaveSlots + o;
            if (slot < valid) atomicAdd(out + base + slot, acc);
        }
    }
}

// --------------------------------------------------------------- main kernel
// One workgroup = one Item.  Wave w works on sub-tile s = w % S with chunk
// c = w / S of the item's rows and seeds (Cw = 16 / S chunks).
//   BL      rows are loaded in block layout (lane t: slots 16t..16t+15), the
//           layout the ChaCha blocks come out in; else coalesced layout.
//   MERGED  every item writes one tile (same-tile, rows-only or mask-only), so
//           rows are added straight into the mask accumulator (needs BL): one
//           16-register accumulator instead of two, no transpose.
//   WPE     minimum waves per SIMD requested from the register allocator.
template <int S, bool BL, bool MERGED, int WPE, int RUM = 2, int AUX = 0, bool SPREAD = false>
__global__ __launch_bounds__(kThreads, WPE) void items_kernel(const Item *__restrict__ items,
                                                              const uint32_t *__restrict__ rows,
                                                              uint64_t row_pitch,
                                                              const SeedRec *__restrict__ recs,
                                                              const uint32_t *__restrict__ meta,
                                                              uint32_t *__restrict__ out) {
    static_assert(!MERGED || BL, "merged accumulation needs block-layout rows");
    constexpr int Cw = kWavesPerGroup / S;
    constexpr int RU = MERGED ? RUM : 4;  // rows in flight per wave in the rows-only loop
    __shared__ u32x4 lds[kWavesPerGroup * 256];  // 64 KiB: one 4 KiB region per wave
    __shared__ uint32_t claim[S];                 // next unclaimed unit of each sub-tile

    const Item it = items[blockIdx.x];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int s = w % S, c = w / S;
    if constexpr (!SPREAD && Cw > 1) {
        if (threadIdx.x < S) claim[threadIdx.x] = 0u;
        __syncthreads();
    }
    const uint32_t flags = it.flags;
    const bool has_rows = flags & kHasRows, has_mask = flags & kHasMask;

    u32x4 racc[4] = {u32x4(0u), u32x4(0u), u32x4(0u), u32x4(0u)};  // unused when MERGED
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = 0;

    // this wave's share of rows and seeds
    uint32_t nr = 0, ns = 0, r0 = 0, q0 = 0;
    if (has_rows) {
        r0 = (uint32_t)(((uint64_t)it.nrows * c) / Cw);
        nr = (uint32_t)(((uint64_t)it.nrows * (c + 1)) / Cw) - r0;
    }
    if (has_mask) {
        q0 = it.k0 + (uint32_t)(((uint64_t)it.nseeds * c) / Cw);
        ns = it.k0 + (uint32_t)(((uint64_t)it.nseeds * (c + 1)) / Cw) - q0;
    }
    const int sub_slot = s * kWaveSlots;
    const int row_valid = (int)it.row_valid - sub_slot;   // may be <= 0: nothing valid
    // bytes of this sub-tile a row load may touch: whole quads up to the last valid slot
    const uint32_t row_bytes =
        row_valid >= kWaveSlots ? 4u * kWaveSlots : (row_valid > 0 ? 16u * (uint32_t)((row_valid + 3) / 4) : 0u);
    const uint32_t *rp = rows + it.row_in + (uint64_t)r0 * row_pitch + sub_slot;
    const uint32_t ctr = (uint32_t)(it.mask_ctr + (uint64_t)(sub_slot / 16) + (uint64_t)lane);
    const SeedRec *rec = recs + q0;
    if (row_valid <= 0) nr = 0;

    auto add_row = [&](const u32x4 (&v)[4]) {
        if constexpr (MERGED) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                m[4 * j + 0] += v[j].x; m[4 * j + 1] += v[j].y; m[4 * j + 2] += v[j].z; m[4 * j + 3] += v[j].w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) racc[j] = racc[j] + v[j];
        }
    };

    if constexpr (SPREAD) {
        // seeds spread evenly over the row stream (Bresenham): every row load is
        // issued before the ChaCha block that hides it, and seed-light items keep
        // HBM busy from the first row instead of front-loading the VALU work
        uint32_t q = 0;
        for (uint32_t r = 0; r < nr; ++r) {
            u32x4 v[4];
            load_row<BL, AUX>(rp, row_bytes, lane, v);
            if (q < ns && (uint64_t)q * nr <= (uint64_t)r * ns) {
                chacha_mask_add(rec, ctr, m);
                ++rec;
                ++q;
            }
            add_row(v);
            rp += row_pitch;
        }
        for (; q < ns; ++q) {
            chacha_mask_add(rec, ctr, m);
            ++rec;
        }
    } else if constexpr (Cw > 1) {
        // Units claimed from a per-sub-tile LDS counter: unit i = seed i of the item, plus row i
        // when there is one.  With a static split (64 seeds per wave at c4) the SIMD's arbiter
        // lets some waves run far ahead, and a workgroup waited at its barrier for its slowest
        // wave: 0.33-0.62 ms workgroup times, wave 0 idle ~0.2 ms of them, 87 % mean residency
        // (tools/probes/wg_trace.py, profiles/r02_wg_trace.log).  Claiming, a fast wave takes more
        // units and the waves of a workgroup finish within about one block of each other.
        // Any split gives the same bits: the partials are summed mod 2^32.
        const uint32_t NR = (has_rows && row_valid > 0) ? it.nrows : 0u;
        const uint32_t NS = has_mask ? it.nseeds : 0u;
        const uint32_t *rb = rows + it.row_in + sub_slot;
        // one lane adds 1 to the counter; in asm so that the compiler's atomic optimizer does not
        // wrap it in a wave reduction (mbcnt/bcnt/readfirstlane: ~8 VALU per unit)
        const uint32_t caddr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)&claim[s];
        auto next = [&]() -> uint32_t {
            uint32_t v = 0;
            if (lane == 0)
                asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(caddr), "v"(1u) : "memory");
            return __builtin_amdgcn_readlane(v, 0);
        };
        // two loops, one body each: a single loop with a row / no-row branch made the compiler
        // copy the 16 accumulators at every unit
        const uint32_t NP = NR < NS ? NR : NS;
        uint32_t i = next();
        for (; i < NP; i = next()) {
            u32x4 v4[4];
            load_row<BL, AUX>(rb + (uint64_t)i * row_pitch, row_bytes, lane, v4);
            chacha_mask_add(recs + it.k0 + i, ctr, m);
            add_row(v4);
        }
        for (; i < NS; i = next()) chacha_mask_add(recs + it.k0 + i, ctr, m);
        // rows past the last seed (seed-light items): the static split, RU rows in flight
        if (NR > NS) {
            const uint32_t a = NS + (uint32_t)(((uint64_t)(NR - NS) * c) / Cw);
            const uint32_t b = NS + (uint32_t)(((uint64_t)(NR - NS) * (c + 1)) / Cw);
            const uint32_t *rq = rb + (uint64_t)a * row_pitch;
            uint32_t rr = b - a;
            for (; rr >= RU; rr -= RU) {
                u32x4 v4[RU][4];
#pragma unroll
                for (int u = 0; u < RU; ++u) load_row<BL, AUX>(rq + u * row_pitch, row_bytes, lane, v4[u]);
#pragma unroll
                for (int u = 0; u < RU; ++u) add_row(v4[u]);
                rq += RU * row_pitch;
            }
            for (; rr > 0; --rr) {
                u32x4 v4[4];
                load_row<BL, AUX>(rq, row_bytes, lane, v4);
                add_row(v4);
                rq += row_pitch;
            }
        }
    } else {
        // paired phase: one row load in flight under one ChaCha block per step
        const uint32_t np = nr < ns ? nr : ns;
        for (uint32_t q = 0; q < np; ++q) {
            u32x4 v[4];
            load_row<BL, AUX>(rp, row_bytes, lane, v);
            chacha_mask_add(rec, ctr, m);
            add_row(v);
            rp += row_pitch;
            ++rec;
        }
        // remaining rows: RU rows (RU x 4 KiB per wave) in flight
        uint32_t rr = nr - np;
        for (; rr >= RU; rr -= RU) {
            u32x4 v[RU][4];
#pragma unroll
            for (int u = 0; u < RU; ++u) load_row<BL, AUX>(rp + u * row_pitch, row_bytes, lane, v[u]);
#pragma unroll
            for (int u = 0; u < RU; ++u) add_row(v[u]);
            rp += RU * row_pitch;
        }
        for (; rr > 0; --rr) {
            u32x4 v[4];
            load_row<BL, AUX>(rp, row_bytes, lane, v);
            add_row(v);
            rp += row_pitch;
        }
        // remaining seeds
        for (uint32_t q = np; q < ns; ++q) {
            chacha_mask_add(rec, ctr, m);
            ++rec;
        }
    }

    // ---- combine through this wave's LDS region (natural slot order), then
    // sum the Cw chunk partials of every sub-tile and write the tile.
    u32x4 *R = lds + w * 256;
    const uint32_t mbias = it.mask_bias + ((flags & kMaskBiasNneg) ? meta_nneg(meta) : 0u);
    if constexpr (MERGED) {
        R[4 * lane + 0] = u32x4{m[0], m[1], m[2], m[3]};
        R[4 * lane + 1] = u32x4{m[4], m[5], m[6], m[7]};
        R[4 * lane + 2] = u32x4{m[8], m[9], m[10], m[11]};
        R[4 * lane + 3] = u32x4{m[12], m[13], m[14], m[15]};
        __syncthreads();
        const uint64_t base = has_mask ? it.mask_out : it.row_out;
        const int valid = has_mask ? (int)it.mask_valid : (int)it.row_valid;
        const uint32_t bias = (has_rows ? it.row_bias : 0u) + (has_mask ? mbias : 0u);
        reduce_out<S>(lds, out, base, valid, bias, (flags & (kRowAtomic | kMaskAtomic)) != 0);
    } else {
        const bool same = flags & kSameTile;
        u32x4 mq[4];
        if (has_mask) {
            if (BL) {
                mq[0] = u32x4{m[0], m[1], m[2], m[3]};
                mq[1] = u32x4{m[4], m[5], m[6], m[7]};
                mq[2] = u32x4{m[8], m[9], m[10], m[11]};
                mq[3] = u32x4{m[12], m[13], m[14], m[15]};
            } else {  // block layout -> coalesced layout
                R[4 * lane + 0] = u32x4{m[0], m[1], m[2], m[3]};
                R[4 * lane + 1] = u32x4{m[4], m[5], m[6], m[7]};
                R[4 * lane + 2] = u32x4{m[8], m[9], m[10], m[11]};
                R[4 * lane + 3] = u32x4{m[12], m[13], m[14], m[15]};
                __syncthreads();
#pragma unroll
                for (int j = 0; j < 4; ++j) mq[j] = R[lane + 64 * j];
            }
            if (same) {
#pragma unroll
                for (int j = 0; j < 4; ++j) racc[j] = racc[j] + mq[j];
            }
        }
        // LDS quad index of accumulator quad j of this lane (natural slot order)
#define FLM_RQ(j) (BL ? 4 * lane + (j) : lane + 64 * (j))
        if (has_rows || same) {
#pragma unroll
            for (int j = 0; j < 4; ++j) R[FLM_RQ(j)] = racc[j];
            __syncthreads();
            const uint64_t base = same ? it.mask_out : it.row_out;
            const int valid = same ? (int)it.mask_valid : (int)it.row_valid;
            const uint32_t bias = it.row_bias + (same ? mbias : 0u);
            const bool atom = same ? ((flags & (kRowAtomic | kMaskAtomic)) != 0) : ((flags & kRowAtomic) != 0);
            reduce_out<S>(lds, out, base, valid, bias, atom);
        }
        if (has_mask && !same) {
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j) R[FLM_RQ(j)] = mq[j];
            __syncthreads();
            reduce_out<S>(lds, out, it.mask_out, (int)it.mask_valid, mbias, (flags & kMaskAtomic) != 0);
        }
#undef FLM_RQ
    }
}

// ------------------------------------------------------- small-round kernel
// The whole round in ONE launch for rounds too small to fill the chip through items_kernel
// (BASELINE c2: N=128 rows, K=128 seeds, L=16384).  There, items_kernel's 1024-thread
// workgroups land on half the CUs, and the seed-schedule launch before it adds its own gap
// (13 us per round measured; ~3 us of ChaCha work).  Here a 256-thread workgroup owns
// T = 16*B output slots outright.  It sums every row over them and adds every seed's mask,
// then stores the tile once: no atomics, no zero-fill, no seed table.
//   lane (b, sl) of wave w: ChaCha block b of the tile for seed s = pass*4*(64/B) + w*(64/B) + sl,
//   keys read straight from the raw 32-byte seeds (no SeedRec precompute: its saving is ~5 %
//   of a block and would cost the extra launch).
//   Rows: thread (quad q, group rg) sums rows rg, rg + RG, ... of quad q with 16-B loads,
//   issued before the ChaCha work so HBM latency hides under it.
//   Combine: lane accumulators and row partials through LDS, 16 entries per thread, then
//   one store per slot.
// Block 0 also writes the sign counts to meta (meta[0] = 1 part) as seed_schedule_kernel does,
// so flm_check_signs keeps working.
// SEG (client masking, SA_ClientAgent.py:304-324): blockIdx.y is output row i; its seeds are
// [seg[i], seg[i+1]), its input is row i of `rows` (none: the all-ones input, `bias` = 1), and
// the row is written at out + i*pitch.  No sign counts (the host validated the signs).
template <int B, bool SEG = false>
__global__ __launch_bounds__(256) void small_round_kernel(const uint32_t *__restrict__ rows, uint64_t pitch, int N,
                                                          const uint8_t *__restrict__ seeds,
                                                          const int8_t *__restrict__ signs, int K, uint64_t L,
                                                          uint64_t mask_lo, uint64_t mask_hi, uint32_t ctr0,
                                                          uint32_t *__restrict__ out, uint32_t *__restrict__ meta,
                                                          const int64_t *__restrict__ seg = nullptr,
                                                          uint32_t bias = 0u) {
    constexpr int T = 16 * B;     // slots per workgroup
    constexpr int SPW = 64 / B;   // seeds per wave per pass
    constexpr int SPP = 4 * SPW;  // seeds per pass
    constexpr int Q = T / 4;      // 16-B quads per row tile
    constexpr int RG = 256 / Q;   // row groups
    constexpr int G = 256 / T;    // slot groups of the combine
    constexpr int RB = 4;         // rows per thread in flight under the ChaCha work
    __shared__ __attribute__((aligned(16))) uint32_t lm[256 * 16];  // lane accumulators, 16 KiB
    __shared__ __attribute__((aligned(16))) uint32_t lr[RG * T];    // row partials
    __shared__ uint32_t lp[G * T];                                  // per-group slot partials (256 words)

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t slot0 = (uint64_t)blockIdx.x * T;
    int k_lo = 0, k_hi = K;
    if constexpr (SEG) {
        const uint64_t y = blockIdx.y;
        k_lo = (int)seg[y];
        k_hi = (int)seg[y + 1];
        N = rows ? 1 : 0;
        if (rows) rows += y * pitch;
        out += y * pitch;
    }

    // ---- rows: the first RB of this thread's rows are loaded before the masks
    const int q = tid % Q, rg = tid / Q;
    const uint64_t qslot = slot0 + 4 * (uint64_t)q;
    const bool qok = qslot < L;  // a quad straddling L stays inside the row (pitch >= round_up(L, 4))
    const uint32_t *rq = rows + qslot;
    u32x4 racc = u32x4(0u), rv[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
        const int r = rg + u * RG;
        rv[u] = (qok && r < N) ? *reinterpret_cast<const u32x4 *>(rq + (uint64_t)r * pitch) : u32x4(0u);
    }

    // ---- masks: one ChaCha block per lane per pass
    uint32_t acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0;
    uint32_t nneg = 0;
    const int b = lane % B, sl = lane / B;
    const uint64_t bslot = slot0 + 16 * (uint64_t)b;
    if (bslot >= mask_lo && bslot < mask_hi) {
        const uint32_t ctr = ctr0 + (uint32_t)(bslot / 16);
        const bool al16 = ((uintptr_t)seeds & 15) == 0;
        for (int s = k_lo + w * SPW + sl; s < k_hi; s += SPP) {
            const uint8_t *p = seeds + 32 * (size_t)s;
            uint32_t k[8];
            if (al16) {
                const uint4 a0 = reinterpret_cast<const uint4 *>(p)[0], a1 = reinterpret_cast<const uint4 *>(p)[1];
                k[0] = a0.x; k[1] = a0.y; k[2] = a0.z; k[3] = a0.w;
                k[4] = a1.x; k[5] = a1.y; k[6] = a1.z; k[7] = a1.w;
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    k[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
                           ((uint32_t)p[4 * i + 3] << 24);
            }
            const bool neg = signs[s] < 0;
            const uint32_t xc = neg ? ~kAbcd : kAbcd;  // -(ks ^ C) = (ks ^ ~C) + 1
            nneg += neg ? 1u : 0u;
            uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
            uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
            uint32_t x12 = ctr, x13 = 0u, x14 = 0u, x15 = 0u;
            if constexpr (SEG) {
                // client masking: throughput-bound, the tuned lockstep rounds (FLM_QR4)
#pragma unroll
                for (int r = 0; r < 10; ++r) {
                    FLM_QR4(x0, x4, x8, x12, x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15);
                    FLM_QR4(x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
                }
            } else {
                // a small round (c2) is one block per lane on a latency path: the s_nop gaps of
                // FLM_QR4 only lengthen it (7.4 -> 9.4 us per c2 round), so the compiler's order
#pragma unroll
                for (int r = 0; r < 10; ++r) {
                    FLM_QR(x0, x4, x8, x12);
                    FLM_QR(x1, x5, x9, x13);
                    FLM_QR(x2, x6, x10, x14);
                    FLM_QR(x3, x7, x11, x15);
                    FLM_QR(x0, x5, x10, x15);
                    FLM_QR(x1, x6, x11, x12);
                    FLM_QR(x2, x7, x8, x13);
                    FLM_QR(x3, x4, x9, x14);
                }
            }
            acc[0] += (x0 + kSigma0) ^ xc;
            acc[1] += (x1 + kSigma1) ^ xc;
            acc[2] += (x2 + kSigma2) ^ xc;
            acc[3] += (x3 + kSigma3) ^ xc;
            acc[4] += (x4 + k[0]) ^ xc;
            acc[5] += (x5 + k[1]) ^ xc;
            acc[6] += (x6 + k[2]) ^ xc;
            acc[7] += (x7 + k[3]) ^ xc;
            acc[8] += (x8 + k[4]) ^ xc;
            acc[9] += (x9 + k[5]) ^ xc;
            acc[10] += (x10 + k[6]) ^ xc;
            acc[11] += (x11 + k[7]) ^ xc;
            acc[12] += (x12 + ctr) ^ xc;
            acc[13] += x13 ^ xc;
            acc[14] += x14 ^ xc;
            acc[15] += x15 ^ xc;
        }
    }

    // ---- rows: add the first batch, stream the rest
#pragma unroll
    for (int u = 0; u < RB; ++u) racc = racc + rv[u];
    if (qok)
        for (int r = rg + RB * RG; r < N; r += RG) racc = racc + *reinterpret_cast<const u32x4 *>(rq + (uint64_t)r * pitch);

    // ---- combine
    u32x4 *lm4 = reinterpret_cast<u32x4 *>(lm) + 4 * tid;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        lm4[j] = u32x4{acc[4 * j] + nneg, acc[4 * j + 1] + nneg, acc[4 * j + 2] + nneg, acc[4 * j + 3] + nneg};
    *reinterpret_cast<u32x4 *>(lr + rg * T + 4 * q) = racc;
    __syncthreads();
    {
        const int j = tid % T, g = tid / T;
        const int jb = j / 16, jw = j % 16;
        uint32_t sum = 0;
#pragma unroll
        for (int e = g * 16; e < g * 16 + 16; ++e) {  // 16 of the 256/B (wave, seed-lane) entries of slot j
            const int wv = e / SPW, sle = e % SPW;
            sum += lm[(wv * 64 + sle * B + jb) * 16 + jw];
        }
#pragma unroll
        for (int r = g; r < RG; r += G) sum += lr[r * T + j];
        lp[g * T + j] = sum;
    }
    __syncthreads();
    if (tid < T) {
        uint32_t total = bias;
#pragma unroll
        for (int g = 0; g < G; ++g) total += lp[g * T + tid];
        if (slot0 + tid < L) out[slot0 + tid] = total;
    }

    // ---- sign counts (block 0), the same meta layout as seed_schedule_kernel with one part
    if (!SEG && blockIdx.x == 0) {
        uint32_t n = 0, bad = 0;
        for (int s = tid; s < K; s += 256) {
            const int sg = signs[s];
            n += sg < 0 ? 1u : 0u;
            bad += (sg != 1 && sg != -1) ? 1u : 0u;
        }
        __syncthreads();  // lp is free again
        lp[tid] = n;
        lm[tid] = bad;
        __syncthreads();
        if (tid == 0) {
            uint32_t tn = 0, tb = 0;
            for (int i = 0; i < 256; ++i) { tn += lp[i]; tb += lm[i]; }
            meta[0] = 1u;
            meta[2] = tn;
            meta[3] = tb;
        }
    }
}

// --------------------------------------------------- byte keystream (host PRF)
// out = in ^ ChaCha20(key, nonce) from block `counter`, one block per thread.
__global__ __launch_bounds__(256) void chacha20_xor_kernel(uint32_t k0, uint32_t k1, uint32_t k2,
                                                           uint32_t k3, uint32_t k4, uint32_t k5,
                                                           uint32_t k6, uint32_t k7, uint32_t n0,
                                                           uint32_t n1, uint64_t counter,
                                                           const uint8_t *__restrict__ in,
                                                           uint8_t *__restrict__ out, uint64_t n) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t off = b * 64;
    if (off >= n) return;
    const uint64_t blk = counter + b;
    uint32_t x0 = kSigma0, x1 = kSigma1, x2 = kSigma2, x3 = kSigma3;
    uint32_t x4 = k0, x5 = k1, x6 = k2, x7 = k3, x8 = k4, x9 = k5, x10 = k6, x11 = k7;
    uint32_t x12 = (uint32_t)blk, x13 = (uint32_t)(blk >> 32), x14 = n0, x15 = n1;
    const uint32_t i12 = x12, i13 = x13;
    for (int r = 0; r < 10; ++r) {
        FLM_QR4(x0, x4, x8, x12, x1, x5, x9, x13, x2, x6, x10, x14, x3, x7, x11, x15);
        FLM_QR4(x0, x5, x10, x15, x1, x6, x11, x12, x2, x7, x8, x13, x3, x4, x9, x14);
    }
    const uint32_t ks[16] = {x0 + kSigma0, x1 + kSigma1, x2 + kSigma2, x3 + kSigma3,
                             x4 + k0,      x5 + k1,      x6 + k2,      x7 + k3,
                             x8 + k4,      x9 + k5,      x10 + k6,     x11 + k7,
                             x12 + i12,    x13 + i13,    x14 + n0,     x15 + n1};
    const uint64_t m = (n - off) < 64 ? (n - off) : 64;
    for (uint64_t i = 0; i < m; ++i) out[off + i] = in[off + i] ^ (uint8_t)(ks[i >> 2] >> (8 * (i & 3)));
}

// ------------------------------------------------------- pair-mask work queue
// The dropout-pair masks of the CU-split reconstruction (reconstruct.py, pair_queue=True;
// SA_ServiceAgent.py:587-603) cut into units of (1024-slot tile, kUnitSeeds seeds), claimed
// from a counter so that two launches on different CU sets share them without a fixed split:
//   SIDE  (the EC CUs, once the combine is done): claims units until ws[1] (set on the
//         self-mask stream by flag_set_kernel when that pass ends) reads non-zero;
//   FINAL (all CUs, after both streams): claims the rest.
// A claimed unit is always finished, so every unit is added exactly once whatever the timing:
// the flag only moves the split.  No wave ever waits on the flag (it is read between units),
// so both grids drain on their own.  One wave per workgroup: the LDS transpose needs only a
// wave-local barrier, and waves that stop at different units never wait for each other.
// Units are chunk-major (consecutive claims hit different tiles); each lane makes ChaCha
// block `tile*64 + lane`, the 16 words go through LDS so that every u32 atomic add of the
// wave covers 64 consecutive slots.
constexpr int kUnitSeeds = 16;  // 32 and 64 measured the same at c5 (profiles/r02_ab_pair_units.log)

template <bool SIDE>
__global__ __launch_bounds__(64) void pair_units_kernel(const SeedRec *__restrict__ recs, int K,
                                                        uint32_t *__restrict__ dst, uint64_t L,
                                                        uint32_t n_tiles, uint32_t n_units,
                                                        uint32_t *__restrict__ ws) {
    __shared__ uint32_t lds[64 * 17];
    const int lane = threadIdx.x;
    for (;;) {
        uint32_t u = 0;
        if (lane == 0) {
            u = n_units;  // "stop"
            if (!SIDE || __hip_atomic_load(&ws[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
                u = __hip_atomic_fetch_add(&ws[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        u = __builtin_amdgcn_readfirstlane(__shfl(u, 0));
        if (u >= n_units) break;
        const uint32_t tile = u % n_tiles, chunk = u / n_tiles;
        const int k0 = (int)chunk * kUnitSeeds;
        const int k1 = min(K, k0 + kUnitSeeds);
        uint32_t m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = 0u;
        uint32_t nneg = 0;
        const uint32_t ctr = tile * 64u + (uint32_t)lane;
        for (int k = k0; k < k1; ++k) {
            chacha_mask_add(&recs[k], ctr, m);
            nneg += (recs[k].xorc != kAbcd);
        }
        __syncthreads();  // the previous unit's reads of lds are done
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[lane * 17 + i] = m[i] + nneg;
        __syncthreads();
        // one address per lane, the 16 stores at immediate offsets j * 256 B; the tile's valid
        // slot count bounds them (full tiles: all 1024)
        const uint64_t base = (uint64_t)tile * 1024u;
        const uint32_t valid = (uint32_t)min<uint64_t>(1024u, L - base);
        // slot e = j*64 + lane sits at lds[(e >> 4) * 17 + (e & 15)] = lds[lb + 68 j]
        uint32_t *p = dst + base + lane;
        const uint32_t lb = (uint32_t)(lane >> 4) * 17u + (uint32_t)(lane & 15);
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if ((uint32_t)(j * 64 + lane) < valid)
                __hip_atomic_fetch_add(p + j * 64, lds[lb + 68 * j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ws[1] = 1 once every earlier launch on this stream has finished (release, device scope).
__global__ void flag_set_kernel(uint32_t *__restrict__ ws) {
    if (threadIdx.x == 0) __hip_atomic_store(&ws[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- mask expansion
// Standalone PRG expansion (north_star (i); the cancel_vec idiom of SA_ServiceAgent.py:596-603 and
// SA_ClientAgent.py:248-250 for a whole batch of seeds): out[k * pitch + l] = PRG(seed k)[slot0 + l]
// for l < L.  A unit is (seed k, 1024-slot chunk), numbered seed-major; one-wave workgroup g takes
// the contiguous run of units [g U / G, (g + 1) U / G), so it loads a seed's SeedRec once (scalar
// registers) for all of that seed's chunks in its run and writes consecutive 4 KiB of its row.
// Lane t makes ChaCha block ctr0 + 64 chunk + t (slots 16t..16t+15 of the chunk); the 16 words
// go through the wave's 4 KiB of LDS and come back in coalesced order, so each 16-B store
// instruction writes 1 KiB contiguous (lane t: slot 4t + 256j).  Measured against storing each
// lane's own 64 B (four 16-B stores at a 64-B lane stride): 1.45 vs 1.53 ms at K = 962, L = 2^20,
// and nontemporal forms the same (LDS-staged) or 4.5x slower (lane-strided partial lines;
// profiles/r06_expand_probe.log).  ~36 VGPRs: the grid is sized for occupancy (flm_set_tuning
// "expand_waves"), not for the unit count.
__global__ __launch_bounds__(64) void prg_expand_kernel(const SeedRec *__restrict__ recs, uint32_t chunks,
                                                        uint32_t n_units, uint64_t L, uint64_t pitch, uint32_t ctr0,
                                                        uint32_t *__restrict__ out) {
    __shared__ u32x4 lds[256];
    const int lane = threadIdx.x;
    const uint32_t u0 = (uint32_t)(((uint64_t)n_units * blockIdx.x) / gridDim.x);
    const uint32_t u1 = (uint32_t)(((uint64_t)n_units * (blockIdx.x + 1)) / gridDim.x);
    for (uint32_t u = u0; u < u1;) {
        const uint32_t k = u / chunks;
        const uint32_t end = min(u1, (k + 1) * chunks);
        const SeedRec rec = recs[k];  // wave-uniform: scalar loads, once per seed of the run
        uint32_t *row = out + (uint64_t)k * pitch;
        for (uint32_t chunk = u - k * chunks; u < end; ++u, ++chunk) {
            uint32_t m[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = 0u;
            chacha_mask_add(&rec, ctr0 + chunk * 64u + (uint32_t)lane, m);
            const int valid = (int)min<uint64_t>(1024u, L - (uint64_t)chunk * 1024u);
            uint32_t *dst = row + (uint64_t)chunk * 1024u;
            __syncthreads();  // one wave per workgroup: the previous chunk's reads are done
#pragma unroll
            for (int j = 0; j < 4; ++j) lds[4 * lane + j] = u32x4{m[4 * j], m[4 * j + 1], m[4 * j + 2], m[4 * j + 3]};
            __syncthreads();
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int slot = 4 * (lane + 64 * j);
                const u32x4 v = lds[lane + 64 * j];
                if (slot + 4 <= valid) {
                    *reinterpret_cast<u32x4 *>(dst + slot) = v;
                } else {
                    if (slot + 0 < valid) dst[slot + 0] = v.x;
                    if (slot + 1 < valid) dst[slot + 1] = v.y;
                    if (slot + 2 < valid) dst[slot + 2] = v.z;
                }
            }
        }
    }
}

// dst = a + b (mod 2^32), 16-B accesses, grid-stride.
__global__ __launch_bounds__(256) void add2_kernel(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                                                   uint32_t *__restrict__ dst, uint64_t n) {
    const uint64_t quads = n / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t q = t0; q < quads; q += stride) {
        const uint4 x = reinterpret_cast<const uint4 *>(a)[q], y = reinterpret_cast<const uint4 *>(b)[q];
        reinterpret_cast<uint4 *>(dst)[q] = make_uint4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
    const uint64_t t = 4 * quads + t0;
    if (t < n) dst[t] = a[t] + b[t];
}

// Loopback exchange of a device group whose ranks share one GPU (flm_group with repeated
// devices; tests and rehearsal only -- distinct GPUs use RCCL's reduce-scatter):
// dst[l] = sum_g parts.p[g][lo + l] for l < n, mod 2^32.  HBM-bound, uint4 when aligned.
__global__ __launch_bounds__(256) void shard_sum_kernel(PartPtrs parts, int G, uint64_t lo, uint64_t n,
                                                        uint32_t *__restrict__ dst) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if ((lo & 3) == 0) {
        const uint64_t quads = n / 4;
        for (uint64_t q = t0; q < quads; q += stride) {
            uint4 acc = make_uint4(0, 0, 0, 0);
            for (int g = 0; g < G; ++g) {
                const uint4 v = reinterpret_cast<const uint4 *>(parts.p[g] + lo)[q];
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
            reinterpret_cast<uint4 *>(dst)[q] = acc;
        }
        for (uint64_t t = 4 * quads + t0; t < n; t += stride) {
            uint32_t a = 0;
            for (int g = 0; g < G; ++g) a += parts.p[g][lo + t];
            dst[t] = a;
        }
        return;
    }
    for (uint64_t t = t0; t < n; t += stride) {
        uint32_t a = 0;
        for (int g = 0; g < G; ++g) a += parts.p[g][lo + t];
        dst[t] = a;
    }
}

#undef FLM_QR
#undef FLM_ROTL

// ----------------------------------------------------------------- launchers
// Workgroups of the seed-schedule launch: one per 256 seeds, more when it also zero-fills
// (about 16 KiB per workgroup, at most 1024).  meta needs 2 + 2 * this many words.
int seed_schedule_groups(int K, uint64_t zero_n) {
    const uint64_t g = (uint64_t)((K + 255) / 256 > 0 ? (K + 255) / 256 : 1);
    const uint64_t z = std::min<uint64_t>(1024, (zero_n + 4095) / 4096);
    return (int)std::max(g, z);
}

hipError_t launch_seed_schedule(const uint8_t *d_seeds, const int8_t *d_signs, int K, SeedRec *d_recs,
                                uint32_t *d_meta, hipStream_t stream, uint32_t *d_zero, uint64_t zero_n) {
    const unsigned grid = (unsigned)seed_schedule_groups(K, d_zero ? zero_n : 0);
    hipLaunchKernelGGL(seed_schedule_kernel, dim3(grid), dim3(256), 0, stream, d_seeds, d_signs, K, d_recs, d_meta,
                       d_zero, d_zero ? zero_n : 0);
    return hipGetLastError();
}

template <int S, bool BL, bool MERGED, int WPE, int RUM = 2, int AUX = 0, bool SPREAD = false>
static void launch_items_t(const Item *d_items, int n_items, const uint32_t *d_rows, uint64_t row_pitch,
                           const SeedRec *d_recs, const uint32_t *d_meta, uint32_t *d_out, hipStream_t stream) {
    hipLaunchKernelGGL((items_kernel<S, BL, MERGED, WPE, RUM, AUX, SPREAD>), dim3(n_items), dim3(kThreads), 0, stream, d_items, d_rows,
                       row_pitch, d_recs, d_meta, d_out);
}

hipError_t launch_items(int subtiles, int variant, const Item *d_items, int n_items, const uint32_t *d_rows,
                        uint64_t row_pitch, const SeedRec *d_recs, const uint32_t *d_meta, uint32_t *d_out,
                        hipStream_t stream) {
    if (n_items <= 0) return hipSuccess;
#define FLM_L(S, BL, MG, W, ...) \
    launch_items_t<S, BL, MG, W, ##__VA_ARGS__>(d_items, n_items, d_rows, row_pitch, d_recs, d_meta, d_out, stream)
#define FLM_V(S)                                                     \
    switch (variant) {                                               \
        case kVarCoalesced: FLM_L(S, false, false, 4); break;        \
        case kVarBlock: FLM_L(S, true, false, 4); break;             \
        case kVarMerged: FLM_L(S, true, true, 4, 2, 0); break;           \
        case kVarMergedW8: FLM_L(S, true, true, 8); break;           \
        case kVarMergedRU4: FLM_L(S, true, true, 4, 4, 0); break;    \
        case kVarMergedNT: FLM_L(S, true, true, 4, 2, 2); break;     \
        case kVarMergedRU4NT: FLM_L(S, true, true, 4, 4, 2); break;  \
        case kVarMergedSpread: FLM_L(S, true, true, 4, 2, 0, true); break; \
        case kVarBlockSpread: FLM_L(S, true, false, 4, 2, 0, true); break; \
        default: return hipErrorInvalidValue;                        \
    }
    switch (subtiles) {
        case 1: FLM_V(1) break;
        case 4: FLM_V(4) break;
        case 16: FLM_V(16) break;
        default: return hipErrorInvalidValue;
    }
#undef FLM_V
#undef FLM_L
    return hipGetLastError();
}

int small_round_slots(int B) { return 16 * B; }

hipError_t launch_small_round(int B, const uint32_t *d_rows, uint64_t pitch, int N, const uint8_t *d_seeds,
                              const int8_t *d_signs, int K, uint64_t L, uint64_t mask_lo, uint64_t mask_hi,
                              uint32_t ctr0, uint32_t *d_out, uint32_t *d_meta, hipStream_t stream) {
    const uint64_t T = (uint64_t)small_round_slots(B);
    const unsigned grid = (unsigned)((L + T - 1) / T);
    switch (B) {
        case 1: hipLaunchKernelGGL(small_round_kernel<1>, dim3(grid), dim3(256), 0, stream, d_rows, pitch, N, d_seeds,
                                   d_signs, K, L, mask_lo, mask_hi, ctr0, d_out, d_meta); break;
        case 2: hipLaunchKernelGGL(small_round_kernel<2>, dim3(grid), dim3(256), 0, stream, d_rows, pitch, N, d_seeds,
                                   d_signs, K, L, mask_lo, mask_hi, ctr0, d_out, d_meta); break;
        case 4: hipLaunchKernelGGL(small_round_kernel<4>, dim3(grid), dim3(256), 0, stream, d_rows, pitch, N, d_seeds,
                                   d_signs, K, L, mask_lo, mask_hi, ctr0, d_out, d_meta); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_small_client_mask(const uint32_t *d_x, uint64_t pitch, int N, const int64_t *d_seg,
                                   const uint8_t *d_seeds, const int8_t *d_signs, uint64_t L, uint32_t bias,
                                   uint32_t *d_out, hipStream_t stream) {
    constexpr int B = 16;  // 256-slot tiles: 4 seeds x 16 blocks per wave, 16 seeds per pass
    const dim3 grid((unsigned)((L + 16 * B - 1) / (16 * B)), (unsigned)N);
    hipLaunchKernelGGL((small_round_kernel<B, true>), grid, dim3(256), 0, stream, d_x, pitch, 0, d_seeds, d_signs, 0,
                       L, (uint64_t)0, L, 0u, d_out, (uint32_t *)nullptr, d_seg, bias);
    return hipGetLastError();
}

uint32_t pair_units_count(int K, uint64_t L, uint32_t *n_tiles) {
    const uint64_t t = (L + 1023) / 1024, c = (uint64_t)((K + kUnitSeeds - 1) / kUnitSeeds);
    if (n_tiles) *n_tiles = (uint32_t)t;
    const uint64_t n = t * c;
    return n > 0xF0000000ull ? 0xFFFFFFFFu : (uint32_t)n;  // caller rejects the sentinel
}

hipError_t launch_pair_units(bool side, const SeedRec *d_recs, int K, uint32_t *d_dst, uint64_t L, uint32_t *d_ws,
                             int groups, hipStream_t stream) {
    uint32_t n_tiles = 0;
    const uint32_t n_units = pair_units_count(K, L, &n_tiles);
    if (n_units == 0 || groups <= 0) return hipSuccess;
    if (side)
        hipLaunchKernelGGL(pair_units_kernel<true>, dim3(groups), dim3(64), 0, stream, d_recs, K, d_dst, L, n_tiles,
                           n_units, d_ws);
    else
        hipLaunchKernelGGL(pair_units_kernel<false>, dim3(groups), dim3(64), 0, stream, d_recs, K, d_dst, L, n_tiles,
                           n_units, d_ws);
    return hipGetLastError();
}

hipError_t launch_prg_expand(const SeedRec *d_recs, int K, uint64_t L, uint64_t pitch, uint32_t ctr0,
                             uint32_t *d_out, int groups, hipStream_t stream) {
    const uint64_t chunks = (L + 1023) / 1024, units = chunks * (uint64_t)K;
    if (K <= 0 || L == 0) return hipSuccess;
    if (units > 0xFFFFFFFFull || groups <= 0) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<uint64_t>(units, (uint64_t)groups);
    hipLaunchKernelGGL(prg_expand_kernel, dim3(grid), dim3(64), 0, stream, d_recs, (uint32_t)chunks, (uint32_t)units,
                       L, pitch, ctr0, d_out);
    return hipGetLastError();
}

hipError_t launch_flag_set(uint32_t *d_ws, hipStream_t stream) {
    hipLaunchKernelGGL(flag_set_kernel, dim3(1), dim3(64), 0, stream, d_ws);
    return hipGetLastError();
}

hipError_t launch_add2(const uint32_t *d_a, const uint32_t *d_b, uint32_t *d_dst, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint64_t g = std::min<uint64_t>(2048, (n / 4 + 255) / 256 + 1);
    hipLaunchKernelGGL(add2_kernel, dim3((unsigned)g), dim3(256), 0, stream, d_a, d_b, d_dst, n);
    return hipGetLastError();
}

hipError_t launch_shard_sum(const uint32_t *const *d_parts, int G, uint64_t lo, uint64_t n, uint32_t *d_dst,
                            hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (G < 1 || G > kMaxParts) return hipErrorInvalidValue;
    PartPtrs pp{};
    for (int g = 0; g < G; ++g) pp.p[g] = d_parts[g];
    const uint64_t grid = std::min<uint64_t>(2048, (n / 4 + 255) / 256 + 1);
    hipLaunchKernelGGL(shard_sum_kernel, dim3((unsigned)grid), dim3(256), 0, stream, pp, G, lo, n, d_dst);
    return hipGetLastError();
}

hipError_t launch_chacha20_xor(const uint32_t key[8], const uint32_t nonce[2], uint64_t counter,
                               const uint8_t *d_in, uint8_t *d_out, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 63) / 64;
    const unsigned grid = (unsigned)((blocks + 255) / 256);
    hipLaunchKernelGGL(chacha20_xor_kernel, dim3(grid), dim3(256), 0, stream, key[0], key[1], key[2], key[3],
                       key[4], key[5], key[6], key[7], nonce[0], nonce[1], counter, d_in, d_out, (uint64_t)n);
    return hipGetLastError();
}

}  // namespace flm

