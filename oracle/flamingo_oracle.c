/*
 * flamingo_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C CPU restatement of Flamingo's per-round mask-and-aggregate path,
 * used as the parity checker for the HIP product path (tests/, the smoke()
 * check in __graft_entry__.py and the cpu_baseline leg of bench.py).  Nothing
 * in flamingo_amd/ links, loads or calls this file.
 *
 * What it restates (reference = /root/reference, eniac/flamingo):
 *   - PRG conventions, util/param.py:8,9,12,32: vector_type uint32,
 *     fixed_key b"abcd", nonce = 8 zero bytes.
 *   - The PRG idiom ChaCha20.new(key=seed, nonce=param.nonce)
 *     .encrypt(param.fixed_key * L) followed by np.frombuffer(.., 'uint32'),
 *     SA_ClientAgent.py:248-250,296-298 and SA_ServiceAgent.py:533-536,596-603.
 *     The cipher lives in pycryptodomex 3.19.1 (requirements.txt:25, not
 *     vendored); its 8-byte-nonce ChaCha20 is D. J. Bernstein's original
 *     layout: 64-bit block counter in state words 12..13, 64-bit nonce in
 *     14..15, counter starting at 0.  Restated here from the published
 *     algorithm (RFC 7539 section 2.1-2.3 quarter round / block function).
 *   - Client masking, SA_ClientAgent.py:304-324:
 *       y_i = x_i + PRG(m_i) + sum_{j>i} PRG(s_ij) - sum_{j<i} PRG(s_ij)
 *   - Server aggregate + unmask, SA_ServiceAgent.py:346-350 (partial sum),
 *     :529-536 (self masks, always subtracted), :587-603 (dropout-pair masks,
 *     sign recon_symbol), :538-540/:605 (final combine), all mod 2^32.
 *
 * PINNED to the reference itself: tests/test_ref_golden_cpu.py compares this
 * code with rounds the reference's own agents produced (tests/golden/
 * make_ref_golden.py imports util/param.py and agent/flamingo/SA_*Agent.py from
 * the reference under a pycryptodomex/libnum stand-in).  Also pinned by the
 * published ChaCha20 vectors (RFC 7539 2.3.2 and A.1), fixtures generated with
 * OpenSSL's independent ChaCha20 (tests/golden/make_golden.py), and the protocol
 * invariant out == |U| (SA_ClientAgent.py:304, SA_ServiceAgent.py:605).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define FLMO_ABCD 0x64636261u /* LE32(b"abcd"), util/param.py:12 */

static inline uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }

static inline uint32_t ld_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static inline void st_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

#define QUARTER(a, b, c, d)                          \
    do {                                             \
        a += b; d ^= a; d = rotl32(d, 16);           \
        c += d; b ^= c; b = rotl32(b, 12);           \
        a += b; d ^= a; d = rotl32(d, 8);            \
        c += d; b ^= c; b = rotl32(b, 7);            \
    } while (0)

/* One 64-byte ChaCha20 block, DJB layout (counter words 12..13, nonce 14..15). */
void flmo_chacha20_block(const uint8_t key[32], const uint8_t nonce[8], uint64_t counter,
                         uint32_t out[16]) {
    uint32_t in[16];
    in[0] = 0x61707865u; in[1] = 0x3320646eu; in[2] = 0x79622d32u; in[3] = 0x6b206574u;
    for (int i = 0; i < 8; ++i) in[4 + i] = ld_le32(key + 4 * i);
    in[12] = (uint32_t)counter;
    in[13] = (uint32_t)(counter >> 32);
    in[14] = ld_le32(nonce);
    in[15] = ld_le32(nonce + 4);
    uint32_t x[16];
    memcpy(x, in, sizeof x);
    for (int r = 0; r < 10; ++r) {
        QUARTER(x[0], x[4], x[8], x[12]);
        QUARTER(x[1], x[5], x[9], x[13]);
        QUARTER(x[2], x[6], x[10], x[14]);
        QUARTER(x[3], x[7], x[11], x[15]);
        QUARTER(x[0], x[5], x[10], x[15]);
        QUARTER(x[1], x[6], x[11], x[12]);
        QUARTER(x[2], x[7], x[8], x[13]);
        QUARTER(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

/* ChaCha20(key, nonce).encrypt(in) starting at block `counter` (byte-exact,
 * any length): the form used by util/param.py:44-46,63-73 and the PRG idiom. */
void flmo_chacha20_xor(const uint8_t key[32], const uint8_t nonce[8], uint64_t counter,
                       const uint8_t *in, uint8_t *out, size_t n) {
    uint32_t ks[16];
    uint8_t kb[64];
    for (size_t off = 0; off < n; off += 64, ++counter) {
        flmo_chacha20_block(key, nonce, counter, ks);
        for (int i = 0; i < 16; ++i) st_le32(kb + 4 * i, ks[i]);
        size_t m = n - off < 64 ? n - off : 64;
        for (size_t i = 0; i < m; ++i) out[off + i] = in[off + i] ^ kb[i];
    }
}

static const uint8_t ZERO_NONCE[8] = {0, 0, 0, 0, 0, 0, 0, 0}; /* util/param.py:32 */

/* PRG(seed)[slot0 : slot0+L] as uint32 words: LE32(keystream word) ^ LE32("abcd").
 * slot l lives in block l>>4, word l&15 (16 uint32 slots per 64-byte block). */
void flmo_prg_words(const uint8_t seed[32], uint64_t slot0, size_t L, uint32_t *out) {
    uint32_t ks[16];
    size_t i = 0;
    while (i < L) {
        uint64_t slot = slot0 + i;
        uint64_t blk = slot >> 4;
        unsigned w = (unsigned)(slot & 15);
        flmo_chacha20_block(seed, ZERO_NONCE, blk, ks);
        for (; w < 16 && i < L; ++w, ++i) out[i] = ks[w] ^ FLMO_ABCD;
    }
}

/* acc[l] += sign * PRG(seed)[slot0 + l]   (mod 2^32), sign in {+1,-1}. */
static void prg_accumulate(const uint8_t seed[32], int sign, uint64_t slot0, size_t L,
                           uint32_t *acc) {
    uint32_t ks[16];
    size_t i = 0;
    while (i < L) {
        uint64_t slot = slot0 + i;
        unsigned w = (unsigned)(slot & 15);
        flmo_chacha20_block(seed, ZERO_NONCE, slot >> 4, ks);
        if (sign > 0)
            for (; w < 16 && i < L; ++w, ++i) acc[i] += ks[w] ^ FLMO_ABCD;
        else
            for (; w < 16 && i < L; ++w, ++i) acc[i] -= ks[w] ^ FLMO_ABCD;
    }
}

/* Server round (SA_ServiceAgent.py:346-350, 529-536, 587-605):
 *   out = sum_{i<N} rows[i] + sum_{k<K} signs[k] * PRG(seeds[k])      (mod 2^32)
 * rows: N rows of `pitch` uint32, first L used.  The slot window
 * [slot0, slot0+L) of every PRG is used (slot0 = 0 for a whole vector).
 * threads > 1 splits the slots into contiguous chunks (OpenMP build only);
 * every chunk runs the same per-slot arithmetic, so the result is identical. */
int flmo_aggregate_unmask(const uint32_t *rows, size_t pitch, int N, const uint8_t *seeds,
                          const int8_t *signs, int K, size_t L, uint64_t slot0, uint32_t *out,
                          int threads) {
    if (N < 0 || K < 0 || (N > 0 && pitch < L)) return -1;
    for (int k = 0; k < K; ++k)
        if (signs[k] != 1 && signs[k] != -1) return -2;
    if (threads < 1) threads = 1;
    /* chunk = multiple of 16 slots so each chunk starts on a block boundary
     * relative to slot0 (correctness does not depend on it). */
    size_t chunk = (L + (size_t)threads - 1) / (size_t)threads;
    chunk = (chunk + 15) & ~(size_t)15;
    if (chunk == 0) chunk = 16;
    long nchunks = (long)((L + chunk - 1) / chunk);
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static)
#endif
    for (long c = 0; c < nchunks; ++c) {
        size_t lo = (size_t)c * chunk;
        size_t n = L - lo < chunk ? L - lo : chunk;
        uint32_t *o = out + lo;
        /* vec_sum_partial = zeros; += user_vectors[id]   (:346-350) */
        memset(o, 0, n * sizeof(uint32_t));
        for (int i = 0; i < N; ++i) {
            const uint32_t *r = rows + (size_t)i * pitch + lo;
            for (size_t l = 0; l < n; ++l) o[l] += r[l];
        }
        /* mi_vec -= PRG(m_i) (:530-536); cancel_vec +-= PRG(s_ij) (:595-603);
         * final_sum = partial + cancel + mi (:605) -- addition is associative
         * and commutative mod 2^32, so accumulating in place is identical. */
        for (int k = 0; k < K; ++k) prg_accumulate(seeds + 32 * (size_t)k, signs[k], slot0 + lo, n, o);
    }
    return 0;
}

/* Client masking (SA_ClientAgent.py:304-324) for a batch of clients.
 *   out[i] = x[i] + sum_{k in [seg[i], seg[i+1])} signs[k] * PRG(seeds[k])
 * x == NULL means the reference's all-ones input (np.ones, :304). */
int flmo_client_mask(const uint32_t *x, size_t x_pitch, int N, const int64_t *seg,
                     const uint8_t *seeds, const int8_t *signs, size_t L, uint32_t *out,
                     size_t out_pitch, int threads) {
    if (threads < 1) threads = 1;
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
#endif
    for (int i = 0; i < N; ++i) {
        uint32_t *o = out + (size_t)i * out_pitch;
        if (x)
            memcpy(o, x + (size_t)i * x_pitch, L * sizeof(uint32_t));
        else
            for (size_t l = 0; l < L; ++l) o[l] = 1u;
        for (int64_t k = seg[i]; k < seg[i + 1]; ++k)
            prg_accumulate(seeds + 32 * (size_t)k, signs[k], 0, L, o);
    }
    return 0;
}

int flmo_has_openmp(void) {
#ifdef _OPENMP
    return 1;
#else
    return 0;
#endif
}
