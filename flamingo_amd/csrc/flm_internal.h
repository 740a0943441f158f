// flm_internal.h -- shared between the gfx950 kernels (flm_kernels.hip) and the
// host runtime (flm_runtime.hip).  Not part of the public ABI.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <hip/hip_runtime.h>

namespace flm {

// b"abcd" as a little-endian word (util/param.py:12).
constexpr uint32_t kAbcd = 0x64636261u;
// ChaCha20 "expand 32-byte k".
constexpr uint32_t kSigma0 = 0x61707865u, kSigma1 = 0x3320646eu, kSigma2 = 0x79622d32u,
                   kSigma3 = 0x6b206574u;

// One wave owns a 1024-slot sub-tile: 64 lanes x one 16-word ChaCha block.
constexpr int kWaveSlots = 1024;
constexpr int kWavesPerGroup = 16;          // 1024-thread workgroups
constexpr int kThreads = 64 * kWavesPerGroup;

// Per-seed schedule, built on the device by seed_schedule_kernel: the key, the
// sign folded into an XOR constant, and everything of ChaCha's first double
// round that does not depend on the block counter (block counter high word is
// 0 for every slot < 2^36, nonce is zero).  128 bytes, read with scalar loads.
struct SeedRec {
    uint32_t k[8];     // key words (LE32 of the 32 seed bytes)
    uint32_t xorc;     // 0x64636261 for sign +1, ~0x64636261 for sign -1
    uint32_t a0;       // sigma0 + k0 (first add of column 0)
    uint32_t col1[4];  // x1, x5, x9, x13 after round-1 column QR(1,5,9,13)
    uint32_t col2[4];  // x2, x6, x10, x14 after QR(2,6,10,14)
    uint32_t col3[4];  // x3, x7, x11, x15 after QR(3,7,11,15)
    uint32_t pad[10];
};
static_assert(sizeof(SeedRec) == 128, "SeedRec must be 128 bytes");

enum ItemFlags : uint32_t {
    kHasRows = 1u,
    kHasMask = 2u,
    kSameTile = 4u,       // row tile == mask tile: combine before writing
    kRowAtomic = 8u,      // row (or combined) tile written with u32 atomic adds
    kMaskAtomic = 16u,
    kMaskBiasNneg = 32u,  // add the device-side count of negative signs to the mask tile
};

// One workgroup's work: a row unit (sum of `nrows` rows over one tile) and/or a
// mask unit (sum of seeds [k0, k0+nseeds) over one tile).  64 bytes.
struct Item {
    uint64_t row_in;     // element offset into rows: first row of the unit, tile start slot
    uint64_t row_out;    // element offset into out of the row tile
    uint64_t mask_out;   // element offset into out of the mask tile
    uint64_t mask_ctr;   // ChaCha block counter at the mask tile start (PRG slot / 16)
    uint32_t nrows;
    uint32_t k0;
    uint32_t nseeds;
    uint32_t row_valid;  // valid slots in the row tile (tail)
    uint32_t mask_valid;
    uint32_t flags;
    uint32_t row_bias;   // added once per slot of the row tile
    uint32_t mask_bias;  // added once per slot of the mask tile
};
static_assert(sizeof(Item) == 64, "Item must be 64 bytes");

// Launchers (flm_kernels.hip).  All enqueue on `stream` and return hipError_t.
// d_zero (optional): zero-fill zero_n u32 words of the round's output in the same launch.
hipError_t launch_seed_schedule(const uint8_t *d_seeds, const int8_t *d_signs, int K, SeedRec *d_recs,
                                uint32_t *d_meta, hipStream_t stream, uint32_t *d_zero = nullptr,
                                uint64_t zero_n = 0);
int seed_schedule_groups(int K, uint64_t zero_n);
// items_kernel variants (see flm_kernels.hip): row load layout / accumulator form.
enum ItemsVariant : int {
    kVarCoalesced = 0,  // coalesced rows, separate row/mask accumulators (any plan)
    kVarBlock = 1,      // block-layout rows, separate accumulators (any plan)
    kVarMerged = 2,     // block-layout rows added into the mask accumulator (single-tile plans)
    kVarMergedW8 = 3,   // kVarMerged at >= 8 waves/SIMD register budget
    kVarMergedRU4 = 4,  // kVarMerged, 4 rows in flight in the rows-only loop
    kVarMergedNT = 5,   // kVarMerged, non-temporal row loads
    kVarMergedRU4NT = 6,
    kVarMergedSpread = 7,  // kVarMerged, seeds spread evenly over the row stream
    kVarBlockSpread = 8,   // kVarBlock (dual-tile plans), seeds spread over the row stream
    kVarCount = 9,
};
// subtiles: 1, 4 or 16 sub-tiles of 1024 slots per workgroup.
hipError_t launch_items(int subtiles, int variant, const Item *d_items, int n_items, const uint32_t *d_rows,
                        uint64_t row_pitch, const SeedRec *d_recs, const uint32_t *d_meta,
                        uint32_t *d_out, hipStream_t stream);
// One-launch round for small rounds (flm_kernels.hip small_round_kernel): a workgroup owns
// 16*B slots (B = 1, 2, 4), sums every row there and adds every seed's mask; meta gets the
// sign counts (one part).  mask_lo % 16 == 0 and (mask_hi % 16 == 0 or mask_hi == L).
int small_round_slots(int B);
hipError_t launch_small_round(int B, const uint32_t *d_rows, uint64_t pitch, int N, const uint8_t *d_seeds,
                              const int8_t *d_signs, int K, uint64_t L, uint64_t mask_lo, uint64_t mask_hi,
                              uint32_t ctr0, uint32_t *d_out, uint32_t *d_meta, hipStream_t stream);
// Client masking with the same kernel (SEG mode): grid (L/256, N), row i gets seeds
// [d_seg[i], d_seg[i+1]) on top of x row i (or the constant `bias` when d_x is NULL).
hipError_t launch_small_client_mask(const uint32_t *d_x, uint64_t pitch, int N, const int64_t *d_seg,
                                   const uint8_t *d_seeds, const int8_t *d_signs, uint64_t L, uint32_t bias,
                                   uint32_t *d_out, hipStream_t stream);
uint32_t pair_units_count(int K, uint64_t L, uint32_t *n_tiles);
hipError_t launch_pair_units(bool side, const SeedRec *d_recs, int K, uint32_t *d_dst, uint64_t L, uint32_t *d_ws,
                             int groups, hipStream_t stream);
hipError_t launch_flag_set(uint32_t *d_ws, hipStream_t stream);
// d_out[k * pitch + l] = PRG(seed k)[16 ctr0 + l], l < L, k < K (prg_expand_kernel): `groups` one-wave
// workgroups take contiguous runs of the K x ceil(L / 1024) seed-major units.
hipError_t launch_prg_expand(const SeedRec *d_recs, int K, uint64_t L, uint64_t pitch, uint32_t ctr0,
                             uint32_t *d_out, int groups, hipStream_t stream);
hipError_t launch_add2(const uint32_t *d_a, const uint32_t *d_b, uint32_t *d_dst, uint64_t n, hipStream_t stream);
// dst[l] = sum_{g<G} d_parts[g][lo + l], l < n (G <= kMaxParts, all on the launching device).
constexpr int kMaxParts = 16;
struct PartPtrs {
    const uint32_t *p[kMaxParts];
};
hipError_t launch_shard_sum(const uint32_t *const *d_parts, int G, uint64_t lo, uint64_t n, uint32_t *d_dst,
                            hipStream_t stream);
hipError_t launch_chacha20_xor(const uint32_t key[8], const uint32_t nonce[2], uint64_t counter,
                               const uint8_t *d_in, uint8_t *d_out, size_t n, hipStream_t stream);

// P-256 (flm_p256.hip). d_jac holds T*D Jacobian results as SoA planes [T][24][D].
hipError_t launch_ec_mul(const uint8_t *d_points, const uint8_t *d_scalars, int per_element, int T, int D,
                         uint32_t *d_jac, uint32_t *d_flags, hipStream_t stream, int threads, int waves,
                         int coop = 0, int terms = 1, unsigned lds_pad = 0);
// Partial sums the combine's ec_mul leaves per element: T, or ceil(T / terms) with Straus lanes.
int ec_mul_groups(int T, int terms);
hipError_t launch_shamir_combine(const uint8_t *d_shares, const uint8_t *d_lambdas, int T, int M, uint8_t *d_out,
                                 hipStream_t stream);
hipError_t launch_ec_finish(const uint8_t *d_base, const uint32_t *d_jac, int T, int D, int negate,
                            uint8_t *d_points_out, uint8_t *d_digests_out, uint32_t *d_flags, hipStream_t stream);
// hash_str_to_curve of n messages (d_msgs: n x 64 bytes + d_lens), or of the decimal strings of
// v0 .. v0+n-1 (d_msgs NULL); d_out n x 64 wire bytes, d_flags n words (written)
hipError_t launch_hash_to_curve(const uint8_t *d_msgs, const uint32_t *d_lens, uint32_t v0, int n, uint8_t *d_out,
                                uint32_t *d_flags, hipStream_t stream);

}  // namespace flm

// Host-runtime hooks shared by flm_runtime.hip and flm_comm.hip (not exported in the header).
struct flm_ctx;
namespace flm {
namespace rt {
int set_error(flm_ctx *ctx, int code, const char *msg);
int device_of(const flm_ctx *ctx);
hipStream_t stream_of(const flm_ctx *ctx);
void **comm_slot(flm_ctx *ctx);
// n bytes between host buffers on the context's copy threads (the CPU side of a pinned-buffer copy)
void host_copy(flm_ctx *ctx, void *dst, const void *src, size_t n);
// The calling thread's current device belongs to the caller: every entry point that selects a
// device (its context's, or each rank's of a group or store) gives the caller's back on return.
// torch and the agents' own HIP code allocate on the current device, and a group call that left
// it on its last rank's GPU would move them there.  set() switches only when needed (hipGetDevice
// is a thread-local read), so a call on the caller's own device costs no hipSetDevice at all.
struct DeviceScope {
    int old = -1;
    DeviceScope() {
        if (hipGetDevice(&old) != hipSuccess) old = -1;
    }
    explicit DeviceScope(int want) : DeviceScope() { (void)set(want); }
    hipError_t set(int want) {
        int now = -1;
        if (hipGetDevice(&now) == hipSuccess && now == want) return hipSuccess;
        return hipSetDevice(want);
    }
    ~DeviceScope() {
        int now = -1;
        if (old >= 0 && hipGetDevice(&now) == hipSuccess && now != old) (void)hipSetDevice(old);
    }
    DeviceScope(const DeviceScope &) = delete;
    DeviceScope &operator=(const DeviceScope &) = delete;
};
// Size of a scratch allocation that must hold `bytes`: half again as much, at most 64 MiB extra,
// in whole 4 KiB pages.  Buffers sized by per-round counts (K seeds, D pairs) change by a few
// percent from round to round; allocating exactly made every new maximum a hipFree + hipMalloc,
// and hipFree waits for the whole device (4.8 ms inside the server's unmask, profiles/r05_hip_api_top.txt).
inline size_t grow_bytes(size_t bytes) {
    const size_t slack = bytes / 2 < (size_t(64) << 20) ? bytes / 2 : (size_t(64) << 20);
    return (bytes + slack + 4095) & ~size_t(4095);
}
// Upload host rows and seeds and enqueue the fused round over mask window [mask_lo, mask_hi) into
// d_out (L words) on the context's stream; returns without synchronising.
int host_round_async(flm_ctx *ctx, const uint32_t *const *rows, int N, const uint8_t *seeds, const int8_t *signs,
                     int K, size_t L, size_t mask_lo, size_t mask_hi, uint32_t *d_out);
}  // namespace rt
void comm_release(flm_ctx *ctx);  // flm_comm.hip: drop the context's communicator (flm_free)
// flm_comm.hip: synchronise every device, finalize a one-thread clique's members in one RCCL group,
// then destroy them (flm_group_free)
void comm_release_clique(flm_ctx *const *ctxs, int n);
}  // namespace flm
