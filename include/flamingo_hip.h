/*
 * flamingo_hip.h -- C ABI of libflamingo_hip.so, the MI355X (gfx950) engine
 * behind Flamingo's per-round mask-and-aggregate path.
 *
 * The reference (eniac/flamingo, pure Python) has no FFI; these entry points
 * replace the bodies of the reference's hot loops under an unchanged agent
 * surface.  Each function cites the reference code it stands in for
 * (paths relative to the reference root).
 *
 * Arithmetic: uint32 mod 2^32 everywhere (util/param.py:9 vector_type).
 * PRG(seed)[l] = LE32(ChaCha20_DJB(key=seed, nonce=0^8).keystream[4l:4l+4])
 *                ^ 0x64636261 (b"abcd", util/param.py:12,32).
 *
 * Conventions
 *  - Return 0 on success, a negative FLM_E* code on failure; the message is
 *    available from flm_last_error(ctx) (or flm_last_error(NULL) when no
 *    context could be created).  The Python layer raises RuntimeError, as the
 *    reference does on its own guard failures (SA_ServiceAgent.py:349,502).
 *  - seeds are K x 32 bytes (the reference's 32-byte ChaCha20 keys:
 *    m_i.to_bytes(32,'big') at SA_ServiceAgent.py:526, SHA-256 digests at
 *    :583-585); signs are K int8 in {+1,-1} (recon_symbol, :375-378; self
 *    masks are always -1, :536).
 *  - Host-pointer functions are synchronous: they copy in, compute on the
 *    GPU and copy out; no host pointer is retained after return.
 *  - *_dev functions take device pointers and enqueue work on `stream`
 *    (a hipStream_t; NULL = the HIP null stream) and return without waiting
 *    for earlier work: the small tables they upload (seg/signs, work items)
 *    go through a pool of pinned staging slots, each reused only after the
 *    launch that read it has completed.  The per-seed device tables a call
 *    builds come from a ring (8 per context) with the same rule: a table is
 *    rebuilt on a stream only after every launch on other streams that reads
 *    it has completed (or, when all are in use, that stream waits for them on
 *    the device), so calls of one context may run on any mix of streams with
 *    any seeds, without ordering by the caller.
 *  - One context per host thread; a context binds one GPU (one process per
 *    GPU).  Create it lazily, after any fork (SA_ServiceAgent.py:562 forks a
 *    multiprocessing.Pool).
 *  - Every entry point leaves the calling thread's current HIP device as it
 *    found it: a call selects its context's device (or each rank's, for a
 *    group or store) only for its own duration.
 */
#ifndef FLAMINGO_HIP_H
#define FLAMINGO_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLM_OK 0
#define FLM_EINVAL (-1)   /* bad argument (length mismatch, sign not +-1, alignment) */
#define FLM_EHIP (-2)     /* HIP runtime error */
#define FLM_ENOMEM (-3)   /* device or pinned allocation failed */
#define FLM_ERANGE (-4)   /* slot range beyond 2^36 (block counter high word must be 0) */

typedef struct flm_ctx flm_ctx;

/* ------------------------------------------------------------ lifecycle */
int flm_device_count(void);
/* Bind a context to HIP device `device` and create its stream. */
int flm_init(flm_ctx **out, int device);
void flm_free(flm_ctx *ctx);
const char *flm_last_error(const flm_ctx *ctx);
/* The context's own non-blocking stream (a hipStream_t): the host-pointer calls and
 * the flm_group rounds run on it, so a caller can order its own streams against them. */
void *flm_ctx_stream(flm_ctx *ctx);
/* Library / kernel build identification string (static storage). */
const char *flm_version(void);

/* ---------------------------------------------------- host-memory path */

/* Server round: replaces SA_ServiceAgent.report_process's partial sum
 * (agent/flamingo/SA_ServiceAgent.py:346-350) and reconstruction_process's
 * self-mask and dropout-pair unmask + final combine (:529-540, :587-605):
 *   out[l] = sum_{i<N} rows[i][l] + sum_{k<K} signs[k] * PRG(seeds[k])[l]
 * rows: N host pointers to L uint32 each (the VECTOR bodies, :210). */
int flm_aggregate_unmask(flm_ctx *ctx, const uint32_t *const *rows, int N, const uint8_t *seeds,
                         const int8_t *signs, int K, size_t L, uint32_t *out);

/* Client masking, batched over N clients: replaces SA_ClientAgent.sendVectors's
 * mask expansion and composition (agent/flamingo/SA_ClientAgent.py:246-324):
 *   out[i][l] = x[i][l] + sum_{k in [seg[i], seg[i+1])} signs[k] * PRG(seeds[k])[l]
 * x: N x L row-major uint32, or NULL for the reference's all-ones input (:304).
 * out: N x L row-major. */
int flm_client_mask(flm_ctx *ctx, const uint32_t *x, int N, const int64_t *seg, const uint8_t *seeds,
                    const int8_t *signs, size_t L, uint32_t *out);

/* Standalone PRG expansion: out[k][l] = PRG(seeds[k])[slot0 + l], K x L
 * row-major (the idiom at SA_ClientAgent.py:248-250 / SA_ServiceAgent.py:533-535
 * for a whole batch).  slot0 must be a multiple of 16. */
int flm_prg_expand(flm_ctx *ctx, const uint8_t *seeds, int K, size_t L, uint64_t slot0, uint32_t *out);

/* acc[l] += sum_k signs[k] * PRG(seeds[k])[slot0 + l], in place on a host
 * vector (the mi_vec / cancel_vec loops, SA_ServiceAgent.py:530-536, 595-603,
 * on a slot window).  slot0 must be a multiple of 16. */
int flm_mask_accumulate(flm_ctx *ctx, const uint8_t *seeds, const int8_t *signs, int K, uint32_t *acc,
                        size_t L, uint64_t slot0);

/* ChaCha20(key, nonce).encrypt(in) from block `counter` on, byte-exact, any
 * length: the PRF/PRG calls of util/param.py:44-46 (choose_committee) and
 * :63-76 (findNeighbors), computed on the GPU. */
int flm_chacha20_xor(flm_ctx *ctx, const uint8_t key[32], const uint8_t nonce[8], uint64_t counter,
                     const uint8_t *in, uint8_t *out, size_t n);

/* -------------------------------------------------- device-resident path */

/* Device-resident server round over a slot window, for single- and multi-GPU use:
 *   out[l]  = sum_{i<N} rows[i*row_pitch + l]                  for l in [0, L)
 *           + sum_k signs[k] * PRG(seeds[k])[prg_slot0 + l]    for l in [mask_lo, mask_hi)
 * (mod 2^32).  With mask_lo=0, mask_hi=L, prg_slot0=0 this is the whole
 * round; on G GPUs each rank passes its own client rows and its own slot
 * shard [mask_lo, mask_hi) and the partial vectors are then reduce-scattered.
 * Requirements: row_pitch % 4 == 0 and row_pitch >= round_up(L, 4);
 * rows and out 16-byte aligned; mask_lo % 16 == 0; prg_slot0 % 16 == 0;
 * prg_slot0 + mask_hi <= 2^36.  d_seeds: K x 32 bytes, d_signs: K int8 (+-1).
 * Enqueued on `stream`; nothing is synchronised. */
int flm_aggregate_unmask_dev(flm_ctx *ctx, const uint32_t *d_rows, size_t row_pitch, int N,
                             const uint8_t *d_seeds, const int8_t *d_signs, int K, size_t L,
                             size_t mask_lo, size_t mask_hi, uint64_t prg_slot0, uint32_t *d_out,
                             void *stream);

/* The same round split in its two launches, so a caller can time the
 * dominant kernel alone: flm_seed_table_dev builds the context's per-seed
 * schedule (ChaCha key words, sign, counter-independent first-round words)
 * from device seeds/signs; flm_aggregate_dev then runs the row-sum + unmask
 * kernel against that table (K must match the table), on any stream: a read
 * on another stream than the table's build waits for the build on the device.
 * The table stays published until the context's next call that builds a seed
 * table (any *_dev round, expansion, client masking, pair units, or another
 * flm_seed_table_dev); flm_aggregate_dev then fails with FLM_EINVAL rather
 * than unmask against other seeds.  Same requirements as flm_aggregate_unmask_dev. */
int flm_seed_table_dev(flm_ctx *ctx, const uint8_t *d_seeds, const int8_t *d_signs, int K, void *stream);
int flm_aggregate_dev(flm_ctx *ctx, const uint32_t *d_rows, size_t row_pitch, int N, int K, size_t L,
                      size_t mask_lo, size_t mask_hi, uint64_t prg_slot0, uint32_t *d_out, void *stream);

/* Device-resident client masking (flm_client_mask on device buffers).  seg and
 * signs are host arrays (they size the launch); seeds, x and out are device
 * pointers; x may be NULL (all-ones input).  x and out rows use `pitch`. */
int flm_client_mask_dev(flm_ctx *ctx, const uint32_t *d_x, size_t pitch, int N, const int64_t *seg,
                        const uint8_t *d_seeds, const int8_t *signs, size_t L, uint32_t *d_out,
                        void *stream);

/* Device-resident PRG expansion: d_out[k*pitch + l] = PRG(seed k)[slot0 + l]. */
int flm_prg_expand_dev(flm_ctx *ctx, const uint8_t *d_seeds, int K, size_t L, uint64_t slot0,
                       uint32_t *d_out, size_t pitch, void *stream);

/* After a *_dev call has completed on its stream: number of signs that were
 * not +-1 in the last seed table (0 when valid). */
int flm_check_signs(flm_ctx *ctx, int *bad_count);

/* ----------------------------------------------------------- diagnostics */

/* Describe the launch plan the last *aggregate* call used:
 * items, tile slots, atomics used (0/1), kernel variant id (100: the one-launch
 * small-round kernel, items = its workgroups; 101: the expansion kernel of
 * flm_prg_expand[_dev], items = its one-wave workgroups). */
int flm_last_plan(const flm_ctx *ctx, int *items, int *tile_slots, int *atomics, int *variant);

/* Tuning knobs for A/B measurement (defaults are the tuned choice):
 *   "variant"  -1 auto | 0 coalesced rows | 1 block-layout rows |
 *              2 merged accumulator | 3 merged, 8 waves/SIMD budget
 *              (2/3 apply only to plans whose items each write one tile)
 *   "subtiles" 0 auto | 1 | 4 | 16 sub-tiles of 1024 slots per workgroup
 *              for aggregate plans.
 *   "pairing"  0 interleaved single-kind items | 1 dual-tile items (default) |
 *              2 same-tile window items (the window's tiles carry rows and seeds in
 *              matching parts, merged kernel), for windows where rows and masks
 *              cover different tiles.
 *   "min_items" planner target for work items per aggregate launch
 *              (default 1024; more items = finer load balance, more atomics).
 *   "ec_threads" 64 (default) | 128 | 256 lanes per workgroup of the P-256
 *              scalar-multiplication kernel.
 *   "ec_waves" 1 (default: uncapped registers) | 4 | 8 minimum waves per SIMD the
 *              scalar-multiplication kernel is compiled for (more waves, more spills).
 *   "ec_coop"  -1 (default: auto) | 0 | 1 | 2: scalar multiplications with four waves per 64 of
 *              them, the field multiplications of each point doubling and addition spread over
 *              the waves (a shorter latency chain for batches that leave most SIMDs idle); 2:
 *              the same with every field element on a 16-lane row (four products per workgroup,
 *              ~93 instructions per multiplication against ~258).
 *              Auto: the row kernel up to 20 products per CU, the cooperative kernel up to 128
 *              per CU (one pass of the device), else one lane per product.
 *   "ec_terms" 1 (default) | 2 | 4: products summed per lane in the reconstruction combine
 *              (Straus: the terms share one chain of doublings); ignored when the combine
 *              runs cooperatively.
 *   "ec_spread" 0 (default) .. 64: KiB of LDS reserved per 64-lane workgroup of the
 *              per-lane combine kernels (caps their workgroups per CU).
 *   "expand_waves" 1..256 (default 128): one-wave workgroups per CU of the expansion kernel
 *              (flm_prg_expand[_dev]), each taking a contiguous run of the K x ceil(L / 1024)
 *              seed-major (seed, 1024-slot chunk) units.
 *   "small"   0 | 1 (default) | 2: flm_aggregate_unmask_dev runs
 *              rounds as ONE small-round launch never | when rows and mask words are both
 *              <= 2^22 (BASELINE c2) | whenever the window allows it (mask_hi % 16 == 0 or
 *              mask_hi == L).  That path builds no device seed table: a following
 *              flm_aggregate_dev needs its own flm_seed_table_dev. */
int flm_set_tuning(flm_ctx *ctx, const char *key, int value);
/* The context's current value of a flm_set_tuning key (whoever set it), FLM_EINVAL for an unknown key. */
int flm_get_tuning(const flm_ctx *ctx, const char *key, int *value);

/* Host-only view of the launch planner (no GPU needed): the work items the
 * aggregate kernel would run for this round shape.  items_out receives up to
 * max_items 64-byte items (layout: flm_internal.h Item); *n_items the total;
 * *plan_flags bit0 zero-fill, bit1 atomics, bit2 single-tile, bit3 seed-light,
 * bits 8.. sub-tiles per workgroup.  subtiles/pairing as flm_set_tuning. */
int flm_plan_aggregate(int subtiles, int pairing, size_t row_pitch, int N, int K, size_t L, size_t mask_lo,
                       size_t mask_hi, uint64_t prg_slot0, void *items_out, int max_items, int *n_items,
                       int *plan_flags);

/* ------------------------------------------------------- P-256 seed recovery */

/* Wire format: a point is 64 bytes x||y, each coordinate a 32-byte big-endian
 * integer < p (what the reference hashes, SA_ServiceAgent.py:583-585); a
 * scalar is 32 bytes big endian.  The point at infinity is returned as 64 zero
 * bytes (pycryptodome's EccPoint(0, 0)); flags bit 2 marks it.
 *
 * Threshold-ElGamal combine + key derivation, replacing
 * SA_ServiceAgent.reconstruction_process's pairwise branch (:542-585):
 *   point_i = c1_i + (negate ? -1 : +1) * sum_{j<T} lambdas[j] * shares[j][i]
 *   seed_i  = SHA-256(point_i wire bytes)          (the 32-byte ChaCha20 key)
 * for i < D, where shares[j][i] = sk_j * c0_i is committee member j's
 * decryption share (SA_ClientAgent.py:397-400) and lambdas are the Lagrange
 * coefficients at 0 (util/crypto/secretsharing points_to_secret_int).  The
 * reference computes -(sum) + c1 (negate = 1).  c1 may be NULL (base = point
 * at infinity).  shares: T*D*64 bytes, term-major; lambdas: T*32 bytes.
 * points_out (D*64), seeds_out (D*32) and flags_out (D) may each be NULL.
 * Returns FLM_EINVAL if any input point is not on P-256 (flags bit 0 = c1,
 * bit 1 = a share), as pycryptodome's EccPoint constructor raises. */
int flm_ec_combine(flm_ctx *ctx, const uint8_t *c1, const uint8_t *shares, const uint8_t *lambdas, int T, int D,
                   int negate, uint8_t *points_out, uint8_t *seeds_out, uint32_t *flags_out);
/* Device-pointer form (enqueued on `stream`; flags are written, not checked).
 * The seeds can feed flm_seed_table_dev directly, so seed recovery and the
 * unmask run back to back without a host round trip. */
int flm_ec_combine_dev(flm_ctx *ctx, const uint8_t *d_c1, const uint8_t *d_shares, const uint8_t *d_lambdas, int T,
                       int D, int negate, uint8_t *d_points_out, uint8_t *d_seeds_out, uint32_t *d_flags,
                       void *stream);
/* Shamir recovery of the self-mask seeds (SA_ServiceAgent.py:506-526):
 *   seed_i = (sum_{j<T} lambdas[j] * shares[j][i] mod n).to_bytes(32, 'big')
 * for i < M (M = |U| online clients), n = the P-256 group order (ecchash.n),
 * shares[j][i] = committee member j's decrypted share of m_i as a 32-byte
 * big-endian integer (any value < 2^256), lambdas[j] < n the Lagrange
 * coefficients at 0.  shares: T*M*32 bytes, term-major.  The seeds are the
 * ChaCha20 keys of the self masks (sign -1), ready for flm_seed_table_dev. */
/* Dropout-pair masks (SA_ServiceAgent.py:587-603) as a work queue shared by two launches on
 * different CU sets, for the CU-split reconstruction (flamingo_amd/reconstruct.py).  Units of
 * (1024 slots, 16 seeds) are claimed from d_ws[0]; every claimed unit is finished, so each unit
 * is added exactly once.
 *   final_pass = 0: d_dst[l] += sum sigma PRG(seed)[l] over the units claimed before d_ws[1]
 *                   reads non-zero (d_dst and d_ws zeroed by the caller beforehand);
 *   final_pass = 1: d_dst = d_p0 + d_p1, then the remaining units are added into d_dst.
 * groups = one-wave workgroups of the launch.  Slot l uses PRG word l (prg_slot0 = 0). */
int flm_pair_units_dev(flm_ctx *ctx, const uint8_t *d_seeds, const int8_t *d_signs, int K, const uint32_t *d_p0,
                       const uint32_t *d_p1, uint32_t *d_dst, size_t L, uint32_t *d_ws, int final_pass, int groups,
                       void *stream);
/* d_ws[1] = 1 once the work enqueued before it on `stream` has finished: the stop flag of a
 * final_pass = 0 launch running on another stream. */
int flm_flag_set_dev(flm_ctx *ctx, uint32_t *d_ws, void *stream);
int flm_shamir_combine(flm_ctx *ctx, const uint8_t *shares, const uint8_t *lambdas, int T, int M,
                       uint8_t *seeds_out);
int flm_shamir_combine_dev(flm_ctx *ctx, const uint8_t *d_shares, const uint8_t *d_lambdas, int T, int M,
                           uint8_t *d_seeds_out, void *stream);
/* Batched scalar multiplication out[i] = scalars[i] * points[i]: the ECDH
 * (SA_ClientAgent.py:256-263), ElGamal (:434-447) and decryption-share
 * (:397-400) products, n independent elements per call. */
int flm_ec_mul(flm_ctx *ctx, const uint8_t *points, const uint8_t *scalars, int n, uint8_t *out, uint32_t *flags_out);
/* Hash to curve, replacing util/crypto/ecchash.hash_str_to_curve (:277-283) as the client calls
 * it for its pairwise seed group element (SA_ClientAgent.py:283-286): expand_message_xmd with
 * SHA-256 and DST "QUUX-V01-CS02-with-P256_XMD:SHA-256_SSWU_RO_" to 96 bytes (:90-133), two field
 * elements OS2IP(48 bytes) mod n (the client passes the group order as the modulus, :285;
 * hash_to_field :50-61), the reference's map_to_curve of each (:233-275), and their sum (:282).
 * flm_hash_to_curve: msgs n x 64 bytes, message i in its first lens[i] <= 64 bytes.
 * flm_hash_to_curve_decimal: the messages are str(v) for v in [v0, v0 + n) -- the client's h_ijt is
 * str(x & 0xFFFF) (:280), so v0 = 0, n = 65536 is every value it can hash: one launch.
 * out: n x 64 wire bytes; flags bit 2: the sum is the point at infinity (out zeros); FLM_EINVAL if
 * a map found no square root (flags bit 3; not expected).  _dev: device buffers, enqueued on
 * `stream`, flags written but not checked.  Square roots are a^((p+1)/4): libnum's sqrtmod root
 * order is assumed to yield that root first (the one convention not pinned by the reference). */
int flm_hash_to_curve(flm_ctx *ctx, const uint8_t *msgs, const uint32_t *lens, int n, uint8_t *out,
                      uint32_t *flags_out);
int flm_hash_to_curve_decimal(flm_ctx *ctx, uint32_t v0, int n, uint8_t *out, uint32_t *flags_out);
int flm_hash_to_curve_decimal_dev(flm_ctx *ctx, uint32_t v0, int n, uint8_t *d_out, uint32_t *d_flags, void *stream);

/* ------------------------------------------------ CU-partitioned streams */

/* A HIP stream whose kernels run only on the CUs set in `mask` (n_words
 * 32-bit words, bit i = logical CU i; hipExtStreamCreateWithCUMask).  The
 * server reconstruction (SA_ServiceAgent.py:499-605) runs its latency-bound
 * EC combine on a few CUs of one such stream while the VALU-bound self-mask
 * unmask fills the complementary set on another, so neither evicts the other's
 * workgroups.  *n_cus receives the device's CU count. */
int flm_cu_count(flm_ctx *ctx, int *n_cus);
int flm_stream_create_cu_mask(flm_ctx *ctx, const uint32_t *mask, int n_words, void **stream_out);
int flm_stream_destroy(flm_ctx *ctx, void *stream);

/* ------------------------------------------------ multi-GPU (RCCL over xGMI) */

/* The round shards two ways over G GPUs: rank r ingests clients
 * [N*r/G, N*(r+1)/G) and sums them over all L slots, regenerates every seed's
 * mask over its own slot shard [lo_r, hi_r) only, and ONE reduce-scatter of the
 * partial vectors (ncclUint32, ncclSum -- mod 2^32, so every ring order gives
 * the same bits) returns rank r the slots [lo_r, hi_r) of the reference's
 * final_sum = vec_sum_partial + cancel_vec + mi_vec (SA_ServiceAgent.py:346-350,
 * 529-605).  Shards are S = round_up(L, 1024*G) / G slots (the partial vectors
 * are S*G long); trailing ranks may own an empty shard. */
int flm_shard_bounds(size_t L, int n_ranks, int rank, size_t *lo, size_t *hi, size_t *shard_words);
int flm_client_bounds(int N, int n_ranks, int rank, int *c0, int *c1);

/* One process per GPU: rank 0 makes a 128-byte RCCL unique id, every rank
 * passes it to flm_comm_init_rank (collective: all ranks must call it), and the
 * context then owns the communicator (released by flm_free).
 * flm_reduce_scatter_dev: d_recv[0..recv_words) = rank's slice of the elementwise
 * uint32 sum over ranks of d_send[0..recv_words*n_ranks).  flm_all_gather_dev:
 * byte all-gather (d_recv = n_ranks * send_bytes), e.g. recovered pair seeds.
 * stream NULL = the HIP null stream, as for every *_dev call.  flm_comm_size
 * returns 1 when no communicator is attached (then *n_ranks = 1, *rank = 0).
 * flm_rccl_available: 1 when RCCL could be loaded (dlopen) and every symbol
 * resolved, else 0 (reason in flm_last_error(NULL)); local, not collective, so
 * every rank can agree on it before any rank enters flm_comm_init_rank.
 * flm_comm_destroy: synchronise the context's device, then ncclCommFinalize + ncclCommDestroy
 * the attached communicator (no-op without one); the context stays usable.  Call it on every
 * rank BEFORE the process's other RCCL users (torch.distributed's nccl process group) are torn
 * down -- the teardown order of distributed.shutdown -- so no library communicator is left for
 * an exit-time destructor. */
int flm_rccl_available(void);
int flm_comm_destroy(flm_ctx *ctx);
int flm_comm_unique_id(uint8_t id_out[128]);
int flm_comm_init_rank(flm_ctx *ctx, int n_ranks, int rank, const uint8_t id[128]);
int flm_comm_size(flm_ctx *ctx, int *n_ranks, int *rank);
int flm_reduce_scatter_dev(flm_ctx *ctx, const uint32_t *d_send, uint32_t *d_recv, size_t recv_words, void *stream);
int flm_all_gather_dev(flm_ctx *ctx, const void *d_send, void *d_recv, size_t send_bytes, void *stream);

/* One process, G GPUs -- the drop-in server's form: the reference server is a
 * single-threaded DES process (Kernel.py:190-271), so the group owns one
 * context per device and an RCCL clique (ncclCommInitAll).  devices: G device
 * ids, all distinct (RCCL) or all equal (loopback: the ranks share one GPU and
 * exchange through a device kernel instead of RCCL -- tests and rehearsal on a
 * one-GPU box); NULL = 0..G-1.  G <= 16.
 * flm_group_aggregate_unmask: flm_aggregate_unmask over every device: host
 * rows in (one host thread per device uploads that device's clients), out (L
 * words, host) back; synchronous.
 * flm_group_aggregate_unmask_dev: rows already resident (d_rows[r]: n_rows[r]
 * rows at row_pitch on device r; d_seeds[r]/d_signs[r] on device r); enqueues
 * every rank's round and the exchange on the ranks' context streams and
 * returns; d_shards[r] (>= S words on device r) receives slots [lo_r, hi_r).
 * The rounds run on the ranks' context streams (flm_ctx_stream(flm_group_ctx(g, r))):
 * the caller orders them after the work that produced the inputs.  A group of
 * one device needs no RCCL: its round writes the shard (the whole vector) directly.
 * flm_group_sync waits for every rank's stream.
 * flm_group_init_flags(..., FLM_GROUP_RCCL): give the group an RCCL clique even
 * when it has one device (ncclCommInitAll(1, {dev})); its rounds then take the
 * multi-GPU path -- partial buffer, grouped ncclReduceScatter, shard -- so the code
 * the 8-GPU node runs is exercised on a one-GPU box.  Refused for loopback groups
 * (RCCL does not allow two ranks on one GPU).  flm_group_has_rccl: 1 when the group
 * has a clique. */
typedef struct flm_group flm_group;
#define FLM_GROUP_RCCL 1u
int flm_group_init(flm_group **out, int n, const int *devices);
int flm_group_init_flags(flm_group **out, int n, const int *devices, unsigned flags);
int flm_group_has_rccl(const flm_group *g);
void flm_group_free(flm_group *g);
const char *flm_group_last_error(const flm_group *g);
int flm_group_size(const flm_group *g);
int flm_group_is_loopback(const flm_group *g);
flm_ctx *flm_group_ctx(flm_group *g, int rank);
int flm_group_sync(flm_group *g);
int flm_group_aggregate_unmask(flm_group *g, const uint32_t *const *rows, int N, const uint8_t *seeds,
                               const int8_t *signs, int K, size_t L, uint32_t *out);
int flm_group_aggregate_unmask_dev(flm_group *g, const uint32_t *const *d_rows, size_t row_pitch, const int *n_rows,
                                   const uint8_t *const *d_seeds, const int8_t *const *d_signs, int K, size_t L,
                                   uint32_t *const *d_shards);

/* ------------------------------------------- device-resident VECTOR ingestion */

/* The server's VECTOR bodies on the GPU(s) from arrival to the final sum: the reference keeps
 * each body in a dict on arrival (SA_ServiceAgent.py:205-210), sums them in report_process
 * (:346-350) and adds the recovered masks in reconstruction_process (:529-540, :587-605).
 * flm_store_create: on one context (ctx) or across a group (g; exactly one of them), L slots,
 *   `capacity` rows expected (the store grows past it).
 * flm_store_add: copies row[0..n) into pinned staging and returns; the DMA onto the sender's
 *   device row runs on a copy stream of the store (rows round-robin over the group's devices in
 *   arrival order; a sender that sends twice overwrites its row, like the reference's dict).
 *   n != L is remembered and makes flm_store_partial fail with the reference's message (:348-349).
 * flm_store_partial: enqueues S = sum of the stored rows after their uploads; S stays on the
 *   device(s) (slot-sharded on a group, after the group's one reduce-scatter).  Returns at once;
 *   flm_store_partial_wait blocks until S is complete and gives the device time in ms.
 * flm_store_partial_host: S to the host (inspection only; the round never needs it there).
 * flm_store_unmask: out[0..L) = S + sum_k signs[k] * PRG(seeds[k]), each device over its own
 *   slot shard (no exchange), then the one copy to the host; synchronous.
 * flm_store_reset: forget the rows (the next arrivals wait for the last partial sum's reads). */
typedef struct flm_store flm_store;
int flm_store_create(flm_store **out, flm_ctx *ctx, flm_group *g, size_t L, int capacity);
void flm_store_free(flm_store *st);
const char *flm_store_last_error(const flm_store *st);
int flm_store_count(const flm_store *st);
int flm_store_add(flm_store *st, int64_t sender, const uint32_t *row, size_t n);
int flm_store_partial(flm_store *st);
int flm_store_partial_wait(flm_store *st, float *gpu_ms);
int flm_store_partial_host(flm_store *st, uint32_t *out);
int flm_store_unmask(flm_store *st, const uint8_t *seeds, const int8_t *signs, int K, uint32_t *out);
/* Device time (ms, rank 0's stream) of the last flm_store_unmask, from its seed upload to the end of
 * its copy of final_sum to the host: the part of the call's wall time the GPU accounts for. */
int flm_store_unmask_ms(const flm_store *st, float *gpu_ms);
int flm_store_reset(flm_store *st);

/* Allocate / free page-locked host memory through HIP (for a pinned arena
 * holding client vectors, so host->device copies are DMA at full PCIe rate). */
void *flm_host_alloc(size_t bytes);
void flm_host_free(void *p);

#ifdef __cplusplus
}
#endif

#endif /* FLAMINGO_HIP_H */
