// flm_runtime.hip -- host runtime and C ABI of libflamingo_hip.so (include/flamingo_hip.h).
//
// Owns one GPU per context: its stream, grow-on-demand device buffers, the
// per-shape launch plans (work-item tables) and the error string.  The launch
// planner turns a round's shape into Items (flm_internal.h) so that every
// workgroup carries an equal share of row streaming and mask generation.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/flamingo_hip.h"
#include "flm_internal.h"

using flm::Item;
using flm::SeedRec;

namespace {

thread_local std::string g_last_error;
constexpr int kCopyStreams = 4;

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = flm::rt::grow_bytes(std::max<size_t>(bytes, 256));
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {  // no room for the slack: exactly what was asked
            (void)hipGetLastError();
            want = std::max<size_t>(bytes, 256);
            e = hipMalloc(&p, want);
        }
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
};

// One contiguous job of the planner: out[out_base + l] for l in [0, L) gets the
// sum of `nrows` rows (rows_base + r*pitch + l) and, for l in [mask_lo, mask_hi),
// seeds [k0, k0+nseeds) at PRG slot prg_slot0 + l, plus mask_bias.
struct Job {
    uint64_t out_base = 0, rows_base = 0;
    uint32_t nrows = 0;
    uint64_t L = 0;
    uint32_t k0 = 0, nseeds = 0;
    uint64_t mask_lo = 0, mask_hi = 0, prg_slot0 = 0;
    uint32_t mask_bias = 0;
    bool bias_nneg = false;
};

struct Plan {
    DevBuf items;
    int n_items = 0;
    int subtiles = 1;
    bool needs_zero = false;
    int atomics = 0;
    bool single_tile = true;  // every item writes one tile (merged accumulator legal)
    bool seed_light = false;  // mask work small next to row streaming
    // a cached plan's items are copied in on the stream of its first launch; a launch on
    // another stream waits for that copy (`ready`) until it is known to have completed
    hipEvent_t ready = nullptr;
    hipStream_t up_stream = nullptr;
    bool ready_known = true;
    // the plan's last launch on each stream it ran on (recorded by run_plan), and when it was last
    // used: the cache recycles its least recently used plan's buffers once those have completed
    std::vector<std::pair<hipStream_t, hipEvent_t>> done;
    uint64_t last_use = 0;
};

// Pinned host + device staging for the small per-call tables the *_dev entry points upload
// (packed seg + signs, signs, work items).  A slot goes back into use only once the launch that
// read its device copy has completed (its event), so a *_dev call never waits for earlier work:
// a busy pool grows (up to kStageSlots slots) instead of blocking the host.
constexpr size_t kStageSlots = 32;
struct StageSlot {
    void *host = nullptr;
    size_t cap = 0;
    DevBuf dev;
    hipEvent_t done = nullptr;
    bool busy = false;
    uint64_t last = 0;
};

using PlanKey = std::tuple<int, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t>;

// A device seed table: the per-seed schedule seed_schedule_kernel builds (SeedRec per seed) and
// its sign counts (meta), read by items_kernel / pair_units_kernel.  A context keeps a ring of
// them so that a call on one stream never rewrites a table that launches queued on other streams
// still read (the r05 cross-stream hazard): each table records its write
// stream (`w_stream`) and its last read on every stream (`readers`: one reused event per stream).
// A write followed at once by a read on the same stream (every fused call) is covered by that read's
// event; only a published table (flm_seed_table_dev: its reads may come on other streams) records
// `written` itself -- one event record per call on the hot path.  A table is rebuilt on stream s
// only once every read and write of it on other streams has completed; when all kSeedTables tables
// are still in use elsewhere, s waits on the device for the least recently used one's events
// (hipStreamWaitEvent, never a host wait).  Reads on the writing stream are in order by
// construction; a read on another stream waits for `written` first.
constexpr size_t kSeedTables = 8;
struct SeedTable {
    DevBuf recs, meta;
    hipEvent_t written = nullptr;
    bool written_valid = false;  // `written` was recorded after the last write (else a read on w_stream covers it)
    hipStream_t w_stream = nullptr;
    std::vector<std::pair<hipStream_t, hipEvent_t>> readers;
    uint64_t last_use = 0;
};

// Host copies between the caller's pageable arrays and the pinned bounce buffer (HostCopies), split
// over a context's few worker threads and the calling thread: a 4 MiB in + 4 MiB out client mask
// takes 0.34 ms of wall this way against 0.47 ms with one thread (profiles/r06_host_path_ab.txt).
// Cutting the copies into 1 MiB pieces pipelined with the DMA, with workers spinning between pieces,
// measured the same (0.34 ms) and was dropped.  Workers start lazily, on the first large copy.
class CopyPool {
  public:
    static constexpr int kWorkers = 3;                      // + the calling thread
    static constexpr size_t kMinSplit = size_t(256) << 10;  // below it the calling thread copies alone
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        work_.notify_all();
        for (auto &t : th_) t.join();
    }
    // rows x width bytes, src rows at spitch, dst rows at dpitch; returns once every byte is copied
    void copy2d(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t rows) {
        const size_t n = width * rows;
        if (n < kMinSplit) return part(dst, dpitch, src, spitch, width, 0, n);
        std::lock_guard<std::mutex> one_job(call_);  // a context's callers are one thread, a store's adds too
        if (th_.empty())
            for (int i = 0; i < kWorkers; ++i) th_.emplace_back([this, i] { run(i + 1); });
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = {dst, dpitch, src, spitch, width, n};
            pending_ = kWorkers;
            ++gen_;
        }
        work_.notify_all();
        slice(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [this] { return pending_ == 0; });
    }

  private:
    struct Job {
        void *dst;
        size_t dpitch;
        const void *src;
        size_t spitch, width, n;
    };
    // bytes [b, e) of the packed rows x width range
    static void part(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t b, size_t e) {
        while (b < e) {
            const size_t r = b / width, c = b % width, m = std::min(width - c, e - b);
            std::memcpy(static_cast<uint8_t *>(dst) + r * dpitch + c, static_cast<const uint8_t *>(src) + r * spitch + c, m);
            b += m;
        }
    }
    void slice(int i) {  // slice i of kWorkers + 1, 4 KiB-aligned bounds
        const size_t per = ((job_.n + kWorkers) / (kWorkers + 1) + 4095) / 4096 * 4096;
        const size_t b = std::min(job_.n, per * i), e = std::min(job_.n, b + per);
        part(job_.dst, job_.dpitch, job_.src, job_.spitch, job_.width, b, e);
    }
    void run(int i) {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> l(m_);
                work_.wait(l, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            slice(i);
            bool last;
            {
                std::lock_guard<std::mutex> g(m_);
                last = --pending_ == 0;
            }
            if (last) done_.notify_one();
        }
    }
    std::mutex call_, m_;
    std::condition_variable work_, done_;
    std::vector<std::thread> th_;
    Job job_{};
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};

}  // namespace

// flm_last_plan's variant for a round run by small_round_kernel (items = its workgroups)
constexpr int kSmallRoundVariant = 100;
// flm_last_plan's variant after a PRG expansion by prg_expand_kernel (items = its workgroups)
constexpr int kExpandVariant = 101;

struct flm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    DevBuf rows, out, seeds, signs, bytes_in, bytes_out;
    std::vector<SeedTable *> tables;  // ring of device seed tables (SeedTable)
    SeedTable *cur_table = nullptr;   // the table the last seed-schedule / small-round launch wrote
    SeedTable *pub_table = nullptr;   // the table flm_seed_table_dev published for flm_aggregate_dev
    DevBuf small_meta;                // sign counts of the one-launch small round (no seed table)
    bool last_small = false;          // the last sign counts came from a small round (flm_check_signs)
    uint64_t table_clock = 0;
    std::vector<StageSlot *> slots;  // staging pool of the *_dev uploads (StageSlot)
    uint64_t slot_clock = 0;
    DevBuf ec_in, ec_base, ec_scal, ec_jac, ec_out, ec_dig, ec_flags;  // P-256 batches
    // pinned staging ring for pageable host rows: two buffers, each reused once
    // the DMA that read it has completed (event per buffer)
    void *stage[2] = {nullptr, nullptr};
    size_t stage_cap = 0;
    hipEvent_t stage_done[2] = {nullptr, nullptr};
    // host->device streams for page-locked rows (several SDMA engines)
    hipStream_t copy[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t copy_done[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t copy_start = nullptr;
    std::map<PlanKey, Plan *> plans;
    uint64_t plan_clock = 0;
    int last_items = 0, last_tile = 0, last_atomics = 0, last_variant = 0;
    int table_k = -1;  // seeds in the published device seed table (pub_table), -1 = none
    int tune_variant = -1;   // items_kernel variant, -1 = auto
    int tune_subtiles = 0;   // aggregate sub-tiles per workgroup, 0 = auto
    int tune_min_items = 1024;  // planner target for work items per aggregate launch (kDefaultMinItems)
    int tune_ec_threads = 64;   // ec_mul workgroup size (64/128/256; 64 measured best, 3.29 vs 3.43 ms)
    int tune_ec_waves = 1;      // ec_mul register budget as min waves/SIMD (1 = uncapped, 4, 8)
    int tune_ec_spread = 0;     // KiB of LDS reserved per 64-lane EC workgroup (0 = none): caps EC waves per CU
                                // so a CU-masked dispatch spreads them one per SIMD instead of packing two
    int tune_ec_terms = 1;      // combine terms per lane (1, 2, 4: Straus, shared doublings)
    int tune_ec_coop = -1;      // 1: four waves per 64 scalar multiplications (ec_mul_coop_kernel); 2: four
                                // waves per 4, each element on a 16-lane row (ec_mul_row_kernel); 0: one
                                // lane each; -1 (auto): cooperative when the batch fits one pass of the chip
    int tune_small = 1;      // one-launch small_round_kernel: 0 never, 1 small rounds (auto), 2 whenever legal
    int tune_pairing = 1;    // rows/masks on different tiles: 0 interleaved items, 1 dual-tile items (measured 1.97 vs 3.46 ms),
                             // 2 same-tile window items (plan_window_same; 0.228 vs 0.188 ms at G = 8, r02_ab_window_same.log)
    int tune_expand_waves = 128;  // prg_expand_kernel one-wave workgroups per CU: 16 / 32 / 64 / 128 -> 1.57 / 1.43 /
                                  // 1.37 / 1.34 ms at K = 962, L = 2^20 (profiles/r06_expand_probe_waves*.log); ~9 fit
                                  // a SIMD at once, the rest queue behind them and even out the runs' ends
    int n_cus = 0;               // the device's CU count (flm_init)
    void *bounce = nullptr;      // pinned bounce buffer of the host-pointer entry points (HostCopies)
    void *bounce_dev = nullptr;  // its address for kernels (hipHostGetDevicePointer)
    size_t bounce_cap = 0;
    CopyPool copies;             // the CPU side of HostCopies' bounce-buffer copies
    void *comm = nullptr;    // RCCL communicator state (flm_comm.hip), owned by the context
};

namespace {

int fail(flm_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_last_error = buf;
    return code;
}

// Select the context's device for the rest of this entry point; the caller's comes back on return.
#define FLM_ON_DEVICE(ctx)                 \
    flm::rt::DeviceScope dev_scope_;       \
    FLM_HIP((ctx), dev_scope_.set((ctx)->device))

#define FLM_HIP(ctx, expr)                                                                            \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail((ctx), FLM_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                    \
    } while (0)

inline uint64_t round_up(uint64_t v, uint64_t m) { return (v + m - 1) / m * m; }

// A staging slot of >= `bytes` that no queued work reads any more (StageSlot).  The host
// waits only when all kStageSlots slots are still queued: then for the oldest.
StageSlot *stage_acquire(flm_ctx *ctx, size_t bytes, int *rc) {
    StageSlot *best = nullptr, *free_small = nullptr, *oldest = nullptr;
    for (StageSlot *s : ctx->slots) {
        if (s->busy) {
            const hipError_t q = hipEventQuery(s->done);
            if (q == hipSuccess) s->busy = false;
            else if (q != hipErrorNotReady) (void)hipGetLastError();
        }
        if (s->busy) {
            if (!oldest || s->last < oldest->last) oldest = s;
        } else if (s->cap >= bytes) {
            if (!best || s->cap < best->cap) best = s;
        } else if (!free_small) {
            free_small = s;
        }
    }
    if (!best) {
        if (ctx->slots.size() < kStageSlots) {
            best = new StageSlot();
            if (hipEventCreateWithFlags(&best->done, hipEventDisableTiming) != hipSuccess) {
                delete best;
                *rc = fail(ctx, FLM_EHIP, "staging slot: hipEventCreate failed");
                return nullptr;
            }
            ctx->slots.push_back(best);
        } else if (free_small) {
            best = free_small;
        } else {
            if (hipEventSynchronize(oldest->done) != hipSuccess) {
                *rc = fail(ctx, FLM_EHIP, "staging slot: hipEventSynchronize failed");
                return nullptr;
            }
            oldest->busy = false;
            best = oldest;
        }
        if (best->cap < bytes) {
            const size_t want = std::max<size_t>(round_up(bytes, 4096), 4096);
            if (best->host) (void)hipHostFree(best->host);
            best->host = nullptr;
            best->cap = 0;
            hipError_t e = hipHostMalloc(&best->host, want, hipHostMallocDefault);
            if (e == hipSuccess) e = best->dev.reserve(want);
            if (e != hipSuccess) {
                *rc = fail(ctx, FLM_ENOMEM, "staging slot of %zu bytes: %s", want, hipGetErrorString(e));
                return nullptr;
            }
            best->cap = want;
        }
    }
    best->last = ++ctx->slot_clock;
    *rc = 0;
    return best;
}

// A few slots made at flm_init, so the first *_dev calls of a context do not pay the pinned and
// device allocations (c2's client masks: 0.196 ms with a slot allocated in the call, 0.065 ms without).
constexpr int kStagePrealloc = 4;
constexpr size_t kStagePreallocBytes = 256u << 10;

void stage_prealloc(flm_ctx *ctx) {
    for (int i = 0; i < kStagePrealloc; ++i) {
        auto *s = new StageSlot();
        if (hipEventCreateWithFlags(&s->done, hipEventDisableTiming) != hipSuccess ||
            hipHostMalloc(&s->host, kStagePreallocBytes, hipHostMallocDefault) != hipSuccess ||
            s->dev.reserve(kStagePreallocBytes) != hipSuccess) {
            if (s->host) (void)hipHostFree(s->host);
            s->dev.release();
            if (s->done) (void)hipEventDestroy(s->done);
            delete s;
            (void)hipGetLastError();
            return;  // the pool fills lazily instead
        }
        s->cap = kStagePreallocBytes;
        ctx->slots.push_back(s);
    }
}

// Copy the slot's first `bytes` host bytes to its device buffer on `s`.
hipError_t stage_upload(StageSlot *slot, size_t bytes, hipStream_t s) {
    return bytes ? hipMemcpyAsync(slot->dev.p, slot->host, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
}

// The slot is free again once the work enqueued on `s` so far (its readers) has completed.
hipError_t stage_commit(StageSlot *slot, hipStream_t s) {
    hipError_t e = hipEventRecord(slot->done, s);
    if (e == hipSuccess) slot->busy = true;
    return e;
}

// ------------------------------------------------------------------ planner
// Split a job into row units (tiles x row parts) and mask units (tiles x seed
// parts) of equal weight, then pair unit i of each list into one Item, so one
// workgroup streams rows (HBM) while it generates masks (VALU).
struct Unit {
    uint64_t tile;  // out slot of the tile start (relative to job)
    uint32_t a, n;  // row or seed sub-range
    uint32_t valid;
    uint32_t part;
};

void plan_job(const Job &j, uint64_t pitch, int subtiles, int parts_r, int parts_m, bool dual_tile,
              std::vector<Item> &items, bool &needs_zero, int &atomics, bool &single_tile) {
    const uint64_t W = (uint64_t)flm::kWaveSlots * subtiles;
    std::vector<Unit> R, M;
    if (j.nrows > 0 && j.L > 0) {
        for (uint64_t t = 0; t < j.L; t += W)
            for (int p = 0; p < parts_r; ++p) {
                uint32_t a = (uint32_t)((uint64_t)j.nrows * p / parts_r);
                uint32_t b = (uint32_t)((uint64_t)j.nrows * (p + 1) / parts_r);
                if (b > a) R.push_back({t, a, b - a, (uint32_t)std::min<uint64_t>(W, j.L - t), (uint32_t)p});
            }
    }
    if (j.nseeds > 0 && j.mask_hi > j.mask_lo) {
        for (uint64_t t = j.mask_lo; t < j.mask_hi; t += W)
            for (int p = 0; p < parts_m; ++p) {
                uint32_t a = (uint32_t)((uint64_t)j.nseeds * p / parts_m);
                uint32_t b = (uint32_t)((uint64_t)j.nseeds * (p + 1) / parts_m);
                if (b > a)
                    M.push_back({t, a, b - a, (uint32_t)std::min<uint64_t>(W, j.mask_hi - t), (uint32_t)p});
            }
    }
    // A tile written by exactly one Item is stored; otherwise every contributor
    // adds atomically into a zeroed output.  Rows and masks share one Item per
    // tile ("same tile") in whole-vector rounds whose rows and seeds are cut into
    // the same number of parts: unit i of each list then covers the same tile, and
    // the item keeps the merged single-accumulator kernel (atomic when parts > 1).
    const bool both = !R.empty() && !M.empty();
    bool paired_same = both && parts_r == parts_m && j.mask_lo == 0 && j.mask_hi == j.L && R.size() == M.size();
    for (size_t i = 0; paired_same && i < R.size(); ++i) paired_same = R[i].tile == M[i].tile;
    const bool atomic = parts_r > 1 || parts_m > 1 || (both && !paired_same);
    if (atomic) needs_zero = true;
    if (R.empty() && (j.mask_lo > 0 || j.mask_hi < j.L || M.empty())) needs_zero = true;
    atomics |= atomic ? 1 : 0;

    // Rows and masks on different tiles: either pair them into dual-tile items
    // (one workgroup streams rows of tile A while generating masks of tile B), or
    // emit single-kind items interleaved R0 M0 R1 M1 ... so row and mask
    // workgroups share CUs and each can use the merged-accumulator kernel.
    if (both && !paired_same && !dual_tile) {
        const size_t n2 = std::max(R.size(), M.size());
        for (size_t i = 0; i < n2; ++i) {
            if (i < R.size()) {
                Item it;
                std::memset(&it, 0, sizeof it);
                const Unit &u = R[i];
                it.flags = flm::kHasRows | flm::kRowAtomic;
                it.row_in = j.rows_base + (uint64_t)u.a * pitch + u.tile;
                it.nrows = u.n;
                it.row_out = j.out_base + u.tile;
                it.row_valid = u.valid;
                items.push_back(it);
            }
            if (i < M.size()) {
                Item it;
                std::memset(&it, 0, sizeof it);
                const Unit &u = M[i];
                it.flags = flm::kHasMask | flm::kMaskAtomic;
                it.k0 = j.k0 + u.a;
                it.nseeds = u.n;
                it.mask_out = j.out_base + u.tile;
                it.mask_ctr = (j.prg_slot0 + u.tile) / 16;
                it.mask_valid = u.valid;
                if (u.part == 0) {
                    it.mask_bias = j.mask_bias;
                    if (j.bias_nneg) it.flags |= flm::kMaskBiasNneg;
                }
                items.push_back(it);
            }
        }
        return;
    }
    if (both && !paired_same) single_tile = false;

    const size_t n = std::max(R.size(), M.size());
    for (size_t i = 0; i < n; ++i) {
        Item it;
        std::memset(&it, 0, sizeof it);
        if (i < R.size()) {
            const Unit &u = R[i];
            it.flags |= flm::kHasRows | (atomic ? flm::kRowAtomic : 0u);
            it.row_in = j.rows_base + (uint64_t)u.a * pitch + u.tile;
            it.nrows = u.n;
            it.row_out = j.out_base + u.tile;
            it.row_valid = u.valid;
        }
        if (i < M.size()) {
            const Unit &u = M[i];
            it.flags |= flm::kHasMask | (atomic ? flm::kMaskAtomic : 0u);
            it.k0 = j.k0 + u.a;
            it.nseeds = u.n;
            it.mask_out = j.out_base + u.tile;
            it.mask_ctr = (j.prg_slot0 + u.tile) / 16;
            it.mask_valid = u.valid;
            if (u.part == 0) {  // per-slot constants are added exactly once
                it.mask_bias = j.mask_bias;
                if (j.bias_nneg) it.flags |= flm::kMaskBiasNneg;
            }
            if (paired_same && i < R.size() && R[i].tile == u.tile) it.flags |= flm::kSameTile;
        }
        items.push_back(it);
    }
}

int choose_parts(uint64_t tiles_r, uint64_t tiles_m, uint32_t nrows, uint32_t nseeds, int &pr, int &pm,
                 uint64_t kTarget = 1024) {
    // Balance mask units against row units, then split both until the grid
    // has a few workgroups per CU (16 waves each), keeping >= 16 rows/seeds
    // per item so every wave of a workgroup has work.
    pr = 1;
    pm = 1;
    if (tiles_r && tiles_m && tiles_r > tiles_m) pm = (int)std::min<uint64_t>(nseeds, (tiles_r + tiles_m - 1) / tiles_m);
    if (tiles_r && tiles_m && tiles_m > tiles_r) pr = (int)std::min<uint64_t>(nrows, (tiles_m + tiles_r - 1) / tiles_r);
    auto units = [&] { return std::max(tiles_r * pr, tiles_m * pm); };
    while (units() < kTarget) {
        bool grew = false;
        if (tiles_r && (uint64_t)pr * 2 * 16 <= nrows) { pr *= 2; grew = true; }
        if (tiles_m && (uint64_t)pm * 2 * 16 <= nseeds) { pm *= 2; grew = true; }
        if (!grew) break;
    }
    return 0;
}

int pick_variant(const flm_ctx *ctx, const Plan &plan) {
    int v = ctx->tune_variant;
    // measured (tools/ab/ab_items.py, profiles/r01_ab_items*.log): merged accumulator
    // fastest where legal (seeds spread over the rows when seed-light), block next
    if (v < 0)
        v = plan.single_tile ? (plan.seed_light ? flm::kVarMergedSpread : flm::kVarMerged)
                             : (plan.seed_light ? flm::kVarBlockSpread : flm::kVarBlock);
    if (!plan.single_tile && v >= flm::kVarMerged) v = (v == flm::kVarMergedSpread || v == flm::kVarBlockSpread)
                                                          ? flm::kVarBlockSpread : flm::kVarBlock;
    return v;
}

// The items go through a staging slot on `s` and the plan records `ready` for launches on
// other streams (run_plan).
int upload_plan(flm_ctx *ctx, Plan &plan, std::vector<Item> &items, hipStream_t s) {
    plan.n_items = (int)items.size();
    if (items.empty()) return 0;
    const size_t bytes = items.size() * sizeof(Item);
    FLM_HIP(ctx, plan.items.reserve(bytes));
    int rc = 0;
    StageSlot *slot = stage_acquire(ctx, bytes, &rc);
    if (!slot) return rc;
    std::memcpy(slot->host, items.data(), bytes);
    FLM_HIP(ctx, hipMemcpyAsync(plan.items.p, slot->host, bytes, hipMemcpyHostToDevice, s));
    FLM_HIP(ctx, stage_commit(slot, s));
    if (!plan.ready) FLM_HIP(ctx, hipEventCreateWithFlags(&plan.ready, hipEventDisableTiming));
    FLM_HIP(ctx, hipEventRecord(plan.ready, s));
    plan.up_stream = s;
    plan.ready_known = false;
    return 0;
}

void plan_free(Plan *plan) {
    plan->items.release();
    if (plan->ready) (void)hipEventDestroy(plan->ready);
    for (auto &d : plan->done) (void)hipEventDestroy(d.second);
    delete plan;
}

constexpr size_t kPlanCache = 64;        // launch plans kept per context (shapes)
constexpr int kDefaultMinItems = 1024;   // flm_set_tuning("min_items") default
constexpr uint64_t kUnsplitTiles = 1024;  // 4 tiles per MI355X CU: from this many a whole-vector round is not split
constexpr uint64_t kSplitItems = 2048;    // item target of a split whole-vector round (8 per CU)
constexpr int kWindowItems = 512;         // item target of a windowed (slot-sharded) round: 2 per CU

// A rank of the slot-sharded round as same-tile items (pairing 2).  The shard's 1024-slot tiles
// carry rows AND seeds, cut into P matching parts (part p of a tile: rows [N p/P, N (p+1)/P) and
// seeds [K p/P, K (p+1)/P), atomics when P > 1); every other tile is one rows-only item, spread
// evenly between the heavy items so that row streaming runs beside the ChaCha work from the
// start.  Every item writes one tile, so the merged single-accumulator kernel runs (63 VGPRs,
// 8 waves/SIMD) instead of the dual-tile kernel (104 VGPRs, 4 waves/SIMD).  Measured slower than
// the dual-tile items at G = 2 / 4 / 8 (0.78 / 0.42 / 0.228 ms against 0.69 / 0.36 / 0.188 ms,
// profiles/r02_ab_window_same.log): a tuning option (flm_set_tuning "pairing" 2), not the default.
void plan_window_same(uint64_t pitch, int N, int K, uint64_t L, uint64_t mask_lo, uint64_t mask_hi,
                      uint64_t prg_slot0, uint64_t heavy_target, std::vector<Item> &items, Plan &plan) {
    const uint64_t W = flm::kWaveSlots;
    const uint64_t tm = (mask_hi - mask_lo + W - 1) / W;
    uint64_t P = tm ? (heavy_target + tm - 1) / tm : 1;
    while (P > 1 && (uint64_t)K < 16 * P) P /= 2;  // >= 16 seeds per part: every wave has work
    if (P < 1) P = 1;
    std::vector<Item> heavy, light;
    for (uint64_t t = mask_lo; t < mask_hi; t += W) {
        const uint32_t valid = (uint32_t)std::min<uint64_t>(W, mask_hi - t);
        for (uint64_t p = 0; p < P; ++p) {
            Item it;
            std::memset(&it, 0, sizeof it);
            const uint32_t ra = (uint32_t)((uint64_t)N * p / P), rb = (uint32_t)((uint64_t)N * (p + 1) / P);
            const uint32_t sa = (uint32_t)((uint64_t)K * p / P), sb = (uint32_t)((uint64_t)K * (p + 1) / P);
            const uint32_t at = P > 1 ? (flm::kRowAtomic | flm::kMaskAtomic) : 0u;
            if (rb > ra) {
                it.flags |= flm::kHasRows | at;
                it.row_in = (uint64_t)ra * pitch + t;
                it.nrows = rb - ra;
                it.row_out = t;
                it.row_valid = valid;
            }
            if (sb > sa) {
                it.flags |= flm::kHasMask | at | (rb > ra ? flm::kSameTile : 0u);
                it.k0 = sa;
                it.nseeds = sb - sa;
                it.mask_out = t;
                it.mask_ctr = (prg_slot0 + t) / 16;
                it.mask_valid = valid;
                if (p == 0) it.flags |= flm::kMaskBiasNneg;
            }
            if (it.flags) heavy.push_back(it);
        }
    }
    auto rows_only = [&](uint64_t a, uint64_t b) {
        for (uint64_t t = a; t < b; t += W) {
            Item it;
            std::memset(&it, 0, sizeof it);
            it.flags = flm::kHasRows;
            it.row_in = t;
            it.nrows = (uint32_t)N;
            it.row_out = t;
            it.row_valid = (uint32_t)std::min<uint64_t>(W, b - t);
            light.push_back(it);
        }
    };
    rows_only(0, mask_lo);
    rows_only(mask_hi, L);
    // interleave: light item j goes after heavy item floor((j + 1) * H / (Lt + 1))
    const size_t H = heavy.size(), Lt = light.size();
    items.reserve(H + Lt);
    size_t j = 0;
    for (size_t h = 0; h < H; ++h) {
        items.push_back(heavy[h]);
        while (j < Lt && (j + 1) * H <= (h + 1) * (Lt + 1)) items.push_back(light[j++]);
    }
    while (j < Lt) items.push_back(light[j++]);
    plan.subtiles = 1;
    plan.seed_light = false;
    plan.single_tile = true;
    plan.needs_zero = P > 1;
    plan.atomics = P > 1 ? 1 : 0;
}

// Host-only planning of one aggregate round (no device state): fills `items`
// and the plan's flags.  Shared by aggregate_plan and the flm_plan_aggregate
// diagnostic entry point.
void build_aggregate_items(int tune_subtiles, int pairing, uint64_t pitch, int N, int K, uint64_t L, uint64_t mask_lo,
                           uint64_t mask_hi, uint64_t prg_slot0, std::vector<Item> &items, Plan &plan,
                           int min_items = 1024) {
    // ChaCha-heavy rounds keep 1024-slot tiles (16 waves split one tile's seeds);
    // row-streaming-heavy rounds (few seeds per slot) prefer 4 sub-tiles per
    // workgroup: 4096-slot tiles, fewer LDS combines (measured 5.77 vs 5.26 TB/s).
    const bool seed_light = (uint64_t)K * (mask_hi - mask_lo) * 2 < (uint64_t)N * L;
    // A rank of the slot-sharded round (rows over all of L, masks over a window): 4096-slot
    // tiles and kWindowItems items, one generation of workgroups on the chip.  One rank of the
    // strong-scaled c4 round, G = 8: 0.179 -> 0.169 ms; G = 4: 0.364 -> 0.350-0.360 ms; G = 2 the
    // same (profiles/r02_ab_strong_plan.log).
    const bool windowed = N > 0 && K > 0 && (mask_lo > 0 || mask_hi < L);
    if (pairing == 2 && windowed && !seed_light && tune_subtiles <= 0) {
        plan_window_same(pitch, N, K, L, mask_lo, mask_hi, prg_slot0, (uint64_t)min_items, items, plan);
        return;
    }
    const int subtiles = tune_subtiles > 0 ? tune_subtiles : ((seed_light || windowed) ? 4 : 1);
    const uint64_t W = (uint64_t)flm::kWaveSlots * subtiles;
    Job j;
    j.nrows = (uint32_t)N;
    j.L = L;
    j.nseeds = (uint32_t)K;
    j.mask_lo = mask_lo;
    j.mask_hi = mask_hi;
    j.prg_slot0 = prg_slot0;
    j.bias_nneg = true;
    const uint64_t tr = N > 0 ? (L + W - 1) / W : 0;
    const uint64_t tm = (K > 0 && mask_hi > mask_lo) ? (mask_hi - mask_lo + W - 1) / W : 0;
    int pr, pm;
    if (!seed_light && min_items == kDefaultMinItems && mask_lo == 0 && mask_hi == L && tr == tm && tm > 0) {
        // A whole-vector ChaCha-heavy round: rows and seeds are cut into the same number of parts P,
        // so part p of both lands in one item and the merged single-accumulator kernel runs
        // (plan_job).  From kUnsplitTiles tiles (4 per CU: c4 / c5, 1024 tiles) one item per tile --
        // no atomics, no zero-fill; 2048 items measured no faster there.  Fewer tiles (c3, N=1024,
        // L=2^18: 256 tiles) are split until kSplitItems items: 0.389 ms at P=8 against 0.414 ms
        // unsplit (one 4-wave/SIMD generation) and 0.410 at P=2 (profiles/r02_ab_split.log).
        pr = pm = 1;
        while (tm < kUnsplitTiles && tm * (uint64_t)pr < kSplitItems && (uint64_t)pr * 2 * 16 <= (uint64_t)N &&
               (uint64_t)pr * 2 * 16 <= (uint64_t)K)
            pr = pm = pr * 2;
    } else {
        const int target = (windowed && !seed_light && tune_subtiles <= 0 && min_items == kDefaultMinItems)
                               ? kWindowItems : min_items;
        choose_parts(tr, tm, (uint32_t)N, (uint32_t)K, pr, pm, (uint64_t)target);
    }
    plan.subtiles = subtiles;
    plan.seed_light = seed_light;
    plan_job(j, pitch, subtiles, pr, pm, pairing != 0, items, plan.needs_zero, plan.atomics, plan.single_tile);
}

Plan *aggregate_plan(flm_ctx *ctx, uint64_t pitch, int N, int K, uint64_t L, uint64_t mask_lo, uint64_t mask_hi,
                     uint64_t prg_slot0, hipStream_t s, int *rc) {
    PlanKey key{ctx->tune_subtiles + 100 * ctx->tune_pairing + 1000 * ctx->tune_min_items, pitch, (uint64_t)N,
                (uint64_t)K, L, mask_lo, mask_hi, prg_slot0};
    auto f = ctx->plans.find(key);
    if (f != ctx->plans.end()) {
        f->second->last_use = ++ctx->plan_clock;
        *rc = 0;
        return f->second;
    }
    // A full cache (kPlanCache shapes; a server whose seed count changes every round makes a new
    // shape every round) hands its least recently used plan's item buffer and events to the new
    // plan once that plan's last launch has completed -- no hipFree, which would wait for the
    // whole device, and no hipMalloc while the buffer is big enough.
    Plan *plan = nullptr;
    if (ctx->plans.size() >= kPlanCache) {
        auto lru = ctx->plans.begin();
        for (auto it = ctx->plans.begin(); it != ctx->plans.end(); ++it)
            if (it->second->last_use < lru->second->last_use) lru = it;
        Plan *old = lru->second;
        hipError_t e = hipSuccess;
        for (auto &d : old->done)  // long done, as a rule
            if (e == hipSuccess) e = hipEventSynchronize(d.second);
        if (e == hipSuccess && old->ready) e = hipEventSynchronize(old->ready);
        if (e != hipSuccess) {
            *rc = fail(ctx, FLM_EHIP, "plan cache: waiting for a recycled plan failed: %s", hipGetErrorString(e));
            return nullptr;
        }
        ctx->plans.erase(lru);
        plan = new Plan();
        plan->items = old->items;  // the buffers move; the old Plan object goes
        plan->ready = old->ready;
        plan->done.swap(old->done);  // (stream, event) pairs: the events are reused per stream
        delete old;
    } else {
        plan = new Plan();
    }
    std::vector<Item> items;
    build_aggregate_items(ctx->tune_subtiles, ctx->tune_pairing, pitch, N, K, L, mask_lo, mask_hi, prg_slot0, items,
                          *plan, ctx->tune_min_items);
    *rc = upload_plan(ctx, *plan, items, s);
    if (*rc) { plan_free(plan); return nullptr; }
    plan->last_use = ++ctx->plan_clock;
    ctx->plans[key] = plan;
    return plan;
}

bool signs_ok(const int8_t *signs, int K, int *nneg) {
    int n = 0;
    for (int k = 0; k < K; ++k) {
        if (signs[k] == -1) ++n;
        else if (signs[k] != 1) return false;
    }
    if (nneg) *nneg = n;
    return true;
}

int check_range(flm_ctx *ctx, uint64_t slot_hi) {
    if (slot_hi > (1ull << 36))
        return fail(ctx, FLM_ERANGE, "PRG slot range ends at %llu > 2^36 (block counter high word must stay 0)",
                    (unsigned long long)slot_hi);
    return 0;
}

// Workgroup width B (16*B slots) of the one-launch small-round kernel for this round, or 0 to
// take the seed-schedule + items_kernel path.  Auto (tune_small 1): rounds whose rows and mask
// words are both <= 2^22 (c2: 2^21 each), where items_kernel's fixed ~10 us dominates.
int small_round_width(const flm_ctx *ctx, int N, int K, uint64_t L, uint64_t mask_lo, uint64_t mask_hi) {
    if (ctx->tune_small == 0) return 0;
    if (mask_lo % 16 || (mask_hi % 16 && mask_hi != L)) return 0;
    if (ctx->tune_small == 1 && ((uint64_t)N * L > (1ull << 22) || (uint64_t)K * (mask_hi - mask_lo) > (1ull << 22)))
        return 0;
    // 2 blocks per 256-thread workgroup keeps 128 seeds per pass (c2: one pass, every lane busy);
    // longer vectors take 4 (64 slots) so the grid stays near 1024 workgroups
    return L >= (1ull << 16) ? 4 : 2;
}

// True when the event has completed (or was never recorded); false while it is pending.
bool event_done(hipEvent_t e) {
    if (!e) return true;
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return true;
    (void)hipGetLastError();  // hipErrorNotReady (an error status would surface at the next launch)
    return false;
}

// No read or write of `t` on a stream other than s is still pending: s may rewrite it at once.
bool table_free_on(const SeedTable *t, hipStream_t s) {
    if (t->w_stream != s && t->written_valid && !event_done(t->written)) return false;
    for (const auto &r : t->readers)
        if (r.first != s && !event_done(r.second)) return false;
    return true;
}

// A seed table stream s may overwrite, grown to hold K records and `meta_words` sign-count words
// (SeedTable).  The write launch follows on s; table_written() records it.
SeedTable *table_acquire(flm_ctx *ctx, int K, size_t meta_words, hipStream_t s, int *rc) {
    SeedTable *t = nullptr;
    for (SeedTable *c : ctx->tables)  // the least recently used of the tables s may rewrite at once
        if (table_free_on(c, s) && (!t || c->last_use < t->last_use)) t = c;
    if (!t && ctx->tables.size() < kSeedTables) {
        t = new SeedTable();
        if (hipEventCreateWithFlags(&t->written, hipEventDisableTiming) != hipSuccess) {
            delete t;
            *rc = fail(ctx, FLM_EHIP, "seed table: hipEventCreate failed");
            return nullptr;
        }
        ctx->tables.push_back(t);
    }
    if (!t) {  // every table is still in use on other streams: s waits (on the device) for the oldest
        t = ctx->tables.front();
        for (SeedTable *c : ctx->tables)
            if (c->last_use < t->last_use) t = c;
        hipError_t e = hipSuccess;
        if (t->w_stream != s && t->written_valid) e = hipStreamWaitEvent(s, t->written, 0);
        for (const auto &r : t->readers)
            if (e == hipSuccess && r.first != s) e = hipStreamWaitEvent(s, r.second, 0);
        if (e != hipSuccess) {
            *rc = fail(ctx, FLM_EHIP, "seed table: hipStreamWaitEvent failed: %s", hipGetErrorString(e));
            return nullptr;
        }
    }
    // growing frees the old buffer: hipFree waits for the device, so no pending launch reads it
    hipError_t e = t->recs.reserve(std::max<size_t>(1, (size_t)K) * sizeof(SeedRec));
    if (e == hipSuccess) e = t->meta.reserve(sizeof(uint32_t) * std::max<size_t>(4, meta_words));
    if (e != hipSuccess) {
        *rc = fail(ctx, FLM_ENOMEM, "seed table of %d seeds: %s", K, hipGetErrorString(e));
        return nullptr;
    }
    t->last_use = ++ctx->table_clock;
    if (ctx->pub_table == t) {  // never left published while it holds other seeds
        ctx->pub_table = nullptr;
        ctx->table_k = -1;
    }
    *rc = 0;
    return t;
}

// The table's write launch has been enqueued on s.  record: mark it with `written` (a published
// table); otherwise the caller's read launch on s follows and table_read() covers both -- or, when
// the read cannot be enqueued, table_cover() records `written` after all.
hipError_t table_written(flm_ctx *ctx, SeedTable *t, hipStream_t s, bool record) {
    t->w_stream = s;
    t->written_valid = record;
    ctx->cur_table = t;
    ctx->last_small = false;
    return record ? hipEventRecord(t->written, s) : hipSuccess;
}

void table_cover(SeedTable *t, hipStream_t s) {
    if (t && !t->written_valid && hipEventRecord(t->written, s) == hipSuccess) t->written_valid = true;
    (void)hipGetLastError();
}

// Before a launch on s that reads t: order it after t's write when that ran on another stream.
hipError_t table_before_read(SeedTable *t, hipStream_t s) {
    if (t->w_stream == s) return hipSuccess;
    if (t->written_valid) return event_done(t->written) ? hipSuccess : hipStreamWaitEvent(s, t->written, 0);
    for (const auto &r : t->readers)  // (not reached: a write recorded no event only when a read followed)
        if (r.first == t->w_stream) return hipStreamWaitEvent(s, r.second, 0);
    return hipSuccess;
}

// A launch that reads t has been enqueued on s: record it as the table's last read on s (one event
// per stream, reused; entries of finished streams are pruned as in Plan::done).
hipError_t table_read(SeedTable *t, hipStream_t s) {
    hipEvent_t *ev = nullptr;
    for (auto &r : t->readers)
        if (r.first == s) ev = &r.second;
    if (!ev) {
        if (t->readers.size() >= 8) {
            std::vector<std::pair<hipStream_t, hipEvent_t>> keep;
            for (auto &r : t->readers) {
                if (event_done(r.second)) (void)hipEventDestroy(r.second);
                else keep.push_back(r);
            }
            t->readers.swap(keep);
        }
        hipEvent_t e = nullptr;
        const hipError_t c = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (c != hipSuccess) return c;
        t->readers.emplace_back(s, e);
        ev = &t->readers.back().second;
    }
    return hipEventRecord(*ev, s);
}

void table_free(SeedTable *t) {
    if (t->written && t->written_valid) (void)hipEventSynchronize(t->written);
    for (auto &r : t->readers) (void)hipEventSynchronize(r.second);
    t->recs.release();
    t->meta.release();
    if (t->written) (void)hipEventDestroy(t->written);
    for (auto &r : t->readers) (void)hipEventDestroy(r.second);
    delete t;
}

// The one-launch small round builds no seed table: it reads the raw seeds and only WRITES its sign
// counts, into a buffer of its own (flm_check_signs reads them; small rounds racing on several
// streams can only race on that diagnostic, never on a sum).  It unpublishes the table like every
// other entry point that takes seeds, so flm_aggregate_dev cannot pair with its seeds.  No event:
// c2's whole round is ~7 us of host time.
int run_small_round(flm_ctx *ctx, int B, const uint32_t *d_rows, uint64_t pitch, int N, const uint8_t *d_seeds,
                    const int8_t *d_signs, int K, uint64_t L, uint64_t mask_lo, uint64_t mask_hi, uint64_t prg_slot0,
                    uint32_t *d_out, hipStream_t s) {
    FLM_HIP(ctx, ctx->small_meta.reserve(4 * sizeof(uint32_t)));
    FLM_HIP(ctx, flm::launch_small_round(B, d_rows, pitch, N, d_seeds, d_signs, K, L, mask_lo, mask_hi,
                                         (uint32_t)(prg_slot0 / 16), d_out, ctx->small_meta.as<uint32_t>(), s));
    ctx->last_small = true;
    ctx->pub_table = nullptr;
    ctx->table_k = -1;
    return 0;
}

// Build a seed table on s (returned in *out).  zero_out (optional): the round's output,
// zero-filled by the same launch (zero_n words).  Only flm_seed_table_dev publishes the table for a
// later flm_aggregate_dev (publish = true); every other entry point that builds one (prg expansion,
// client masking, pair units, the fused round) withdraws the publication, so aggregate_dev only
// ever unmasks against the seeds of the latest flm_seed_table_dev call, and only until another
// entry point runs.
int run_seed_schedule(flm_ctx *ctx, const uint8_t *d_seeds, const int8_t *d_signs, int K, hipStream_t s,
                      SeedTable **out, uint32_t *zero_out = nullptr, uint64_t zero_n = 0, bool publish = false) {
    const int groups = flm::seed_schedule_groups(K, zero_out ? zero_n : 0);
    int rc = 0;
    SeedTable *t = table_acquire(ctx, K, 2 + 2 * (size_t)groups, s, &rc);
    if (!t) return rc;
    const hipError_t e = flm::launch_seed_schedule(d_seeds, d_signs, K, t->recs.as<SeedRec>(), t->meta.as<uint32_t>(),
                                                   s, zero_out, zero_n);
    if (e != hipSuccess) {
        table_cover(t, s);  // whatever part of it got enqueued
        return fail(ctx, FLM_EHIP, "seed schedule launch: %s", hipGetErrorString(e));
    }
    FLM_HIP(ctx, table_written(ctx, t, s, /*record=*/publish));
    ctx->pub_table = publish ? t : nullptr;
    ctx->table_k = publish ? K : -1;
    *out = t;
    return 0;
}

// zeroed: the output was already zero-filled on this stream (by the seed-schedule launch)
int run_plan(flm_ctx *ctx, Plan &plan, SeedTable *table, const uint32_t *d_rows, uint64_t pitch, uint32_t *d_out,
             size_t out_elems, hipStream_t s, bool zeroed = false) {
    if (!plan.ready_known) {  // the items' copy was enqueued on another stream: order after it
        const hipError_t q = hipEventQuery(plan.ready);
        if (q == hipSuccess) plan.ready_known = true;
        else if (q != hipErrorNotReady) FLM_HIP(ctx, q);
        else if (s != plan.up_stream) FLM_HIP(ctx, hipStreamWaitEvent(s, plan.ready, 0));
    }
    if (plan.needs_zero && !zeroed) FLM_HIP(ctx, hipMemsetAsync(d_out, 0, out_elems * sizeof(uint32_t), s));
    const int variant_id = pick_variant(ctx, plan);
    FLM_HIP(ctx, table_before_read(table, s));
    FLM_HIP(ctx, flm::launch_items(plan.subtiles, variant_id, plan.items.as<Item>(), plan.n_items, d_rows, pitch,
                                   table->recs.as<SeedRec>(), table->meta.as<uint32_t>(), d_out, s));
    FLM_HIP(ctx, table_read(table, s));
    // one event per stream the plan ran on, after its last launch there: the cache recycles the
    // items only once all of them have completed (no dependency is added between the streams)
    hipEvent_t *ev = nullptr;
    for (auto &d : plan.done)
        if (d.first == s) ev = &d.second;
    if (!ev) {
        if (plan.done.size() >= 8) {  // many streams over time: drop the entries already completed
            std::vector<std::pair<hipStream_t, hipEvent_t>> keep;
            for (auto &d : plan.done) {
                if (hipEventQuery(d.second) == hipSuccess) (void)hipEventDestroy(d.second);
                else keep.push_back(d);
            }
            (void)hipGetLastError();  // hipErrorNotReady from the queries
            plan.done.swap(keep);
        }
        hipEvent_t e = nullptr;
        FLM_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        plan.done.emplace_back(s, e);
        ev = &plan.done.back().second;
    }
    FLM_HIP(ctx, hipEventRecord(*ev, s));
    ctx->last_items = plan.n_items;
    ctx->last_tile = flm::kWaveSlots * plan.subtiles;
    ctx->last_atomics = plan.atomics;
    ctx->last_variant = variant_id;
    return 0;
}

// Upload N host rows (pageable or pinned) into the context's row buffer at `pitch`.
bool host_pinned(const void *p) {
    hipPointerAttribute_t a;
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable memory is not an error here
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Upload N host rows into the context's row buffer at `pitch`.  Page-locked
// rows (e.g. from flm_host_alloc / PinnedArena) are DMA'd directly; pageable
// rows are packed into a pinned staging ring (kStageBytes per buffer, two
// buffers) so the copy engine sees few large transfers while the CPU fills
// the other buffer.  The VECTOR bodies of the reference are pageable numpy
// arrays (SA_ServiceAgent.py:210).  No pageable row is ever handed to a HIP copy
// (HostCopies below says why).
constexpr size_t kStageBytes = 32u << 20;

// The two kStageBytes pinned staging buffers of the context (upload_rows, HostCopies' large copies).
int ensure_stage(flm_ctx *ctx) {
    if (ctx->stage_cap >= kStageBytes) return 0;
    for (int b = 0; b < 2; ++b) {
        if (ctx->stage[b]) (void)hipHostFree(ctx->stage[b]);
        ctx->stage[b] = nullptr;
        FLM_HIP(ctx, hipHostMalloc(&ctx->stage[b], kStageBytes, hipHostMallocDefault));
        if (!ctx->stage_done[b]) FLM_HIP(ctx, hipEventCreateWithFlags(&ctx->stage_done[b], hipEventDisableTiming));
    }
    ctx->stage_cap = kStageBytes;
    return 0;
}

int upload_rows(flm_ctx *ctx, const uint32_t *const *rows, int N, size_t L, uint64_t pitch) {
    FLM_HIP(ctx, ctx->rows.reserve(std::max<size_t>(1, (size_t)N) * pitch * sizeof(uint32_t)));
    uint32_t *dst = ctx->rows.as<uint32_t>();
    const size_t row_bytes = L * sizeof(uint32_t);
    const size_t slot_bytes = pitch * sizeof(uint32_t);
    std::vector<int> pageable, pinned;
    for (int i = 0; i < N; ++i) {
        if (!rows[i]) return fail(ctx, FLM_EINVAL, "row %d is NULL", i);
        (host_pinned(rows[i]) ? pinned : pageable).push_back(i);
    }
    if (!pinned.empty()) {
        // Page-locked rows go straight to the device, spread over kCopyStreams
        // streams (several SDMA engines: one stream tops out near 49 GB/s, four
        // reach the link's ~57 GB/s, tools/probes/h2d_probe.hip).  Runs of rows that are
        // contiguous on the host (an arena) move as one copy of up to 16 rows.
        if (!ctx->copy[0]) {
            for (int c = 0; c < kCopyStreams; ++c) {
                FLM_HIP(ctx, hipStreamCreateWithFlags(&ctx->copy[c], hipStreamNonBlocking));
                FLM_HIP(ctx, hipEventCreateWithFlags(&ctx->copy_done[c], hipEventDisableTiming));
            }
            FLM_HIP(ctx, hipEventCreateWithFlags(&ctx->copy_start, hipEventDisableTiming));
        }
        // the row buffer may still be read by the previous round on ctx->stream
        FLM_HIP(ctx, hipEventRecord(ctx->copy_start, ctx->stream));
        for (int c = 0; c < kCopyStreams; ++c) FLM_HIP(ctx, hipStreamWaitEvent(ctx->copy[c], ctx->copy_start, 0));
        int next = 0;
        for (size_t k = 0; k < pinned.size();) {
            const int first = pinned[k];
            size_t n = 1;
            while (pitch == L && n < 16 && k + n < pinned.size() && pinned[k + n] == first + (int)n &&
                   rows[first + n] == rows[first] + n * L)
                ++n;
            FLM_HIP(ctx, hipMemcpyAsync(dst + (size_t)first * pitch, rows[first], (n - 1) * slot_bytes + row_bytes,
                                        hipMemcpyHostToDevice, ctx->copy[next]));
            next = (next + 1) % kCopyStreams;
            k += n;
        }
        for (int c = 0; c < kCopyStreams; ++c) {
            FLM_HIP(ctx, hipEventRecord(ctx->copy_done[c], ctx->copy[c]));
            FLM_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->copy_done[c], 0));
        }
    }
    if (pageable.empty()) return 0;
    if (int rc = ensure_stage(ctx)) return rc;
    size_t k = 0;
    int b = 0;
    bool used[2] = {false, false};
    if (slot_bytes > kStageBytes) {  // very long rows: each in kStageBytes pieces through the same ring
        for (int i : pageable)
            for (size_t off = 0; off < row_bytes; off += kStageBytes) {
                const size_t n = std::min(kStageBytes, row_bytes - off);
                if (used[b]) FLM_HIP(ctx, hipEventSynchronize(ctx->stage_done[b]));
                ctx->copies.copy2d(ctx->stage[b], n, reinterpret_cast<const uint8_t *>(rows[i]) + off, n, n, 1);
                FLM_HIP(ctx, hipMemcpyAsync(reinterpret_cast<uint8_t *>(dst + (size_t)i * pitch) + off, ctx->stage[b], n,
                                            hipMemcpyHostToDevice, ctx->stream));
                FLM_HIP(ctx, hipEventRecord(ctx->stage_done[b], ctx->stream));
                used[b] = true;
                b ^= 1;
            }
        return 0;
    }
    const size_t per_buf = kStageBytes / slot_bytes;  // rows per staging buffer
    while (k < pageable.size()) {
        if (used[b]) FLM_HIP(ctx, hipEventSynchronize(ctx->stage_done[b]));  // DMA out of this buffer done
        uint8_t *st = static_cast<uint8_t *>(ctx->stage[b]);
        // a run of consecutive row indices packs into one contiguous device range
        const int first = pageable[k];
        size_t n = 0;
        while (k + n < pageable.size() && n < per_buf && pageable[k + n] == first + (int)n) {
            ctx->copies.copy2d(st + n * slot_bytes, row_bytes, rows[pageable[k + n]], row_bytes, row_bytes, 1);
            ++n;
        }
        FLM_HIP(ctx, hipMemcpyAsync(dst + (size_t)first * pitch, st, n * slot_bytes - (slot_bytes - row_bytes),
                                    hipMemcpyHostToDevice, ctx->stream));
        FLM_HIP(ctx, hipEventRecord(ctx->stage_done[b], ctx->stream));
        used[b] = true;
        k += n;
        b ^= 1;
    }
    return 0;
}

// The host-pointer entry points move the caller's arrays through the context's pinned bounce
// buffer (ctx->bounce), never straight between a HIP copy and the caller's pageable pages.  For a
// large pageable copy the HIP runtime pins those pages for the DMA (a KFD userptr allocation; its log:
// "HSA Copy Using Pinned resource"); when the process later unmaps them (a numpy array freed), the
// driver evicts ALL of the process's GPU queues while it revalidates: 20-40 ms in which nothing of
// ours runs.  That was the agent run's unmask stall (the driver's per-process
// evicted_ms grows by exactly the stall, and the stalls go away when the runtime never pins,
// GPU_PINNED_MIN_XFER_SIZE).  The runtime's rect path (hipMemcpy2DAsync straight on the caller's
// array) logs no pinning but brings the evictions back all the same (5 of 5 runs,
// profiles/r06_rect_path_evictions.log), so every caller array, small or large, goes through the
// bounce buffer; the CPU side of the copies is split over the context's CopyPool, and a call whose
// arrays fit may run its kernel on the bounce buffer in place (mapped(), dev()).  One bounce buffer per context: these calls are synchronous (or, for a
// group's ranks, synchronised before the call returns), so a call reuses it only after the last
// call's copies out of it have completed; reserve() sizes it for the whole call before its first copy.
// Copies of kStageBytes or more skip it and stream through the context's two staging buffers instead
// (inputs at once, outputs in finish()), so no call pins more host memory than its small copies plus
// 2 x 32 MiB, whatever its size (a 962 x 2^20 prg_expand returns 4 GiB).
class HostCopies {
  public:
    HostCopies(flm_ctx *ctx, hipStream_t s) : ctx_(ctx), s_(s) {}
    static size_t room(size_t n) { return n >= kStageBytes ? 0 : round_up(n, 256); }
    int reserve(size_t bytes) {  // the sum of room(n) over the call's copies
        if (bytes > ctx_->bounce_cap) {
            if (ctx_->bounce) (void)hipHostFree(ctx_->bounce);  // waits for the device: nothing reads it after
            ctx_->bounce = nullptr;
            ctx_->bounce_cap = 0;
            const size_t want = flm::rt::grow_bytes(bytes);
            const hipError_t e = hipHostMalloc(&ctx_->bounce, want, hipHostMallocDefault);
            if (e != hipSuccess) return fail(ctx_, FLM_ENOMEM, "pinned bounce buffer of %zu bytes: %s", want, hipGetErrorString(e));
            ctx_->bounce_cap = want;
            FLM_HIP(ctx_, hipHostGetDevicePointer(&ctx_->bounce_dev, ctx_->bounce, 0));
        }
        cap_ = bytes;
        return 0;
    }
    // d_dst <- h_src (n bytes): copied into the bounce buffer now, DMA enqueued on the stream
    int in(void *d_dst, const void *h_src, size_t n) { return in2d(d_dst, n, h_src, n, n, 1); }
    // rows x width bytes, host rows at h_pitch, device rows at d_pitch
    int in2d(void *d_dst, size_t d_pitch, const void *h_src, size_t h_pitch, size_t width, size_t rows) {
        if (!width || !rows) return 0;
        if (width * rows >= kStageBytes) return stream_in(d_dst, d_pitch, h_src, h_pitch, width, rows);
        uint8_t *b = take(width * rows);
        if (!b) return fail(ctx_, FLM_EINVAL, "host bounce: %zu bytes past the reserved %zu", width * rows, cap_);
        ctx_->copies.copy2d(b, width, h_src, h_pitch, width, rows);
        FLM_HIP(ctx_, rows == 1 ? hipMemcpyAsync(d_dst, b, width, hipMemcpyHostToDevice, s_)
                                : hipMemcpy2DAsync(d_dst, d_pitch, b, width, width, rows, hipMemcpyHostToDevice, s_));
        return 0;
    }
    // h_dst <- d_src: DMA into the bounce buffer now, handed to the caller by finish()
    int out(void *h_dst, const void *d_src, size_t n) { return out2d(h_dst, n, d_src, n, n, 1); }
    int out2d(void *h_dst, size_t h_pitch, const void *d_src, size_t d_pitch, size_t width, size_t rows) {
        if (!width || !rows) return 0;
        if (width * rows >= kStageBytes) {
            bigs_.push_back({h_dst, h_pitch, static_cast<const uint8_t *>(d_src), d_pitch, width, rows});
            return 0;
        }
        uint8_t *b = take(width * rows);
        if (!b) return fail(ctx_, FLM_EINVAL, "host bounce: %zu bytes past the reserved %zu", width * rows, cap_);
        FLM_HIP(ctx_, rows == 1 ? hipMemcpyAsync(b, d_src, width, hipMemcpyDeviceToHost, s_)
                                : hipMemcpy2DAsync(b, width, d_src, d_pitch, width, rows, hipMemcpyDeviceToHost, s_));
        outs_.push_back({h_dst, h_pitch, b, width, width, rows});
        return 0;
    }
    // n bytes of the bounce buffer for a kernel to read or write in place (the GPU reaches pinned host
    // memory over the link), nullptr for n of kStageBytes or more: a caller then copies as above
    uint8_t *mapped(size_t n) { return n < kStageBytes ? take(n) : nullptr; }
    // the kernel-side address of host address b of the bounce buffer
    template <class T>
    T *dev(const uint8_t *b) const {
        return b ? reinterpret_cast<T *>(static_cast<uint8_t *>(ctx_->bounce_dev) + (b - static_cast<uint8_t *>(ctx_->bounce)))
                 : nullptr;
    }
    // rows x width bytes a kernel wrote in place at b (mapped) at b_pitch, to the caller's rows at h_pitch
    void out_mapped(void *h_dst, size_t h_pitch, const uint8_t *b, size_t b_pitch, size_t width, size_t rows) {
        outs_.push_back({h_dst, h_pitch, b, b_pitch, width, rows});
    }
    // wait for the stream, then copy the outputs to the caller (large ones through the staging ring)
    int finish() {
        FLM_HIP(ctx_, hipStreamSynchronize(s_));
        for (const Out &o : outs_) ctx_->copies.copy2d(o.dst, o.pitch, o.src, o.spitch, o.width, o.rows);
        outs_.clear();
        for (const Big &g : bigs_)
            if (int rc = stream_out(g)) return rc;
        bigs_.clear();
        return 0;
    }

  private:
    struct Out {
        void *dst;
        size_t pitch;
        const uint8_t *src;
        size_t spitch, width, rows;
    };
    struct Big {  // a large output: device rows at d_pitch -> host rows at h_pitch
        void *dst;
        size_t h_pitch;
        const uint8_t *src;
        size_t d_pitch, width, rows;
    };
    // Pieces of at most kStageBytes of a rows x width copy: whole rows, or one row's columns.
    struct Piece {
        size_t r, c, w, nr;  // first row, first column, bytes per row, rows
    };
    static std::vector<Piece> pieces(size_t width, size_t rows) {
        std::vector<Piece> v;
        if (width > kStageBytes) {
            for (size_t r = 0; r < rows; ++r)
                for (size_t c = 0; c < width; c += kStageBytes) v.push_back({r, c, std::min(kStageBytes, width - c), 1});
        } else {
            const size_t per = kStageBytes / width;
            for (size_t r = 0; r < rows; r += per) v.push_back({r, 0, width, std::min(per, rows - r)});
        }
        return v;
    }
    // a large input: each piece copied into the next free staging buffer, then DMA'd from it
    int stream_in(void *d_dst, size_t d_pitch, const void *h_src, size_t h_pitch, size_t width, size_t rows) {
        if (int rc = ensure_stage(ctx_)) return rc;
        const auto *src = static_cast<const uint8_t *>(h_src);
        auto *dst = static_cast<uint8_t *>(d_dst);
        int b = 0;
        for (const Piece &p : pieces(width, rows)) {
            FLM_HIP(ctx_, hipEventSynchronize(ctx_->stage_done[b]));  // the DMA out of this buffer is done
            auto *st = static_cast<uint8_t *>(ctx_->stage[b]);
            ctx_->copies.copy2d(st, p.w, src + p.r * h_pitch + p.c, h_pitch, p.w, p.nr);
            FLM_HIP(ctx_, hipMemcpy2DAsync(dst + p.r * d_pitch + p.c, d_pitch, st, p.w, p.w, p.nr, hipMemcpyHostToDevice, s_));
            FLM_HIP(ctx_, hipEventRecord(ctx_->stage_done[b], s_));
            b ^= 1;
        }
        return 0;
    }
    // a large output, after the stream has drained: piece i + 1 lands in one staging buffer while
    // piece i is copied out of the other
    int stream_out(const Big &g) {
        if (int rc = ensure_stage(ctx_)) return rc;
        const std::vector<Piece> ps = pieces(g.width, g.rows);
        auto issue = [&](size_t i) -> int {
            const Piece &p = ps[i];
            FLM_HIP(ctx_, hipMemcpy2DAsync(ctx_->stage[i & 1], p.w, g.src + p.r * g.d_pitch + p.c, g.d_pitch, p.w, p.nr,
                                           hipMemcpyDeviceToHost, s_));
            FLM_HIP(ctx_, hipEventRecord(ctx_->stage_done[i & 1], s_));
            return 0;
        };
        for (size_t i = 0; i < ps.size() && i < 2; ++i)
            if (int rc = issue(i)) return rc;
        for (size_t i = 0; i < ps.size(); ++i) {
            const Piece &p = ps[i];
            FLM_HIP(ctx_, hipEventSynchronize(ctx_->stage_done[i & 1]));
            ctx_->copies.copy2d(static_cast<uint8_t *>(g.dst) + p.r * g.h_pitch + p.c, g.h_pitch, ctx_->stage[i & 1], p.w,
                                p.w, p.nr);
            if (i + 2 < ps.size())
                if (int rc = issue(i + 2)) return rc;
        }
        return 0;
    }
    uint8_t *take(size_t n) {
        if (off_ + room(n) > cap_) return nullptr;
        uint8_t *b = static_cast<uint8_t *>(ctx_->bounce) + off_;
        off_ += room(n);
        return b;
    }
    flm_ctx *ctx_;
    hipStream_t s_;
    size_t cap_ = 0, off_ = 0;
    std::vector<Out> outs_;
    std::vector<Big> bigs_;
};

size_t seeds_room(int K) { return K > 0 ? HostCopies::room((size_t)K * 32) + HostCopies::room((size_t)K) : 0; }

int upload_seeds(flm_ctx *ctx, HostCopies &hc, const uint8_t *seeds, const int8_t *signs, int K) {
    FLM_HIP(ctx, ctx->seeds.reserve(std::max<size_t>(1, (size_t)K) * 32));
    FLM_HIP(ctx, ctx->signs.reserve(std::max<size_t>(1, (size_t)K)));
    if (K > 0) {
        if (int rc = hc.in(ctx->seeds.p, seeds, (size_t)K * 32)) return rc;
        if (int rc = hc.in(ctx->signs.p, signs, (size_t)K)) return rc;
    }
    return 0;
}

// Client masking / expansion plan: one job per output row, 16 sub-tiles per
// workgroup (each wave its own 1024 slots, all of the row's seeds).
// out[i] = (x[i] or base_bias) + sum of row i's seeds (+1 per negative seed).
// seg NULL: row i has seed i alone.  signs: K host signs, or NULL for all +1 (expansion).
// The items and the signs travel in one staging slot (StageSlot): nothing here waits on the host.
int run_rows_jobs(flm_ctx *ctx, const uint32_t *d_x, uint64_t pitch, int N, const int64_t *seg, const int8_t *signs,
                  const uint8_t *d_seeds, int K, uint32_t base_bias, size_t L, uint64_t slot0, uint32_t *d_out,
                  hipStream_t s) {
    const int subtiles = 16;
    std::vector<Item> items;
    bool needs_zero = false, single_tile = true;
    int atomics = 0;
    for (int i = 0; i < N; ++i) {
        Job j;
        j.out_base = (uint64_t)i * pitch;
        j.L = L;
        const uint32_t k0 = seg ? (uint32_t)seg[i] : (uint32_t)i;
        const uint32_t k1 = seg ? (uint32_t)seg[i + 1] : (uint32_t)i + 1;
        uint32_t nneg = 0;
        if (signs)
            for (uint32_t k = k0; k < k1; ++k) nneg += signs[k] < 0;
        const uint32_t bias = (d_x ? 0u : base_bias) + nneg;
        if (k1 == k0) {
            // no seeds: out = x (copy) or the constant bias, as a rows-only item
            const uint64_t W = (uint64_t)flm::kWaveSlots * subtiles;
            for (uint64_t t = 0; t < L; t += W) {
                Item it;
                std::memset(&it, 0, sizeof it);
                it.flags = flm::kHasRows;
                it.row_in = j.out_base + t;
                it.nrows = d_x ? 1 : 0;
                it.row_out = j.out_base + t;
                it.row_valid = (uint32_t)std::min<uint64_t>(W, L - t);
                it.row_bias = bias;
                items.push_back(it);
            }
            continue;
        }
        if (d_x) {
            j.rows_base = (uint64_t)i * pitch;
            j.nrows = 1;
        }
        j.k0 = k0;
        j.nseeds = k1 - k0;
        j.mask_lo = 0;
        j.mask_hi = L;
        j.prg_slot0 = slot0;
        j.mask_bias = bias;
        plan_job(j, pitch, subtiles, 1, 1, false, items, needs_zero, atomics, single_tile);
    }
    Plan plan;
    plan.subtiles = subtiles;
    plan.needs_zero = needs_zero;
    plan.atomics = atomics;
    plan.single_tile = single_tile;
    plan.n_items = (int)items.size();
    const size_t item_bytes = items.size() * sizeof(Item);
    int rc = 0;
    StageSlot *slot = stage_acquire(ctx, item_bytes + std::max(K, 1), &rc);
    if (!slot) return rc;
    uint8_t *h = static_cast<uint8_t *>(slot->host);
    if (item_bytes) std::memcpy(h, items.data(), item_bytes);
    if (K > 0) {
        if (signs) std::memcpy(h + item_bytes, signs, (size_t)K);
        else std::memset(h + item_bytes, 1, (size_t)K);
    }
    FLM_HIP(ctx, stage_upload(slot, item_bytes + (size_t)K, s));
    const uint8_t *d = slot->dev.as<uint8_t>();
    SeedTable *table = nullptr;
    rc = run_seed_schedule(ctx, d_seeds, reinterpret_cast<const int8_t *>(d + item_bytes), K, s, &table);
    if (!rc && needs_zero) {
        const hipError_t e = hipMemsetAsync(d_out, 0, (size_t)N * pitch * sizeof(uint32_t), s);
        if (e != hipSuccess) rc = fail(ctx, FLM_EHIP, "hipMemsetAsync: %s", hipGetErrorString(e));
    }
    const int variant_id = pick_variant(ctx, plan);
    if (!rc && plan.n_items) {
        hipError_t e = flm::launch_items(subtiles, variant_id, reinterpret_cast<const Item *>(d), plan.n_items, d_x,
                                         pitch, table->recs.as<SeedRec>(), table->meta.as<uint32_t>(), d_out, s);
        if (e == hipSuccess) e = table_read(table, s);
        if (e != hipSuccess) rc = fail(ctx, FLM_EHIP, "items launch: %s", hipGetErrorString(e));
    }
    if (table && (rc || !plan.n_items)) table_cover(table, s);  // no read recorded after the table's write
    // the slot is busy until the work enqueued so far has run, whether or not it all got enqueued
    FLM_HIP(ctx, stage_commit(slot, s));
    if (rc) return rc;
    ctx->last_items = plan.n_items;
    ctx->last_tile = flm::kWaveSlots * subtiles;
    ctx->last_atomics = atomics;
    ctx->last_variant = variant_id;
    return 0;
}

}  // namespace

namespace flm {
namespace rt {
int set_error(flm_ctx *ctx, int code, const char *msg) { return fail(ctx, code, "%s", msg); }
int device_of(const flm_ctx *ctx) { return ctx->device; }
hipStream_t stream_of(const flm_ctx *ctx) { return ctx->stream; }
void **comm_slot(flm_ctx *ctx) { return &ctx->comm; }
void host_copy(flm_ctx *ctx, void *dst, const void *src, size_t n) { ctx->copies.copy2d(dst, n, src, n, n, 1); }

int host_round_async(flm_ctx *ctx, const uint32_t *const *rows, int N, const uint8_t *seeds, const int8_t *signs,
                     int K, size_t L, size_t mask_lo, size_t mask_hi, uint32_t *d_out) {
    if (N < 0 || K < 0) return fail(ctx, FLM_EINVAL, "negative N or K");
    if ((N > 0 && !rows) || (K > 0 && (!seeds || !signs)) || !d_out) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (!signs_ok(signs, K, nullptr)) return fail(ctx, FLM_EINVAL, "signs must be +1 or -1");
    if (int rc = check_range(ctx, L)) return rc;
    FLM_ON_DEVICE(ctx);
    const uint64_t pitch = round_up(L, 64);
    if (int rc = upload_rows(ctx, rows, N, L, pitch)) return rc;
    HostCopies hc(ctx, ctx->stream);  // the group synchronises every rank before its call returns
    if (int rc = hc.reserve(seeds_room(K))) return rc;
    if (int rc = upload_seeds(ctx, hc, seeds, signs, K)) return rc;
    return flm_aggregate_unmask_dev(ctx, ctx->rows.as<uint32_t>(), pitch, N, ctx->seeds.as<uint8_t>(),
                                    ctx->signs.as<int8_t>(), K, L, mask_lo, mask_hi, 0, d_out, ctx->stream);
}

}  // namespace rt
}  // namespace flm

// ======================================================================= ABI
extern "C" {

int flm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *flm_version(void) { return "flamingo_hip 0.4 gfx950 items_kernel<S={1,4,16}>"; }

int flm_init(flm_ctx **out, int device) {
    if (!out) return fail(nullptr, FLM_EINVAL, "flm_init: out is NULL");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(nullptr, FLM_EHIP, "flm_init: no HIP device visible (%s)", hipGetErrorString(e));
    if (device < 0 || device >= n) return fail(nullptr, FLM_EINVAL, "flm_init: device %d out of range [0,%d)", device, n);
    flm::rt::DeviceScope dev_scope_;
    e = dev_scope_.set(device);
    if (e != hipSuccess) return fail(nullptr, FLM_EHIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    flm_ctx *ctx = new flm_ctx();
    ctx->device = device;
    e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return fail(nullptr, FLM_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    if (hipDeviceGetAttribute(&ctx->n_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) {
        (void)hipGetLastError();
        ctx->n_cus = 256;  // MI355X
    }
    stage_prealloc(ctx);
    *out = ctx;
    return 0;
}

void flm_free(flm_ctx *ctx) {
    if (!ctx) return;
    flm::rt::DeviceScope dev_scope_(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    // collectives may sit on a caller's stream (a torch comm stream), not the context's: the whole
    // device completes before the communicator is finalised (flm_comm_destroy does the same)
    if (ctx->comm) (void)hipDeviceSynchronize();
    flm::comm_release(ctx);
    for (StageSlot *s : ctx->slots) (void)hipEventSynchronize(s->done);  // launches on other streams
    for (auto &kv : ctx->plans) plan_free(kv.second);
    for (SeedTable *t : ctx->tables) table_free(t);  // waits for the table's readers on every stream
    if (ctx->small_meta.p) (void)hipDeviceSynchronize();  // small rounds on any stream may still write it
    ctx->small_meta.release();
    for (DevBuf *b : {&ctx->rows, &ctx->out, &ctx->seeds, &ctx->signs, &ctx->bytes_in, &ctx->bytes_out, &ctx->ec_in,
                      &ctx->ec_base, &ctx->ec_scal, &ctx->ec_jac, &ctx->ec_out, &ctx->ec_dig, &ctx->ec_flags})
        b->release();
    for (StageSlot *s : ctx->slots) {
        if (s->host) (void)hipHostFree(s->host);
        s->dev.release();
        (void)hipEventDestroy(s->done);
        delete s;
    }
    if (ctx->bounce) (void)hipHostFree(ctx->bounce);
    for (int i = 0; i < 2; ++i) {
        if (ctx->stage[i]) (void)hipHostFree(ctx->stage[i]);
        if (ctx->stage_done[i]) (void)hipEventDestroy(ctx->stage_done[i]);
    }
    for (int c = 0; c < 4; ++c) {
        if (ctx->copy[c]) (void)hipStreamSynchronize(ctx->copy[c]);
        if (ctx->copy[c]) (void)hipStreamDestroy(ctx->copy[c]);
        if (ctx->copy_done[c]) (void)hipEventDestroy(ctx->copy_done[c]);
    }
    if (ctx->copy_start) (void)hipEventDestroy(ctx->copy_start);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void *flm_ctx_stream(flm_ctx *ctx) { return ctx ? static_cast<void *>(ctx->stream) : nullptr; }

const char *flm_last_error(const flm_ctx *ctx) {
    if (ctx) return ctx->err.c_str();
    return g_last_error.c_str();
}

int flm_aggregate_unmask(flm_ctx *ctx, const uint32_t *const *rows, int N, const uint8_t *seeds, const int8_t *signs,
                         int K, size_t L, uint32_t *out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (N < 0 || K < 0) return fail(ctx, FLM_EINVAL, "negative N or K");
    if (L == 0) return 0;
    if (!out || (N > 0 && !rows) || (K > 0 && (!seeds || !signs))) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (!signs_ok(signs, K, nullptr)) return fail(ctx, FLM_EINVAL, "signs must be +1 or -1");
    if (int rc = check_range(ctx, L)) return rc;
    FLM_ON_DEVICE(ctx);
    const uint64_t pitch = round_up(L, 64);
    if (int rc = upload_rows(ctx, rows, N, L, pitch)) return rc;
    HostCopies hc(ctx, ctx->stream);
    if (int rc = hc.reserve(seeds_room(K) + HostCopies::room(L * sizeof(uint32_t)))) return rc;
    if (int rc = upload_seeds(ctx, hc, seeds, signs, K)) return rc;
    FLM_HIP(ctx, ctx->out.reserve(L * sizeof(uint32_t)));
    if (int rc = flm_aggregate_unmask_dev(ctx, ctx->rows.as<uint32_t>(), pitch, N, ctx->seeds.as<uint8_t>(),
                                          ctx->signs.as<int8_t>(), K, L, 0, L, 0, ctx->out.as<uint32_t>(), ctx->stream))
        return rc;
    if (int rc = hc.out(out, ctx->out.p, L * sizeof(uint32_t))) return rc;
    return hc.finish();
}

static int check_aggregate_args(flm_ctx *ctx, const uint32_t *d_rows, size_t row_pitch, int N, int K, size_t L,
                                size_t mask_lo, size_t mask_hi, uint64_t prg_slot0, const uint32_t *d_out) {
    if (N < 0 || K < 0) return fail(ctx, FLM_EINVAL, "negative N or K");
    if (N > 0 && (row_pitch % 4 != 0 || row_pitch < round_up(L, 4)))
        return fail(ctx, FLM_EINVAL, "row_pitch %zu must be a multiple of 4 and >= round_up(L=%zu, 4)", row_pitch, L);
    if ((N > 0 && ((uintptr_t)d_rows & 15)) || ((uintptr_t)d_out & 15))
        return fail(ctx, FLM_EINVAL, "rows and out must be 16-byte aligned");
    if (mask_hi > L || mask_lo > mask_hi)
        return fail(ctx, FLM_EINVAL, "mask window [%zu,%zu) outside [0,%zu)", mask_lo, mask_hi, L);
    if ((mask_hi > mask_lo && mask_lo % 16) || prg_slot0 % 16)
        return fail(ctx, FLM_EINVAL, "mask_lo and prg_slot0 must be multiples of 16");
    if (int rc = check_range(ctx, prg_slot0 + mask_hi)) return rc;
    if (N > 0 && !d_rows) return fail(ctx, FLM_EINVAL, "rows is NULL");
    if (!d_out) return fail(ctx, FLM_EINVAL, "out is NULL");
    return 0;
}

int flm_seed_table_dev(flm_ctx *ctx, const uint8_t *d_seeds, const int8_t *d_signs, int K, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (K < 0) return fail(ctx, FLM_EINVAL, "negative K");
    if (K > 0 && (!d_seeds || !d_signs)) return fail(ctx, FLM_EINVAL, "seeds/signs NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    FLM_ON_DEVICE(ctx);
    SeedTable *t = nullptr;
    return run_seed_schedule(ctx, d_seeds, d_signs, K, s, &t, nullptr, 0, /*publish=*/true);
}

int flm_aggregate_dev(flm_ctx *ctx, const uint32_t *d_rows, size_t row_pitch, int N, int K, size_t L, size_t mask_lo,
                      size_t mask_hi, uint64_t prg_slot0, uint32_t *d_out, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (L == 0) return 0;
    if (int rc = check_aggregate_args(ctx, d_rows, row_pitch, N, K, L, mask_lo, mask_hi, prg_slot0, d_out)) return rc;
    if (!ctx->pub_table || K != ctx->table_k)
        return fail(ctx, FLM_EINVAL, "K=%d does not match the seed table (%d)", K, ctx->table_k);
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    FLM_ON_DEVICE(ctx);
    int rc = 0;
    Plan *plan = aggregate_plan(ctx, row_pitch, N, K, L, mask_lo, mask_hi, prg_slot0, s, &rc);
    if (!plan) return rc;
    return run_plan(ctx, *plan, ctx->pub_table, d_rows, row_pitch, d_out, L, s);
}

int flm_aggregate_unmask_dev(flm_ctx *ctx, const uint32_t *d_rows, size_t row_pitch, int N, const uint8_t *d_seeds,
                             const int8_t *d_signs, int K, size_t L, size_t mask_lo, size_t mask_hi,
                             uint64_t prg_slot0, uint32_t *d_out, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (L == 0) return 0;
    if (int rc = check_aggregate_args(ctx, d_rows, row_pitch, N, K, L, mask_lo, mask_hi, prg_slot0, d_out)) return rc;
    if (K > 0 && (!d_seeds || !d_signs)) return fail(ctx, FLM_EINVAL, "seeds/signs NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    FLM_ON_DEVICE(ctx);
    int rc = 0;
    if (const int B = small_round_width(ctx, N, K, L, mask_lo, mask_hi)) {
        // one submission; the device seed table is not built, so flm_aggregate_dev must not reuse it
        if ((rc = run_small_round(ctx, B, d_rows, row_pitch, N, d_seeds, d_signs, K, L, mask_lo, mask_hi, prg_slot0,
                                  d_out, s)))
            return rc;
        ctx->last_items = (int)((L + flm::small_round_slots(B) - 1) / flm::small_round_slots(B));
        ctx->last_tile = flm::small_round_slots(B);
        ctx->last_atomics = 0;
        ctx->last_variant = kSmallRoundVariant;
        return 0;
    }
    Plan *plan = aggregate_plan(ctx, row_pitch, N, K, L, mask_lo, mask_hi, prg_slot0, s, &rc);
    if (!plan) return rc;
    // two submissions: seed schedule (+ the zero-fill an atomics plan needs), then the items
    SeedTable *table = nullptr;
    if ((rc = run_seed_schedule(ctx, d_seeds, d_signs, K, s, &table, plan->needs_zero ? d_out : nullptr, L))) return rc;
    if ((rc = run_plan(ctx, *plan, table, d_rows, row_pitch, d_out, L, s, plan->needs_zero))) table_cover(table, s);
    return rc;
}

int flm_client_mask(flm_ctx *ctx, const uint32_t *x, int N, const int64_t *seg, const uint8_t *seeds,
                    const int8_t *signs, size_t L, uint32_t *out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (N < 0) return fail(ctx, FLM_EINVAL, "negative N");
    if (N == 0 || L == 0) return 0;
    if (!seg || !out) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (seg[0] != 0) return fail(ctx, FLM_EINVAL, "seg[0] must be 0");
    for (int i = 0; i < N; ++i)
        if (seg[i + 1] < seg[i]) return fail(ctx, FLM_EINVAL, "seg must be non-decreasing");
    const int64_t K = seg[N];
    if (K > 0 && (!seeds || !signs)) return fail(ctx, FLM_EINVAL, "NULL seeds/signs");
    if (K > 0x7fffffff) return fail(ctx, FLM_EINVAL, "too many seeds");
    if (!signs_ok(signs, (int)K, nullptr)) return fail(ctx, FLM_EINVAL, "signs must be +1 or -1");
    if (int rc = check_range(ctx, L)) return rc;
    FLM_ON_DEVICE(ctx);
    const uint64_t pitch = round_up(L, 64);
    const size_t plane = (size_t)N * L * 4;
    HostCopies hc(ctx, ctx->stream);
    const uint64_t hp = round_up(L, 4);  // pitch of the in-place planes
    const size_t hplane = (size_t)N * hp * 4;
    if (hplane < kStageBytes) {
        // one client's call (c5: 4 MiB in, 4 MiB out): the kernel reads x from and writes y to the
        // pinned bounce buffer in place, so the link carries both at once instead of a DMA each way
        if (int rc = hc.reserve((x ? HostCopies::room(hplane) : 0) + seeds_room((int)K) + HostCopies::room(hplane))) return rc;
        uint8_t *bx = x ? hc.mapped(hplane) : nullptr;
        if (bx) ctx->copies.copy2d(bx, hp * 4, x, L * 4, L * 4, (size_t)N);
        if (int rc = upload_seeds(ctx, hc, seeds, signs, (int)K)) return rc;
        uint8_t *by = hc.mapped(hplane);
        if (int rc = flm_client_mask_dev(ctx, hc.dev<const uint32_t>(bx), hp, N, seg, ctx->seeds.as<uint8_t>(), signs, L,
                                         hc.dev<uint32_t>(by), ctx->stream))
            return rc;
        hc.out_mapped(out, L * 4, by, hp * 4, L * 4, (size_t)N);
        return hc.finish();
    }
    if (int rc = hc.reserve((x ? HostCopies::room(plane) : 0) + seeds_room((int)K) + HostCopies::room(plane))) return rc;
    uint32_t *d_x = nullptr;
    if (x) {
        FLM_HIP(ctx, ctx->rows.reserve((size_t)N * pitch * sizeof(uint32_t)));
        if (int rc = hc.in2d(ctx->rows.p, pitch * 4, x, L * 4, L * 4, (size_t)N)) return rc;
        d_x = ctx->rows.as<uint32_t>();
    }
    if (int rc = upload_seeds(ctx, hc, seeds, signs, (int)K)) return rc;
    FLM_HIP(ctx, ctx->out.reserve((size_t)N * pitch * sizeof(uint32_t)));
    if (int rc = flm_client_mask_dev(ctx, d_x, pitch, N, seg, ctx->seeds.as<uint8_t>(), signs, L, ctx->out.as<uint32_t>(),
                                     ctx->stream))
        return rc;
    if (int rc = hc.out2d(out, L * 4, ctx->out.p, pitch * 4, L * 4, (size_t)N)) return rc;
    return hc.finish();
}

int flm_client_mask_dev(flm_ctx *ctx, const uint32_t *d_x, size_t pitch, int N, const int64_t *seg,
                        const uint8_t *d_seeds, const int8_t *signs, size_t L, uint32_t *d_out, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (N <= 0 || L == 0) return 0;
    if (!seg || !d_out) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (pitch % 4 || pitch < round_up(L, 4)) return fail(ctx, FLM_EINVAL, "pitch must be a multiple of 4 and >= L");
    if (((uintptr_t)d_out & 15) || ((uintptr_t)d_x & 15)) return fail(ctx, FLM_EINVAL, "x/out must be 16-byte aligned");
    // seg sizes the launch: a decreasing pair would wrap a seed count and read past the table
    if (seg[0] != 0) return fail(ctx, FLM_EINVAL, "seg[0] must be 0");
    for (int i = 0; i < N; ++i)
        if (seg[i + 1] < seg[i]) return fail(ctx, FLM_EINVAL, "seg must be non-decreasing");
    const int64_t K = seg[N];
    if (K > 0x7fffffff) return fail(ctx, FLM_EINVAL, "too many seeds");
    if (K > 0 && (!d_seeds || !signs)) return fail(ctx, FLM_EINVAL, "NULL seeds/signs");
    if (!signs_ok(signs, (int)K, nullptr)) return fail(ctx, FLM_EINVAL, "signs must be +1 or -1");
    if (int rc = check_range(ctx, L)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    FLM_ON_DEVICE(ctx);
    // small batches (c2: 128 clients x ~15 seeds x 16384 slots): one launch of the small-round
    // kernel, one workgroup per (client, 256-slot tile), instead of a seed schedule + one 1024-thread
    // workgroup per client row.  seg and signs travel in ONE host-to-device copy.
    if (N <= 65535 /* grid.y */ && (ctx->tune_small == 2 || (ctx->tune_small == 1 && (uint64_t)K * L <= (1ull << 26)))) {
        const size_t seg_bytes = (size_t)(N + 1) * sizeof(int64_t), need = seg_bytes + (size_t)K;
        int rc = 0;
        StageSlot *slot = stage_acquire(ctx, need, &rc);  // never waits on queued work (StageSlot)
        if (!slot) return rc;
        std::memcpy(slot->host, seg, seg_bytes);
        if (K > 0) std::memcpy(static_cast<uint8_t *>(slot->host) + seg_bytes, signs, (size_t)K);
        FLM_HIP(ctx, stage_upload(slot, need, s));
        const hipError_t e = flm::launch_small_client_mask(
            d_x, pitch, N, slot->dev.as<int64_t>(), d_seeds,
            reinterpret_cast<const int8_t *>(slot->dev.as<uint8_t>() + seg_bytes), L, d_x ? 0u : 1u, d_out, s);
        FLM_HIP(ctx, stage_commit(slot, s));
        FLM_HIP(ctx, e);
        ctx->last_items = (int)(((L + 255) / 256) * (uint64_t)N);
        ctx->last_tile = 256;
        ctx->last_atomics = 0;
        ctx->last_variant = kSmallRoundVariant;
        return 0;
    }
    // signs go to the device with the work items (the schedule folds them into xorc)
    return run_rows_jobs(ctx, d_x, pitch, N, seg, signs, d_seeds, (int)K, 1u, L, 0, d_out, s);
}

int flm_prg_expand(flm_ctx *ctx, const uint8_t *seeds, int K, size_t L, uint64_t slot0, uint32_t *out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (K < 0) return fail(ctx, FLM_EINVAL, "negative K");
    if (K == 0 || L == 0) return 0;
    if (!seeds || !out) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (slot0 % 16) return fail(ctx, FLM_EINVAL, "slot0 must be a multiple of 16");
    if (int rc = check_range(ctx, slot0 + L)) return rc;
    FLM_ON_DEVICE(ctx);
    const uint64_t pitch = round_up(L, 64);
    HostCopies hc(ctx, ctx->stream);
    const uint64_t hp = round_up(L, 4);  // pitch of rows written in place
    if (int rc = hc.reserve(HostCopies::room((size_t)K * 32) + HostCopies::room((size_t)K * hp * 4))) return rc;
    FLM_HIP(ctx, ctx->seeds.reserve((size_t)K * 32));
    if (int rc = hc.in(ctx->seeds.p, seeds, (size_t)K * 32)) return rc;
    if ((size_t)K * hp * 4 < kStageBytes) {  // rows written in place in the bounce buffer (flm_client_mask)
        uint8_t *bo = hc.mapped((size_t)K * hp * 4);
        if (int rc = flm_prg_expand_dev(ctx, ctx->seeds.as<uint8_t>(), K, L, slot0, hc.dev<uint32_t>(bo), hp, ctx->stream))
            return rc;
        hc.out_mapped(out, L * 4, bo, hp * 4, L * 4, (size_t)K);
        return hc.finish();
    }
    FLM_HIP(ctx, ctx->out.reserve((size_t)K * pitch * sizeof(uint32_t)));
    if (int rc = flm_prg_expand_dev(ctx, ctx->seeds.as<uint8_t>(), K, L, slot0, ctx->out.as<uint32_t>(), pitch,
                                    ctx->stream))
        return rc;
    if (int rc = hc.out2d(out, L * 4, ctx->out.p, pitch * 4, L * 4, (size_t)K)) return rc;
    return hc.finish();
}

int flm_prg_expand_dev(flm_ctx *ctx, const uint8_t *d_seeds, int K, size_t L, uint64_t slot0, uint32_t *d_out,
                       size_t pitch, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (K <= 0 || L == 0) return 0;
    if (slot0 % 16) return fail(ctx, FLM_EINVAL, "slot0 must be a multiple of 16");
    if (pitch % 4 || pitch < round_up(L, 4)) return fail(ctx, FLM_EINVAL, "pitch must be a multiple of 4 and >= L");
    if ((uintptr_t)d_out & 15) return fail(ctx, FLM_EINVAL, "out must be 16-byte aligned");
    if (int rc = check_range(ctx, slot0 + L)) return rc;
    if ((uint64_t)K * ((L + 1023) / 1024) > 0xFFFFFFFFull)
        return fail(ctx, FLM_EINVAL, "K=%d x %zu slots: more than 2^32 1024-slot units", K, L);
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    FLM_ON_DEVICE(ctx);
    // +1 signs through a staging slot (no host wait), the seed schedule, then prg_expand_kernel
    int rc = 0;
    StageSlot *slot = stage_acquire(ctx, (size_t)K, &rc);
    if (!slot) return rc;
    std::memset(slot->host, 1, (size_t)K);
    FLM_HIP(ctx, stage_upload(slot, (size_t)K, s));
    SeedTable *table = nullptr;
    const int groups = std::max(1, ctx->n_cus * ctx->tune_expand_waves);
    rc = run_seed_schedule(ctx, d_seeds, slot->dev.as<int8_t>(), K, s, &table);
    if (!rc) {
        hipError_t e = flm::launch_prg_expand(table->recs.as<SeedRec>(), K, L, pitch, (uint32_t)(slot0 / 16), d_out,
                                              groups, s);
        if (e == hipSuccess) e = table_read(table, s);
        if (e != hipSuccess) rc = fail(ctx, FLM_EHIP, "prg_expand launch: %s", hipGetErrorString(e));
        if (rc) table_cover(table, s);
    }
    // the slot is busy until the work enqueued so far has run, whether or not it all got enqueued
    FLM_HIP(ctx, stage_commit(slot, s));
    if (rc) return rc;
    const uint64_t units = (uint64_t)K * ((L + 1023) / 1024);
    ctx->last_items = (int)std::min<uint64_t>(units, (uint64_t)groups);
    ctx->last_tile = flm::kWaveSlots;
    ctx->last_atomics = 0;
    ctx->last_variant = kExpandVariant;
    return 0;
}

int flm_mask_accumulate(flm_ctx *ctx, const uint8_t *seeds, const int8_t *signs, int K, uint32_t *acc, size_t L,
                        uint64_t slot0) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (K < 0) return fail(ctx, FLM_EINVAL, "negative K");
    if (L == 0) return 0;
    if (!acc || (K > 0 && (!seeds || !signs))) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (slot0 % 16) return fail(ctx, FLM_EINVAL, "slot0 must be a multiple of 16");
    if (!signs_ok(signs, K, nullptr)) return fail(ctx, FLM_EINVAL, "signs must be +1 or -1");
    if (int rc = check_range(ctx, slot0 + L)) return rc;
    FLM_ON_DEVICE(ctx);
    const uint64_t pitch = round_up(L, 64);
    HostCopies hc(ctx, ctx->stream);
    if (int rc = hc.reserve(2 * HostCopies::room(L * 4) + seeds_room(K))) return rc;
    if (L * 4 < kStageBytes) {  // acc read and written in place in the bounce buffer (flm_client_mask)
        uint8_t *bx = hc.mapped(L * 4), *by = hc.mapped(L * 4);
        ctx->copies.copy2d(bx, L * 4, acc, L * 4, L * 4, 1);
        if (int rc = upload_seeds(ctx, hc, seeds, signs, K)) return rc;
        if (int rc = flm_aggregate_unmask_dev(ctx, hc.dev<const uint32_t>(bx), round_up(L, 4), 1, ctx->seeds.as<uint8_t>(),
                                              ctx->signs.as<int8_t>(), K, L, 0, L, slot0, hc.dev<uint32_t>(by),
                                              ctx->stream))
            return rc;
        hc.out_mapped(acc, L * 4, by, L * 4, L * 4, 1);
        return hc.finish();
    }
    FLM_HIP(ctx, ctx->rows.reserve(pitch * sizeof(uint32_t)));
    if (int rc = hc.in(ctx->rows.p, acc, L * 4)) return rc;
    if (int rc = upload_seeds(ctx, hc, seeds, signs, K)) return rc;
    FLM_HIP(ctx, ctx->out.reserve(pitch * sizeof(uint32_t)));
    if (int rc = flm_aggregate_unmask_dev(ctx, ctx->rows.as<uint32_t>(), pitch, 1, ctx->seeds.as<uint8_t>(),
                                          ctx->signs.as<int8_t>(), K, L, 0, L, slot0, ctx->out.as<uint32_t>(),
                                          ctx->stream))
        return rc;
    if (int rc = hc.out(acc, ctx->out.p, L * 4)) return rc;
    return hc.finish();
}

int flm_chacha20_xor(flm_ctx *ctx, const uint8_t key[32], const uint8_t nonce[8], uint64_t counter, const uint8_t *in,
                     uint8_t *out, size_t n) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (n == 0) return 0;
    if (!key || !nonce || !in || !out) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    uint32_t k[8], nn[2];
    for (int i = 0; i < 8; ++i)
        k[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
               ((uint32_t)key[4 * i + 3] << 24);
    for (int i = 0; i < 2; ++i)
        nn[i] = (uint32_t)nonce[4 * i] | ((uint32_t)nonce[4 * i + 1] << 8) | ((uint32_t)nonce[4 * i + 2] << 16) |
                ((uint32_t)nonce[4 * i + 3] << 24);
    HostCopies hc(ctx, ctx->stream);
    if (int rc = hc.reserve(2 * HostCopies::room(n))) return rc;
    if (n < kStageBytes) {  // read and written in place in the bounce buffer (flm_client_mask)
        uint8_t *bi = hc.mapped(n), *bo = hc.mapped(n);
        ctx->copies.copy2d(bi, n, in, n, n, 1);
        FLM_HIP(ctx, flm::launch_chacha20_xor(k, nn, counter, hc.dev<const uint8_t>(bi), hc.dev<uint8_t>(bo), n, ctx->stream));
        hc.out_mapped(out, n, bo, n, n, 1);
        return hc.finish();
    }
    FLM_HIP(ctx, ctx->bytes_in.reserve(n));
    FLM_HIP(ctx, ctx->bytes_out.reserve(n));
    if (int rc = hc.in(ctx->bytes_in.p, in, n)) return rc;
    FLM_HIP(ctx, flm::launch_chacha20_xor(k, nn, counter, ctx->bytes_in.as<uint8_t>(), ctx->bytes_out.as<uint8_t>(), n,
                                          ctx->stream));
    if (int rc = hc.out(out, ctx->bytes_out.p, n)) return rc;
    return hc.finish();
}

int flm_plan_aggregate(int subtiles, int pairing, size_t row_pitch, int N, int K, size_t L, size_t mask_lo,
                       size_t mask_hi, uint64_t prg_slot0, void *items_out, int max_items, int *n_items,
                       int *plan_flags) {
    if (N < 0 || K < 0 || mask_hi > L || mask_lo > mask_hi || !n_items)
        return fail(nullptr, FLM_EINVAL, "flm_plan_aggregate: bad arguments");
    std::vector<Item> items;
    Plan plan;
    build_aggregate_items(subtiles, pairing, row_pitch, N, K, L, mask_lo, mask_hi, prg_slot0, items, plan);
    *n_items = (int)items.size();
    if (plan_flags)
        *plan_flags = (plan.needs_zero ? 1 : 0) | (plan.atomics ? 2 : 0) | (plan.single_tile ? 4 : 0) |
                      (plan.seed_light ? 8 : 0) | (plan.subtiles << 8);
    if (items_out && max_items > 0)
        std::memcpy(items_out, items.data(), sizeof(Item) * (size_t)std::min<int>(max_items, (int)items.size()));
    return 0;
}

int flm_set_tuning(flm_ctx *ctx, const char *key, int value) {
    if (!ctx || !key) return fail(ctx, FLM_EINVAL, "NULL argument");
    const std::string k(key);
    if (k == "variant") {
        if (value < -1 || value >= flm::kVarCount) return fail(ctx, FLM_EINVAL, "variant %d out of range", value);
        ctx->tune_variant = value;
    } else if (k == "pairing") {
        if (value < 0 || value > 2) return fail(ctx, FLM_EINVAL, "pairing must be 0, 1 or 2");
        ctx->tune_pairing = value;
    } else if (k == "subtiles") {
        if (value != 0 && value != 1 && value != 4 && value != 16)
            return fail(ctx, FLM_EINVAL, "subtiles must be 0 (auto), 1, 4 or 16");
        ctx->tune_subtiles = value;
    } else if (k == "ec_waves") {
        if (value != 1 && value != 4 && value != 8) return fail(ctx, FLM_EINVAL, "ec_waves must be 1, 4 or 8");
        ctx->tune_ec_waves = value;
    } else if (k == "small") {
        if (value < 0 || value > 2) return fail(ctx, FLM_EINVAL, "small must be 0 (never), 1 (auto) or 2 (when legal)");
        ctx->tune_small = value;
    } else if (k == "min_items") {
        if (value < 64 || value > (1 << 20)) return fail(ctx, FLM_EINVAL, "min_items must be in [64, 2^20]");
        ctx->tune_min_items = value;
    } else if (k == "ec_spread") {
        if (value < 0 || value > 64) return fail(ctx, FLM_EINVAL, "ec_spread must be in [0, 64] KiB");
        ctx->tune_ec_spread = value;
    } else if (k == "ec_terms") {
        if (value != 1 && value != 2 && value != 4) return fail(ctx, FLM_EINVAL, "ec_terms must be 1, 2 or 4");
        ctx->tune_ec_terms = value;
    } else if (k == "ec_coop") {
        if (value < -1 || value > 2) return fail(ctx, FLM_EINVAL, "ec_coop must be -1, 0, 1 or 2");
        ctx->tune_ec_coop = value;
    } else if (k == "expand_waves") {
        if (value < 1 || value > 256) return fail(ctx, FLM_EINVAL, "expand_waves must be in [1, 256]");
        ctx->tune_expand_waves = value;
    } else if (k == "ec_threads") {
        if (value != 64 && value != 128 && value != 256)
            return fail(ctx, FLM_EINVAL, "ec_threads must be 64, 128 or 256");
        ctx->tune_ec_threads = value;
    } else {
        return fail(ctx, FLM_EINVAL, "unknown tuning key '%s'", key);
    }
    return 0;
}

int flm_get_tuning(const flm_ctx *ctx, const char *key, int *value) {
    flm_ctx *c = const_cast<flm_ctx *>(ctx);  // only its error string is written
    if (!ctx || !key || !value) return fail(c, FLM_EINVAL, "NULL argument");
    const std::string k(key);
    const std::pair<const char *, int> knobs[] = {
        {"variant", ctx->tune_variant},       {"pairing", ctx->tune_pairing},     {"subtiles", ctx->tune_subtiles},
        {"ec_waves", ctx->tune_ec_waves},     {"small", ctx->tune_small},         {"min_items", ctx->tune_min_items},
        {"ec_spread", ctx->tune_ec_spread},   {"ec_terms", ctx->tune_ec_terms},   {"ec_coop", ctx->tune_ec_coop},
        {"ec_threads", ctx->tune_ec_threads}, {"expand_waves", ctx->tune_expand_waves}};
    for (const auto &kv : knobs)
        if (k == kv.first) {
            *value = kv.second;
            return 0;
        }
    return fail(c, FLM_EINVAL, "unknown tuning key '%s'", key);
}

int flm_check_signs(flm_ctx *ctx, int *bad_count) {
    if (!ctx || !bad_count) return fail(ctx, FLM_EINVAL, "NULL argument");
    *bad_count = 0;
    const SeedTable *t = ctx->last_small ? nullptr : ctx->cur_table;
    const DevBuf *meta = ctx->last_small ? &ctx->small_meta : (t ? &t->meta : nullptr);
    if (!meta || !meta->p) return 0;
    FLM_ON_DEVICE(ctx);
    if (t && t->written_valid) FLM_HIP(ctx, hipEventSynchronize(t->written));
    if (t)
        for (const auto &r : t->readers)
            if (r.first == t->w_stream) FLM_HIP(ctx, hipEventSynchronize(r.second));
    uint32_t parts = 0;
    FLM_HIP(ctx, hipMemcpy(&parts, meta->p, sizeof parts, hipMemcpyDeviceToHost));
    if (2 + 2 * (size_t)parts > meta->cap / sizeof(uint32_t))
        return fail(ctx, FLM_EHIP, "seed table sign counts: %u parts overrun the table", parts);
    std::vector<uint32_t> m(2 + 2 * (size_t)parts);
    FLM_HIP(ctx, hipMemcpy(m.data(), meta->p, m.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (uint32_t p = 0; p < parts; ++p) *bad_count += (int)m[3 + 2 * p];
    return 0;
}

int flm_last_plan(const flm_ctx *ctx, int *items, int *tile_slots, int *atomics, int *variant) {
    if (!ctx) return FLM_EINVAL;
    if (items) *items = ctx->last_items;
    if (tile_slots) *tile_slots = ctx->last_tile;
    if (atomics) *atomics = ctx->last_atomics;
    if (variant) *variant = ctx->last_variant;
    return 0;
}

// ------------------------------------------------------------------ P-256
static int ec_dims(flm_ctx *ctx, int T, int D) {
    if (T < 0 || D < 0) return fail(ctx, FLM_EINVAL, "negative batch size (T=%d, D=%d)", T, D);
    if ((size_t)T * (size_t)D > (size_t)1 << 26) return fail(ctx, FLM_EINVAL, "batch too large (T*D=%zu)", (size_t)T * D);
    return 0;
}

// Cooperative scalar multiplication when the whole batch fits one pass of the device -- the
// latency-bound case: the row-field kernel (four waves per 4 products, ec_mul_row_kernel) up to
// 20 products per CU, e.g. one G = 8 rank's pair chunk (ceil(962/8) x 20 = 2,420: 0.77 against
// 1.20 ms per-lane-field cooperative, tools/probes/ec_kernel_sweep.py, profiles/r04_ec_kernel_sweep.log;
// still 13 % ahead at 4,800, 39 % behind at 9,620), then the per-lane-field cooperative kernel (four
// waves per 64 products, 78 KiB of LDS: two workgroups per CU) up to 128 per CU, e.g. the whole c5
// seed recovery (19,240 products); bigger batches, and launches the caller confines to a few CUs
// (ServerReconstruction's CU-split stream sets 0), keep one lane per product.
int ec_coop(flm_ctx *ctx, size_t n) {
    if (ctx->tune_ec_coop >= 0) return ctx->tune_ec_coop;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return 0;
    if (n <= (size_t)cus * 20) return 2;
    return n <= (size_t)cus * 2 * 64 ? 1 : 0;
}

int flm_ec_combine_dev(flm_ctx *ctx, const uint8_t *d_c1, const uint8_t *d_shares, const uint8_t *d_lambdas, int T,
                       int D, int negate, uint8_t *d_points_out, uint8_t *d_seeds_out, uint32_t *d_flags,
                       void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, T, D)) return rc;
    if (D == 0) return 0;
    if ((T > 0 && (!d_shares || !d_lambdas)) || !d_flags) return fail(ctx, FLM_EINVAL, "NULL argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    FLM_ON_DEVICE(ctx);
    FLM_HIP(ctx, ctx->ec_jac.reserve((size_t)std::max(T, 1) * D * 96));
    FLM_HIP(ctx, hipMemsetAsync(d_flags, 0, (size_t)D * 4, s));
    const int coop = ec_coop(ctx, (size_t)T * D);
    const int terms = coop ? 1 : ctx->tune_ec_terms;
    FLM_HIP(ctx, flm::launch_ec_mul(d_shares, d_lambdas, 0, T, D, ctx->ec_jac.as<uint32_t>(), d_flags, s,
                                    ctx->tune_ec_threads, ctx->tune_ec_waves, coop, terms,
                                    1024u * (unsigned)ctx->tune_ec_spread));
    FLM_HIP(ctx, flm::launch_ec_finish(d_c1, ctx->ec_jac.as<uint32_t>(), flm::ec_mul_groups(T, terms), D, negate,
                                       d_points_out, d_seeds_out,
                                       d_flags, s));
    return 0;
}

int flm_ec_combine(flm_ctx *ctx, const uint8_t *c1, const uint8_t *shares, const uint8_t *lambdas, int T, int D,
                   int negate, uint8_t *points_out, uint8_t *seeds_out, uint32_t *flags_out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, T, D)) return rc;
    if (D == 0) return 0;
    if (T > 0 && (!shares || !lambdas)) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    const size_t nsh = (size_t)T * D * 64;
    FLM_HIP(ctx, ctx->ec_in.reserve(nsh));
    FLM_HIP(ctx, ctx->ec_scal.reserve((size_t)T * 32));
    FLM_HIP(ctx, ctx->ec_base.reserve((size_t)D * 64));
    FLM_HIP(ctx, ctx->ec_out.reserve((size_t)D * 64));
    FLM_HIP(ctx, ctx->ec_dig.reserve((size_t)D * 32));
    FLM_HIP(ctx, ctx->ec_flags.reserve((size_t)D * 4));
    hipStream_t s = ctx->stream;
    HostCopies hc(ctx, s);
    using HC = HostCopies;
    if (int rc = hc.reserve(HC::room(nsh) + HC::room((size_t)T * 32) + HC::room((size_t)D * 64) + HC::room((size_t)D * 4) +
                            HC::room((size_t)D * 64) + HC::room((size_t)D * 32)))
        return rc;
    if (T > 0) {
        if (int rc = hc.in(ctx->ec_in.p, shares, nsh)) return rc;
        if (int rc = hc.in(ctx->ec_scal.p, lambdas, (size_t)T * 32)) return rc;
    }
    if (c1)
        if (int rc = hc.in(ctx->ec_base.p, c1, (size_t)D * 64)) return rc;
    if (int rc = flm_ec_combine_dev(ctx, c1 ? ctx->ec_base.as<uint8_t>() : nullptr, ctx->ec_in.as<uint8_t>(),
                                    ctx->ec_scal.as<uint8_t>(), T, D, negate, ctx->ec_out.as<uint8_t>(),
                                    ctx->ec_dig.as<uint8_t>(), ctx->ec_flags.as<uint32_t>(), s))
        return rc;
    std::vector<uint32_t> fl(D);
    if (int rc = hc.out(fl.data(), ctx->ec_flags.p, (size_t)D * 4)) return rc;
    if (points_out)
        if (int rc = hc.out(points_out, ctx->ec_out.p, (size_t)D * 64)) return rc;
    if (seeds_out)
        if (int rc = hc.out(seeds_out, ctx->ec_dig.p, (size_t)D * 32)) return rc;
    if (int rc = hc.finish()) return rc;
    if (flags_out) std::copy(fl.begin(), fl.end(), flags_out);
    for (int i = 0; i < D; ++i)
        if (fl[i] & 3u)
            return fail(ctx, FLM_EINVAL, "element %d: %s is not a point on P-256", i,
                        (fl[i] & 1u) ? "ciphertext c1" : "a decryption share");
    return 0;
}

int flm_shamir_combine_dev(flm_ctx *ctx, const uint8_t *d_shares, const uint8_t *d_lambdas, int T, int M,
                           uint8_t *d_seeds_out, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, T, M)) return rc;
    if (M == 0) return 0;
    if (!d_seeds_out || (T > 0 && (!d_shares || !d_lambdas))) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    hipStream_t s = static_cast<hipStream_t>(stream);
    FLM_HIP(ctx, flm::launch_shamir_combine(d_shares, d_lambdas, T, M, d_seeds_out, s));
    return 0;
}

int flm_pair_units_dev(flm_ctx *ctx, const uint8_t *d_seeds, const int8_t *d_signs, int K, const uint32_t *d_p0,
                       const uint32_t *d_p1, uint32_t *d_dst, size_t L, uint32_t *d_ws, int final_pass, int groups,
                       void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (K < 0) return fail(ctx, FLM_EINVAL, "negative K");
    if (groups <= 0) return fail(ctx, FLM_EINVAL, "groups must be positive");
    if (!d_dst || !d_ws || (K > 0 && (!d_seeds || !d_signs))) return fail(ctx, FLM_EINVAL, "NULL argument");
    if (final_pass && (!d_p0 || !d_p1)) return fail(ctx, FLM_EINVAL, "the final pass needs both partial rows");
    if (final_pass && (((uintptr_t)d_p0 | (uintptr_t)d_p1 | (uintptr_t)d_dst) & 15))
        return fail(ctx, FLM_EINVAL, "partial rows and dst must be 16-byte aligned");
    if (L > ((uint64_t)1 << 36)) return fail(ctx, FLM_EINVAL, "L=%zu beyond the 2^32-block ChaCha counter", L);
    if (flm::pair_units_count(K, L, nullptr) == 0xFFFFFFFFu) return fail(ctx, FLM_EINVAL, "too many units");
    FLM_ON_DEVICE(ctx);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (final_pass) FLM_HIP(ctx, flm::launch_add2(d_p0, d_p1, d_dst, L, s));
    if (L == 0 || K == 0) return 0;
    SeedTable *table = nullptr;
    if (int rc = run_seed_schedule(ctx, d_seeds, d_signs, K, s, &table)) return rc;
    hipError_t e = flm::launch_pair_units(!final_pass, table->recs.as<flm::SeedRec>(), K, d_dst, L, d_ws, groups, s);
    if (e == hipSuccess) e = table_read(table, s);
    if (e != hipSuccess) {
        table_cover(table, s);
        return fail(ctx, FLM_EHIP, "pair units launch: %s", hipGetErrorString(e));
    }
    return 0;
}

int flm_flag_set_dev(flm_ctx *ctx, uint32_t *d_ws, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (!d_ws) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    FLM_HIP(ctx, flm::launch_flag_set(d_ws, static_cast<hipStream_t>(stream)));
    return 0;
}

int flm_shamir_combine(flm_ctx *ctx, const uint8_t *shares, const uint8_t *lambdas, int T, int M,
                       uint8_t *seeds_out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, T, M)) return rc;
    if (M == 0) return 0;
    if (!seeds_out || (T > 0 && (!shares || !lambdas))) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    hipStream_t s = ctx->stream;
    FLM_HIP(ctx, ctx->ec_in.reserve((size_t)std::max(T, 1) * M * 32));
    FLM_HIP(ctx, ctx->ec_scal.reserve((size_t)std::max(T, 1) * 32));
    FLM_HIP(ctx, ctx->ec_dig.reserve((size_t)M * 32));
    HostCopies hc(ctx, s);
    if (int rc = hc.reserve(HostCopies::room((size_t)T * M * 32) + HostCopies::room((size_t)T * 32) +
                            HostCopies::room((size_t)M * 32)))
        return rc;
    if (T > 0) {
        if (int rc = hc.in(ctx->ec_in.p, shares, (size_t)T * M * 32)) return rc;
        if (int rc = hc.in(ctx->ec_scal.p, lambdas, (size_t)T * 32)) return rc;
    }
    FLM_HIP(ctx, flm::launch_shamir_combine(ctx->ec_in.as<uint8_t>(), ctx->ec_scal.as<uint8_t>(), T, M,
                                            ctx->ec_dig.as<uint8_t>(), s));
    if (int rc = hc.out(seeds_out, ctx->ec_dig.p, (size_t)M * 32)) return rc;
    return hc.finish();
}

int flm_ec_mul(flm_ctx *ctx, const uint8_t *points, const uint8_t *scalars, int n, uint8_t *out, uint32_t *flags_out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, 1, n)) return rc;
    if (n == 0) return 0;
    if (!points || !scalars || !out) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    FLM_HIP(ctx, ctx->ec_in.reserve((size_t)n * 64));
    FLM_HIP(ctx, ctx->ec_scal.reserve((size_t)n * 32));
    FLM_HIP(ctx, ctx->ec_jac.reserve((size_t)n * 96));
    FLM_HIP(ctx, ctx->ec_out.reserve((size_t)n * 64));
    FLM_HIP(ctx, ctx->ec_flags.reserve((size_t)n * 4));
    hipStream_t s = ctx->stream;
    HostCopies hc(ctx, s);
    if (int rc = hc.reserve(2 * HostCopies::room((size_t)n * 64) + HostCopies::room((size_t)n * 32) +
                            HostCopies::room((size_t)n * 4)))
        return rc;
    if (int rc = hc.in(ctx->ec_in.p, points, (size_t)n * 64)) return rc;
    if (int rc = hc.in(ctx->ec_scal.p, scalars, (size_t)n * 32)) return rc;
    FLM_HIP(ctx, hipMemsetAsync(ctx->ec_flags.p, 0, (size_t)n * 4, s));
    FLM_HIP(ctx, flm::launch_ec_mul(ctx->ec_in.as<uint8_t>(), ctx->ec_scal.as<uint8_t>(), 1, 1, n,
                                    ctx->ec_jac.as<uint32_t>(), ctx->ec_flags.as<uint32_t>(), s,
                                    ctx->tune_ec_threads, ctx->tune_ec_waves, ec_coop(ctx, (size_t)n)));
    FLM_HIP(ctx, flm::launch_ec_finish(nullptr, ctx->ec_jac.as<uint32_t>(), 1, n, 0, ctx->ec_out.as<uint8_t>(),
                                       nullptr, ctx->ec_flags.as<uint32_t>(), s));
    std::vector<uint32_t> fl(n);
    if (int rc = hc.out(fl.data(), ctx->ec_flags.p, (size_t)n * 4)) return rc;
    if (int rc = hc.out(out, ctx->ec_out.p, (size_t)n * 64)) return rc;
    if (int rc = hc.finish()) return rc;
    if (flags_out) std::copy(fl.begin(), fl.end(), flags_out);
    for (int i = 0; i < n; ++i)
        if (fl[i] & 2u) return fail(ctx, FLM_EINVAL, "element %d: input is not a point on P-256", i);
    return 0;
}

static int h2c_run(flm_ctx *ctx, const uint8_t *msgs, const uint32_t *lens, uint32_t v0, int n, uint8_t *out,
                   uint32_t *flags_out) {
    FLM_ON_DEVICE(ctx);
    hipStream_t s = ctx->stream;
    FLM_HIP(ctx, ctx->ec_out.reserve((size_t)n * 64));
    FLM_HIP(ctx, ctx->ec_flags.reserve((size_t)n * 4));
    HostCopies hc(ctx, s);
    if (int rc = hc.reserve(2 * HostCopies::room((size_t)n * 64) + 2 * HostCopies::room((size_t)n * 4))) return rc;
    if (msgs) {
        FLM_HIP(ctx, ctx->ec_in.reserve((size_t)n * 64));
        FLM_HIP(ctx, ctx->ec_scal.reserve((size_t)n * 4));
        if (int rc = hc.in(ctx->ec_in.p, msgs, (size_t)n * 64)) return rc;
        if (int rc = hc.in(ctx->ec_scal.p, lens, (size_t)n * 4)) return rc;
    }
    FLM_HIP(ctx, flm::launch_hash_to_curve(msgs ? ctx->ec_in.as<uint8_t>() : nullptr,
                                           msgs ? ctx->ec_scal.as<uint32_t>() : nullptr, v0, n,
                                           ctx->ec_out.as<uint8_t>(), ctx->ec_flags.as<uint32_t>(), s));
    std::vector<uint32_t> fl(n);
    if (int rc = hc.out(fl.data(), ctx->ec_flags.p, (size_t)n * 4)) return rc;
    if (int rc = hc.out(out, ctx->ec_out.p, (size_t)n * 64)) return rc;
    if (int rc = hc.finish()) return rc;
    if (flags_out) std::copy(fl.begin(), fl.end(), flags_out);
    for (int i = 0; i < n; ++i)
        if (fl[i] & 8u) return fail(ctx, FLM_EINVAL, "message %d: map_to_curve found no square root", i);
    return 0;
}

int flm_hash_to_curve(flm_ctx *ctx, const uint8_t *msgs, const uint32_t *lens, int n, uint8_t *out,
                      uint32_t *flags_out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, 1, n)) return rc;
    if (n == 0) return 0;
    if (!msgs || !lens || !out) return fail(ctx, FLM_EINVAL, "NULL argument");
    for (int i = 0; i < n; ++i)
        if (lens[i] > 64) return fail(ctx, FLM_EINVAL, "message %d is %u bytes (at most 64)", i, lens[i]);
    return h2c_run(ctx, msgs, lens, 0, n, out, flags_out);
}

int flm_hash_to_curve_decimal(flm_ctx *ctx, uint32_t v0, int n, uint8_t *out, uint32_t *flags_out) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, 1, n)) return rc;
    if (n == 0) return 0;
    if (!out) return fail(ctx, FLM_EINVAL, "NULL argument");
    if ((uint64_t)v0 + (uint64_t)n > (1ull << 32)) return fail(ctx, FLM_EINVAL, "v0 + n exceeds 2^32");
    return h2c_run(ctx, nullptr, nullptr, v0, n, out, flags_out);
}

int flm_hash_to_curve_decimal_dev(flm_ctx *ctx, uint32_t v0, int n, uint8_t *d_out, uint32_t *d_flags, void *stream) {
    if (!ctx) return fail(nullptr, FLM_EINVAL, "ctx is NULL");
    if (int rc = ec_dims(ctx, 1, n)) return rc;
    if (n == 0) return 0;
    if (!d_out || !d_flags) return fail(ctx, FLM_EINVAL, "NULL argument");
    if ((uint64_t)v0 + (uint64_t)n > (1ull << 32)) return fail(ctx, FLM_EINVAL, "v0 + n exceeds 2^32");
    FLM_ON_DEVICE(ctx);
    FLM_HIP(ctx, flm::launch_hash_to_curve(nullptr, nullptr, v0, n, d_out, d_flags, static_cast<hipStream_t>(stream)));
    return 0;
}

void *flm_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void flm_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

int flm_cu_count(flm_ctx *ctx, int *n_cus) {
    if (!ctx || !n_cus) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_HIP(ctx, hipDeviceGetAttribute(n_cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    return 0;
}

int flm_stream_create_cu_mask(flm_ctx *ctx, const uint32_t *mask, int n_words, void **stream_out) {
    if (!ctx || !mask || !stream_out || n_words <= 0) return fail(ctx, FLM_EINVAL, "NULL argument or empty mask");
    int n_cus = 0;
    FLM_HIP(ctx, hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    int set = 0;
    for (int w = 0; w < n_words; ++w)
        for (int b = 0; b < 32; ++b)
            if ((mask[w] >> b) & 1u) {
                if (w * 32 + b >= n_cus)
                    return fail(ctx, FLM_EINVAL, "CU mask names CU %d of %d", w * 32 + b, n_cus);
                ++set;
            }
    if (set == 0) return fail(ctx, FLM_EINVAL, "CU mask selects no CU");
    FLM_ON_DEVICE(ctx);
    hipStream_t s = nullptr;
    FLM_HIP(ctx, hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask));
    *stream_out = s;
    return 0;
}

int flm_stream_destroy(flm_ctx *ctx, void *stream) {
    if (!ctx || !stream) return fail(ctx, FLM_EINVAL, "NULL argument");
    FLM_ON_DEVICE(ctx);
    FLM_HIP(ctx, hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return 0;
}

}  // extern "C"
