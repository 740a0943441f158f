// flm_store.hip -- device-resident VECTOR ingestion for the drop-in server (include/flamingo_hip.h).
//
// The reference server keeps every client's VECTOR body in a dict on arrival
// (SA_ServiceAgent.py:205-210), sums them in report_process (:346-350) and, one step later,
// adds the regenerated masks to that sum in reconstruction_process (:529-540, :587-605).  A
// store keeps those three moments on the GPU(s):
//   flm_store_add      on arrival: the body is copied into a pinned staging ring and DMA'd onto
//                      its device row on a copy stream of its own, so the upload overlaps the
//                      simulation's message handling; the call returns once the host copy is made;
//   flm_store_partial  at report: S = sum of the stored rows, device-resident (on a group:
//                      client-sharded rows, slot-sharded S after one reduce-scatter);
//   flm_store_unmask   at reconstruction: final = S + sum sign*PRG(seed) over each device's own
//                      slot shard (S is already sharded: no exchange), then the one copy out.
// No L-vector crosses PCIe between report and reconstruction.  Rows are placed round-robin over
// the devices in arrival order; a sender that sends twice overwrites its row, like the
// reference's dict assignment.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/flamingo_hip.h"
#include "flm_internal.h"

namespace {
constexpr int kStoreRing = 8;  // pinned staging buffers per device

struct StoreRank {
    flm_ctx *ctx = nullptr;
    int device = 0;
    hipStream_t copy = nullptr;   // uploads
    uint32_t *rows = nullptr;     // cap x pitch words
    int cap = 0, n = 0;
    uint32_t *S = nullptr;        // this rank's slots of the partial sum (S words)
    uint32_t *out = nullptr;      // unmask output (S words)
    uint8_t *seeds = nullptr;     // K x 32 + K signs, per unmask
    size_t seeds_cap = 0;
    void *stage[kStoreRing] = {};
    hipEvent_t stage_done[kStoreRing] = {};
    bool stage_busy[kStoreRing] = {};
    int next = 0;
    hipEvent_t uploaded = nullptr;  // copy stream: every add so far
    hipEvent_t consumed = nullptr;  // the last partial sum has read the rows
    bool consumed_pending = false;
    size_t lo = 0, hi = 0;          // output slots of this rank
};
}  // namespace

struct flm_store {
    flm_group *group = nullptr;
    bool via_group = false;      // partial sums through the group's sharded round (G > 1, or an RCCL clique)
    size_t L = 0, pitch = 0, S = 0;
    std::vector<StoreRank> rk;
    std::unordered_map<int64_t, std::pair<int, int>> slot;
    int bad = 0;                 // bodies of the wrong length since the last reset
    bool have_partial = false;
    hipEvent_t t0 = nullptr, t1 = nullptr;  // device time of the last partial sum (rank 0)
    hipEvent_t u0 = nullptr, u1 = nullptr;  // device time of the last unmask, uploads to D2H (rank 0)
    float unmask_ms = -1.0f;
    // pinned bounce buffers of the host-facing calls (flm_store_unmask, flm_store_partial_host): the
    // caller's seeds and output are pageable numpy memory, which HIP would stage or pin per call
    uint8_t *hseeds = nullptr;   // K x 32 seeds + K signs
    size_t hseeds_cap = 0;
    uint32_t *hout = nullptr;    // L words: every rank's shard lands at its offset lo
    bool bounce_busy = false;    // a call that failed after enqueueing may have left DMAs reading them
    std::string err;
};

namespace {

int sfail(flm_store *st, int code, const std::string &msg) {
    if (st) st->err = msg;
    flm::rt::set_error(nullptr, code, msg.c_str());
    return code;
}

#define FLM_SHIP(st, expr)                                                                           \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) return sfail((st), FLM_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

int grow_rows(flm_store *st, StoreRank &r, int want) {
    if (want <= r.cap) return 0;
    const int cap = std::max(want, std::max(1, 2 * r.cap));
    FLM_SHIP(st, hipSetDevice(r.device));
    uint32_t *p = nullptr;
    FLM_SHIP(st, hipMalloc(&p, (size_t)cap * st->pitch * sizeof(uint32_t)));
    if (r.rows) {
        // growth is rare (capacity is the expected client count): copy in stream order, then free
        hipError_t e = hipMemcpyAsync(p, r.rows, (size_t)r.cap * st->pitch * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                      r.copy);
        if (e == hipSuccess) e = hipStreamSynchronize(r.copy);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return sfail(st, FLM_EHIP, std::string("store row growth: ") + hipGetErrorString(e));
        }
        (void)hipFree(r.rows);
    }
    r.rows = p;
    r.cap = cap;
    return 0;
}

// The pinned bounce buffers are free once every rank's stream has drained (only after a call that
// returned an error between its enqueues and its synchronisation can they still be in use).
int bounce_idle(flm_store *st) {
    if (!st->bounce_busy) return 0;
    for (StoreRank &k : st->rk) {
        FLM_SHIP(st, hipSetDevice(k.device));
        FLM_SHIP(st, hipStreamSynchronize(flm::rt::stream_of(k.ctx)));
    }
    st->bounce_busy = false;
    return 0;
}

// Only the store's own objects are touched: the context or group may already be gone (a caller
// that frees its group first).  Its own events cover every queued use of its buffers: uploads on
// the copy stream, the partial sum (consumed, t1); flm_store_unmask is synchronous.
void release(flm_store *st) {
    if (st->have_partial && st->t1) {
        (void)hipSetDevice(st->rk[0].device);
        (void)hipEventSynchronize(st->t1);
    }
    for (StoreRank &r : st->rk) {
        (void)hipSetDevice(r.device);
        if (r.copy) (void)hipStreamSynchronize(r.copy);
        if (r.consumed && r.consumed_pending) (void)hipEventSynchronize(r.consumed);
        for (int b = 0; b < kStoreRing; ++b) {
            if (r.stage[b]) (void)hipHostFree(r.stage[b]);
            if (r.stage_done[b]) (void)hipEventDestroy(r.stage_done[b]);
        }
        if (r.rows) (void)hipFree(r.rows);
        if (r.S) (void)hipFree(r.S);
        if (r.out) (void)hipFree(r.out);
        if (r.seeds) (void)hipFree(r.seeds);
        if (r.uploaded) (void)hipEventDestroy(r.uploaded);
        if (r.consumed) (void)hipEventDestroy(r.consumed);
        if (r.copy) (void)hipStreamDestroy(r.copy);
    }
    if (st->hseeds) (void)hipHostFree(st->hseeds);
    if (st->hout) (void)hipHostFree(st->hout);
    if (st->t0) (void)hipEventDestroy(st->t0);
    if (st->t1) (void)hipEventDestroy(st->t1);
    if (st->u0) (void)hipEventDestroy(st->u0);
    if (st->u1) (void)hipEventDestroy(st->u1);
}

}  // namespace

extern "C" {

int flm_store_create(flm_store **out, flm_ctx *ctx, flm_group *g, size_t L, int capacity) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!out) return sfail(nullptr, FLM_EINVAL, "flm_store_create: out is NULL");
    *out = nullptr;
    if ((ctx == nullptr) == (g == nullptr)) return sfail(nullptr, FLM_EINVAL, "flm_store_create: give a context or a group");
    if (L == 0 || L > (1ull << 36)) return sfail(nullptr, FLM_EINVAL, "flm_store_create: L must be in [1, 2^36]");
    auto *st = new flm_store();
    st->group = g;
    st->L = L;
    st->pitch = (L + 63) / 64 * 64;  // rows 256-B aligned, pitch a multiple of 4 words
    const int G = g ? flm_group_size(g) : 1;
    // a one-device group with an RCCL clique (FLM_GROUP_RCCL) goes through the group's round too
    st->via_group = g && (G > 1 || flm_group_has_rccl(g));
    size_t lo = 0, hi = L, S = st->pitch;
    st->rk.resize(G);
    for (int r = 0; r < G; ++r) {
        StoreRank &k = st->rk[r];
        k.ctx = g ? flm_group_ctx(g, r) : ctx;
        k.device = flm::rt::device_of(k.ctx);
        if (st->via_group) flm_shard_bounds(L, G, r, &lo, &hi, &S);
        k.lo = lo;
        k.hi = hi;
    }
    st->S = st->via_group ? S : st->pitch;
    int rc = 0;
    const int per = std::max(1, (capacity + G - 1) / G);
    for (int r = 0; r < G && !rc; ++r) {
        StoreRank &k = st->rk[r];
        hipError_t e = hipSetDevice(k.device);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&k.copy, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&k.uploaded, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&k.consumed, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMalloc(&k.S, st->S * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMalloc(&k.out, st->S * sizeof(uint32_t));
        // the unmask's seeds + signs (33 B each): |U| + D seeds, D about a quarter of N at 1 %
        // dropouts and neighbourhood ~22 (c5), so 2 N seeds now and grow_bytes' slack later
        if (e == hipSuccess) {
            k.seeds_cap = flm::rt::grow_bytes((size_t)std::max(1, capacity) * 2 * 33);
            e = hipMalloc(&k.seeds, k.seeds_cap);
            if (e != hipSuccess) k.seeds_cap = 0;
        }
        for (int b = 0; b < kStoreRing && e == hipSuccess; ++b) {
            e = hipHostMalloc(&k.stage[b], L * sizeof(uint32_t), hipHostMallocDefault);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&k.stage_done[b], hipEventDisableTiming);
        }
        if (e != hipSuccess) rc = sfail(st, FLM_ENOMEM, std::string("flm_store_create: ") + hipGetErrorString(e));
        if (!rc) rc = grow_rows(st, k, per);
    }
    if (!rc) {
        (void)hipSetDevice(st->rk[0].device);
        if (hipEventCreate(&st->t0) != hipSuccess || hipEventCreate(&st->t1) != hipSuccess ||
            hipEventCreate(&st->u0) != hipSuccess || hipEventCreate(&st->u1) != hipSuccess)
            rc = sfail(st, FLM_EHIP, "flm_store_create: hipEventCreate");
        else if (hipHostMalloc(&st->hout, L * sizeof(uint32_t), hipHostMallocPortable) != hipSuccess)
            rc = sfail(st, FLM_ENOMEM, "flm_store_create: pinned output buffer");
    }
    if (rc) {
        std::string m = st->err;
        release(st);
        delete st;
        return sfail(nullptr, rc, m);
    }
    *out = st;
    return 0;
}

void flm_store_free(flm_store *st) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st) return;
    release(st);
    delete st;
}

const char *flm_store_last_error(const flm_store *st) { return st ? st->err.c_str() : flm_last_error(nullptr); }

int flm_store_count(const flm_store *st) { return st ? (int)st->slot.size() : 0; }

int flm_store_add(flm_store *st, int64_t sender, const uint32_t *row, size_t n) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st) return sfail(nullptr, FLM_EINVAL, "store is NULL");
    if (!row || n != st->L) {  // report_process raises on it (:348-349): remembered for flm_store_partial
        ++st->bad;
        return 0;
    }
    int r, i;
    auto f = st->slot.find(sender);
    if (f != st->slot.end()) {
        r = f->second.first;
        i = f->second.second;
    } else {
        r = (int)(st->slot.size() % st->rk.size());
        i = st->rk[r].n;
        if (int rc = grow_rows(st, st->rk[r], i + 1)) return rc;
        st->rk[r].n = i + 1;
        st->slot.emplace(sender, std::make_pair(r, i));
    }
    StoreRank &k = st->rk[r];
    FLM_SHIP(st, hipSetDevice(k.device));
    if (k.consumed_pending) {
        // an add between flm_store_partial and flm_store_reset (a late VECTOR the caller forwards
        // anyway) may overwrite a row the partial sum is still reading: the upload waits for it
        FLM_SHIP(st, hipStreamWaitEvent(k.copy, k.consumed, 0));
        k.consumed_pending = false;
    }
    const int b = k.next;
    k.next = (b + 1) % kStoreRing;
    if (k.stage_busy[b]) FLM_SHIP(st, hipEventSynchronize(k.stage_done[b]));  // its last DMA has read it
    flm::rt::host_copy(k.ctx, k.stage[b], row, st->L * sizeof(uint32_t));
    FLM_SHIP(st, hipMemcpyAsync(k.rows + (size_t)i * st->pitch, k.stage[b], st->L * sizeof(uint32_t),
                                hipMemcpyHostToDevice, k.copy));
    FLM_SHIP(st, hipEventRecord(k.stage_done[b], k.copy));
    k.stage_busy[b] = true;
    return 0;
}

int flm_store_partial(flm_store *st) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st) return sfail(nullptr, FLM_EINVAL, "store is NULL");
    if (st->bad) return sfail(st, FLM_EINVAL, "Client sends vector of incorrect length.");
    const int G = (int)st->rk.size();
    FLM_SHIP(st, hipSetDevice(st->rk[0].device));
    FLM_SHIP(st, hipEventRecord(st->t0, flm::rt::stream_of(st->rk[0].ctx)));
    for (StoreRank &k : st->rk) {  // each rank's round runs after its uploads
        FLM_SHIP(st, hipSetDevice(k.device));
        FLM_SHIP(st, hipEventRecord(k.uploaded, k.copy));
        FLM_SHIP(st, hipStreamWaitEvent(flm::rt::stream_of(k.ctx), k.uploaded, 0));
    }
    if (!st->via_group) {
        StoreRank &k = st->rk[0];
        hipStream_t s = flm::rt::stream_of(k.ctx);
        if (k.n) {
            if (int rc = flm_aggregate_unmask_dev(k.ctx, k.rows, st->pitch, k.n, nullptr, nullptr, 0, st->L, 0, 0, 0,
                                                  k.S, s))
                return sfail(st, rc, std::string("store partial: ") + flm_last_error(k.ctx));
        } else {
            FLM_SHIP(st, hipMemsetAsync(k.S, 0, st->S * sizeof(uint32_t), s));
        }
    } else {
        std::vector<const uint32_t *> rows(G);
        std::vector<int> n(G);
        std::vector<uint32_t *> shards(G);
        for (int r = 0; r < G; ++r) {
            rows[r] = st->rk[r].n ? st->rk[r].rows : nullptr;
            n[r] = st->rk[r].n;
            shards[r] = st->rk[r].S;
        }
        if (int rc = flm_group_aggregate_unmask_dev(st->group, rows.data(), st->pitch, n.data(), nullptr, nullptr, 0,
                                                    st->L, shards.data()))
            return sfail(st, rc, std::string("store partial: ") + flm_group_last_error(st->group));
    }
    for (StoreRank &k : st->rk) {
        FLM_SHIP(st, hipSetDevice(k.device));
        FLM_SHIP(st, hipEventRecord(k.consumed, flm::rt::stream_of(k.ctx)));
        k.consumed_pending = true;
    }
    // rank 0's stream marks the end once every rank's S is complete (the group's exchange)
    FLM_SHIP(st, hipSetDevice(st->rk[0].device));
    hipStream_t s0 = flm::rt::stream_of(st->rk[0].ctx);
    for (int r = 1; r < G; ++r) FLM_SHIP(st, hipStreamWaitEvent(s0, st->rk[r].consumed, 0));
    FLM_SHIP(st, hipEventRecord(st->t1, s0));
    st->have_partial = true;
    return 0;
}

int flm_store_partial_wait(flm_store *st, float *gpu_ms) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st) return sfail(nullptr, FLM_EINVAL, "store is NULL");
    if (!st->have_partial) return sfail(st, FLM_EINVAL, "no partial sum enqueued");
    FLM_SHIP(st, hipSetDevice(st->rk[0].device));
    FLM_SHIP(st, hipEventSynchronize(st->t1));
    if (gpu_ms) FLM_SHIP(st, hipEventElapsedTime(gpu_ms, st->t0, st->t1));
    return 0;
}

int flm_store_partial_host(flm_store *st, uint32_t *out) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st || !out) return sfail(st, FLM_EINVAL, "NULL argument");
    if (!st->have_partial) return sfail(st, FLM_EINVAL, "no partial sum enqueued");
    if (int rc = bounce_idle(st)) return rc;
    st->bounce_busy = true;
    for (StoreRank &k : st->rk) {
        if (k.hi <= k.lo) continue;
        FLM_SHIP(st, hipSetDevice(k.device));
        FLM_SHIP(st, hipMemcpyAsync(st->hout + k.lo, k.S, (k.hi - k.lo) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                    flm::rt::stream_of(k.ctx)));
    }
    for (StoreRank &k : st->rk) {
        FLM_SHIP(st, hipSetDevice(k.device));
        FLM_SHIP(st, hipStreamSynchronize(flm::rt::stream_of(k.ctx)));
    }
    st->bounce_busy = false;
    flm::rt::host_copy(st->rk[0].ctx, out, st->hout, st->L * sizeof(uint32_t));
    return 0;
}

int flm_store_unmask(flm_store *st, const uint8_t *seeds, const int8_t *signs, int K, uint32_t *out) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st || !out || K < 0 || (K > 0 && (!seeds || !signs))) return sfail(st, FLM_EINVAL, "bad argument");
    if (!st->have_partial) return sfail(st, FLM_EINVAL, "no partial sum: call flm_store_partial at report");
    for (int k = 0; k < K; ++k)
        if (signs[k] != 1 && signs[k] != -1) return sfail(st, FLM_EINVAL, "signs must be +1 or -1");
    const size_t sb = (size_t)K * 33;
    st->unmask_ms = -1.0f;
    if (int rc = bounce_idle(st)) return rc;
    if (K > 0) {  // one pinned copy of seeds + signs, read by every rank's upload (idle: the last call synced)
        if (st->hseeds_cap < sb) {
            if (st->hseeds) (void)hipHostFree(st->hseeds);
            st->hseeds = nullptr;
            st->hseeds_cap = 0;
            const size_t want = flm::rt::grow_bytes(sb);
            FLM_SHIP(st, hipHostMalloc(&st->hseeds, want, hipHostMallocPortable));
            st->hseeds_cap = want;
        }
        std::memcpy(st->hseeds, seeds, (size_t)K * 32);
        std::memcpy(st->hseeds + (size_t)K * 32, signs, (size_t)K);
    }
    FLM_SHIP(st, hipSetDevice(st->rk[0].device));
    FLM_SHIP(st, hipEventRecord(st->u0, flm::rt::stream_of(st->rk[0].ctx)));
    st->bounce_busy = true;
    for (StoreRank &k : st->rk) {
        const size_t n = k.hi - k.lo;
        if (n == 0) continue;
        FLM_SHIP(st, hipSetDevice(k.device));
        hipStream_t s = flm::rt::stream_of(k.ctx);
        if (K > 0) {
            if (k.seeds_cap < sb) {
                if (k.seeds) FLM_SHIP(st, hipStreamSynchronize(s));  // the last unmask may still read it
                if (k.seeds) (void)hipFree(k.seeds);
                k.seeds = nullptr;
                k.seeds_cap = 0;
                const size_t want = flm::rt::grow_bytes(sb);  // K moves by a few % per iteration
                FLM_SHIP(st, hipMalloc(&k.seeds, want));
                k.seeds_cap = want;
            }
            FLM_SHIP(st, hipMemcpyAsync(k.seeds, st->hseeds, sb, hipMemcpyHostToDevice, s));
        }
        // final[lo + l] = S[l] + sum_k sign_k PRG(seed_k)[lo + l], l < n: S as one row, PRG words lo..
        if (int rc = flm_aggregate_unmask_dev(k.ctx, k.S, st->S, 1, K ? k.seeds : nullptr,
                                              K ? reinterpret_cast<const int8_t *>(k.seeds + (size_t)K * 32) : nullptr,
                                              K, n, 0, n, k.lo, k.out, s))
            return sfail(st, rc, std::string("store unmask: ") + flm_last_error(k.ctx));
        FLM_SHIP(st, hipMemcpyAsync(st->hout + k.lo, k.out, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
    FLM_SHIP(st, hipSetDevice(st->rk[0].device));
    FLM_SHIP(st, hipEventRecord(st->u1, flm::rt::stream_of(st->rk[0].ctx)));
    for (StoreRank &k : st->rk) {
        FLM_SHIP(st, hipSetDevice(k.device));
        FLM_SHIP(st, hipStreamSynchronize(flm::rt::stream_of(k.ctx)));
    }
    st->bounce_busy = false;
    flm::rt::host_copy(st->rk[0].ctx, out, st->hout, st->L * sizeof(uint32_t));
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, st->u0, st->u1) == hipSuccess) st->unmask_ms = ms;
    return 0;
}

int flm_store_unmask_ms(const flm_store *st, float *gpu_ms) {
    if (!st || !gpu_ms) return FLM_EINVAL;
    if (st->unmask_ms < 0.0f) return sfail(const_cast<flm_store *>(st), FLM_EINVAL, "no unmask has completed");
    *gpu_ms = st->unmask_ms;
    return 0;
}

int flm_store_reset(flm_store *st) {
    flm::rt::DeviceScope dev_scope_;  // the caller's device comes back on return
    if (!st) return sfail(nullptr, FLM_EINVAL, "store is NULL");
    st->slot.clear();
    st->bad = 0;
    for (StoreRank &k : st->rk) {
        k.n = 0;
        if (k.consumed_pending) {  // the next arrivals overwrite rows the last partial sum reads
            FLM_SHIP(st, hipSetDevice(k.device));
            FLM_SHIP(st, hipStreamWaitEvent(k.copy, k.consumed, 0));
            k.consumed_pending = false;
        }
    }
    return 0;
}

}  // extern "C"
