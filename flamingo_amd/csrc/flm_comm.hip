// flm_comm.hip -- RCCL over xGMI for the multi-GPU server round.
//
// The reference server is one single-threaded discrete-event process
// (Kernel.py:190-271); its partial sum and unmask (SA_ServiceAgent.py:346-350,
// 529-605) are one vector of L uint32.  On G GPUs the work shards two ways:
//   * rows by client: rank r ingests clients [N*r/G, N*(r+1)/G) over its own link
//     and sums them over all L slots;
//   * masks by slot: rank r regenerates every seed's mask over its own shard
//     [r*S, (r+1)*S) only, S = round_up(L, 1024*G) / G (the VALU-bound part);
// then ONE reduce-scatter (ncclUint32, ncclSum: mod 2^32, so any ring order gives
// the same bits) returns each rank its shard of S + C + M.
//
// Two ways to drive it:
//   * one process per GPU (torchrun): each process attaches a communicator to its
//     context (flm_comm_init_rank) and calls flm_reduce_scatter_dev on its partial;
//   * one process for all GPUs (the drop-in DES server): flm_group owns one context
//     per device plus a communicator clique (ncclCommInitAll), and
//     flm_group_aggregate_unmask runs the whole round from host rows.
//
// RCCL is resolved at run time (dlopen) so the library links against no RCCL:
// the copy already loaded in the process (PyTorch's, which matches the HIP runtime
// PyTorch loaded) is preferred, else /opt/rocm's librccl.so.1.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/flamingo_hip.h"
#include "flm_internal.h"

namespace {

struct Rccl {
    void *h = nullptr;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommFinalize)(ncclComm_t) = nullptr;  // optional: RCCL builds before 2.18 lack it
    ncclResult_t (*ReduceScatter)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                  hipStream_t) = nullptr;
    ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl &rccl_state() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *env = getenv("FLM_RCCL_LIBRARY");
        const char *names[] = {"librccl.so", "librccl.so.1"};
        if (env && *env) r.h = dlopen(env, RTLD_NOW | RTLD_GLOBAL);
        for (const char *n : names)  // a copy some other library (PyTorch) already loaded
            if (!r.h) r.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
        if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!r.h) {
            r.err = std::string("cannot load RCCL: ") + dlerror();
            return;
        }
#define FLM_SYM(field, name)                                                   \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.h, name));           \
    if (!r.field) {                                                            \
        r.err = std::string("RCCL symbol missing: ") + name;                   \
        r.h = nullptr;                                                         \
        return;                                                                \
    }
        FLM_SYM(GetUniqueId, "ncclGetUniqueId");
        FLM_SYM(CommInitRank, "ncclCommInitRank");
        FLM_SYM(CommInitAll, "ncclCommInitAll");
        FLM_SYM(CommDestroy, "ncclCommDestroy");
        FLM_SYM(ReduceScatter, "ncclReduceScatter");
        FLM_SYM(AllGather, "ncclAllGather");
        FLM_SYM(GroupStart, "ncclGroupStart");
        FLM_SYM(GroupEnd, "ncclGroupEnd");
        FLM_SYM(GetErrorString, "ncclGetErrorString");
#undef FLM_SYM
        r.CommFinalize = reinterpret_cast<decltype(r.CommFinalize)>(dlsym(r.h, "ncclCommFinalize"));
    });
    return r;
}

Rccl *rccl() {
    Rccl &r = rccl_state();
    return r.h ? &r : nullptr;
}

struct CommState {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
};

CommState *comm_of(flm_ctx *ctx) { return static_cast<CommState *>(*flm::rt::comm_slot(ctx)); }

int fail_ctx(flm_ctx *ctx, int code, const char *fmt, ...) __attribute__((format(printf, 3, 4)));
int fail_ctx(flm_ctx *ctx, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return flm::rt::set_error(ctx, code, buf);
}

int rccl_missing(flm_ctx *ctx) {
    return fail_ctx(ctx, FLM_EHIP, "RCCL unavailable (set FLM_RCCL_LIBRARY to librccl.so's path)");
}

#define FLM_NCCL(ctx, expr)                                                                           \
    do {                                                                                              \
        ncclResult_t r_ = (expr);                                                                     \
        if (r_ != ncclSuccess)                                                                        \
            return fail_ctx((ctx), FLM_EHIP, "%s failed: %s", #expr, rccl()->GetErrorString(r_));    \
    } while (0)

#define FLM_HIPC(ctx, expr)                                                                           \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return fail_ctx((ctx), FLM_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

}  // namespace

namespace flm {
// Finalize (flushes the communicator's outstanding operations and joins its proxy work) and then
// destroy, with the context's device current.  Callers synchronise the device first (flm_free and
// flm_comm_destroy call hipDeviceSynchronize when a communicator is attached): the collectives may
// have been enqueued on streams other than the context's own (a torch comm stream).  One process
// per GPU: each rank finalizes its own communicator.  A one-thread clique goes through
// comm_release_clique instead.
void comm_release(flm_ctx *ctx) {
    CommState *cs = comm_of(ctx);
    if (!cs) return;
    if (cs->comm && rccl()) {
        if (rccl()->CommFinalize) (void)rccl()->CommFinalize(cs->comm);
        (void)rccl()->CommDestroy(cs->comm);
    }
    delete cs;
    *flm::rt::comm_slot(ctx) = nullptr;
}

// A clique driven by one thread (ncclCommInitAll, flm_group): every device is synchronised, then
// all members are finalized inside ONE group -- a member's finalize waits for the clique to be
// quiescent, so finalizing them one after another from this thread could wait on members not yet
// finalized -- and only then destroyed.  Without ncclCommFinalize (RCCL before 2.18) the members are
// destroyed one by one, as NCCL's single-thread examples do.
void comm_release_clique(flm_ctx *const *ctxs, int n) {
    Rccl *r = rccl();
    std::vector<CommState *> cs;
    for (int q = 0; q < n; ++q)
        if (CommState *c = comm_of(ctxs[q])) cs.push_back(c);
    if (cs.empty()) return;
    for (int q = 0; q < n; ++q) {
        if (hipSetDevice(flm::rt::device_of(ctxs[q])) == hipSuccess) (void)hipDeviceSynchronize();
        (void)hipGetLastError();
    }
    if (r && r->CommFinalize) {
        (void)r->GroupStart();
        for (CommState *c : cs)
            if (c->comm) (void)r->CommFinalize(c->comm);
        (void)r->GroupEnd();
    }
    for (int q = 0; q < n; ++q) {
        CommState *c = comm_of(ctxs[q]);
        if (!c) continue;
        (void)hipSetDevice(flm::rt::device_of(ctxs[q]));
        if (c->comm && r) (void)r->CommDestroy(c->comm);
        delete c;
        *flm::rt::comm_slot(ctxs[q]) = nullptr;
    }
}
}  // namespace flm

// =========================================================== shard geometry
namespace {
constexpr uint64_t kShardAlign = 1024;  // one wave's sub-tile: every shard start is a multiple of 16 slots

uint64_t padded_len(uint64_t L, int G) {
    const uint64_t q = kShardAlign * (uint64_t)G;
    return (L + q - 1) / q * q;
}
}  // namespace

extern "C" {

int flm_shard_bounds(size_t L, int n_ranks, int rank, size_t *lo, size_t *hi, size_t *shard_words) {
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || !lo || !hi) return FLM_EINVAL;
    const uint64_t S = padded_len(L, n_ranks) / n_ranks;
    *lo = (size_t)std::min<uint64_t>((uint64_t)rank * S, L);
    *hi = (size_t)std::min<uint64_t>((uint64_t)(rank + 1) * S, L);
    if (shard_words) *shard_words = (size_t)S;
    return 0;
}

int flm_client_bounds(int N, int n_ranks, int rank, int *c0, int *c1) {
    if (N < 0 || n_ranks < 1 || rank < 0 || rank >= n_ranks || !c0 || !c1) return FLM_EINVAL;
    *c0 = (int)((int64_t)N * rank / n_ranks);
    *c1 = (int)((int64_t)N * (rank + 1) / n_ranks);
    return 0;
}

// ======================================================= one process per GPU
int flm_rccl_available(void) {
    Rccl *r = rccl();
    if (!r) {
        flm::rt::set_error(nullptr, FLM_EHIP, rccl_state().err.c_str());
        return 0;
    }
    return 1;
}

int flm_comm_unique_id(uint8_t id_out[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId must be 128 bytes");
    if (!id_out) return FLM_EINVAL;
    Rccl *r = rccl();
    if (!r) return flm::rt::set_error(nullptr, FLM_EHIP, "RCCL unavailable");
    ncclUniqueId id;
    ncclResult_t e = r->GetUniqueId(&id);
    if (e != ncclSuccess) return flm::rt::set_error(nullptr, FLM_EHIP, r->GetErrorString(e));
    std::memcpy(id_out, &id, sizeof id);
    return 0;
}

int flm_comm_init_rank(flm_ctx *ctx, int n_ranks, int rank, const uint8_t id[128]) {
    if (!ctx) return flm::rt::set_error(nullptr, FLM_EINVAL, "ctx is NULL");
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || !id) return fail_ctx(ctx, FLM_EINVAL, "bad rank %d of %d", rank, n_ranks);
    Rccl *r = rccl();
    if (!r) return rccl_missing(ctx);
    flm::comm_release(ctx);
    flm::rt::DeviceScope dev_scope_;
    FLM_HIPC(ctx, dev_scope_.set(flm::rt::device_of(ctx)));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    auto *cs = new CommState();
    ncclResult_t e = r->CommInitRank(&cs->comm, n_ranks, uid, rank);
    if (e != ncclSuccess) {
        delete cs;
        return fail_ctx(ctx, FLM_EHIP, "ncclCommInitRank(%d of %d): %s", rank, n_ranks, r->GetErrorString(e));
    }
    cs->nranks = n_ranks;
    cs->rank = rank;
    *flm::rt::comm_slot(ctx) = cs;
    return 0;
}

int flm_comm_destroy(flm_ctx *ctx) {
    if (!ctx) return flm::rt::set_error(nullptr, FLM_EINVAL, "ctx is NULL");
    if (!comm_of(ctx)) return 0;
    flm::rt::DeviceScope dev_scope_;
    FLM_HIPC(ctx, dev_scope_.set(flm::rt::device_of(ctx)));
    // every stream of the device: the collectives may sit on a caller's stream, not the context's
    FLM_HIPC(ctx, hipDeviceSynchronize());
    flm::comm_release(ctx);
    return 0;
}

int flm_comm_size(flm_ctx *ctx, int *n_ranks, int *rank) {
    if (!ctx || !n_ranks || !rank) return FLM_EINVAL;
    CommState *cs = comm_of(ctx);
    *n_ranks = cs ? cs->nranks : 1;
    *rank = cs ? cs->rank : 0;
    return cs ? 0 : 1;  // 1: no communicator attached
}

int flm_reduce_scatter_dev(flm_ctx *ctx, const uint32_t *d_send, uint32_t *d_recv, size_t recv_words, void *stream) {
    if (!ctx) return flm::rt::set_error(nullptr, FLM_EINVAL, "ctx is NULL");
    CommState *cs = comm_of(ctx);
    if (!cs) return fail_ctx(ctx, FLM_EINVAL, "no communicator: call flm_comm_init_rank first");
    if (!d_send || !d_recv) return fail_ctx(ctx, FLM_EINVAL, "NULL buffer");
    flm::rt::DeviceScope dev_scope_;
    FLM_HIPC(ctx, dev_scope_.set(flm::rt::device_of(ctx)));
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream, as every *_dev call
    FLM_NCCL(ctx, rccl()->ReduceScatter(d_send, d_recv, recv_words, ncclUint32, ncclSum, cs->comm, s));
    return 0;
}

int flm_all_gather_dev(flm_ctx *ctx, const void *d_send, void *d_recv, size_t send_bytes, void *stream) {
    if (!ctx) return flm::rt::set_error(nullptr, FLM_EINVAL, "ctx is NULL");
    CommState *cs = comm_of(ctx);
    if (!cs) return fail_ctx(ctx, FLM_EINVAL, "no communicator: call flm_comm_init_rank first");
    if (!d_send || !d_recv) return fail_ctx(ctx, FLM_EINVAL, "NULL buffer");
    flm::rt::DeviceScope dev_scope_;
    FLM_HIPC(ctx, dev_scope_.set(flm::rt::device_of(ctx)));
    hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the HIP null stream
    FLM_NCCL(ctx, rccl()->AllGather(d_send, d_recv, send_bytes, ncclUint8, cs->comm, s));
    return 0;
}

}  // extern "C"

// ======================================================= one process, G GPUs
struct flm_group {
    int n = 0;
    std::vector<int> dev;
    std::vector<flm_ctx *> ctx;
    bool loopback = false;  // every rank on one device: exchange by shard_sum_kernel, no RCCL
    bool clique = false;    // RCCL communicators attached (distinct devices; one device with FLM_GROUP_RCCL)
    struct Rank {
        uint32_t *partial = nullptr, *shard = nullptr;
        size_t cap_partial = 0, cap_shard = 0;
        hipEvent_t done = nullptr;
        hipEvent_t xdone = nullptr;  // loopback: this rank's shard_sum (it reads every rank's partial)
        bool xpending = false;
        size_t dirty = 0;  // partial words [0, dirty) may hold an earlier round's data
    };
    std::vector<Rank> rk;
    // pinned landing buffer of flm_group_aggregate_unmask's shards: the caller's `out` is pageable, and
    // a HIP copy into pageable memory pins it for the driver (flm_runtime.hip HostCopies: DESIGN.md 6)
    uint32_t *hout = nullptr;
    size_t hout_cap = 0;
    std::string err;
};

namespace {

int gfail(flm_group *g, int code, const std::string &msg) {
    if (g) g->err = msg;
    flm::rt::set_error(nullptr, code, msg.c_str());
    return code;
}

// The round goes through partial buffers and an exchange: more than one rank, or a one-device
// group given a real RCCL clique (FLM_GROUP_RCCL: the 8-GPU code path, collective included, run
// on one GPU).  Otherwise the one device's round writes its shard -- the whole vector -- directly.
bool sharded(const flm_group *g) { return g->n > 1 || g->clique; }

int grow(flm_group *g, int r, uint32_t *&p, size_t &cap, size_t words) {
    if (words <= cap) return 0;
    (void)hipSetDevice(g->dev[r]);
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(words, 64) * sizeof(uint32_t));
    // zeroed on the rank's own stream, ahead of the round that writes it: a plain hipMemset is
    // enqueued on the null stream, which the non-blocking rank streams do not wait for, so it
    // could land after the round behind the caller's earlier work (tools/probes/group_order_probe.py)
    if (e == hipSuccess)
        e = hipMemsetAsync(p, 0, std::max<size_t>(words, 64) * sizeof(uint32_t), flm::rt::stream_of(g->ctx[r]));
    if (e != hipSuccess) return gfail(g, FLM_ENOMEM, std::string("group buffer: ") + hipGetErrorString(e));
    cap = words;
    return 0;
}

int rank_error(flm_group *g, int r, int rc) {
    return gfail(g, rc, "rank " + std::to_string(r) + ": " + flm_last_error(g->ctx[r]));
}

// The exchange: partial[r] (Lp words each) -> shards[r] (S words each), on each rank's stream.
int exchange(flm_group *g, uint64_t S, const std::vector<uint32_t *> &shards) {
    const int G = g->n;
    if (g->loopback) {
        std::vector<const uint32_t *> parts(G);
        for (int r = 0; r < G; ++r) parts[r] = g->rk[r].partial;
        for (int r = 0; r < G; ++r) {
            hipStream_t s = flm::rt::stream_of(g->ctx[r]);
            for (int q = 0; q < G; ++q)
                if (q != r && hipStreamWaitEvent(s, g->rk[q].done, 0) != hipSuccess)
                    return gfail(g, FLM_EHIP, "hipStreamWaitEvent");
            hipError_t e = flm::launch_shard_sum(parts.data(), G, (uint64_t)r * S, S, shards[r], s);
            if (e != hipSuccess) return gfail(g, FLM_EHIP, std::string("shard_sum: ") + hipGetErrorString(e));
            if (hipEventRecord(g->rk[r].xdone, s) != hipSuccess) return gfail(g, FLM_EHIP, "hipEventRecord");
            g->rk[r].xpending = true;
        }
        return 0;
    }
    Rccl *rc = rccl();
    ncclResult_t e = rc->GroupStart();
    for (int r = 0; r < G && e == ncclSuccess; ++r)
        e = rc->ReduceScatter(g->rk[r].partial, shards[r], S, ncclUint32, ncclSum, comm_of(g->ctx[r])->comm,
                              flm::rt::stream_of(g->ctx[r]));
    const ncclResult_t e2 = rc->GroupEnd();
    if (e != ncclSuccess || e2 != ncclSuccess)
        return gfail(g, FLM_EHIP, std::string("ncclReduceScatter: ") + rc->GetErrorString(e != ncclSuccess ? e : e2));
    return 0;
}

// The reduce-scatter reads partial[r] over all Lp = G*S words; the round writes [0, L).  Words
// [L, Lp) must be zero: they are at allocation (grow), but an earlier round with a larger L left
// its sums there, which would reach the last shard's padding.
int clear_stale_tail(flm_group *g, int r, size_t L) {
    auto &k = g->rk[r];
    if (k.dirty > L) {
        (void)hipSetDevice(g->dev[r]);
        const size_t hi = std::min(k.dirty, k.cap_partial);
        hipError_t e = hipMemsetAsync(k.partial + L, 0, (hi - L) * sizeof(uint32_t), flm::rt::stream_of(g->ctx[r]));
        if (e != hipSuccess) return gfail(g, FLM_EHIP, std::string("partial tail: ") + hipGetErrorString(e));
    }
    k.dirty = L;
    return 0;
}

// Loopback: rank r's next round rewrites its partial, which the other ranks' shard_sum of the
// previous round read on their own streams; make stream r wait for those reads first.
int wait_previous_exchange(flm_group *g, int r) {
    if (!g->loopback) return 0;  // RCCL: the collective is ordered on each rank's own stream
    hipStream_t s = flm::rt::stream_of(g->ctx[r]);
    for (int q = 0; q < g->n; ++q)
        if (q != r && g->rk[q].xpending && hipStreamWaitEvent(s, g->rk[q].xdone, 0) != hipSuccess)
            return gfail(g, FLM_EHIP, "hipStreamWaitEvent");
    return 0;
}

}  // namespace

extern "C" {

int flm_group_init(flm_group **out, int n, const int *devices) { return flm_group_init_flags(out, n, devices, 0); }

int flm_group_init_flags(flm_group **out, int n, const int *devices, unsigned flags) {
    flm::rt::DeviceScope dev_scope_;  // the rank loops below switch devices
    if (!out) return gfail(nullptr, FLM_EINVAL, "flm_group_init: out is NULL");
    *out = nullptr;
    if (n < 1 || n > flm::kMaxParts) return gfail(nullptr, FLM_EINVAL, "flm_group_init: n must be in [1, 16]");
    if (flags & ~(unsigned)FLM_GROUP_RCCL) return gfail(nullptr, FLM_EINVAL, "flm_group_init: unknown flags");
    auto *g = new flm_group();
    g->n = n;
    for (int r = 0; r < n; ++r) g->dev.push_back(devices ? devices[r] : r);
    bool all_same = true, distinct = true;
    for (int r = 0; r < n; ++r)
        for (int q = 0; q < r; ++q) {
            all_same &= g->dev[r] == g->dev[q];
            distinct &= g->dev[r] != g->dev[q];
        }
    if (!distinct && !all_same) {
        delete g;
        return gfail(nullptr, FLM_EINVAL, "flm_group_init: devices must be all distinct (RCCL) or all equal (loopback)");
    }
    g->loopback = n > 1 && all_same;
    if (g->loopback && (flags & FLM_GROUP_RCCL)) {  // RCCL refuses two ranks on one device
        delete g;
        return gfail(nullptr, FLM_EINVAL, "flm_group_init: FLM_GROUP_RCCL needs distinct devices (RCCL refuses "
                                          "two ranks on one GPU)");
    }
    g->rk.resize(n);
    for (int r = 0; r < n; ++r) {
        flm_ctx *c = nullptr;
        if (int rc = flm_init(&c, g->dev[r])) {
            std::string m = flm_last_error(nullptr);
            flm_group_free(g);
            return gfail(nullptr, rc, "flm_group_init: rank " + std::to_string(r) + ": " + m);
        }
        g->ctx.push_back(c);
        (void)hipSetDevice(g->dev[r]);
        if (hipEventCreateWithFlags(&g->rk[r].done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->rk[r].xdone, hipEventDisableTiming) != hipSuccess) {
            flm_group_free(g);
            return gfail(nullptr, FLM_EHIP, "flm_group_init: hipEventCreate");
        }
    }
    // one device needs no communicator (its shard is the whole vector) unless FLM_GROUP_RCCL asks
    // for the clique anyway: ncclCommInitAll(1, {dev}) and the grouped reduce-scatter below then
    // run on a one-GPU box exactly as on the 8-GPU node
    if (!g->loopback && (n > 1 || (flags & FLM_GROUP_RCCL))) {
        Rccl *r = rccl();
        if (!r) {
            flm_group_free(g);
            return gfail(nullptr, FLM_EHIP, "flm_group_init: RCCL unavailable");
        }
        std::vector<ncclComm_t> comms(n);
        ncclResult_t e = r->CommInitAll(comms.data(), n, g->dev.data());
        if (e != ncclSuccess) {
            flm_group_free(g);
            return gfail(nullptr, FLM_EHIP, std::string("ncclCommInitAll: ") + r->GetErrorString(e));
        }
        for (int q = 0; q < n; ++q) {
            auto *cs = new CommState();
            cs->comm = comms[q];
            cs->nranks = n;
            cs->rank = q;
            *flm::rt::comm_slot(g->ctx[q]) = cs;
        }
        g->clique = true;
    }
    *out = g;
    return 0;
}

void flm_group_free(flm_group *g) {
    flm::rt::DeviceScope dev_scope_;  // the rank loops below switch devices
    if (!g) return;
    if (g->clique) flm::comm_release_clique(g->ctx.data(), (int)g->ctx.size());  // before any flm_free
    for (int r = 0; r < (int)g->ctx.size(); ++r) {
        (void)hipSetDevice(g->dev[r]);
        (void)hipStreamSynchronize(flm::rt::stream_of(g->ctx[r]));
        if (g->rk[r].partial) (void)hipFree(g->rk[r].partial);
        if (g->rk[r].shard) (void)hipFree(g->rk[r].shard);
        if (g->rk[r].done) (void)hipEventDestroy(g->rk[r].done);
        if (g->rk[r].xdone) (void)hipEventDestroy(g->rk[r].xdone);
        flm_free(g->ctx[r]);
    }
    if (g->hout) (void)hipHostFree(g->hout);
    delete g;
}

const char *flm_group_last_error(const flm_group *g) { return g ? g->err.c_str() : flm_last_error(nullptr); }

int flm_group_size(const flm_group *g) { return g ? g->n : 0; }

int flm_group_is_loopback(const flm_group *g) { return g && g->loopback ? 1 : 0; }

int flm_group_has_rccl(const flm_group *g) { return g && g->clique ? 1 : 0; }

flm_ctx *flm_group_ctx(flm_group *g, int rank) {
    if (!g || rank < 0 || rank >= g->n) return nullptr;
    return g->ctx[rank];
}

int flm_group_sync(flm_group *g) {
    flm::rt::DeviceScope dev_scope_;  // the rank loops below switch devices
    if (!g) return FLM_EINVAL;
    for (int r = 0; r < g->n; ++r) {
        (void)hipSetDevice(g->dev[r]);
        hipError_t e = hipStreamSynchronize(flm::rt::stream_of(g->ctx[r]));
        if (e != hipSuccess) return gfail(g, FLM_EHIP, std::string("rank sync: ") + hipGetErrorString(e));
    }
    return 0;
}

// Host rows in, unmasked sum out, over every device of the group (the drop-in server's round,
// SA_ServiceAgent.py:346-350 + 529-605): one host thread per device uploads that device's
// clients and enqueues its fused round; then one reduce-scatter; then each shard comes back.
int flm_group_aggregate_unmask(flm_group *g, const uint32_t *const *rows, int N, const uint8_t *seeds,
                               const int8_t *signs, int K, size_t L, uint32_t *out) {
    flm::rt::DeviceScope dev_scope_;  // the rank loops below switch devices
    if (!g) return gfail(nullptr, FLM_EINVAL, "group is NULL");
    if (N < 0 || K < 0) return gfail(g, FLM_EINVAL, "negative N or K");
    if (L == 0) return 0;
    if (!out || (N > 0 && !rows) || (K > 0 && (!seeds || !signs))) return gfail(g, FLM_EINVAL, "NULL argument");
    int rc_ = 0;
    const int G = g->n;
    const bool X = sharded(g);
    const uint64_t Lp = padded_len(L, G), S = Lp / G;
    for (int r = 0; r < G; ++r) {
        if (X && (rc_ = grow(g, r, g->rk[r].partial, g->rk[r].cap_partial, Lp))) return rc_;
        if ((rc_ = grow(g, r, g->rk[r].shard, g->rk[r].cap_shard, S))) return rc_;
    }
    for (int r = 0; r < G; ++r)
        if ((rc_ = wait_previous_exchange(g, r))) return rc_;
    for (int r = 0; X && r < G; ++r)
        if ((rc_ = clear_stale_tail(g, r, L))) return rc_;
    if (g->hout_cap < L) {  // the last call synchronised every rank: nothing reads the old buffer
        if (g->hout) (void)hipHostFree(g->hout);
        g->hout = nullptr;
        g->hout_cap = 0;
        if (hipHostMalloc(&g->hout, L * sizeof(uint32_t), hipHostMallocPortable) != hipSuccess)
            return gfail(g, FLM_ENOMEM, "group: pinned output buffer");
        g->hout_cap = L;
    }
    std::vector<int> rcs(G, 0);
    auto work = [&](int r) {
        int c0, c1;
        size_t lo, hi;
        flm_client_bounds(N, G, r, &c0, &c1);
        flm_shard_bounds(L, G, r, &lo, &hi, nullptr);
        // one device without a clique: the round writes its shard (the whole vector) directly
        rcs[r] = flm::rt::host_round_async(g->ctx[r], rows ? rows + c0 : nullptr, c1 - c0, seeds, signs, K, L, lo, hi,
                                           X ? g->rk[r].partial : g->rk[r].shard);
        if (!rcs[r] && hipEventRecord(g->rk[r].done, flm::rt::stream_of(g->ctx[r])) != hipSuccess) rcs[r] = FLM_EHIP;
    };
    if (G == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int r = 0; r < G; ++r) th.emplace_back(work, r);
        for (auto &t : th) t.join();
    }
    for (int r = 0; r < G; ++r)
        if (rcs[r]) return rank_error(g, r, rcs[r]);
    std::vector<uint32_t *> shards(G);
    for (int r = 0; r < G; ++r) shards[r] = g->rk[r].shard;
    if (X && (rc_ = exchange(g, S, shards))) return rc_;
    for (int r = 0; r < G; ++r) {
        size_t lo, hi;
        flm_shard_bounds(L, G, r, &lo, &hi, nullptr);
        if (hi <= lo) continue;
        (void)hipSetDevice(g->dev[r]);
        hipError_t e = hipMemcpyAsync(g->hout + lo, g->rk[r].shard, (hi - lo) * sizeof(uint32_t),
                                      hipMemcpyDeviceToHost, flm::rt::stream_of(g->ctx[r]));
        if (e != hipSuccess) return gfail(g, FLM_EHIP, std::string("shard D2H: ") + hipGetErrorString(e));
    }
    if (int rc = flm_group_sync(g)) return rc;
    flm::rt::host_copy(g->ctx[0], out, g->hout, L * sizeof(uint32_t));
    return 0;
}

// Device-resident form: rank r's rows are already in its HBM (d_rows[r], n_rows[r] rows at
// row_pitch), seeds/signs on every device.  Enqueues each rank's fused round and the exchange on
// the ranks' streams (flm_group_ctx(g, r)'s stream) and returns; d_shards[r] (>= S words, S =
// round_up(L, 1024*G)/G, on device r) receives rank r's slots [lo_r, hi_r) at offset 0.
int flm_group_aggregate_unmask_dev(flm_group *g, const uint32_t *const *d_rows, size_t row_pitch, const int *n_rows,
                                   const uint8_t *const *d_seeds, const int8_t *const *d_signs, int K, size_t L,
                                   uint32_t *const *d_shards) {
    flm::rt::DeviceScope dev_scope_;  // the rank loops below switch devices
    if (!g) return gfail(nullptr, FLM_EINVAL, "group is NULL");
    if (!n_rows || !d_shards || (K > 0 && (!d_seeds || !d_signs))) return gfail(g, FLM_EINVAL, "NULL argument");
    if (L == 0) return 0;
    const int G = g->n;
    const bool X = sharded(g);
    const uint64_t Lp = padded_len(L, G), S = Lp / G;
    for (int r = 0; X && r < G; ++r)
        if (int rc = grow(g, r, g->rk[r].partial, g->rk[r].cap_partial, Lp)) return rc;
    for (int r = 0; r < G; ++r)
        if (int rc = wait_previous_exchange(g, r)) return rc;
    for (int r = 0; X && r < G; ++r)
        if (int rc = clear_stale_tail(g, r, L)) return rc;
    for (int r = 0; r < G; ++r) {
        size_t lo, hi;
        flm_shard_bounds(L, G, r, &lo, &hi, nullptr);
        flm_ctx *c = g->ctx[r];
        // one device without a clique: the round writes the caller's shard (the whole vector) directly
        int rc = flm_aggregate_unmask_dev(c, d_rows ? d_rows[r] : nullptr, row_pitch, n_rows[r],
                                          K ? d_seeds[r] : nullptr, K ? d_signs[r] : nullptr, K, L, lo, hi, 0,
                                          X ? g->rk[r].partial : d_shards[r], flm::rt::stream_of(c));
        if (rc) return rank_error(g, r, rc);
        if (hipEventRecord(g->rk[r].done, flm::rt::stream_of(c)) != hipSuccess) return gfail(g, FLM_EHIP, "event");
    }
    if (!X) return 0;
    // the exchange writes the caller's shard buffers directly
    return exchange(g, S, std::vector<uint32_t *>(d_shards, d_shards + G));
}

}  // extern "C"
