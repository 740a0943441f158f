"""Multi-GPU server round: client-sharded rows, slot-sharded unmask, RCCL reduce-scatter.

One process per GPU.  Rank r of G holds the masked vectors of its own clients
(the VECTOR bodies it ingested over its own PCIe link) and owns slot shard
[r*S, (r+1)*S) of the output, S = Lp / G with Lp = L rounded up to 1024*G:

  partial_r[l] = sum_{i in clients(r)} y_i[l]                    l in [0, L)
               + sum_k sign_k * PRG(seed_k)[l]                   l in shard(r)
  out_r        = reduce_scatter_sum(partial_0..G-1)[shard(r)]

The mask term is added by exactly one rank per slot, so the reduce-scatter
returns S + C + M of SA_ServiceAgent.py:605 for that shard.  Integer addition
is associative and commutative mod 2^32, so every ring order gives the same
bits.  Each rank regenerates all K masks but only over its own slots, which
splits the VALU-bound ChaCha work G ways; the row sum (HBM-bound) is split by
clients.  The only collective is one reduce-scatter of Lp*4 bytes per round.

The collective runs through the library's own RCCL communicator
(flm_comm_init_rank / flm_reduce_scatter_dev: ncclReduceScatter with ncclUint32,
enqueued on the same HIP stream as the kernel that wrote the partial) when one
is attached -- ``init_rccl`` does that over an existing torch.distributed group.
Without one (gloo tests on CPU, or several ranks sharing one GPU, where RCCL
refuses duplicate devices) the same exchange goes through torch.distributed.
The shard geometry is the library's (flm_shard_bounds / flm_client_bounds), so
the single-process DeviceGroup and these per-process ranks cut the round alike.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

SHARD_ALIGN = 1024  # a wave's sub-tile; keeps every shard start a multiple of 16 slots


def padded_length(L: int, world: int) -> int:
    q = SHARD_ALIGN * world
    return (L + q - 1) // q * q


def shard_bounds(L: int, world: int, rank: int):
    """[lo, hi) of output slots owned by `rank` (hi clipped to L; may be empty).  Same as flm_shard_bounds."""
    S = padded_length(L, world) // world
    lo = min(rank * S, L)
    hi = min((rank + 1) * S, L)
    return lo, hi


def client_bounds(N: int, world: int, rank: int):
    """Contiguous block of clients ingested by `rank` (flm_client_bounds)."""
    return N * rank // world, N * (rank + 1) // world


def init_rccl(engine, group=None):
    """Attach an RCCL communicator over `group`'s ranks to `engine` (collective).

    Every rank makes the same torch.distributed calls in the same order whatever fails, so
    a failure surfaces as the same RuntimeError on every rank instead of mismatched
    collectives: (1) all ranks agree that RCCL loads (flm_rccl_available, local);
    (2) rank 0 makes the unique id and broadcasts (id, error) -- an error on rank 0 reaches
    everyone; (3) every rank joins with flm_comm_init_rank; (4) all ranks agree it worked.
    A rank that fails INSIDE ncclCommInitRank leaves the others blocked in RCCL's bootstrap
    until RCCL's own timeout: that step alone cannot be made recoverable from here.
    Returns (world, rank)."""
    from .engine import comm_unique_id, rccl_available
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    src = dist.get_global_rank(group, 0) if group is not None else 0
    ok, why = rccl_available()
    oks = [None] * world
    dist.all_gather_object(oks, (ok, why), group=group)
    bad = [f"rank {r}: {w}" for r, (o, w) in enumerate(oks) if not o]
    if bad:
        raise RuntimeError("RCCL unavailable on " + "; ".join(bad))
    box = [None]
    if rank == 0:
        try:
            box = [(comm_unique_id(), "")]
        except Exception as e:                       # still broadcast: the others are waiting for it
            box = [(None, f"{type(e).__name__}: {e}")]
    dist.broadcast_object_list(box, src=src, group=group)
    uid, err = box[0]
    if uid is None:
        raise RuntimeError(f"RCCL unique id on rank 0 failed: {err}")
    err = ""
    try:
        engine.comm_init(world, rank, uid)
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    errs = [None] * world
    dist.all_gather_object(errs, err, group=group)
    bad = [f"rank {r}: {e}" for r, e in enumerate(errs) if e]
    if bad:
        raise RuntimeError("flm_comm_init_rank failed on " + "; ".join(bad))
    return world, rank


def shutdown(*owners, group_initialized: bool | None = None):
    """Ordered teardown of one process's RCCL users; every rank calls it at the end of its run.

    torch's nccl process group and the library's communicators come from the same librccl.so
    (flm_comm.hip resolves the copy torch loaded).  Destroying torch's group first and leaving the
    library communicator to flm_free -- or to a __del__ at interpreter exit -- ended the process in
    an exit-time destructor (__cxa_finalize) after every check had passed (the rccl
    clique smoke under rocprofv3 with the nccl backend).  The order here:
      1. synchronise the device (the collectives may sit on a comm stream of their own);
      2. finalize + destroy every library communicator (MaskEngine.comm_destroy; a DeviceGroup's
         clique is destroyed by closing the group);
      3. a barrier, so no rank tears down torch's group while a peer is still in step 2;
      4. torch.distributed.destroy_process_group();
      5. close every owner (contexts, CU streams, device buffers) and collect, so nothing of ours is
         left for a finalizer at interpreter exit.
    owners: MaskEngine / DeviceGroup / anything with close(); a VectorStore must come before the
    group it lives on."""
    import gc
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
    from .engine import MaskEngine
    rest = []
    for o in owners:
        if isinstance(o, MaskEngine):
            o.comm_destroy()
            rest.append(o)
        elif o is not None:
            o.close()                    # stores, then the groups they live on (clique destroyed here)
    init = dist.is_initialized() if group_initialized is None else group_initialized
    if init:
        dist.barrier()
        dist.destroy_process_group()
    for o in rest:
        o.close()
    gc.collect()


def _torch_stream(stream):
    if stream is None or isinstance(stream, torch.cuda.Stream):
        return stream
    return torch.cuda.ExternalStream(int(stream))


class ShardedRound:
    """Runs one rank's share of a round on its GPU and reduce-scatters the partials.

    With buffers=2, launch() leaves the reduce-scatter in flight and the next round's
    kernel writes the other partial buffer, so round k's collective over xGMI runs under
    round k+1's kernel; a buffer is reused only after the collective that read it has
    completed (a stream-side wait, the host never blocks).  On the RCCL path the
    collective runs on a comm stream of its own, ordered after the kernel by an event.

    force_collective: at world 1 reduce-scatter anyway (and pipeline it with buffers=2) instead of
    returning the partial, so a one-GPU box runs the multi-GPU exchange code."""

    def __init__(self, engine, L: int, group=None, device=None, buffers: int = 1, comm: str | None = None,
                 force_collective: bool = False):
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.force_collective = bool(force_collective)
        if self.force_collective and not dist.is_initialized():
            raise RuntimeError("force_collective needs an initialised torch.distributed group")
        self._solo = self.world == 1 and not self.force_collective    # world 1: the partial is the result
        self.L = L
        self.Lp = padded_length(L, self.world)
        self.S = self.Lp // self.world
        self.lo, self.hi = shard_bounds(L, self.world, self.rank)
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if buffers not in (1, 2):
            raise ValueError("buffers must be 1 or 2")
        if comm is None:
            comm = "rccl" if (engine is not None and not self._solo and engine.has_comm()
                              and engine.comm_size() == (self.world, self.rank)) else "torch"
        if comm not in ("rccl", "torch"):
            raise ValueError("comm must be 'rccl' or 'torch'")
        if comm == "rccl" and (not engine.has_comm() or engine.comm_size() != (self.world, self.rank)):
            raise RuntimeError("comm='rccl' needs init_rccl(engine, group) first")
        self.comm = comm
        self._partials = [torch.zeros(self.Lp, dtype=torch.int32, device=dev) for _ in range(buffers)]
        self._outs = [torch.empty(self.S, dtype=torch.int32, device=dev) for _ in range(buffers)]
        self._pending = [None] * buffers          # torch Work (torch path) or comm-done Event (rccl path)
        self._comm_stream = torch.cuda.Stream(device=dev) if (comm == "rccl" and buffers == 2) else None
        self._k = 0
        self.partial, self.out = self._partials[0], self._outs[0]

    def prepare_seeds(self, d_seeds, d_signs, stream=None):
        self.K = d_seeds.shape[0]
        self.engine.seed_table_dev(d_seeds, d_signs, stream=stream)

    def compute(self, d_rows, stream=None):
        """Row sum over all slots + unmask over this rank's shard (one kernel)."""
        self.engine.aggregate_dev(d_rows, self.K, self.partial, L=self.L, mask_lo=self.lo, mask_hi=self.hi,
                                  stream=stream)

    def _torch_exchange(self, async_op: bool = False):
        if self.partial.is_cuda and dist.get_backend(self.group) == "gloo":
            # test path only (several ranks sharing one GPU, where RCCL refuses duplicate
            # devices): the same reduce-scatter on host copies
            cpu_out = torch.empty(self.out.shape, dtype=self.out.dtype)
            dist.reduce_scatter_tensor(cpu_out, self.partial.cpu(), op=dist.ReduceOp.SUM, group=self.group)
            self.out.copy_(cpu_out)
            return None
        return dist.reduce_scatter_tensor(self.out, self.partial, op=dist.ReduceOp.SUM, group=self.group,
                                          async_op=async_op)

    def exchange(self, stream=None):
        """The reduce-scatter of the current partial, ordered after the work on `stream`."""
        if self._solo:
            return self.partial[: self.L]
        if self.comm == "rccl":
            self.engine.reduce_scatter_dev(self.partial, self.out, self.S, stream=stream)
        else:
            st = _torch_stream(stream)
            if st is not None and self.partial.is_cuda:
                with torch.cuda.stream(st):           # torch's collective orders against the CURRENT stream
                    self._torch_exchange()
            else:
                self._torch_exchange()
        return self.out[: self.hi - self.lo]

    def step(self, d_rows, d_seeds, d_signs, stream=None):
        self.prepare_seeds(d_seeds, d_signs, stream)
        self.compute(d_rows, stream)
        return self.exchange(stream)

    def _async_ok(self):
        # RCCL (or gloo on host tensors) can leave the collective in flight; the gloo path
        # over a shared GPU (tests only) goes through host copies and stays synchronous
        if self._solo:
            return False
        if self.comm == "rccl":
            return self._comm_stream is not None
        return not (self.partial.is_cuda and dist.get_backend(self.group) == "gloo")

    def launch(self, d_rows, d_seeds, d_signs, stream=None) -> int:
        """Enqueue one round; returns its buffer index for result()."""
        b = self._k % len(self._partials)
        st = _torch_stream(stream)
        if self._pending[b] is not None:
            # the collective that last read this buffer must finish before the kernel rewrites it
            if self.comm == "rccl":
                (st or torch.cuda.current_stream()).wait_event(self._pending[b])
            elif st is not None and self.partial.is_cuda:
                with torch.cuda.stream(st):            # Work.wait() makes the CURRENT stream wait
                    self._pending[b].wait()
            else:
                self._pending[b].wait()
            self._pending[b] = None
        self.partial, self.out = self._partials[b], self._outs[b]
        self.prepare_seeds(d_seeds, d_signs, stream)
        self.compute(d_rows, stream)
        if not self._async_ok():
            self.exchange(stream)
        elif self.comm == "rccl":
            ready = torch.cuda.Event()
            ready.record(st or torch.cuda.current_stream())
            self._comm_stream.wait_event(ready)
            self.engine.reduce_scatter_dev(self.partial, self.out, self.S, stream=self._comm_stream)
            done = torch.cuda.Event()
            done.record(self._comm_stream)
            self._pending[b] = done
        elif st is not None and self.partial.is_cuda:
            with torch.cuda.stream(st):
                self._pending[b] = self._torch_exchange(async_op=True)
        else:
            self._pending[b] = self._torch_exchange(async_op=True)
        self._k += 1
        return b

    def result(self, b: int | None = None):
        """This rank's shard of round `b` (default: the last launched), after its collective."""
        b = (self._k - 1) % len(self._partials) if b is None else b
        if self._pending[b] is not None:
            if self.comm == "rccl":
                torch.cuda.current_stream().wait_event(self._pending[b])
            else:
                self._pending[b].wait()
            self._pending[b] = None
        if self._solo:
            return self._partials[b][: self.L]
        return self._outs[b][: self.hi - self.lo]
