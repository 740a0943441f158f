"""Multi-GPU server reconstruction (BASELINE c5 on G GPUs): seed recovery + unmask, sharded.

SA_ServiceAgent.reconstruction_process (:499-605) on G ranks, one process per GPU.  Every
rank needs every seed -- it regenerates all K masks over its own slot shard -- so the
question is who recovers which seeds:

* m_i (Shamir, :506-526): every rank recovers all M of them.  It is one tiny launch
  (0.06 ms at c5 for M = 4055), cheaper than any exchange.
* s_ij (threshold ElGamal + SHA-256, :542-585): rank r recovers only pairs
  [r*Dc, (r+1)*Dc), Dc = ceil(D/G), then ONE all-gather of 32*Dc bytes per rank gives
  every rank all D keys.  The combine is latency-bound (one scalar multiplication is a
  ~2.7 ms chain per lane whatever the batch), so the split does not shorten it, but it
  takes G times fewer lanes on each GPU and runs on a side stream under the self-mask pass.

Per rank, in stream order:
  side:  ec_combine(my pairs) -> chunk ------------------------------------\\
  main:  shamir(all m_i) -> rows(my clients) + self masks(my shard) -> part -+-> all_gather(chunk)
         -> part + pair masks(my shard) -> part2 -> reduce_scatter -> out shard

The two exchanges go through the library's RCCL communicator (flm_all_gather_dev,
flm_reduce_scatter_dev) when one is attached (distributed.init_rccl), else through
torch.distributed (gloo on host copies: ranks sharing one GPU in tests).

The reference itself splits the round in two steps (report_process :346-350 sums the rows
before any share exists; reconstruction_process :499-605 adds the masks).  report() +
run_from_partial() keep that split on G ranks: report reduce-scatters the rows' partial sums
into each rank's S shard; once the shares arrive, each rank adds every mask over its own S
shard -- the all-gather of the pair keys is then the only exchange on the shares-to-final
path, and no row is read there:
  side:  ec_combine(my pairs) -> chunk -------------------------\
  main:  shamir(all m_i) -> S shard + self masks -> part ------+-> all_gather(chunk)
         -> part + pair masks -> out shard
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .distributed import padded_length, shard_bounds


def pair_chunk(D: int, world: int, rank: int):
    """[a, b) of the dropout pairs rank recovers; every rank's chunk is Dc = ceil(D/G) long (padded)."""
    Dc = (D + world - 1) // world if D else 0
    a = min(rank * Dc, D)
    return a, min(a + Dc, D), Dc


class ShardedReconstruction:
    """ec_cus > 0 partitions the rank's CUs (flm_stream_create_cu_mask): the combine runs on the first
    `ec_cus` CUs (cu_pick), Shamir and the self-mask pass on the rest, and the caller's stream joins
    both before the all-gather.  One rank's share of the pairs is a few dozen cooperative workgroups,
    so on its own CUs the chain keeps its lone-wave speed instead of sharing SIMDs with the pass:
    one rank of G = 8 at c5 from its S shard 1.63 ms unpartitioned against 1.39-1.40 ms on 72 or 96
    EC CUs (tools/probes/rank8_overlap_probe.py, profiles/r03_rank8_overlap_*.log; 64 and 80 CUs
    came out bimodal there).  At G = 4 / 2 the self-mask pass on the remaining CUs is the longer leg
    and the partitioned schedule loses (1.75 -> 2.21 ms, 3.01 -> 4.07 ms; r03_rank_overlap_G{4,2}.log).
    Default 0: unpartitioned.

    force_collective: at world 1 run both exchanges through the collective anyway (the library's RCCL
    communicator when init_rccl attached one, else torch.distributed) instead of the world-1 copies,
    so a one-GPU box executes the exact code the G-GPU run takes."""

    def __init__(self, engine, L: int, group=None, device=None, comm: str | None = None, ec_cus: int = 0,
                 cu_pick: str = "first", force_collective: bool = False, ec_coop: int = 1):
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.force_collective = bool(force_collective)
        if self.force_collective and not dist.is_initialized():
            raise RuntimeError("force_collective needs an initialised torch.distributed group")
        self.L = L
        self.Lp = padded_length(L, self.world)
        self.S = self.Lp // self.world
        self.lo, self.hi = shard_bounds(L, self.world, self.rank)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if comm is None:
            comm = "rccl" if ((self.world > 1 or self.force_collective) and engine.has_comm()
                              and engine.comm_size() == (self.world, self.rank)) else "torch"
        self.comm = comm
        self.ec_cus = int(ec_cus)
        # the scalar-multiplication kernel on the confined CUs (flm_set_tuning ec_coop; unconfined, the
        # library's auto choice stands): the per-lane-field cooperative kernel, 1.45 ms for one G = 8
        # rank's shares -> final on 72 CUs against 1.83 / 1.53 ms for the row-field kernel on 64 / 128
        # (its 16x more waves crowd a confined set; tools/probes/rank8_overlap_probe.py --row,
        # profiles/r04_rank8_row.log)
        self.ec_coop = int(ec_coop)
        self.pass_stream = None
        if self.ec_cus > 0:
            from .reconstruct import pick_cus
            n = engine.cu_count()
            if not 0 < self.ec_cus < n:
                raise ValueError(f"ec_cus={ec_cus} must be in (0, {n})")
            ec = pick_cus(n, self.ec_cus, cu_pick)
            self.side = engine.cu_stream(ec)
            self.pass_stream = engine.cu_stream([c for c in range(n) if c not in set(ec)])
        else:
            self.side = torch.cuda.Stream(device=self.device)
        self._bufs = {}

    def _buf(self, name, shape, dtype, fill=None):
        b = self._bufs.get(name)
        if b is None or tuple(b.shape) != tuple(shape) or b.dtype != dtype:
            b = torch.empty(shape, dtype=dtype, device=self.device)
            if fill is not None:
                b.fill_(fill)
            self._bufs[name] = b
        return b

    def _ec_combine(self, c1, shares, lambdas, seeds, flags):
        """The rank's pair chunk on the side stream; on confined CUs with the ec_coop kernel."""
        prev = self.eng.get_tuning("ec_coop")
        if self.ec_cus > 0:
            self.eng.set_tuning("ec_coop", self.ec_coop)
        try:
            self.eng.ec_combine_dev(c1, shares, lambdas, seeds, flags, stream=self.side)
        finally:
            if self.ec_cus > 0:
                self.eng.set_tuning("ec_coop", prev)          # the caller's own setting, not auto

    def _pass_begin(self, ready, main):
        """The stream Shamir and the self-mask pass run on: the caller's, or (ec_cus > 0) the
        CU-partitioned pass stream, ordered after the caller's work so far."""
        if self.pass_stream is None:
            return main
        self.pass_stream.wait_event(ready)
        return self.pass_stream

    def _pass_end(self, ps, main):
        if ps is not main:
            ev = torch.cuda.Event()
            ev.record(ps)
            main.wait_event(ev)

    def _all_gather(self, chunk, gathered, stream):
        if self.world == 1 and not self.force_collective:
            with torch.cuda.stream(stream):             # torch copies run on the CURRENT stream
                gathered[: chunk.shape[0]].copy_(chunk)
        elif self.comm == "rccl":
            self.eng.all_gather_dev(chunk, gathered, stream=stream)
        else:
            with torch.cuda.stream(stream):
                if dist.get_backend(self.group) == "gloo":
                    host = torch.empty((gathered.shape[0],) + tuple(chunk.shape[1:]), dtype=chunk.dtype)
                    dist.all_gather_into_tensor(host, chunk.cpu(), group=self.group)
                    gathered.copy_(host)
                else:
                    dist.all_gather_into_tensor(gathered, chunk, group=self.group)

    def _reduce_scatter(self, part, out, stream):
        if self.world == 1 and not self.force_collective:
            with torch.cuda.stream(stream):
                out[: self.L].copy_(part[: self.L])
        elif self.comm == "rccl":
            self.eng.reduce_scatter_dev(part, out, self.S, stream=stream)
        else:
            with torch.cuda.stream(stream):
                if dist.get_backend(self.group) == "gloo":
                    host = torch.empty(self.S, dtype=part.dtype)
                    dist.reduce_scatter_tensor(host, part.cpu(), op=dist.ReduceOp.SUM, group=self.group)
                    out[: self.S].copy_(host)
                else:
                    dist.reduce_scatter_tensor(out[: self.S], part, op=dist.ReduceOp.SUM, group=self.group)

    def run(self, rows, lambdas, mi_shares, c1_mine, pair_shares_mine, pair_signs, D: int, out, stream=None):
        """rows (N_r, pitch) int32: this rank's online clients; lambdas (T, 32); mi_shares (T, M, 32) -- all
        online clients; c1_mine (Dr, 64), pair_shares_mine (T, Dr, 64): this rank's pair chunk
        (pair_chunk(D, G, rank)); pair_signs (D,) int8 -- all pairs, recon_symbol order; out (>= S,) int32
        receives this rank's slots [lo, hi) (world 1: out[:L] is the whole sum).  Enqueued on `stream`."""
        eng = self.eng
        main = torch.cuda.current_stream(self.device) if stream is None else stream
        M = mi_shares.shape[1]
        _, _, Dc = pair_chunk(D, self.world, self.rank)
        Dr = c1_mine.shape[0] if c1_mine is not None else 0
        with torch.cuda.stream(main):
            m_seeds = self._buf("m_seeds", (M, 32), torch.uint8)
            neg = self._buf("neg", (M,), torch.int8, -1)
            chunk = self._buf("chunk", (max(Dc, 1), 32), torch.uint8, 0)
            gathered = self._buf("gathered", (max(Dc, 1) * self.world, 32), torch.uint8)
            flags = self._buf("flags", (max(Dr, 1),), torch.int32)
            part = self._buf("part", (1, self.Lp), torch.int32, 0)
            part2 = self._buf("part2", (self.Lp,), torch.int32, 0)
        ready = torch.cuda.Event()
        ready.record(main)
        if Dr:
            self.side.wait_event(ready)
            self._ec_combine(c1_mine, pair_shares_mine, lambdas, chunk[:Dr], flags)
        done = torch.cuda.Event()
        done.record(self.side)
        ps = self._pass_begin(ready, main)
        eng.shamir_combine_dev(mi_shares, lambdas, m_seeds, stream=ps)
        eng.aggregate_unmask_dev(rows, m_seeds, neg, part[0], L=self.L, mask_lo=self.lo, mask_hi=self.hi,
                                 stream=ps)
        self._pass_end(ps, main)
        if D:
            main.wait_event(done)
            self._all_gather(chunk, gathered, main)
            eng.aggregate_unmask_dev(part, gathered[:D], pair_signs, part2, L=self.L, mask_lo=self.lo,
                                     mask_hi=self.hi, stream=main)
            src = part2
        else:
            src = part[0]
        self._reduce_scatter(src, out, main)
        return out, flags

    # ----------------------------------------------- the reference's two-step split
    def report(self, rows, S_out, stream=None):
        """report_process on G ranks: S_out[:S] = this rank's slots of sum over every rank's rows
        (one rows-only launch over all L, then the reduce-scatter).  rows (N_r, pitch) int32."""
        main = torch.cuda.current_stream(self.device) if stream is None else stream
        with torch.cuda.stream(main):
            part = self._buf("report_part", (self.Lp,), torch.int32, 0)
        if rows is not None and rows.shape[0]:
            self.eng.aggregate_unmask_dev(rows, None, None, part, L=self.L, stream=main)
        else:
            with torch.cuda.stream(main):
                part[: self.L].zero_()
        self._reduce_scatter(part, S_out, main)
        return S_out

    def run_from_partial(self, S_shard, lambdas, mi_shares, c1_mine, pair_shares_mine, pair_signs, D: int, out,
                         stream=None):
        """reconstruction_process on G ranks over the report's S shard (S_shard (>= S,) int32):
        out[:hi-lo] = S_shard[:hi-lo] + sum of every mask over this rank's slots [lo, hi).
        Other arguments as run()."""
        eng = self.eng
        main = torch.cuda.current_stream(self.device) if stream is None else stream
        M = mi_shares.shape[1]
        _, _, Dc = pair_chunk(D, self.world, self.rank)
        Dr = c1_mine.shape[0] if c1_mine is not None else 0
        n = self.hi - self.lo
        with torch.cuda.stream(main):
            m_seeds = self._buf("m_seeds", (M, 32), torch.uint8)
            neg = self._buf("neg", (M,), torch.int8, -1)
            chunk = self._buf("chunk", (max(Dc, 1), 32), torch.uint8, 0)
            gathered = self._buf("gathered", (max(Dc, 1) * self.world, 32), torch.uint8)
            flags = self._buf("flags", (max(Dr, 1),), torch.int32)
            part = self._buf("fp_part", (1, self.S), torch.int32, 0)
        ready = torch.cuda.Event()
        ready.record(main)
        if Dr:
            self.side.wait_event(ready)
            self._ec_combine(c1_mine, pair_shares_mine, lambdas, chunk[:Dr], flags)
        done = torch.cuda.Event()
        done.record(self.side)
        ps = self._pass_begin(ready, main)
        eng.shamir_combine_dev(mi_shares, lambdas, m_seeds, stream=ps)
        src = S_shard[: self.S].view(1, self.S)
        if n > 0:
            eng.aggregate_unmask_dev(src, m_seeds, neg, part[0] if D else out, L=n, prg_slot0=self.lo, stream=ps)
        self._pass_end(ps, main)
        if D:
            main.wait_event(done)
            self._all_gather(chunk, gathered, main)
            if n > 0:
                eng.aggregate_unmask_dev(part, gathered[:D], pair_signs, out, L=n, prg_slot0=self.lo, stream=main)
        return out, flags
