"""Device-resident server reconstruction with seed recovery overlapped (one GPU).

SA_ServiceAgent.reconstruction_process (:499-605) in order: recover every
online client's m_i from the decryptors' Shamir shares (:506-526), recover
every dropout pair's s_ij by threshold-ElGamal decryption (:542-585), then
final_sum = S - sum PRG(m_i) + sum sigma PRG(s_ij) (:529-540, :587-605).

Here the m_i recovery is tiny (flm_shamir_combine_dev, ~0.06 ms at c5) and
unblocks the self-mask unmask of the row sum, the bulk of the VALU work.
The EC combine (flm_ec_combine_dev) is latency-bound on ~300 waves, far from
filling the chip, so it runs on a second HIP stream under that unmask.  The
D pair masks are then added in a second pass over the one partial vector,
seeds taken straight from the combine (no host round trip):

  main stream:  shamir -> unmask(rows, m seeds)  -> tmp ---wait---> unmask(tmp, pair seeds) -> out
  side stream:  ec_combine -> pair seeds --------------event--^

`overlap=False` runs the same steps on one stream with a single unmask over all
K seeds (the sequential schedule) for comparison.

With `ec_cus > 0` the two streams are CU-partitioned (flm_stream_create_cu_mask):
the combine runs on `ec_cus` CUs only and the Shamir step + self-mask unmask on
the rest.  Unpartitioned, an EC wave resident on a SIMD leaves too few VGPRs for
a second unmask workgroup on that CU, so those CUs run at half rate for the
whole combine and finish last; partitioned, the unmask is evenly spread over
the CUs it owns.  The pair pass then runs on the caller's stream over all CUs.

`pair_split = f > 0` (with `ec_cus`): once the combine is done, the EC CUs do not idle
until the self-mask pass ends.  They add the pair masks of slots [0, f*L) into a second
partial row while the self-mask pass still runs on the other CUs.  The last pass then
sums the two partial rows over all L and adds the pair masks of [f*L, L) only:

  side (EC CUs):   ec_combine -> pair masks [0, fL) -> part[1] ------------\
  part (the rest): shamir -> rows + self masks       -> part[0] -----------+-> part[0] + part[1]
                                                                              + pair masks [fL, L) -> out

`pair_queue=True` (with `ec_cus`) makes that split dynamic.  The pair masks are cut into
units of (1024 slots, 16 seeds) claimed from one device counter (flm_pair_units_dev).  The
EC CUs claim units into part[1] from the end of the combine until the self-mask stream sets
a stop flag; the last pass writes part[0] + part[1] and claims the rest on all CUs.  A static f
has a cliff (the side pass outlasting the self-mask pass costs more than it saves); the queue
stops at the flag whatever the box's EC and unmask times are:

  side (EC CUs):   ec_combine -> claim units -> part[1] (until the flag) --\
  part (the rest): shamir -> rows + self masks -> part[0] -> set flag -----+-> part[0] + part[1]
                                                                              + units left -> out
"""
from __future__ import annotations

import torch


class ServerReconstruction:
    def __init__(self, engine, device=None, pass1_min_items: int = 1024, ec_cus: int = 0, cu_pick: str = "stride",
                 pair_split: float = 0.0, pair_queue: bool = False, ec_terms: int = 1, ec_spread: int = 0,
                 ec_coop: int = 0):
        self.eng = engine
        if ec_terms not in (1, 2, 4):
            raise ValueError("ec_terms must be 1, 2 or 4")
        self.ec_terms = int(ec_terms)
        self.ec_spread = int(ec_spread)   # KiB of LDS per EC workgroup on the confined CUs (flm_set_tuning ec_spread)
        self.ec_coop = int(ec_coop)       # on the confined CUs: 0 one lane per product, 1 four cooperating waves,
                                          # 2 the same with the row field (flm_fe_row.h)
        self.pass1_min_items = pass1_min_items
        if not 0.0 <= pair_split < 1.0:
            raise ValueError("pair_split must be in [0, 1)")
        if (pair_split or pair_queue) and ec_cus <= 0:
            raise ValueError("pair_split / pair_queue need CU-partitioned streams (ec_cus > 0)")
        if pair_split and pair_queue:
            raise ValueError("pair_split and pair_queue are alternatives")
        self.pair_split = float(pair_split)
        self.pair_queue = bool(pair_queue)
        # the side stream's pair pass builds a device seed table while the self-mask pass builds
        # another on the other stream: a context of its own, so the two never share recs/meta
        self.side_eng = None
        if self.pair_split or self.pair_queue:
            from .engine import MaskEngine
            self.side_eng = MaskEngine(engine.device)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self._bufs = {}
        self._cu_streams = []
        self.ec_cus = int(ec_cus)
        self.part = None
        if self.ec_cus > 0:
            n = engine.cu_count()
            if not 0 < self.ec_cus < n:
                raise ValueError(f"ec_cus={ec_cus} must be in (0, {n})")
            ec = pick_cus(n, self.ec_cus, cu_pick)
            self.side = engine.cu_stream(ec)
            self.part = engine.cu_stream([c for c in range(n) if c not in set(ec)])
            self._cu_streams = [self.side, self.part]
        else:
            self.side = torch.cuda.Stream(device=self.device)

    def close(self):
        """The CU-partitioned streams belong to the engine (cached per CU set, destroyed
        by MaskEngine.close()); nothing of ours outlives the last run's events."""
        self._cu_streams = []
        if self.side_eng is not None:
            torch.cuda.synchronize(self.device)
            self.side_eng.close()
            self.side_eng = None

    def _buf(self, name, shape, dtype, fill=None):
        b = self._bufs.get(name)
        if b is None or tuple(b.shape) != tuple(shape) or b.dtype != dtype:
            b = torch.empty(shape, dtype=dtype, device=self.device)
            if fill is not None:
                b.fill_(fill)
            self._bufs[name] = b
        return b

    def _ec_combine(self, c1, pair_shares, lambdas, p_seeds, flags):
        """The threshold-ElGamal combine on the side stream.  Confined to ec_cus CUs it fills them,
        so the one-lane-per-product kernel (fewer instructions) beats the cooperative one there
        (profiles/r02_recon_coop.log; re-checked after round 3's shorter chain, ec_coop=1 on 24-48
        first CUs: 6.71-8.72 ms against 6.63-7.70 for two Straus terms per lane,
        profiles/r03_recon_coop_confined_sweep.log), and `ec_terms` products per lane share one chain of
        doublings (Straus: 2 terms on 24 CUs 8.05 ms vs 1 term on 32 CUs 8.46, profiles/r02_straus_recon.log);
        unconfined, the library's auto choice stands."""
        keys = ("ec_coop", "ec_terms", "ec_spread")
        prev = {k: self.eng.get_tuning(k) for k in keys}
        if self.ec_cus > 0:
            self.eng.set_tuning("ec_coop", self.ec_coop)
            self.eng.set_tuning("ec_terms", self.ec_terms)
            self.eng.set_tuning("ec_spread", self.ec_spread)
        try:
            self.eng.ec_combine_dev(c1, pair_shares, lambdas, p_seeds, flags, stream=self.side)
        finally:
            if self.ec_cus > 0:
                for k in keys:                        # the caller's own settings, not the defaults
                    self.eng.set_tuning(k, prev[k])

    def run(self, rows, L: int, lambdas, mi_shares, c1, pair_shares, pair_signs, out, stream=None,
            overlap: bool = True):
        """rows (N, pitch) int32; lambdas (T, 32), mi_shares (T, M, 32), c1 (D, 64), pair_shares
        (T, D, 64) uint8; pair_signs (D,) int8; out (>= L,) int32 -- all CUDA tensors on this device.
        Enqueues on `stream` (default: torch's current stream); returns (out, flags), flags (D,)
        int32 from the combine (bits 0/1: a point was not on P-256, bit 2: result at infinity)."""
        eng = self.eng
        main = torch.cuda.current_stream(self.device) if stream is None else stream
        M = mi_shares.shape[1]
        D = c1.shape[0] if c1 is not None else 0
        # Every buffer (and every fill) is made on the caller's stream BEFORE the `ready`
        # event below, so the side and CU-partitioned streams that wait on `ready` see it
        # initialised, on the first run and whenever a shape changes.
        with torch.cuda.stream(main):
            seeds = self._buf("seeds", (M + D, 32), torch.uint8)
            flags = self._buf("flags", (max(D, 1),), torch.int32)
            neg = self._buf("neg", (M,), torch.int8, -1)
            if D and not overlap:
                signs = self._buf("signs_all", (M + D,), torch.int8)
                signs[:M].fill_(-1)
                signs[M:].copy_(pair_signs)
        m_seeds, p_seeds = seeds[:M], seeds[M:]
        if D == 0:
            eng.shamir_combine_dev(mi_shares, lambdas, m_seeds, stream=main)
            eng.aggregate_unmask_dev(rows, m_seeds, neg, out, L=L, stream=main)
            return out, flags[:0]
        if not overlap:
            eng.shamir_combine_dev(mi_shares, lambdas, m_seeds, stream=main)
            eng.ec_combine_dev(c1, pair_shares, lambdas, p_seeds, flags, stream=main)
            eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L, stream=main)
            return out, flags
        if self.pair_queue:
            return self._run_queue(rows, L, lambdas, mi_shares, c1, pair_shares, pair_signs, out, main,
                                   m_seeds, p_seeds, flags, neg)
        caller = main
        with torch.cuda.stream(caller):
            part = self._buf("tmp", (2 if self.pair_split else 1, rows.shape[1]), torch.int32)
        ready = torch.cuda.Event()
        ready.record(main)                       # inputs enqueued on main are visible to the side stream
        self.side.wait_event(ready)
        self._ec_combine(c1, pair_shares, lambdas, p_seeds, flags)
        done = torch.cuda.Event()
        done.record(self.side)
        if self.part is not None:
            self.part.wait_event(ready)
            main = self.part
        eng.shamir_combine_dev(mi_shares, lambdas, m_seeds, stream=main)
        # part[0]: rows + self masks; part[1]: the side stream's share of the pair masks
        tmp = part[:1]
        lo = int(self.pair_split * L) // 1024 * 1024 if self.pair_split else 0
        if lo:
            self.side_eng.aggregate_unmask_dev(None, p_seeds, pair_signs, part[1], L=L, mask_lo=0, mask_hi=lo,
                                               stream=self.side)
            done = torch.cuda.Event()
            done.record(self.side)
        if self.pass1_min_items != 1024:
            eng.set_tuning("min_items", self.pass1_min_items)
        try:
            eng.aggregate_unmask_dev(rows, m_seeds, neg, tmp[0], L=L, stream=main)
        finally:
            if self.pass1_min_items != 1024:
                eng.set_tuning("min_items", 1024)
        if main is not caller:
            fin = torch.cuda.Event()
            fin.record(main)
            caller.wait_event(fin)
            main = caller
        # the caller's stream now waits for both streams' work, so every buffer they
        # touched is safe to free or reuse in the caller's stream order (no
        # record_stream, which would tie the allocator to a stream we may destroy)
        main.wait_event(done)
        eng.aggregate_unmask_dev(part if lo else tmp, p_seeds, pair_signs, out, L=L, mask_lo=lo, mask_hi=L,
                                 stream=main)
        return out, flags


    def _run_queue(self, rows, L, lambdas, mi_shares, c1, pair_shares, pair_signs, out, caller, m_seeds, p_seeds,
                   flags, neg):
        eng, side_eng = self.eng, self.side_eng
        pitch = rows.shape[1]
        with torch.cuda.stream(caller):
            part = self._buf("tmp", (2, pitch), torch.int32)
            ws = self._buf("ws", (4,), torch.int32)
            ws.zero_()                           # unit counter, stop flag
            part[1].zero_()                      # the side pass adds into it
        ready = torch.cuda.Event()
        ready.record(caller)
        self.side.wait_event(ready)
        self.part.wait_event(ready)
        self._ec_combine(c1, pair_shares, lambdas, p_seeds, flags)
        side_groups = self.ec_cus * 32           # one-wave workgroups, 8 per SIMD
        side_eng.pair_units_dev(p_seeds, pair_signs, part[1], L, ws, side_groups, stream=self.side)
        done = torch.cuda.Event()
        done.record(self.side)
        eng.shamir_combine_dev(mi_shares, lambdas, m_seeds, stream=self.part)
        if self.pass1_min_items != 1024:
            eng.set_tuning("min_items", self.pass1_min_items)
        try:
            eng.aggregate_unmask_dev(rows, m_seeds, neg, part[0], L=L, stream=self.part)
        finally:
            if self.pass1_min_items != 1024:
                eng.set_tuning("min_items", 1024)
        eng.flag_set_dev(ws, stream=self.part)
        fin = torch.cuda.Event()
        fin.record(self.part)
        caller.wait_event(fin)
        caller.wait_event(done)
        side_eng.pair_units_dev(p_seeds, pair_signs, out, L, ws, eng.cu_count() * 32, p0=part[0], p1=part[1],
                                final=True, stream=caller)
        return out, flags


def pick_cus(n: int, k: int, how: str = "stride"):
    """k of n logical CU ids: evenly strided over the id space, the first k, "xcd_stride": k/8 per XCD
    (logical id i sits on XCD i % 8, profiles/r01_cu_map_probe.log) spread over each XCD's CUs, or
    "xcd": whole XCDs, XCD 0's CUs first."""
    if how == "first":
        return list(range(k))
    if how == "xcd" and n % 8 == 0 and k <= n:
        per = n // 8
        return sorted((i % per) * 8 + i // per for i in range(k))  # whole XCDs: XCD 0's CUs, then XCD 1's, ...
    if how == "xcd_stride" and n % 8 == 0 and k % 8 == 0 and k > 0:
        per, m = n // 8, k // 8
        return sorted(x + 8 * ((j * per) // m) for x in range(8) for j in range(m))
    return sorted({(i * n) // k for i in range(k)})
