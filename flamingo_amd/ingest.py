"""Device-resident VECTOR ingestion for the drop-in server.

The reference server stores each client's VECTOR body on arrival
(SA_ServiceAgent.py:205-210), sums the stored vectors in report_process
(:346-350) and, one step later, adds the regenerated masks to that partial sum
in reconstruction_process (:529-540, :587-605).  VectorStore keeps the same
three moments on the GPU(s):

  add(sender, vec)   on arrival: the body is copied through a pinned staging
                     ring onto its device row (async, a copy stream per device),
                     so the uploads overlap the simulation's message handling;
  partial_sum()      at report: S = sum of the stored rows, one launch per device
                     (a DeviceGroup: client-sharded rows, one reduce-scatter);
                     S stays on the device(s), sharded by slot on a group;
  unmask(seeds, sg)  at reconstruction: final = S + sum sg*PRG(seed) over each
                     device's own slot shard (no exchange: S is already sharded),
                     the only device-to-host copy of the round.

No L-vector goes device -> host -> device between the two steps.  Rows are
placed round-robin over the devices in arrival order; a sender that sends
twice overwrites its row, as the reference's dict assignment does.
"""
from __future__ import annotations

import numpy as np

RING = 8   # pinned staging buffers per device


class VectorStore:
    def __init__(self, engine, L: int, capacity: int):
        import torch
        from .engine import DeviceGroup
        self.L = int(L)
        self.group = engine if isinstance(engine, DeviceGroup) else None
        self.engines = engine.engines if self.group is not None else [engine]
        self.devices = [torch.device("cuda", e.device) for e in self.engines]
        self.G = len(self.engines)
        self.cap = max(1, -(-int(capacity) // self.G))
        self.pitch = -(-self.L // 64) * 64     # row pitch: a multiple of 4 words (flm_aggregate_unmask_dev)
        self._rows = [torch.empty((self.cap, self.pitch), dtype=torch.int32, device=d) for d in self.devices]
        self._copy = [torch.cuda.Stream(device=d) for d in self.devices]
        self._stage = [[torch.empty(self.L, dtype=torch.int32).pin_memory() for _ in range(RING)]
                       for _ in self.devices]
        self._stage_ev = [[None] * RING for _ in self.devices]
        self._next = [0] * self.G
        self._consumed = [None] * self.G    # the last partial sum's read of the rows, per device
        self.reset()

    # ------------------------------------------------------------ ingestion
    def reset(self):
        """Forget the stored rows (a new iteration's VECTORs go into the same device rows once
        the last partial sum has read them: the copy streams wait for it)."""
        self._slot = {}
        self._n = [0] * self.G
        self.bad = []
        for r in range(self.G):
            if self._consumed[r] is not None:
                self._copy[r].wait_event(self._consumed[r])
                self._consumed[r] = None

    def __len__(self):
        return len(self._slot)

    def add(self, sender, vec):
        """Store one VECTOR body (uint32[L]); a wrong length (or a non-32-bit-integer body) is
        remembered for partial_sum to raise, as report_process does (:348-349)."""
        import torch
        v = np.asarray(vec)
        if v.ndim != 1 or v.shape[0] != self.L or v.dtype.kind not in "ui" or v.dtype.itemsize != 4:
            self.bad.append(sender)
            return
        if sender in self._slot:
            r, i = self._slot[sender]
        else:
            r = len(self._slot) % self.G
            i = self._n[r]
            if i == self._rows[r].shape[0]:
                self._grow(r)
            self._n[r] += 1
            self._slot[sender] = (r, i)
        b = self._next[r]
        self._next[r] = (b + 1) % RING
        if self._stage_ev[r][b] is not None:
            self._stage_ev[r][b].synchronize()        # this staging buffer's last DMA has been read
        st = self._stage[r][b]
        st.numpy()[:] = v.view(np.int32)
        with torch.cuda.stream(self._copy[r]):
            self._rows[r][i, : self.L].copy_(st, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._copy[r])
        self._stage_ev[r][b] = ev

    def _grow(self, r):
        import torch
        old = self._rows[r]
        new = torch.empty((2 * old.shape[0], self.pitch), dtype=torch.int32, device=old.device)
        self._copy[r].wait_stream(torch.cuda.current_stream(old.device))
        with torch.cuda.stream(self._copy[r]):
            new[: old.shape[0]].copy_(old)
        old.record_stream(self._copy[r])      # freed only after the copy that reads it
        self._rows[r] = new

    # ------------------------------------------------------------ the round
    def partial_sum(self):
        """Enqueue S = sum of the stored rows (SA_ServiceAgent.py:346-350); returns the device
        event that completes it (S stays device-resident, see unmask / host_partial)."""
        import torch
        if self.bad:
            raise RuntimeError("Client sends vector of incorrect length.")
        self._t0 = torch.cuda.Event(enable_timing=True)
        self._t0.record(torch.cuda.current_stream(self.devices[0]))
        for r, d in enumerate(self.devices):
            torch.cuda.current_stream(d).wait_stream(self._copy[r])
        if self.group is None:
            d = self.devices[0]
            s = torch.cuda.current_stream(d)
            self.S = [torch.empty(self.pitch, dtype=torch.int32, device=d)]
            n = self._n[0]
            if n:
                self.engines[0].aggregate_unmask_dev(self._rows[0][:n], None, None, self.S[0], L=self.L, stream=s)
            else:
                self.S[0].zero_()
            self._consumed[0] = torch.cuda.Event()
            self._consumed[0].record(s)
            self.bounds = [(0, self.L)]
        else:
            from .engine import shard_bounds
            g = self.group
            sb = [shard_bounds(self.L, self.G, r) for r in range(self.G)]
            self.S = [torch.empty(S, dtype=torch.int32, device=d) for (_, _, S), d in zip(sb, self.devices)]
            g.aggregate_unmask_dev([self._rows[r][: self._n[r]] for r in range(self.G)], [None] * self.G,
                                   [None] * self.G, self.S, self.L)
            for r in range(self.G):
                ev = torch.cuda.Event()
                ev.record(g.rank_stream(r))
                self._consumed[r] = ev
            g.wait()
            self.bounds = [(lo, hi) for lo, hi, _ in sb]
        self.done = torch.cuda.Event(enable_timing=True)
        self.done.record(torch.cuda.current_stream(self.devices[0]))
        return self.done

    def wait_partial(self) -> float:
        """Block until S is complete; the device time (ms) from partial_sum's call to S done --
        the uploads still in flight at that call included."""
        self.done.synchronize()
        return self._t0.elapsed_time(self.done)

    def host_partial(self) -> np.ndarray:
        """S on the host (uint32[L]) -- only for inspection; the round itself never copies it."""
        out = np.empty(self.L, np.uint32)
        for (lo, hi), s in zip(self.bounds, self.S):
            out[lo:hi] = s[: hi - lo].cpu().numpy().view(np.uint32)
        return out

    def unmask(self, seeds, signs) -> np.ndarray:
        """final = S + sum_k signs[k] * PRG(seeds[k]) (SA_ServiceAgent.py:529-540, 587-605), each
        device over its own slot shard [lo, hi) (PRG words lo.. of every seed), host out."""
        import torch
        from .engine import _seeds_array, _signs_array
        seeds = _seeds_array(seeds)
        signs = _signs_array(signs, seeds.shape[0])
        K = seeds.shape[0]
        if getattr(self, "_host_out", None) is None:
            self._host_out = torch.empty(self.L, dtype=torch.int32).pin_memory()
        host = self._host_out
        outs = []
        for r, d in enumerate(self.devices):
            lo, hi = self.bounds[r]
            n = hi - lo
            if n <= 0:
                continue
            s = torch.cuda.current_stream(d)
            out = torch.empty(n, dtype=torch.int32, device=d)
            d_seeds = torch.from_numpy(seeds).to(d, non_blocking=False) if K else None
            d_signs = torch.from_numpy(signs).to(d, non_blocking=False) if K else None
            self.engines[r].aggregate_unmask_dev(self.S[r].view(1, -1), d_seeds, d_signs, out, L=n,
                                                 mask_lo=0, mask_hi=n, prg_slot0=lo, stream=s)
            with torch.cuda.stream(s):
                host[lo:hi].copy_(out, non_blocking=True)
            outs.append((d_seeds, d_signs, out))
        for d in set(self.devices):
            torch.cuda.synchronize(d)
        return host.numpy().view(np.uint32).copy()
