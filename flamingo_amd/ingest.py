"""Device-resident VECTOR ingestion for the drop-in server (flm_store_*, csrc/flm_store.hip).

The reference server stores each client's VECTOR body on arrival
(SA_ServiceAgent.py:205-210), sums the stored vectors in report_process
(:346-350) and, one step later, adds the regenerated masks to that partial sum
in reconstruction_process (:529-540, :587-605).  VectorStore keeps the same
three moments on the GPU(s), in the library:

  add(sender, vec)   on arrival: the body is copied into pinned staging and DMA'd
                     onto its device row on the store's copy stream, so the uploads
                     overlap the simulation's message handling;
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

import ctypes

import numpy as np

from . import _lib
from ._lib import p_i8, p_u32, p_u8


class VectorStore:
    def __init__(self, engine, L: int, capacity: int):
        from .engine import DeviceGroup
        self.lib = _lib.load()
        self.L = int(L)
        grp = engine if isinstance(engine, DeviceGroup) else None
        self.G = grp.n if grp is not None else 1
        self.devices = list(grp.devices) if grp is not None else [engine.device]
        self._owner = engine                       # keeps the context / group alive
        h = ctypes.c_void_p()
        rc = self.lib.flm_store_create(ctypes.byref(h), None if grp is not None else engine.ctx,
                                       grp.g if grp is not None else None, self.L, max(1, int(capacity)))
        if rc != 0:
            raise RuntimeError(f"flm_store_create: {self.lib.flm_store_last_error(None).decode()}")
        self.h = h
        self.bad = []
        self.has_partial = False                   # a partial sum S has been enqueued since the last reset
        self._grp = grp
        if grp is not None:
            grp._stores += 1                       # the group refuses to close while its stores are open

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: {self.lib.flm_store_last_error(self.h).decode()}")

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.flm_store_free(self.h)
            self.h = None
            if self._grp is not None:
                self._grp._stores -= 1
                if self._grp._stores == 0 and self._grp.retired:
                    self._grp.close()              # a group replaced under this store (protocol.server_engine)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ ingestion
    def __len__(self):
        return int(self.lib.flm_store_count(self.h))

    def add(self, sender, vec):
        """Store one VECTOR body (uint32[L]); a wrong length (or a non-32-bit-integer body) is
        remembered and makes partial_sum raise, as report_process does (:348-349)."""
        v = np.asarray(vec)
        if v.ndim != 1 or v.shape[0] != self.L or v.dtype.kind not in "ui" or v.dtype.itemsize != 4:
            self.bad.append(sender)
            self._check(self.lib.flm_store_add(self.h, int(sender), None, 0), "flm_store_add")
            return
        v = np.ascontiguousarray(v)
        self._check(self.lib.flm_store_add(self.h, int(sender), v.ctypes.data, self.L), "flm_store_add")

    def reset(self):
        """Forget the stored rows (the next iteration's VECTORs wait for the last partial sum's reads)."""
        self.bad = []
        self.has_partial = False
        self._check(self.lib.flm_store_reset(self.h), "flm_store_reset")

    # ------------------------------------------------------------ the round
    def partial_sum(self):
        """Enqueue S = sum of the stored rows (SA_ServiceAgent.py:346-350); S stays device-resident."""
        if self.bad:
            raise RuntimeError("Client sends vector of incorrect length.")
        self._check(self.lib.flm_store_partial(self.h), "flm_store_partial")
        self.has_partial = True

    def wait_partial(self) -> float:
        """Block until S is complete; the device time (ms) from partial_sum's call to S done --
        the uploads still in flight at that call included."""
        ms = ctypes.c_float()
        self._check(self.lib.flm_store_partial_wait(self.h, ctypes.byref(ms)), "flm_store_partial_wait")
        return float(ms.value)

    def host_partial(self) -> np.ndarray:
        """S on the host (uint32[L]) -- only for inspection; the round itself never copies it."""
        out = np.empty(self.L, np.uint32)
        self._check(self.lib.flm_store_partial_host(self.h, p_u32(out)), "flm_store_partial_host")
        return out

    def unmask(self, seeds, signs) -> np.ndarray:
        """final = S + sum_k signs[k] * PRG(seeds[k]) (SA_ServiceAgent.py:529-540, 587-605), each
        device over its own slot shard (PRG words lo.. of every seed), host out."""
        from .engine import _seeds_array, _signs_array
        seeds = _seeds_array(seeds)
        signs = _signs_array(signs, seeds.shape[0])
        out = np.empty(self.L, np.uint32)
        self._check(self.lib.flm_store_unmask(self.h, p_u8(seeds), p_i8(signs), seeds.shape[0], p_u32(out)),
                    "flm_store_unmask")
        return out

    def unmask_ms(self) -> float:
        """Device time (ms) of the last unmask, seed upload to the end of the D2H (flm_store_unmask_ms)."""
        ms = ctypes.c_float()
        self._check(self.lib.flm_store_unmask_ms(self.h, ctypes.byref(ms)), "flm_store_unmask_ms")
        return float(ms.value)
