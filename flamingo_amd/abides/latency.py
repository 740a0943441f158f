"""Per-message network latency (model/LatencyModel.py surface).

``cubic``: latency = min + (a / x^3) * (min / unit), x ~ U(clip, 1]
(model/LatencyModel.py:126-140); ``deterministic``: latency = min (:142-143).
Parameters are scalars or numpy arrays indexed by sender (1-D) or
[sender, recipient] (2-D).  Late VECTOR messages are the only source of
client dropouts in the reference simulation.
"""
from __future__ import annotations

import numpy as np

_DEFAULTS = {"connected": True, "jitter": 0.5, "jitter_clip": 0.1, "jitter_unit": 10.0}


def _pick(v, s, r):
    if np.isscalar(v):
        return v
    v = np.asarray(v)
    if v.ndim == 1:
        return v[s]
    if v.ndim == 2:
        return v[s, r]
    raise ValueError("LatencyModel parameter must be a scalar, 1-D or 2-D array")


class LatencyModel:
    def __init__(self, latency_model: str = "cubic", random_state=None, **kwargs):
        if "kwargs" in kwargs:
            kwargs = kwargs["kwargs"]
        self.latency_model = latency_model.lower()
        if self.latency_model not in ("cubic", "deterministic"):
            raise ValueError(f"unknown latency model {latency_model!r}")
        if "min_latency" not in kwargs:
            raise ValueError(f"{self.latency_model} latency model requires 'min_latency'")
        self.kwargs = dict(kwargs)
        if self.latency_model == "cubic":
            for k, v in _DEFAULTS.items():
                self.kwargs.setdefault(k, v)
        self.random_state = random_state

    def get_latency(self, sender_id=None, recipient_id=None):
        kw = self.kwargs
        lo = _pick(kw["min_latency"], sender_id, recipient_id)
        if self.latency_model == "deterministic":
            return lo
        if not _pick(kw["connected"], sender_id, recipient_id):
            return -1
        a = _pick(kw["jitter"], sender_id, recipient_id)
        clip = _pick(kw["jitter_clip"], sender_id, recipient_id)
        unit = _pick(kw["jitter_unit"], sender_id, recipient_id)
        x = self.random_state.uniform(low=clip, high=1.0)
        return lo + (a / x ** 3) * (lo / unit)
