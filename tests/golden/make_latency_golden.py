"""Golden vectors for the ABIDES latency model, produced by the REFERENCE'S OWN module.

model/LatencyModel.py imports only numpy and sys, so it loads unmodified in the
build container (no shim).  This script is run there, once, reading the file from the
read-only reference tree; its output tests/golden/latency.json is what travels.
Each case fixes a RandomState seed and parameters (scalar, 1-D, 2-D, connected mask,
deterministic) and records get_latency(sender, recipient) for a fixed call sequence, so
the test pins both the formula and the order of random draws.

usage: python tests/golden/make_latency_golden.py /root/reference
"""
import importlib.util
import json
import os
import sys

import numpy as np

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
spec = importlib.util.spec_from_file_location("ref_latency", os.path.join(ref, "model", "LatencyModel.py"))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)

n = 6
rs = np.random.RandomState(5)
min_lat = rs.uniform(low=10_000_000, high=100_000_000, size=(n, n))
calls = [(s, r) for s in range(n) for r in range(n) if s != r] * 3
cases = {
    "config_flamingo": dict(model="cubic", seed=11, kwargs={"connected": True, "min_latency": min_lat.tolist(),
                                                              "jitter": 0.3, "jitter_clip": 0.05, "jitter_unit": 5}),
    "defaults": dict(model="cubic", seed=12, kwargs={"min_latency": min_lat.tolist()}),
    "vector_params": dict(model="cubic", seed=13, kwargs={"min_latency": min_lat.tolist(),
                                                          "jitter": np.linspace(0.1, 0.9, n).tolist(),
                                                          "jitter_clip": 0.2, "jitter_unit": np.arange(1, n + 1.0).tolist()}),
    "scalar_min": dict(model="cubic", seed=14, kwargs={"min_latency": 21000, "jitter": 0.5}),
    "deterministic": dict(model="deterministic", seed=15, kwargs={"min_latency": min_lat.tolist()}),
}
out = {"calls": calls, "cases": {}}
for name, c in cases.items():
    kw = {k: (np.array(v) if isinstance(v, list) else v) for k, v in c["kwargs"].items()}
    m = mod.LatencyModel(c["model"], random_state=np.random.RandomState(c["seed"]), kwargs=kw)
    out["cases"][name] = dict(c, latencies=[float(m.get_latency(s, r)) for s, r in calls])
# connected mask: one direction disabled returns -1 and consumes no draw
conn = np.ones((n, n), bool)
conn[1, 2] = False
m = mod.LatencyModel("cubic", random_state=np.random.RandomState(16),
                     kwargs={"min_latency": min_lat, "connected": conn})
out["cases"]["connected_mask"] = dict(model="cubic", seed=16,
                                      kwargs={"min_latency": min_lat.tolist(), "connected": conn.tolist()},
                                      latencies=[float(m.get_latency(s, r)) for s, r in calls])
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "latency.json"), "w") as f:
    json.dump(out, f)
print("wrote latency.json:", {k: len(v["latencies"]) for k, v in out["cases"].items()})
