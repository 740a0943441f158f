"""One rank's kernel of the strong-scaled c4 round (BASELINE configs[3]: 1024 clients in all, L = 2^20,
1024 self-mask seeds) at G = 1, 2, 4, 8, on one GPU: N/G rows over all L slots plus the K masks
over rank G-1's slot shard, after a clock settle.  Median of 50 launches (seed schedule excluded),
plus the seed-schedule + kernel pair as one step.  Predicts the per-GPU time of bench.py --gpus G
before the reduce-scatter."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.distributed import shard_bounds  # noqa: E402

N, K, L = 1024, 1024, 1 << 20
eng = MaskEngine(0)
s = torch.cuda.current_stream()
g = torch.Generator(device="cuda").manual_seed(1)
rows_all = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
out = torch.empty(L, dtype=torch.int32, device="cuda")
eng.seed_table_dev(seeds, signs)
e0 = torch.cuda.Event(enable_timing=True)
e0.record(s)
while True:
    for _ in range(10):
        eng.aggregate_dev(rows_all, K, out, L=L)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(s)
    torch.cuda.synchronize()
    if e0.elapsed_time(e1) > 200:
        break
base = None
for G in (1, 2, 4, 8):
    rows = rows_all[: N // G]
    lo, hi = shard_bounds(L, G, G - 1)
    for _ in range(5):
        eng.aggregate_dev(rows, K, out, L=L, mask_lo=lo, mask_hi=hi)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(51)]
    ev[0].record(s)
    for i in range(50):
        eng.aggregate_dev(rows, K, out, L=L, mask_lo=lo, mask_hi=hi)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(50)]
    ms = float(np.median(t))
    es = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    es[0].record(s)
    for i in range(50):
        eng.seed_table_dev(seeds, signs)
        eng.aggregate_dev(rows, K, out, L=L, mask_lo=lo, mask_hi=hi)
    es[1].record(s)
    torch.cuda.synchronize()
    step = es[0].elapsed_time(es[1]) / 50
    base = base or step
    p = eng.last_plan()
    print(json.dumps({"G": G, "rows": N // G, "mask_slots": hi - lo, "items": p["items"], "variant": p["variant"],
                      "atomics": p["atomics"], "kernel_ms": round(ms, 4), "step_ms": round(step, 4),
                      "speedup_vs_G1": round(base / step, 2)}), flush=True)
