"""Rank G-1 of the strong-scaled c4 round at G = 8 (128 rows over all L = 2^20 slots, 1024 seeds over
the last 1/8 of the slots), split into its parts and planner settings: rows only, masks only, both;
min_items 256 / 512 / 1024 / 2048 / 4096.  Median of 40 launches after a clock settle."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

N, K, L, G = 1024, 1024, 1 << 20, int(os.environ.get("G", "8"))
eng = MaskEngine(0)
s = torch.cuda.current_stream()
gen = torch.Generator(device="cuda").manual_seed(1)
rows = torch.randint(-2**31, 2**31 - 1, (N // G, L), dtype=torch.int32, device="cuda", generator=gen)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=gen)
signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
out = torch.empty(L, dtype=torch.int32, device="cuda")
lo, hi = (G - 1) * L // G, L


def run(r, k, mi, reps=40):
    eng.set_tuning("min_items", mi)
    eng.seed_table_dev(seeds[:k], signs[:k])
    for _ in range(5):
        eng.aggregate_dev(r, k, out, L=L, mask_lo=lo, mask_hi=hi)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        eng.aggregate_dev(r, k, out, L=L, mask_lo=lo, mask_hi=hi)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    return float(np.median(t)), eng.last_plan()


e0 = torch.cuda.Event(enable_timing=True)
e0.record(s)
while True:
    run(rows, K, 1024, reps=10)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(s)
    torch.cuda.synchronize()
    if e0.elapsed_time(e1) > 200:
        break
for what, r, k in (("rows", rows, 0), ("masks", None, K), ("both", rows, K)):
    for mi in (256, 512, 1024, 2048, 4096):
        ms, p = run(r, k, mi)
        print(json.dumps({"G": G, "what": what, "min_items": mi, "items": p["items"], "variant": p["variant"],
                          "kernel_ms": round(ms, 4)}), flush=True)
