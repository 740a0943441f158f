"""Plan sweep for the c3 round shape (N = 1024 rows, K = 1024 seeds, L = 2^18, whole vector): the
default plan against sub-tile counts and item targets (flm_set_tuning "subtiles" / "min_items"),
median of 40 launches each after a clock settle, every plan checked against the default's output;
three interleaved passes."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

N, K, L = 1024, 1024, 1 << 18
eng = MaskEngine(0)
s = torch.cuda.current_stream()
g = torch.Generator(device="cuda").manual_seed(3)
rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
out = torch.empty(L, dtype=torch.int32, device="cuda")
ref = torch.empty(L, dtype=torch.int32, device="cuda")
eng.seed_table_dev(seeds, signs)
eng.aggregate_dev(rows, K, ref, L=L)
e0 = torch.cuda.Event(enable_timing=True)
e0.record(s)
while True:
    for _ in range(20):
        eng.aggregate_dev(rows, K, out, L=L)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(s)
    torch.cuda.synchronize()
    if e0.elapsed_time(e1) > 200:
        break
plans = [dict()] + [dict(subtiles=st, min_items=mi) for st in (1, 4) for mi in (512, 1024, 2048, 4096)]
for _ in range(3):
    for pl in plans:
        for k, v in pl.items():
            eng.set_tuning(k, v)
        for _ in range(4):
            eng.aggregate_dev(rows, K, out, L=L)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
        ev[0].record(s)
        for i in range(40):
            eng.aggregate_dev(rows, K, out, L=L)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        ms = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(40)]))
        p = eng.last_plan()
        print(json.dumps({**pl, "items": p["items"], "variant": p["variant"], "atomics": p["atomics"],
                          "kernel_ms": round(ms, 4), "same_as_default": bool(torch.equal(out, ref))}), flush=True)
        eng.set_tuning("subtiles", 0)
        eng.set_tuning("min_items", 1024)
eng.close()
