"""Why does the c4 round run at ~704 G words/s while client masking (same ChaCha core) reaches
~771?  Mask-only items_kernel launches (no rows) of K seeds over L slots at several shapes:
more tiles per launch (more workgroup generations per CU) vs more seeds per tile, and the
planner's seed split (min_items).  Every launch runs after >= 100 ms of back-to-back load.
Also a 300-launch time series of the c4 shape to see the steady clock."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

eng = MaskEngine(0)
s = torch.cuda.current_stream()
g = torch.Generator(device="cuda").manual_seed(1)


def run(K, L, reps=20, min_items=None, variant=None, series=False):
    if min_items:
        eng.set_tuning("min_items", min_items)
    if variant is not None:
        eng.set_tuning("variant", variant)
    seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
    signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.seed_table_dev(seeds, signs)
    t_warm = 0
    n_warm = max(3, int(100e-3 / (K * L / 700e9)))
    for _ in range(n_warm):
        eng.aggregate_dev(None, K, out, L=L)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        eng.aggregate_dev(None, K, out, L=L)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    p = eng.last_plan()
    ms = float(np.median(t))
    rec = {"K": K, "L": L, "items": p.get("items"), "variant": p.get("variant"), "min_items": min_items,
           "median_ms": round(ms, 4), "min_ms": round(min(t), 4), "Gwords/s": round(K * L / ms / 1e6, 1)}
    if series:
        rec["series"] = [round(x, 3) for x in t]
    print(rec, flush=True)
    eng.set_tuning("min_items", 1024)
    eng.set_tuning("variant", -1)


for K, L in ((1024, 1 << 20), (1024, 1 << 21), (1024, 1 << 22), (2048, 1 << 20), (4096, 1 << 20),
             (256, 1 << 22), (512, 1 << 21), (1024, 1 << 19), (1024, 1 << 18)):
    run(K, L)
for mi in (2048, 4096, 8192):
    run(1024, 1 << 20, min_items=mi)
run(1024, 1 << 20, reps=300, series=True)
