"""One rank of the strong-scaled c4 round (N/G rows over all L = 2^20 slots, 1024 seeds over the
rank's slot shard) planned as dual-tile items (pairing 1) or as same-tile window items (pairing 2,
merged kernel); G = 2, 4, 8, ranks 0 and G-1.  Outputs compared bit for bit between the plans;
median of 40 launches after a clock settle, alternating plans."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.engine import shard_bounds  # noqa: E402

N, K, L = 1024, 1024, 1 << 20
eng = MaskEngine(0)
s = torch.cuda.current_stream()
gen = torch.Generator(device="cuda").manual_seed(1)
rows_all = torch.randint(-2**31, 2**31 - 1, (N // 2, L), dtype=torch.int32, device="cuda", generator=gen)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=gen)
signs = torch.where(torch.rand(K, device="cuda", generator=gen) < 0.5, 1, -1).to(torch.int8)
eng.seed_table_dev(seeds, signs)
out = {p: torch.empty(L, dtype=torch.int32, device="cuda") for p in (1, 2)}


def run(rows, lo, hi, pairing, reps=40, min_items=1024):
    eng.set_tuning("pairing", pairing)
    eng.set_tuning("min_items", min_items)
    for _ in range(5):
        eng.aggregate_dev(rows, K, out[pairing], L=L, mask_lo=lo, mask_hi=hi)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        eng.aggregate_dev(rows, K, out[pairing], L=L, mask_lo=lo, mask_hi=hi)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    return float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)])), eng.last_plan()


e0 = torch.cuda.Event(enable_timing=True)
e0.record(s)
while True:
    run(rows_all, 0, L // 8, 1, reps=10)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(s)
    torch.cuda.synchronize()
    if e0.elapsed_time(e1) > 200:
        break
for G in (2, 4, 8):
    rows = rows_all[: N // G]
    for r in (0, G - 1):
        lo, hi, _ = shard_bounds(L, G, r)
        res = {}
        for rep in range(2):
            for p in (1, 2):
                ms, plan = run(rows, lo, hi, p)
                res.setdefault(p, []).append(ms)
                res[f"plan{p}"] = {"items": plan["items"], "variant": plan["variant"]}
        same = bool(torch.equal(out[1], out[2]))
        print(json.dumps({"G": G, "rank": r, "dual_ms": res[1], "same_tile_ms": res[2], "bit_equal": same,
                          "dual_plan": res["plan1"], "same_plan": res["plan2"]}), flush=True)
        if not same:
            sys.exit(1)
        if os.environ.get("SWEEP"):
            for mi in (256, 512, 2048):
                ms, plan = run(rows, lo, hi, 2, min_items=mi)
                print(json.dumps({"G": G, "rank": r, "min_items": mi, "same_tile_ms": ms, "plan": plan}), flush=True)
