"""Plan sweep for one rank of the strong-scaled c4 round (N/G rows over all L, K = 1024 masks over
the last rank's slot shard) at G = 2, 4, 8: the default plan against windowed plans with other
sub-tile counts and item targets (flm_set_tuning "subtiles" / "min_items" / "pairing"), median of
40 launches each after a clock settle; every plan checked against the default's output."""
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
ref = torch.empty(L, dtype=torch.int32, device="cuda")
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


def timed(rows, lo, hi, n=40):
    for _ in range(4):
        eng.aggregate_dev(rows, K, out, L=L, mask_lo=lo, mask_hi=hi)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record(s)
    for i in range(n):
        eng.aggregate_dev(rows, K, out, L=L, mask_lo=lo, mask_hi=hi)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    return float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(n)]))


FOCUS = "--focus" in sys.argv   # the default against 4-sub-tile plans of 128 / 256 items, 3 interleaved passes
plans = ([dict()] + [dict(subtiles=st, min_items=mi) for st in (1, 4, 16) for mi in (256, 512, 1024, 2048)] +
         [dict(pairing=2, min_items=mi) for mi in (512, 1024, 2048)]) if not FOCUS else \
        [dict(), dict(subtiles=4, min_items=256), dict(subtiles=4, min_items=128)] * 3
for G in (2, 4, 8):
    rows = rows_all[: N // G]
    lo, hi = shard_bounds(L, G, G - 1)[:2]
    eng.aggregate_dev(rows, K, ref, L=L, mask_lo=lo, mask_hi=hi)
    for pl in plans:
        for k, v in pl.items():
            eng.set_tuning(k, v)
        ms = timed(rows, lo, hi)
        ok = bool(torch.equal(out, ref))
        p = eng.last_plan()
        print(json.dumps({"G": G, **pl, "items": p["items"], "variant": p["variant"], "kernel_ms": round(ms, 4),
                          "same_as_default": ok}), flush=True)
        eng.set_tuning("subtiles", 0)
        eng.set_tuning("min_items", 1024)
        eng.set_tuning("pairing", 1)
