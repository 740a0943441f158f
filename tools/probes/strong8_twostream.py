"""Rank G-1 of the strong-scaled c4 round at G = 2, 4, 8: rows (N/G over all L) and masks (1024 seeds
over the last 1/G slots) as two kernels on two streams (two engines, two outputs, then one add)
against the one dual-tile kernel.  Median over 40 rounds after a clock settle."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

N, K, L = 1024, 1024, 1 << 20
eng, eng_r = MaskEngine(0), MaskEngine(0)
gen = torch.Generator(device="cuda").manual_seed(1)
rows_all = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=gen)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=gen)
signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
out, o1, o2 = (torch.empty(L, dtype=torch.int32, device="cuda") for _ in range(3))
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
eng.seed_table_dev(seeds, signs, stream=sa)
eng_r.seed_table_dev(seeds[:0], signs[:0], stream=sb)
torch.cuda.synchronize()


def one(rows, lo, hi):
    eng.aggregate_dev(rows, K, out, L=L, mask_lo=lo, mask_hi=hi, stream=sa)


def two(rows, lo, hi):
    ev = torch.cuda.Event()
    ev.record(sa)
    sb.wait_event(ev)
    eng_r.aggregate_dev(rows, 0, o1, L=L, stream=sb)
    eng.aggregate_dev(None, K, o2, L=L, mask_lo=lo, mask_hi=hi, stream=sa)
    ev2 = torch.cuda.Event()
    ev2.record(sb)
    sa.wait_event(ev2)
    torch.add(o1, o2, out=out)  # (stands in for the library's add; same stream as the masks)


def timeit(f, *a, reps=40):
    for _ in range(5):
        with torch.cuda.stream(sa):
            f(*a)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    with torch.cuda.stream(sa):
        ev[0].record(sa)
        for i in range(reps):
            f(*a)
            ev[i + 1].record(sa)
    torch.cuda.synchronize()
    return float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))


e0 = torch.cuda.Event(enable_timing=True)
e0.record(sa)
while True:
    for _ in range(10):
        one(rows_all, 0, L)
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(sa)
    torch.cuda.synchronize()
    if e0.elapsed_time(e1) > 200:
        break
for G in (2, 4, 8):
    rows = rows_all[: N // G]
    lo, hi = (G - 1) * L // G, L
    t1 = timeit(one, rows, lo, hi)
    t2 = timeit(two, rows, lo, hi)
    print(json.dumps({"G": G, "one_dual_kernel_ms": round(t1, 4), "two_streams_ms": round(t2, 4)}), flush=True)
