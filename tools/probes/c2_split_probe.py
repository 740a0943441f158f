"""c2-shaped round (N=128, L=16384): where do its ~13.5 us go?  Times (HIP events, 200 rounds)
the full round, the rows-only round (K=0), the masks-only round (N=0), the aggregate launch alone
against a prebuilt seed table, and the seed-table launch alone."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

N, K, L = 128, 128, 16384
eng = MaskEngine(0)
g = np.random.Generator(np.random.PCG64(1))
rows = torch.from_numpy(g.integers(0, 2**31, size=(N, L), dtype=np.int64).astype(np.int32)).cuda()
seeds = torch.from_numpy(g.integers(0, 256, size=(K, 32), dtype=np.uint8)).cuda()
signs = torch.from_numpy(np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)).cuda()
out = torch.empty(L, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
e_seeds = seeds[:0]
e_signs = signs[:0]


def timed(name, fn, n=200):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    print(f"{name:34s} {e0.elapsed_time(e1) / n * 1e3:7.2f} us  plan={eng.last_plan()}", flush=True)


timed("full round", lambda: eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L))
timed("rows only (K=0)", lambda: eng.aggregate_unmask_dev(rows, e_seeds, e_signs, out, L=L))
timed("masks only (N=0)", lambda: eng.aggregate_unmask_dev(None, seeds, signs, out, L=L))
timed("rows 16 only (K=0)", lambda: eng.aggregate_unmask_dev(rows[:16], e_seeds, e_signs, out, L=L))
timed("masks 16 only (N=0)", lambda: eng.aggregate_unmask_dev(None, seeds[:16], signs[:16], out, L=L))
eng.seed_table_dev(seeds, signs)
timed("aggregate launch alone", lambda: eng.aggregate_dev(rows, K, out, L=L))
timed("seed table launch alone", lambda: eng.seed_table_dev(seeds, signs))
timed("torch empty-ish kernel (out.zero_)", lambda: out.zero_())
