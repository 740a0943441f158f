"""pairs-only variant (K = D dropout-pair seeds over 1024 rows x 2^20): bench.py's measurement vs
tools/ab/ab_items.py's (per-launch events, median), same process, same rows."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd import params as P  # noqa: E402

eng = MaskEngine(0)
N, L = 1024, 1 << 20
g = torch.Generator(device="cuda")
g.manual_seed(1)
rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g)
m = np.zeros((N, 32), np.uint8)
nbrs = P.neighbor_graph(b"\x00" * 32, 1, N, 1, encrypt=eng.chacha20_encrypt)
s = torch.cuda.Stream()
for rep in range(3):
    r = bench.variant_pairs_only(eng, torch, rows, m, nbrs, np.arange(N), L, s, P)["pairs_only"]
    print("bench loop:", r["kernel_ms"], "ms", flush=True)
    K = r["seeds_K"]
    seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
    signs = (torch.randint(0, 2, (K,), device="cuda", generator=g) * 2 - 1).to(torch.int8)
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.seed_table_dev(seeds, signs, stream=s)
    for _ in range(3):
        eng.aggregate_dev(rows, K, out, L=L, stream=s)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    ev[0].record(s)
    for i in range(20):
        eng.aggregate_dev(rows, K, out, L=L, stream=s)
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(20)]
    print("per-launch: median", round(float(np.median(ms)), 4), "mean", round(float(np.mean(ms)), 4),
          "min", round(min(ms), 4), "plan", eng.last_plan(), flush=True)
