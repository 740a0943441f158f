#!/usr/bin/env python3
"""Same ChaCha work (2^30 mask words), two launch plans of items_kernel, timed back to back:

  agg      flm_aggregate_dev mask-only: K=1024 seeds over L=2^20 slots (the c4 round's plan:
           1024 items of one 1024-slot tile, 16 waves splitting the seeds, LDS combine)
  client   flm_client_mask_dev: 16 rows x 64 seeds over 2^20 slots each (client-masking plan:
           16 sub-tiles per workgroup, each wave its own 1024 slots with all 64 of its row's seeds)
  fused    the c4 round itself (1024 rows + 1024 seeds)

Prints ms and G words/s per case (median of --reps launches); --case runs just one (for PMC passes)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--case", default="all")
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--subtiles", type=int, default=0)
ap.add_argument("--min-items", type=int, default=1024)
args = ap.parse_args()
torch.cuda.set_device(0)
eng = MaskEngine(0)
eng.set_tuning("variant", args.variant)
eng.set_tuning("subtiles", args.subtiles)
eng.set_tuning("min_items", args.min_items)
L = 1 << 20
g = torch.Generator(device="cuda")
g.manual_seed(5)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
K = 1024
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
signs = -torch.ones(K, dtype=torch.int8, device="cuda")
out = torch.empty(L, dtype=torch.int32, device="cuda")
rows = None
cases = ["agg", "client", "fused"] if args.case == "all" else args.case.split(",")
if "fused" in cases:
    rows = torch.randint(-2**31, 2**31 - 1, (1024, L), dtype=torch.int32, device="cuda", generator=g)
cm_out = torch.empty((16, L), dtype=torch.int32, device="cuda")
seg = np.arange(0, K + 1, 64, dtype=np.int64)
signs_h = -np.ones(K, np.int8)


def run(case):
    if case == "agg":
        eng.aggregate_dev(None, K, out, L=L, stream=s)
    elif case == "fused":
        eng.aggregate_dev(rows, K, out, L=L, stream=s)
    else:
        eng.client_mask_dev(seg, seeds, signs_h, cm_out, L, stream=s)


res = []
for rnd in range(2):
    for case in cases:
        if case != "client":
            eng.seed_table_dev(seeds, signs, stream=s)
        for _ in range(5):
            run(case)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
        ev[0].record(s)
        for i in range(args.reps):
            run(case)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        ms = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(args.reps)]))
        words = float(K) * L
        res.append({"round": rnd, "case": case, "ms": round(ms, 4), "Gwords/s": round(words / ms / 1e6, 1),
                    "plan": eng.last_plan()})
for r in res:
    print(json.dumps(r), flush=True)
