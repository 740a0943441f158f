"""Where the row kernel's time goes: one combine (T = 20) timed with Lagrange scalars and with
doubling-only scalars (every lambda = 2^255: ~258 doublings, no additions), for the per-lane
cooperative kernel (ec_coop 1) and the row kernel (ec_coop 2), at a lone-wave batch (D = 4) and at
one G = 8 rank's share (D = 120).  Doubling time = pow2 time / 258 (minus the shared ec_finish),
addition time = (Lagrange - pow2) / additions.  Usage: python tools/probes/ec_row_split.py"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from flamingo_amd import MaskEngine
from flamingo_amd import crypto as C
from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero

T = 20
rng = random.Random(1)
base = [C.mul(rng.randrange(1, C.N)) for _ in range(64)]
lag = lagrange_at_zero(sorted(rng.sample(range(1, 61), T)))
dev = torch.device("cuda:0")
eng = MaskEngine(0)
s = torch.cuda.Stream()


def naf_adds(k):
    """Non-zero digits of k's width-5 NAF (the additions of one scalar multiplication)."""
    n = 0
    while k:
        if k & 1:
            d = k & 31
            d = d - 32 if d >= 16 else d
            k -= d
            n += 1
        k >>= 1
    return n


def timed(coop, D, lams, reps=10):
    shares = np.stack([C.points_to_wire([base[(j * 7 + i) % 64] for i in range(D)]) for j in range(T)])
    c1_t = torch.from_numpy(C.points_to_wire([base[(i * 3) % 64] for i in range(D)])).to(dev)
    sh_t = torch.from_numpy(shares).to(dev)
    lam_t = torch.from_numpy(C.scalars_to_wire(lams)).to(dev)
    seeds = torch.empty((D, 32), dtype=torch.uint8, device=dev)
    flags = torch.empty(D, dtype=torch.int32, device=dev)
    eng.set_tuning("ec_coop", coop)
    with torch.cuda.stream(s):
        for _ in range(3):
            eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds, flags, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds, flags, stream=s)
        e1.record(s)
        s.synchronize()
    return e0.elapsed_time(e1) / reps


adds = max(naf_adds(x) for x in lag)
out = []
for D in (4, 120):
    for coop in (1, 2):
        tl = timed(coop, D, lag)
        tp = timed(coop, D, [1 << 255] * T)
        r = {"D": D, "kernel": {1: "coop (per-lane field)", 2: "row"}[coop], "lagrange_ms": round(tl, 4),
             "doublings_only_ms": round(tp, 4), "us_per_doubling_upper": round(tp / 258 * 1e3, 3),
             "us_per_addition": round((tl - tp) / adds * 1e3, 3), "additions": adds}
        print(json.dumps(r), flush=True)
        out.append(r)
eng.close()
