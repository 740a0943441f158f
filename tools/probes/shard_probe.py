"""Decompose one rank's round at G ranks (weak scaling, 1024 clients/rank, L = 2^20) on one GPU:
rows over all L + K = 1024*G seeds over the rank's L/G window, against its parts (rows only,
masks only) and the G = 1 round.  Prints one JSON line per case (median kernel ms of both launches)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402


def timed(eng, rows, seeds, signs, out, L, lo, hi, reps, stream):
    for _ in range(2):
        eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L, mask_lo=lo, mask_hi=hi, stream=stream)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L, mask_lo=lo, mask_hi=hi, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), eng.last_plan()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=9)
    a = ap.parse_args()
    eng = MaskEngine(0)
    N, L = 1024, 1 << 20
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device=dev, generator=g)
    none = torch.empty((0, L), dtype=torch.int32, device=dev)
    out = torch.empty(L, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for G in [int(x) for x in a.G.split(",")]:
            K = 1024 * G
            seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device=dev, generator=g)
            signs = torch.full((K,), -1, dtype=torch.int8, device=dev)
            lo, hi = (G - 1) * (L // G), L                   # the last rank's window
            for case, r, k in (("fused", rows, K), ("rows_only", rows, 0), ("masks_only", none, K)):
                sd = seeds[:k] if k else None
                sg = signs[:k] if k else None
                ms, plan = timed(eng, r if r.shape[0] else None, sd, sg, out, L, lo, hi, a.reps, stream)
                words = k * (hi - lo)
                print(json.dumps({"G": G, "case": case, "ms": round(ms, 4), "K": k, "window": hi - lo,
                                  "mask_Gw/s": round(words / ms / 1e6, 1),
                                  "row_TB/s": round(4.0 * r.shape[0] * L / ms / 1e9, 3), "plan": plan}),
                      flush=True)


if __name__ == "__main__":
    main()
