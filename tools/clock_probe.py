"""One launch shape of the c4 round, repeated after a clock settle, for PMC passes.

usage: clock_probe.py MODE [--reps R] [--settle-ms T]
  MODE = full  (1024 rows + 1024 self masks over L = 2^20: the bench's c4 kernel)
       | mask  (the same 1024 seeds, no rows: the same-run ChaCha ceiling launch)
       | rows  (1024 rows, no seeds: the HBM half)
       | client (flm_client_mask_dev: 1024 clients x 24 seeds over L, all-ones inputs)
  --subtiles S  the aggregate planner's sub-tiles per workgroup (0 = auto)

Run each mode in its own process under rocprofv3 --pmc (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES,
SQ_INSTS_VALU, ...) to compare the shader clock and cycles per VALU instruction of the c4
launch against the mask-only launch (tools/clock_summary.py).  Prints one JSON line with the
HIP-event times of the timed launches."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flamingo_amd import MaskEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("full", "mask", "rows", "client"))
    ap.add_argument("--subtiles", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=200.0)
    a = ap.parse_args()
    N, K, L = 1024, 1024, 1 << 20
    eng = MaskEngine(0)
    eng.set_tuning("subtiles", a.subtiles)
    g = torch.Generator(device="cuda").manual_seed(1)
    if a.mode == "client":
        per = 24
        seeds = torch.randint(0, 256, (N * per, 32), dtype=torch.uint8, device="cuda", generator=g)
        signs = np.where(np.arange(N * per) % 3 == 0, -1, 1).astype(np.int8)
        seg = np.arange(0, N * per + 1, per, dtype=np.int64)
        out2 = torch.empty((N, L), dtype=torch.int32, device="cuda")
        run = lambda: eng.client_mask_dev(seg, seeds, signs, out2, L=L)  # noqa: E731
        K = N * per
    else:
        run = None
    rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g) \
        if a.mode not in ("mask", "client") else None
    k = 0 if a.mode == "rows" else K
    s = torch.cuda.current_stream()
    if run is None:
        seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
        signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
        out = torch.empty(L, dtype=torch.int32, device="cuda")
        eng.seed_table_dev(seeds[:k], signs[:k])
        run = lambda: eng.aggregate_dev(rows, k, out, L=L)  # noqa: E731
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record(s)
    while True:
        for _ in range(10):
            run()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(s)
        torch.cuda.synchronize()
        if e0.elapsed_time(e1) >= a.settle_ms:
            break
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
    ev[0].record(s)
    for i in range(a.reps):
        run()
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    t = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.reps)]
    print(json.dumps({"mode": a.mode, "subtiles": a.subtiles, "rows": 0 if rows is None else N, "K": k, "L": L,
                      "plan": eng.last_plan(), "gwords_per_s": round(k * L / (float(np.median(t)) * 1e-3) / 1e9, 1),
                      "median_ms": round(float(np.median(t)), 4), "min_ms": round(min(t), 4),
                      "max_ms": round(max(t), 4)}), flush=True)


if __name__ == "__main__":
    main()
