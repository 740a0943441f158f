#!/usr/bin/env python3
"""A/B the items_kernel variants in one process (interleaved rounds, same device).

Workloads (all N=1024 rows x L=2^20 slots, device resident, random rows):
  full     K=1024 self-mask seeds over all slots (G=1 round)
  pairs    K=204 dropout-pair seeds (HBM-bound half)
  shard8   K=8192 seeds over a 1/8 slot window (one rank of the 8-GPU weak-scaled round)
  mask     K=1024 seeds, no rows (the same-run ChaCha ceiling launch)
  client   client masking, 1024 clients x 24 seeds over L (flm_client_mask_dev; variant and
           subtiles do not apply: one line per round)
Prints median/min kernel ms and GB/s per (workload, variant, subtiles), and
checks every variant returns identical bits.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

VARIANTS = {"auto": -1, "coalesced": 0, "block": 1, "merged": 2, "merged_w8": 3, "merged_ru4": 4, "merged_nt": 5,
            "merged_ru4_nt": 6, "merged_spread": 7, "block_spread": 8}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workloads", default="full,pairs,shard8")
    ap.add_argument("--variants", default="coalesced,block,merged,merged_w8")
    ap.add_argument("--subtiles", default="1,4")
    ap.add_argument("--pairing", default="0")
    ap.add_argument("--min-items", default="1024")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed back-to-back launches first: MI355X ramps its clock over ~100 ms of load")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    eng = MaskEngine(0)
    N, L = 1024, 1 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g)
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    res = []
    for wl in args.workloads.split(","):
        if wl == "client":
            client_round(eng, g, s, L, args)
            continue
        K = 1024 if wl.startswith("strong") else {"full": 1024, "pairs": 204, "shard8": 8192, "rows": 0, "c3": 1024,
                                                   "mask": 1024}[wl]
        Lw = (1 << 18) if wl == "c3" else L        # c3: N=1024, L=2^18 (BASELINE configs[2])
        lo, hi = (0, Lw) if wl != "shard8" else (3 * L // 8, 4 * L // 8)
        rows_w = None if wl == "mask" else rows
        if wl.startswith("strong"):                # one rank of the strong-scaled c4 round: N/G rows, last shard
            G = int(wl[6:])
            rows_w = rows[: N // G]
            lo, hi = (G - 1) * L // G, L
        seeds = torch.randint(0, 256, (max(K, 1), 32), dtype=torch.uint8, device="cuda", generator=g)[:K]
        signs = (torch.randint(0, 2, (max(K, 1),), device="cuda", generator=g) * 2 - 1).to(torch.int8)[:K]
        eng.seed_table_dev(seeds, signs, stream=s)
        times, plans = {}, {}
        ref = None
        if args.settle_ms > 0:
            t_end, e0 = 0.0, torch.cuda.Event(enable_timing=True)
            e0.record(s)
            while t_end < args.settle_ms:
                for _ in range(10):
                    eng.aggregate_dev(rows_w, K, out, L=Lw, mask_lo=lo, mask_hi=hi, stream=s)
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(s)
                torch.cuda.synchronize()
                t_end = e0.elapsed_time(e1)
        combos = [(v, st, pa, mi) for v in args.variants.split(",") for st in map(int, args.subtiles.split(","))
                  for pa in map(int, args.pairing.split(",")) for mi in map(int, args.min_items.split(","))]
        for rnd in range(args.rounds):
            for v, st, pa, mi in combos:
                eng.set_tuning("variant", VARIANTS[v])
                eng.set_tuning("subtiles", st)
                eng.set_tuning("pairing", pa)
                eng.set_tuning("min_items", mi)
                eng.aggregate_dev(rows_w, K, out, L=Lw, mask_lo=lo, mask_hi=hi, stream=s)  # warm / plan
                e = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
                e[0].record(s)
                for r in range(args.reps):
                    eng.aggregate_dev(rows_w, K, out, L=Lw, mask_lo=lo, mask_hi=hi, stream=s)
                    e[r + 1].record(s)
                torch.cuda.synchronize()
                ms = [e[i].elapsed_time(e[i + 1]) for i in range(args.reps)]
                times.setdefault((v, st, pa, mi), []).extend(ms)
                o = out.cpu().numpy()
                if ref is None:
                    ref = o.copy()
                elif not np.array_equal(ref, o):
                    print(f"MISMATCH {wl} {v} st={st} pairing={pa} min_items={mi}", flush=True)
                plans[(v, st, pa, mi)] = eng.last_plan()
        for (v, st, pa, mi), ms in times.items():
            med, mn = float(np.median(ms)), float(np.min(ms))
            nrw = N // int(wl[6:]) if wl.startswith("strong") else (0 if wl == "mask" else N)
            gbs = (4.0 * nrw * Lw + 4.0 * Lw) / (med * 1e-3) / 1e9
            r = {"workload": wl, "variant": v, "subtiles": st, "pairing": pa, "min_items": mi,
                 "items": plans[(v, st, pa, mi)]["items"], "median_ms": round(med, 4), "min_ms": round(mn, 4),
                 "GB/s": round(gbs, 1), "mask_gwords_per_s": round(K * (hi - lo) / (med * 1e-3) / 1e9, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    eng.close()


def client_round(eng, g, s, L, args, N=1024, per=24):
    """flm_client_mask_dev over N clients x `per` seeds (all-ones inputs): the launch shape of
    bench.py's client_masks (S=16 sub-tiles per workgroup, each wave its own 1024 slots)."""
    K = N * per
    seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
    signs = np.where(np.arange(K) % 3 == 0, -1, 1).astype(np.int8)
    seg = np.arange(0, K + 1, per, dtype=np.int64)
    out = torch.empty((N, L), dtype=torch.int32, device="cuda")
    for _ in range(3):
        eng.client_mask_dev(seg, seeds, signs, out, L=L, stream=s)
    ms = []
    for _ in range(args.rounds):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(args.reps + 1)]
        e[0].record(s)
        for r in range(args.reps):
            eng.client_mask_dev(seg, seeds, signs, out, L=L, stream=s)
            e[r + 1].record(s)
        torch.cuda.synchronize()
        ms += [e[i].elapsed_time(e[i + 1]) for i in range(args.reps)]
    med = float(np.median(ms))
    print(json.dumps({"workload": "client", "clients": N, "seeds_per_client": per, "items": eng.last_plan()["items"],
                      "median_ms": round(med, 4), "min_ms": round(min(ms), 4),
                      "mask_gwords_per_s": round(K * L / (med * 1e-3) / 1e9, 1)}), flush=True)
    del out


if __name__ == "__main__":
    main()
