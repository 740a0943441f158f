#!/usr/bin/env python3
"""Workgroup timeline of one items_kernel launch (probe build with -DFLM_WG_TRACE, loaded through
FLM_LIB_PATH): per workgroup the s_memrealtime (100 MHz) stamps at start, after wave 0's seed loop,
and after the store, plus XCC / CU ids.  Prints the launch span, the start/end spread of the two
workgroup generations, and the mean workgroup residency over the span (slots = 2 per CU).

usage: FLM_LIB_PATH=.../libflamingo_hip.so wg_trace.py MODE [--subtiles S] [--min-items M]
  MODE = mask | full (the c4 launch shapes of tools/clock_probe.py) | c3 (N=K=1024, L=2^18)"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("mask", "full", "c3"))
    ap.add_argument("--subtiles", type=int, default=0)
    ap.add_argument("--min-items", type=int, default=1024)
    ap.add_argument("--settle-ms", type=float, default=200.0)
    a = ap.parse_args()
    N, K, L = 1024, 1024, (1 << 18) if a.mode == "c3" else (1 << 20)
    eng = MaskEngine(0)
    eng.set_tuning("subtiles", a.subtiles)
    eng.set_tuning("min_items", a.min_items)
    g = torch.Generator(device="cuda").manual_seed(1)
    rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g) \
        if a.mode in ("full", "c3") else None
    seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
    signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.seed_table_dev(seeds, signs)
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    while True:
        for _ in range(10):
            eng.aggregate_dev(rows, K, out, L=L)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        torch.cuda.synchronize()
        if e0.elapsed_time(e1) >= a.settle_ms:
            break
    res = []
    for rep in range(3):
        eng.aggregate_dev(rows, K, out, L=L)
        torch.cuda.synchronize()
        n = eng.last_plan()["items"]
        buf = np.zeros((n, 4), dtype=np.uint64)
        rc = eng.lib.flm_debug_wg_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int(n))
        assert rc == 0, rc
        t = buf[:, :3].astype(np.float64) * 10.0   # ns (100 MHz)
        t -= t[:, 0].min()
        hw, xcc = (buf[:, 3] & 0xFFFFFFFF).astype(np.int64), (buf[:, 3] >> 32).astype(np.int64)
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 0x7
        start, mid, end = t[:, 0], t[:, 1], t[:, 2]
        span = end.max()
        dur = end - start
        # generation: a workgroup whose start is after the earliest end began in the second wave
        gen2 = start > np.sort(end)[0] * 0.5
        slots = 2 * 256
        if os.environ.get("WG_TRACE_DUMP"):
            np.save(os.environ["WG_TRACE_DUMP"] + f".{rep}.npy", buf)
        busy = dur.sum() / (slots * span)
        r = {"mode": a.mode, "subtiles": a.subtiles, "items": int(n), "span_us": round(span / 1e3, 1),
             "wg_us_p0_p50_p100": [round(float(np.percentile(dur, q)) / 1e3, 1) for q in (0, 50, 100)],
             "combine_us_p50": round(float(np.median(end - mid)) / 1e3, 2),
             "gen1_start_us_max": round(float(start[~gen2].max()) / 1e3, 2) if (~gen2).any() else None,
             "gen1_end_us_p0_p50_p100": [round(float(np.percentile(end[~gen2], q)) / 1e3, 1) for q in (0, 50, 100)],
             "gen2_start_us_p0_p50_p100": [round(float(np.percentile(start[gen2], q)) / 1e3, 1) for q in (0, 50, 100)]
             if gen2.any() else None,
             "gen2_end_us_p0_p50_p100": [round(float(np.percentile(end[gen2], q)) / 1e3, 1) for q in (0, 50, 100)]
             if gen2.any() else None,
             "n_gen1": int((~gen2).sum()), "n_gen2": int(gen2.sum()),
             "residency": round(float(busy), 3),
             "end_us_by_xcc": [round(float(end[xcc == x].max()) / 1e3, 1) for x in range(8)],
             "wg_us_p50_by_xcc": [round(float(np.median(dur[xcc == x])) / 1e3, 1) for x in range(8)],
             "wgs_by_xcc": [int((xcc == x).sum()) for x in range(8)],
             "distinct_cu": int(len(set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))))}
        res.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
