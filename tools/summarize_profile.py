#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel trace/stats + separate PMC passes) into JSON.

usage: summarize_profile.py OUT.json TRACE_DIR [PMC_DIR ...]

Per kernel: dispatch count, average duration; per PMC counter: per-dispatch
average summed over XCD/SE dimensions.  HBM traffic follows
MI355X_MICROARCH.md "HBM": FETCH_SIZE reads half the bytes of a wide
coalesced stream on gfx950, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE
is exact for 16 B/lane stores (KB units).  Clock = GRBM_GUI_ACTIVE / 8 / duration.
"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_key(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def main():
    out, trace = sys.argv[1], sys.argv[2]
    pmcs = sys.argv[3:]
    res = {"kernels": {}, "counters": {}}
    stats = glob.glob(os.path.join(trace, "*kernel_stats.csv"))
    if stats:
        for r in csv.DictReader(open(stats[0])):
            res["kernels"][kernel_key(r["Name"])] = {
                "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                "max_ns": float(r["MaxNs"]), "pct": float(r["Percentage"])}
    durations = collections.defaultdict(list)
    for f in glob.glob(os.path.join(trace, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            durations[kernel_key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for d in pmcs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            dur = {}
            for r in csv.DictReader(open(f)):
                k = kernel_key(r["Kernel_Name"])
                per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[(k, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            agg = collections.defaultdict(lambda: collections.defaultdict(list))
            for (k, disp), cs in per.items():
                for c, v in cs.items():
                    agg[k][c].append(v)
                agg[k]["_duration_ns"].append(dur[(k, disp)])
            for k, cs in agg.items():
                dst = res["counters"].setdefault(k, {})
                for c, vs in cs.items():
                    if c == "_duration_ns":
                        dst.setdefault("pmc_pass_avg_ns", []).append(sum(vs) / len(vs))
                    else:
                        dst[c] = sum(vs) / len(vs)
    for k, cs in res["counters"].items():
        if "FETCH_SIZE" in cs:
            cs["hbm_read_bytes_corrected"] = 2.0 * cs["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in cs:
            cs["hbm_write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "GRBM_GUI_ACTIVE" in cs and cs.get("pmc_pass_avg_ns"):
            ns = cs["pmc_pass_avg_ns"][-1]
            cs["clock_ghz"] = cs["GRBM_GUI_ACTIVE"] / 8 / ns
        if "hbm_read_bytes_corrected" in cs and "hbm_write_bytes" in cs:
            cs["hbm_traffic_bytes"] = cs["hbm_read_bytes_corrected"] + cs["hbm_write_bytes"]
    for k, v in durations.items():
        res["kernels"].setdefault(k, {})["trace_avg_ns"] = sum(v) / len(v)
    res["workload"] = {"rows": 1024, "L": 1 << 20, "K": 1024,
                       "command": "python3 bench.py --profile --steps 20 --warmup 3"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1)[:4000])


if __name__ == "__main__":
    main()
