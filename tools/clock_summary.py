#!/usr/bin/env python3
"""Summarise tools/gpu_clock.sh: per mode (full / mask / rows), the items_kernel dispatches of the
timed part (the last R), averaged: duration, shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration),
VALU instructions, and cycles per VALU instruction per SIMD (256 CUs x 4 SIMDs).

usage: clock_summary.py OUT.json DIR_full DIR_mask DIR_rows [R]"""
import collections
import csv
import glob
import json
import os
import sys


def load(d, last):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "items_kernel" not in r["Kernel_Name"]:
                continue
            i = int(r["Dispatch_Id"])
            per[i][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[i] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(per)[-last:]
    avg = {c: sum(per[i][c] for i in ids) / len(ids) for c in per[ids[0]]}
    ns = sum(dur[i] for i in ids) / len(ids)
    avg["duration_ns"] = ns
    avg["dispatches"] = len(ids)
    if "GRBM_GUI_ACTIVE" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        avg["clock_ghz"] = cyc / ns
        if avg.get("SQ_INSTS_VALU"):
            avg["cycles_per_valu_inst_per_simd"] = cyc * 1024 / avg["SQ_INSTS_VALU"]
    return avg


def main():
    out, dirs = sys.argv[1], sys.argv[2:5]
    last = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    res = {m: load(d, last) for m, d in zip(("full", "mask", "rows"), dirs)}
    res["what"] = ("c4 launch shapes after a 200 ms clock settle (tools/clock_probe.py), one rocprofv3 --pmc pass "
                   "per mode: full = 1024 rows + 1024 self masks, mask = the same seeds without rows, rows = the "
                   "rows without seeds; L = 2^20")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
