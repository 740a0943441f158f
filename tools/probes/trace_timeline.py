#!/usr/bin/env python3
"""Print a rocprofv3 kernel trace (run_kernel_trace.csv) as a timeline relative to the start of the
N-th launch of a kernel whose name contains ANCHOR (default: the last ec_mul_kernel launch),
up to LIMIT rows.  usage: trace_timeline.py TRACE_CSV [ANCHOR] [LIMIT]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "ec_mul_kernel"
limit = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = starts[-1] if starts else 0
t0 = int(rows[i0]["Start_Timestamp"])
lo = max(0, i0 - 5)
print(f"# start_ms end_ms dur_ms kernel (t=0: the last {anchor} launch)")
for r in rows[lo:lo + limit]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f}  {r['Kernel_Name'][:90]}")
