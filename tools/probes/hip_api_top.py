"""Summarise a rocprofv3 --hip-trace CSV: per HIP API function (count, total, max ms) and the N
longest calls with their start time relative to the first call and the calls just before them.

    python tools/probes/hip_api_top.py DIR/run_hip_api_trace.csv [N]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top_n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], int(r.get("Thread_Id", 0))))
    rows.sort()
    t0 = rows[0][0]
    agg = defaultdict(lambda: [0, 0, 0])
    for s, e, fn, _ in rows:
        a = agg[fn]
        a[0] += 1
        a[1] += e - s
        a[2] = max(a[2], e - s)
    print(f"{len(rows)} HIP API calls over {(rows[-1][1] - t0) / 1e9:.2f} s")
    print(f"{'function':40s} {'count':>8s} {'total ms':>10s} {'max ms':>9s}")
    for fn, (n, tot, mx) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        print(f"{fn:40s} {n:8d} {tot / 1e6:10.3f} {mx / 1e6:9.3f}")
    print(f"\nthe {top_n} longest calls (t = start since the first call, s):")
    idx = sorted(range(len(rows)), key=lambda i: rows[i][0] - rows[i][1])[:top_n]
    for i in sorted(idx):
        s, e, fn, tid = rows[i]
        before = " < ".join(r[2] for r in rows[max(0, i - 3):i][::-1])
        print(f"t={(s - t0) / 1e9:9.4f}  {(e - s) / 1e6:9.3f} ms  {fn:28s} tid {tid}  after: {before}")


if __name__ == "__main__":
    main()
