"""Where do the drop-in server's reconstruction wall spikes come from?  (profiles/r05_sim_c5*.log:
iterations 1, 5 and 9 of the c5 agent run take 34-43 ms of wall for a 6.5-6.9 ms GPU unmask.)

Runs the ABIDES flamingo simulation (python -m flamingo_amd.abides arguments after `--`) with
gc.callbacks recording every garbage collection (generation, start, duration) and the server's
unmask calls (VectorStore.unmask) wrapped to record their windows, then prints per unmask window its
wall time and the collector time inside it, and the run's collector totals per generation.

    python tools/probes/sim_gc_probe.py [--freeze] -- -n 4096 --vector_len 1048576 -i 10 --dropout 0.01 ...

--threshold N: gc.set_threshold(N, 10, 10) (fewer young collections, so fewer full ones).
--freeze: gc.freeze() when the Kernel starts its event loop (after the agents are built), so the
          full collections no longer walk the simulation's setup objects.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--freeze", action="store_true")
    ap.add_argument("--threshold", type=int, default=0, help="gc.set_threshold(N, 10, 10) before the run")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    argv = [x for x in a.rest if x != "--"]

    collections = []          # (generation, t_start, seconds)
    start = {}

    def cb(phase, info):
        t = time.perf_counter()
        if phase == "start":
            start["t"] = t
        else:
            collections.append((info["generation"], start.get("t", t), t - start.get("t", t)))

    gc.callbacks.append(cb)
    if a.threshold:
        gc.set_threshold(a.threshold, 10, 10)

    from flamingo_amd import ingest
    from flamingo_amd.abides import kernel as K
    windows = []              # (t0, t1)
    orig_unmask = ingest.VectorStore.unmask

    def unmask(self, seeds, signs):
        t0 = time.perf_counter()
        out = orig_unmask(self, seeds, signs)
        windows.append((t0, time.perf_counter()))
        return out

    ingest.VectorStore.unmask = unmask
    if a.freeze:
        orig_runner = K.Kernel.runner

        def runner(self, *args, **kw):
            gc.collect()
            gc.freeze()
            print(f"[gc probe] froze {gc.get_freeze_count()} objects at the start of the event loop", flush=True)
            return orig_runner(self, *args, **kw)

        K.Kernel.runner = runner

    from flamingo_amd.abides.__main__ import main as sim_main
    t_run = time.perf_counter()
    sim_main(["-c", "flamingo"] + argv)
    t_run = time.perf_counter() - t_run

    rows = []
    for i, (t0, t1) in enumerate(windows):
        inside = [(g, s, d) for g, s, d in collections if s >= t0 and s + d <= t1 + 1e-9]
        rows.append({"call": i + 1, "wall_ms": round((t1 - t0) * 1e3, 3),
                     "gc_ms_inside": round(sum(d for _, _, d in inside) * 1e3, 3),
                     "gc_inside": [[g, round(d * 1e3, 3)] for g, _, d in inside]})
    per_gen = {}
    for g, _, d in collections:
        n, tot, mx = per_gen.get(g, (0, 0.0, 0.0))
        per_gen[g] = (n + 1, tot + d, max(mx, d))
    rec = {"freeze": a.freeze, "threshold": gc.get_threshold(), "run_s": round(t_run, 2), "unmask_calls": rows,
           "gc": {str(g): {"count": n, "total_ms": round(tot * 1e3, 1), "max_ms": round(mx * 1e3, 3)}
                  for g, (n, tot, mx) in sorted(per_gen.items())}}
    print("[gc probe] " + json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
