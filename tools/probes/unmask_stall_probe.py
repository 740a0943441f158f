"""The server's reconstruction step outside the simulation: the s_ij recovery (MaskEngine.ec_combine_wire,
host in/out, D = 960 pairs x T = 20 shares) and then VectorStore.unmask over a c5-shaped store
(4055 rows of L = 2^20 already summed, K = 5015 seeds), as SA_ServiceAgent.reconstruction does --
after an idle gap of `idle` seconds, as the simulation leaves the GPU idle between its steps.
Prints per trial the unmask wall time and its device time (flm_store_unmask_ms), to see whether
the occasional 15-35 ms walls of the agent run (profiles/r05_sim_c5*.log) follow idle gaps.

    python tools/probes/unmask_stall_probe.py [trials]
"""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import numpy as np

from flamingo_amd import MaskEngine
from flamingo_amd import crypto as C
from flamingo_amd.ingest import VectorStore


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    L, N, U, K, D, T = 1 << 20, 4096, 4055, 5015, 960, 20
    eng = MaskEngine(0)
    rng = random.Random(1)
    base = [C.mul(rng.randrange(1, C.N)) for _ in range(32)]
    shares = np.stack([C.points_to_wire([base[(j * 7 + i) % 32] for i in range(D)]) for j in range(T)])
    c1 = C.points_to_wire([base[(i * 3) % 32] for i in range(D)])
    lams = C.scalars_to_wire([rng.randrange(1, C.N) for _ in range(T)])
    st = VectorStore(eng, L, N)
    row = np.ones(L, np.uint32)
    for i in range(U):
        st.add(i, row)
    st.partial_sum()
    g = np.random.Generator(np.random.PCG64(5))
    seeds = g.integers(0, 256, (K, 32), dtype=np.uint8)
    signs = np.where(g.integers(0, 2, K) == 1, 1, -1).astype(np.int8)
    out = {}
    for idle in (0.0, 0.5, 2.0):
        for ec in (False, True):
            rows = []
            for _ in range(trials):
                time.sleep(idle)
                t_ec = 0.0
                if ec:
                    t0 = time.perf_counter()
                    eng.ec_combine_wire(c1, shares, lams)
                    t_ec = (time.perf_counter() - t0) * 1e3
                t0 = time.perf_counter()
                st.unmask(seeds, signs)
                wall = (time.perf_counter() - t0) * 1e3
                rows.append([round(t_ec, 2), round(wall, 2), round(st.unmask_ms(), 2)])
            out[f"idle{idle}_ec{int(ec)}"] = rows
            print(f"idle {idle} s, EC before: {ec}:  [ec ms, unmask wall ms, unmask GPU ms] {rows}", flush=True)
    # a new seed count K every call, as every simulation iteration has (|U| + D moves): a new launch
    # plan (its work-item table allocated and uploaded) inside the unmask
    for idle in (0.0, 0.5):
        rows = []
        for t in range(3 * trials):
            time.sleep(idle)
            Kt = K + 1 + t + int(idle * 100)
            eng.ec_combine_wire(c1, shares, lams)
            t0 = time.perf_counter()
            st.unmask(seeds[:Kt] if Kt <= K else np.concatenate([seeds, seeds[:Kt - K]]),
                      signs[:Kt] if Kt <= K else np.concatenate([signs, signs[:Kt - K]]))
            wall = (time.perf_counter() - t0) * 1e3
            rows.append([Kt, round(wall, 2), round(st.unmask_ms(), 2)])
        out[f"new_K_idle{idle}"] = rows
        print(f"a new K every call, idle {idle} s, EC before:  [K, unmask wall ms, unmask GPU ms] {rows}", flush=True)
    # the simulation's client traffic before each reconstruction: every client's y_i made on the
    # GPU and copied into a fresh pageable 4 MiB array (MaskEngine.client_mask, as sendVectors
    # does), handed to the store and dropped
    seg = np.array([0, 23], np.int64)
    cseeds = g.integers(0, 256, (23, 32), dtype=np.uint8)
    csigns = np.ones(23, np.int8)
    rows = []
    for it in range(trials):
        t0 = time.perf_counter()
        for i in range(U):
            y = eng.client_mask(seg, cseeds, csigns, L)[0]
            st.add(i, y)
            del y
        t_cl = (time.perf_counter() - t0) * 1e3 / U
        st.partial_sum()
        eng.ec_combine_wire(c1, shares, lams)
        t0 = time.perf_counter()
        st.unmask(seeds, signs)
        wall = (time.perf_counter() - t0) * 1e3
        rows.append([round(t_cl, 3), round(wall, 2), round(st.unmask_ms(), 2)])
        st.reset()
    out["clients_then_ec"] = rows
    print(f"after {U} client_mask + add:  [ms per client, unmask wall ms, unmask GPU ms] {rows}", flush=True)
    # the same with the VECTOR bodies kept until the reconstruction (the simulation's messages hold
    # them) and then released all at once, right before the server's GPU work
    rows = []
    for it in range(trials):
        t0 = time.perf_counter()
        held = []
        for i in range(U):
            y = eng.client_mask(seg, cseeds, csigns, L)[0]
            st.add(i, y)
            held.append(y)
        t_cl = (time.perf_counter() - t0) * 1e3 / U
        st.partial_sum()
        t0 = time.perf_counter()
        del held, y
        t_free = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        eng.ec_combine_wire(c1, shares, lams)
        t_ec = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        st.unmask(seeds, signs)
        wall = (time.perf_counter() - t0) * 1e3
        rows.append([round(t_cl, 3), round(t_free, 2), round(t_ec, 2), round(wall, 2), round(st.unmask_ms(), 2)])
        st.reset()
    out["clients_held_then_freed"] = rows
    print(f"bodies held, freed before the EC:  [ms per client, free ms, ec ms, unmask wall ms, unmask GPU ms] {rows}",
          flush=True)
    st.close()
    eng.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
