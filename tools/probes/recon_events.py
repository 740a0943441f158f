"""c5 reconstruction (pair queue): HIP-event timeline of one run without a profiler attached --
pass 1 (Shamir + self-mask unmask on the non-EC CUs), the EC combine and the side pair-unit pass
on the EC CUs, and the final pair pass -- to see which stream bounds the round.
Env: EC_CUS (24), EC_TERMS (2), MIN_ITEMS (4096).  Prints one JSON line per run (ms from start)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import flamingo_amd.params as P  # noqa: E402
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.reconstruct import ServerReconstruction  # noqa: E402
from flamingo_amd.synthetic import recovery_round  # noqa: E402

N, L = 4096, 1 << 20
eng = MaskEngine(0)
dev = torch.device("cuda:0")
m = np.frombuffer(b"".join(P.bench_seed("c5", i) for i in range(N)), np.uint8).reshape(N, 32)
nbrs = P.neighbor_graph(b"\x00" * 32, 1, N, 1, encrypt=eng.chacha20_encrypt)
off = np.sort(np.random.Generator(np.random.PCG64(1)).choice(N, N // 100, replace=False))
on = np.setdiff1d(np.arange(N), off)
R = recovery_round(eng, m, nbrs, on, off, T=20, committee=60, seed=1)
rows = torch.empty((N, L), dtype=torch.int32, device=dev)
eng.client_mask_dev(R["seg"], torch.from_numpy(R["client_seeds"]).to(dev), R["client_signs"], rows, L)
r_on = rows[torch.from_numpy(on).to(dev)].contiguous()
del rows
t = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares", "c1", "pair_shares", "pair_signs")}
out = torch.empty(L, dtype=torch.int32, device=dev)
main = torch.cuda.Stream()
rec = ServerReconstruction(eng, pass1_min_items=int(os.environ.get("MIN_ITEMS", "4096")),
                           ec_cus=int(os.environ.get("EC_CUS", "24")), cu_pick=os.environ.get("EC_PICK", "first"), pair_queue=True,
                           ec_terms=int(os.environ.get("EC_TERMS", "2")), ec_spread=int(os.environ.get("EC_SPREAD", "0")))
args = (r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out)

# instrument: events recorded on the side / part streams around the pieces of _run_queue
marks = {}
orig_ec, orig_pu, orig_agg, orig_flag = rec._ec_combine, rec.side_eng.pair_units_dev, eng.aggregate_unmask_dev, \
    eng.flag_set_dev


def ev(name, stream):
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    marks[name] = e


def ec_combine(*a, **k):
    r = orig_ec(*a, **k)
    ev("ec_done", rec.side)
    return r


def pair_units(*a, **k):
    final = k.get("final", False)
    r = orig_pu(*a, **k)
    ev("final_done" if final else "side_pairs_done", k["stream"])
    return r


def agg(*a, **k):
    ev("pass1_start", k["stream"])
    r = orig_agg(*a, **k)
    ev("pass1_done", k["stream"])
    return r


rec._ec_combine = ec_combine
rec.side_eng.pair_units_dev = pair_units
eng.aggregate_unmask_dev = agg
with torch.cuda.stream(main):
    for it in range(6):
        torch.cuda.synchronize()
        ev("start", main)
        rec.run(*args, stream=main)
        torch.cuda.synchronize()
        ok = bool(torch.all(out == len(on)).item())
        t0 = marks["start"]
        print(json.dumps({k: round(t0.elapsed_time(v), 3) for k, v in marks.items() if k != "start"} | {"ok": ok}),
              flush=True)
