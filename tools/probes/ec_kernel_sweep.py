"""A/B of the cooperative scalar-multiplication kernels over the combine's batch sizes: the per-lane
Montgomery field (ec_coop 1, ec_mul_coop_kernel) against the 16-lane row field (ec_coop 2,
ec_mul_row_kernel), and the per-lane kernel (ec_coop 0) for reference.  T = 20 Lagrange scalars,
D dropout pairs; the two cooperative kernels alternate within each D (interleaved repetitions) so
clock drift hits both.  Every result is checked against OpenSSL on a sample of pairs.
Usage: python tools/probes/ec_kernel_sweep.py [D ...]"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from flamingo_amd import MaskEngine
from flamingo_amd import crypto as C
from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero

Ds = [int(x) for x in sys.argv[1:]] or [4, 16, 60, 120, 240, 481, 962]
T = 20
rng = random.Random(1)
base = [C.mul(rng.randrange(1, C.N)) for _ in range(64)]
lams = lagrange_at_zero(sorted(rng.sample(range(1, 61), T)))
dev = torch.device("cuda:0")
eng = MaskEngine(0)
s = torch.cuda.Stream()
lam_t = torch.from_numpy(C.scalars_to_wire(lams)).to(dev)


def run(coop, D, c1_t, sh_t, seeds, pts, flags, reps):
    eng.set_tuning("ec_coop", coop)
    with torch.cuda.stream(s):
        eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds, flags, points_out=pts, stream=s)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(s)
        for _ in range(reps):
            eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds, flags, points_out=pts, stream=s)
        ev1.record(s)
        s.synchronize()
    assert int(flags.abs().sum()) == 0
    return ev0.elapsed_time(ev1) / reps


print("D  T  products  per_lane_ms  coop_ms  row_ms  row/coop", flush=True)
out = []
for D in Ds:
    shares = np.stack([C.points_to_wire([base[(j * 7 + i) % 64] for i in range(D)]) for j in range(T)])
    c1 = C.points_to_wire([base[(i * 3) % 64] for i in range(D)])
    c1_t, sh_t = torch.from_numpy(c1).to(dev), torch.from_numpy(shares).to(dev)
    seeds = torch.empty((D, 32), dtype=torch.uint8, device=dev)
    pts = torch.empty((D, 64), dtype=torch.uint8, device=dev)
    flags = torch.empty(D, dtype=torch.int32, device=dev)
    want = None
    res = {0: [], 1: [], 2: []}
    for rep in range(4):
        for coop in ((1, 2) if rep % 2 == 0 else (2, 1)) + ((0,) if rep == 0 else ()):
            res[coop].append(run(coop, D, c1_t, sh_t, seeds, pts, flags, 5))
            got = pts.cpu().numpy().copy()
            if want is None:
                want = got
                for i in range(0, D, max(1, D // 4)):     # OpenSSL check on a sample of pairs
                    acc = None
                    for j in range(T):
                        acc = C.add(acc, C.mul(lams[j], base[(j * 7 + i) % 64]))
                    assert C.points_from_wire(got[i:i + 1])[0] == C.add(C.points_from_wire(c1[i:i + 1])[0], C.neg(acc))
            assert np.array_equal(got, want), (D, coop)          # every kernel the same points, bit for bit
    lane, coop, row = (float(np.median(res[k])) for k in (0, 1, 2))
    print(f"{D} {T} {D * T} {lane:.4f} {coop:.4f} {row:.4f} {row / coop:.3f}", flush=True)
    out.append({"D": D, "T": T, "per_lane_ms": round(lane, 4), "coop_ms": round(coop, 4), "row_ms": round(row, 4)})
print(json.dumps({"sweep": out}))
eng.close()
