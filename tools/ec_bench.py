"""Time the P-256 seed-recovery kernels on the GPU vs OpenSSL on the host.

D dropped pairs x T committee shares (c5: D ~ 1000, T = 20).  Inputs are
random points (scalar multiples of G) made by OpenSSL; the GPU result is
checked against OpenSSL's sum for a few pairs."""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from flamingo_amd import MaskEngine
from flamingo_amd import crypto as C

ap = argparse.ArgumentParser()
ap.add_argument("--D", type=int, default=1000)
ap.add_argument("--T", type=int, default=20)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--cpu-sample", type=int, default=100, help="scalar mults timed on the host")
ap.add_argument("--threads", type=int, default=64)
ap.add_argument("--scalars", choices=["random", "lagrange", "pow2"], default="random",
                help="pow2: every lambda = 2^255 (one wNAF digit: ~258 doublings and no additions, to split the chain)")
ap.add_argument("--coop", type=int, default=0, help="flm_set_tuning ec_coop (four waves per 64 products)")
ap.add_argument("--terms", type=int, default=1, help="flm_set_tuning ec_terms (Straus: combine terms per lane)")
ap.add_argument("--spread", type=int, default=0, help="flm_set_tuning ec_spread (KiB of LDS per EC workgroup)")
ap.add_argument("--pick", default="first", choices=("first", "stride", "xcd_stride", "xcd"), help="which CUs --cus selects (pick_cus)")
ap.add_argument("--cus", type=int, default=0, help="run on a CU-masked stream of this many CUs ('first' pick)")
a = ap.parse_args()

rng = random.Random(1)
base = [C.mul(rng.randrange(1, C.N)) for _ in range(64)]
shares = np.stack([C.points_to_wire([base[(j * 7 + i) % 64] for i in range(a.D)]) for j in range(a.T)])
if a.scalars == "lagrange":
    from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero
    lams = lagrange_at_zero(sorted(rng.sample(range(1, 61), a.T)))
elif a.scalars == "pow2":
    lams = [1 << 255] * a.T
else:
    lams = [rng.randrange(1, C.N) for _ in range(a.T)]
c1 = C.points_to_wire([base[(i * 3) % 64] for i in range(a.D)])
dev = torch.device("cuda:0")
eng = MaskEngine(0)
eng.set_tuning("ec_threads", a.threads)
eng.set_tuning("ec_coop", a.coop)
eng.set_tuning("ec_terms", a.terms)
eng.set_tuning("ec_spread", a.spread)
c1_t = torch.from_numpy(c1).to(dev)
sh_t = torch.from_numpy(shares).to(dev)
lam_t = torch.from_numpy(C.scalars_to_wire(lams)).to(dev)
seeds = torch.empty((a.D, 32), dtype=torch.uint8, device=dev)
pts = torch.empty((a.D, 64), dtype=torch.uint8, device=dev)
flags = torch.empty(a.D, dtype=torch.int32, device=dev)
if a.cus:
    from flamingo_amd.reconstruct import pick_cus
    s = eng.cu_stream(pick_cus(eng.cu_count(), a.cus, a.pick))
else:
    s = torch.cuda.Stream()
with torch.cuda.stream(s):
    eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds, flags, points_out=pts, stream=s)
    s.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(s)
    for _ in range(a.reps):
        eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds, flags, points_out=pts, stream=s)
    ev1.record(s)
    s.synchronize()
gpu_ms = ev0.elapsed_time(ev1) / a.reps
assert int(flags.abs().sum()) == 0
got = C.points_from_wire(pts.cpu().numpy())
for i in range(0, a.D, max(1, a.D // 5)):
    acc = None
    for j in range(a.T):
        acc = C.add(acc, C.mul(lams[j], base[(j * 7 + i) % 64]))
    want = C.add(C.points_from_wire(c1[i:i + 1])[0], C.neg(acc))
    assert got[i] == want, i
t = time.perf_counter()
for i in range(a.cpu_sample):
    C.mul(lams[i % a.T], base[i % 64])
cpu_per_mul = (time.perf_counter() - t) / a.cpu_sample
print(json.dumps({"lib": os.environ.get("FLM_LIB_PATH", "default"), "coop": a.coop, "terms": a.terms, "cus": a.cus, "threads": a.threads, "D": a.D, "T": a.T, "scalars": a.scalars, "lambda_hex": [hex(x)[:12] for x in lams[:4]], "gpu_ms": round(gpu_ms, 4),
                  "gpu_scalar_mults_per_s": round(a.D * a.T / gpu_ms * 1e3),
                  "cpu_openssl_ms_est": round(cpu_per_mul * a.D * a.T * 1e3, 1),
                  "cpu_openssl_us_per_mul": round(cpu_per_mul * 1e6, 1), "cpu_cores": 1}))
