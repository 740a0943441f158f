"""One rank of the 8-GPU c5 reconstruction from the report partial, on one GPU: its S shard
(L/8 slots), all M self-mask seeds from Shamir shares and its ceil(D/8) dropout pairs from
threshold-ElGamal shares (c5 inputs, the pair arrays sliced to the rank's chunk), through
ServerReconstruction: sequential, the unpartitioned overlap (EC on a side stream beside the
self-mask pass) and the CU-split pair queue.  Each schedule is checked against the sequential
one.  Median of 7 runs."""
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
G = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--G=")), 8))   # the rank shape of G GPUs
L8 = L // G
eng = MaskEngine(0)
dev = torch.device("cuda:0")
m = np.frombuffer(b"".join(P.bench_seed("c5", i) for i in range(N)), np.uint8).reshape(N, 32)
nbrs = P.neighbor_graph(b"\x00" * 32, 1, N, 1, encrypt=eng.chacha20_encrypt)
off = np.sort(np.random.Generator(np.random.PCG64(1)).choice(N, N // 100, replace=False))
on = np.setdiff1d(np.arange(N), off)
R = recovery_round(eng, m, nbrs, on, off, T=20, committee=60, seed=1)
D = len(R["c1"])
d8 = -(-D // G)
S = torch.randint(-2**31, 2**31 - 1, (1, L8), dtype=torch.int32, device=dev)
t = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares")}
t["c1"] = torch.from_numpy(R["c1"][:d8]).to(dev)
t["pair_shares"] = torch.from_numpy(np.ascontiguousarray(R["pair_shares"][:, :d8])).to(dev)
t["pair_signs"] = torch.from_numpy(R["pair_signs"][:d8]).to(dev)
print(f"one rank of G = {G}: S shard {L8} slots, M = {len(on)}, pairs {d8} of D = {D}", flush=True)
main = torch.cuda.Stream()
ref = torch.empty(L8, dtype=torch.int32, device=dev)
out = torch.empty(L8, dtype=torch.int32, device=dev)
cases = [("sequential", dict(), False), ("overlap", dict(), True),
         ("cu_split_queue_24", dict(ec_cus=24, cu_pick="first", pair_queue=True, ec_terms=2, pass1_min_items=4096), True),
         ("cu_split_queue_32", dict(ec_cus=32, cu_pick="first", pair_queue=True, ec_terms=2, pass1_min_items=4096), True)]
# the cooperative kernel confined to about as many CUs as it has workgroups (ceil(D/8) x T / 64)
for cus in (40, 48, 64):
    for mi in (1024, 4096):
        cases.append((f"cu_split_coop_{cus}_items{mi}",
                       dict(ec_cus=cus, cu_pick="first", pair_queue=True, ec_terms=1, ec_coop=1, pass1_min_items=mi), True))
if "--coop-only" in sys.argv:
    cases = cases[:2] + cases[4:]
if "--shapes" in sys.argv:   # the unpartitioned overlap against the partitioned schedule at 72 / 96 / 128 CUs
    cases = cases[:2] + [(f"cu_split_coop_{c}_items4096",
                          dict(ec_cus=c, cu_pick="first", pair_queue=True, ec_terms=1, ec_coop=1, pass1_min_items=4096), True)
                         for c in (72, 96, 128)] * 2
if "--coop-fine" in sys.argv:   # around the best of --coop-only, two passes
    cases = cases[:2] + [(f"cu_split_coop_{c}_items{mi}",
                           dict(ec_cus=c, cu_pick="first", pair_queue=True, ec_terms=1, ec_coop=1, pass1_min_items=mi), True)
                          for c in (56, 64, 72, 80, 96) for mi in (2048, 4096)] * 2
if "--row" in sys.argv:   # round 4: the row-field cooperative kernel (ec_coop 2), unpartitioned and on its own CUs
    cases = cases[:2] + [(f"cu_split_row_{c}_items4096",
                          dict(ec_cus=c, cu_pick="first", pair_queue=True, ec_terms=1, ec_coop=2, pass1_min_items=4096), True)
                         for c in (64, 96, 128, 160)] + [
                        (f"cu_split_coop_{c}_items4096",
                         dict(ec_cus=c, cu_pick="first", pair_queue=True, ec_terms=1, ec_coop=1, pass1_min_items=4096), True)
                        for c in (72, 96)]
# round 5's --straus cases (Straus inside the row kernel) were retired with ec_mul_row_straus_kernel (-3 %)
for ci, (name, kw, ovl) in enumerate(cases):
    rec = ServerReconstruction(eng, **kw)
    dst = ref if name == "sequential" else out
    args = (S, L8, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], dst)
    ms = []
    with torch.cuda.stream(main):
        for _ in range(3):
            rec.run(*args, stream=main, overlap=ovl)
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            rec.run(*args, stream=main, overlap=ovl)
            e1.record(main)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
    rec.close()
    same = True if name == "sequential" else bool(torch.equal(out, ref))
    print(f"{name}: {float(np.median(ms)):.3f} ms (min {min(ms):.3f}) same_as_sequential={same}", flush=True)
eng.close()
