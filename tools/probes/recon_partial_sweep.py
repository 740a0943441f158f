"""c5 reconstruction with the reference's report/reconstruction split: S (the row sum) made once,
then the shares -> final_sum schedules run over the one row S.  Sweeps the pair-queue schedule's EC
CU count, CU pick and combine terms per lane, plus the unpartitioned overlap, each checked
out == |U| (round 3; bench.py's from_report_partial uses ec_cus = 24, first, 2 terms)."""
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
S = torch.empty((1, L), dtype=torch.int32, device=dev)
eng.aggregate_unmask_dev(r_on, None, None, S[0], L=L)
del r_on
t = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares", "c1", "pair_shares", "pair_signs")}
out = torch.empty(L, dtype=torch.int32, device=dev)
main = torch.cuda.Stream()
print(f"c5 from S: M={len(on)} D={len(R['c1'])}", flush=True)

cases = [dict()]                                              # unpartitioned overlap
for cus in (16, 24, 32, 40):
    for pick in ("first", "stride"):
        for terms in (1, 2):
            cases.append(dict(ec_cus=cus, cu_pick=pick, pair_queue=True, ec_terms=terms, pass1_min_items=4096))
if "--coop" in sys.argv:   # round 3: the cooperative kernel on the confined EC CUs against the per-lane Straus default
    cases = [dict(ec_cus=c, cu_pick="first", pair_queue=True, ec_terms=t, ec_coop=k, pass1_min_items=4096)
             for c in (24, 32, 40, 48) for (t, k) in ((2, 0), (1, 1))] * 2
for kw in cases:
    rec = ServerReconstruction(eng, **kw)
    args = (S, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out)
    with torch.cuda.stream(main):
        for _ in range(2):
            rec.run(*args, stream=main)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for _ in range(5):
            rec.run(*args, stream=main)
        e1.record(main)
    torch.cuda.synchronize()
    rec.close()
    ok = bool(torch.all(out == len(on)).item())
    print(f"{kw or 'overlap, no CU split'}: {e0.elapsed_time(e1) / 5:.3f} ms correct={ok}", flush=True)
eng.close()
