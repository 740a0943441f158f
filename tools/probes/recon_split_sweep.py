"""c5-shaped server reconstruction, CU-partitioned, with the pair masks of the first f*L slots
added on the EC CUs once the combine is done (ServerReconstruction pair_split): sweep EC CU
count x f.  f = "q" is the dynamic split instead (pair_queue: the EC CUs claim pair-mask units
until the self-mask pass ends).  CU_PICK = first | stride.  Prints one line per case with the
mean of 6 runs and the out == |U| check."""
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
cases = [(int(c), f) for c in os.environ.get("EC_CUS", "24,32,40").split(",")
         for f in os.environ.get("SPLIT", "0,0.2,0.35,0.5").split(",")]
# EC_TUNE="threads:waves,..." (flm_set_tuning ec_threads / ec_waves) multiplies the cases
tunes = [tuple(int(v) for v in x.split(":")) for x in os.environ.get("EC_TUNE", "64:1").split(",")]
cases = [(c, f, tn) for tn in tunes for c, f in cases]
for ec_cus, f, (ec_threads, ec_waves) in cases:
    eng.set_tuning("ec_threads", ec_threads)
    eng.set_tuning("ec_waves", ec_waves)
    eng.set_tuning("ec_coop", int(os.environ.get("EC_COOP", "0")))
    eng.set_tuning("ec_terms", int(os.environ.get("EC_TERMS", "1")))
    q = f == "q"
    rec = ServerReconstruction(eng, pass1_min_items=int(os.environ.get("MIN_ITEMS", "4096")), ec_cus=ec_cus, cu_pick=os.environ.get("CU_PICK", "first"),
                               pair_split=0.0 if q else float(f), pair_queue=q,
                               ec_terms=int(os.environ.get("EC_TERMS", "1")))
    if os.environ.get("PASS1_ALL") == "1":
        rec.part = torch.cuda.Stream()   # probe: pass 1 on every CU, the EC still confined to its CUs
    args = (r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out)
    with torch.cuda.stream(main):
        for _ in range(2):
            rec.run(*args, stream=main)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for _ in range(6):
            rec.run(*args, stream=main)
        e1.record(main)
    torch.cuda.synchronize()
    ok = bool(torch.all(out == len(on)).item())
    rec.close()
    print(f"ec_coop={os.environ.get('EC_COOP', '0')} ec_terms={os.environ.get('EC_TERMS', '1')} ec_cus={ec_cus} ec_threads={ec_threads} ec_waves={ec_waves} pair_split={f} ms={e0.elapsed_time(e1) / 6:.3f} correct={ok}", flush=True)
