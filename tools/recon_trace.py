"""c5-shaped reconstruction with the CU-split schedule, a few rounds, for rocprofv3 --kernel-trace:
the timeline of pass 1 (Shamir + self-mask unmask), the EC combine and pass 2 (pair masks)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import flamingo_amd.params as P  # noqa: E402
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.reconstruct import ServerReconstruction  # noqa: E402
from flamingo_amd.synthetic import recovery_round  # noqa: E402

N, L = 4096, 1 << 20
EC_CUS = int(os.environ.get("EC_CUS", "24"))
MIN_ITEMS = int(os.environ.get("MIN_ITEMS", "4096"))
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
rec = ServerReconstruction(eng, pass1_min_items=MIN_ITEMS, ec_cus=EC_CUS, cu_pick="first")
with torch.cuda.stream(main):
    for _ in range(4):
        rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out, stream=main)
        torch.cuda.synchronize()
print("correct", bool(torch.all(out == len(on)).item()), flush=True)
