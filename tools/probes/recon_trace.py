"""c5-shaped reconstruction with the CU-split schedule, a few rounds, for rocprofv3 --kernel-trace:
the timeline of pass 1 (Shamir + self-mask unmask), the EC combine and pass 2 (pair masks).
QUEUE=1: the pair_queue schedule, then the pair masks alone once through the work queue
(pair_units_kernel) and once through items_kernel, to compare the two kernels."""
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
QUEUE = os.environ.get("QUEUE", "0") == "1"
rec = ServerReconstruction(eng, pass1_min_items=MIN_ITEMS, ec_cus=EC_CUS, cu_pick="first", pair_queue=QUEUE,
                           ec_terms=int(os.environ.get("EC_TERMS", "1")))
with torch.cuda.stream(main):
    for _ in range(4):
        rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out, stream=main)
        torch.cuda.synchronize()
print("correct", bool(torch.all(out == len(on)).item()), flush=True)
if QUEUE:
    D = R["c1"].shape[0]
    p_seeds = rec._bufs["seeds"][len(on):]
    ws = rec._bufs["ws"]
    print("units claimed by the side pass (last round): see the trace; total units",
          ((L + 1023) // 1024) * ((D + 15) // 16), flush=True)
    zero = torch.zeros((2, L), dtype=torch.int32, device=dev)
    for _ in range(3):
        ws.zero_()
        eng.flag_set_dev(ws)
        rec.side_eng.pair_units_dev(p_seeds, t["pair_signs"], out, L, ws, eng.cu_count() * 32, p0=zero[0], p1=zero[1],
                                    final=True)
        eng.aggregate_unmask_dev(None, p_seeds, t["pair_signs"], zero[1], L=L)
    torch.cuda.synchronize()
rec.close()
