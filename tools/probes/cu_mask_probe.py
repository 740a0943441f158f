"""Self-mask unmask of a c5-shaped round (4055 rows + 4055 seeds, L=2^20) on a CU-masked stream,
alone (no EC beside it): does a CU mask by itself cost more than the lost CUs?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.reconstruct import pick_cus  # noqa: E402

N, K, L = 4055, 4055, 1 << 20
eng = MaskEngine(0)
g = torch.Generator(device="cuda")
g.manual_seed(1)
rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
out = torch.empty(L, dtype=torch.int32, device="cuda")
ncu = eng.cu_count()
for mi in (1024, 4096):
    eng.set_tuning("min_items", mi)
    for excl, how in ((0, "none"), (24, "first"), (32, "first"), (24, "stride"), (64, "first")):
        if excl:
            ec = set(pick_cus(ncu, excl, how))
            st = eng.cu_stream([c for c in range(ncu) if c not in ec])
        else:
            st = torch.cuda.Stream()
        for _ in range(2):
            eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print(f"min_items={mi} excluded={excl} ({how}) CUs={ncu - excl} ms={ms:.3f} "
              f"ms*CUs/256={ms * (ncu - excl) / 256:.3f}", flush=True)
eng.close()
