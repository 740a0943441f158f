"""c2-shaped round (N=128, L=16384) for rocprofv3 --kernel-trace: where do its ~14 us go?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

N, K, L = 128, 128, 16384
eng = MaskEngine(0)
g = np.random.Generator(np.random.PCG64(1))
rows = torch.from_numpy(g.integers(0, 2**31, size=(N, L), dtype=np.int64).astype(np.int32)).cuda()
seeds = torch.from_numpy(g.integers(0, 256, size=(K, 32), dtype=np.uint8)).cuda()
signs = torch.from_numpy(np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)).cuda()
out = torch.empty(L, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
for mi in (1024, 256, 4096):
    eng.set_tuning("min_items", mi)
    for _ in range(3):
        eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(50):
        eng.aggregate_unmask_dev(rows, seeds, signs, out, L=L)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"min_items={mi} plan={eng.last_plan()} us/round={e0.elapsed_time(e1) / 50 * 1e3:.2f}", flush=True)
