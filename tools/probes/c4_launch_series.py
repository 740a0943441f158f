"""c4 round (N=1024, L=2^20, K=1024) launched 60 times back to back: per-launch kernel time
(HIP events on the launch stream) in order, to tell a thermal/clock drift from random spread."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

N, K, L = 1024, 1024, 1 << 20
eng = MaskEngine(0)
g = torch.Generator(device="cuda").manual_seed(1)
rows = torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g)
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
signs = torch.full((K,), -1, dtype=torch.int8, device="cuda")
out = torch.empty(L, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
eng.seed_table_dev(seeds, signs)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(60)]
for a, b in ev:
    a.record(s)
    eng.aggregate_dev(rows, K, out, L=L)
    b.record(s)
torch.cuda.synchronize()
t = [a.elapsed_time(b) for a, b in ev]
print(" ".join(f"{x:.3f}" for x in t))
print(f"min {min(t):.3f} median {float(np.median(t)):.3f} max {max(t):.3f} first10 {np.mean(t[:10]):.3f} "
      f"last10 {np.mean(t[-10:]):.3f}")
