"""BASELINE c2 client masking (N = 128 clients, L = 16384, the real o = 1 graph: ~14 seeds per
client) -- one flm_client_mask_dev launch of small_round_kernel<16, SEG> -- timed back to back, for
a rocprofv3 PMC pass (451-494 G words/s against ~980 at c5).  Prints the
launch's words, time and rate.  Usage: python tools/probes/c2_client_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd import params as P  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
N, L = 128, 16384
eng = MaskEngine(0)
m = np.frombuffer(b"".join(P.bench_seed("c2-probe", i) for i in range(N)), np.uint8).reshape(N, 32)
nbrs = P.neighbor_graph(b"\x00" * 32, 1, N, 1, encrypt=eng.chacha20_encrypt)
seg, cs, csg = P.client_seed_table(m, nbrs, P.synthetic_pair_seed)
d_cs = torch.from_numpy(cs).cuda()
rows = torch.empty((N, L), dtype=torch.int32, device="cuda")
s = torch.cuda.Stream()
words = int(seg[-1]) * L
with torch.cuda.stream(s):
    for _ in range(20):
        eng.client_mask_dev(seg, d_cs, csg, rows, L, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        eng.client_mask_dev(seg, d_cs, csg, rows, L, stream=s)
    e1.record(s)
    s.synchronize()
us = e0.elapsed_time(e1) / reps * 1e3
print(f"c2 client masks: {int(seg[-1])} seeds, {words / 1e6:.1f} M words, {us:.1f} us per launch, "
      f"{words / us / 1e3:.1f} G words/s", flush=True)
