"""The standalone mask expansion at the bench's shape, default settings, for rocprofv3 sessions
(tools/gpu_prof.sh): K = 962 pair seeds (c5's D) x L = 2^20 slots through flm_prg_expand_dev,
`--reps` launches back to back on one stream after 3 warm-up launches; prints one JSON line with
the HIP-event time per launch.  The bench's `prg_expand` leg measures the same thing in its run."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flamingo_amd import MaskEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--K", type=int, default=962)
ap.add_argument("--log2-L", type=int, default=20)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
K, L = a.K, 1 << a.log2_L
eng = MaskEngine(0)
s = torch.cuda.Stream()
seeds = torch.from_numpy(np.random.Generator(np.random.PCG64(962)).integers(0, 256, (K, 32), dtype=np.uint8)).cuda()
out = torch.empty((K, L), dtype=torch.int32, device="cuda")
with torch.cuda.stream(s):
    for _ in range(3):
        eng.prg_expand_dev(seeds, out, L, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        eng.prg_expand_dev(seeds, out, L, stream=s)
    e1.record(s)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.reps
print(json.dumps({"K": K, "L": L, "reps": a.reps, "ms_per_launch": round(ms, 4),
                  "GB/s_written": round(4.0 * K * L / (ms * 1e-3) / 1e9, 1), "plan": eng.last_plan(),
                  "note": "per launch = seed schedule + prg_expand_kernel (HIP events over the loop)"}))
