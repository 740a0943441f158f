"""A/B of the expansion kernel (flm_prg_expand_dev, prg_expand_kernel): one-wave workgroups per CU
(expand_waves; round 6's first pass also swept the store form, profiles/r06_expand_probe.log), at the bench's
shape (K = 962 pair seeds x L = 2^20), median of 7 launches each, rounds interleaved so the clock
drifts alike; every configuration's output is checked against oracle.prg on windows (checker only).
Also times the summing kernel's mask-only launch of the same seeds (the same-run ChaCha ceiling)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (checker only)
from flamingo_amd import MaskEngine  # noqa: E402

K, L = 962, 1 << 20
eng = MaskEngine(0)
dev = torch.device("cuda", 0)
s = torch.cuda.Stream()
seeds = np.random.Generator(np.random.PCG64(962)).integers(0, 256, (K, 32), dtype=np.uint8)
d_seeds = torch.from_numpy(seeds).to(dev)
d_signs = torch.ones(K, dtype=torch.int8, device=dev)
out = torch.empty((K, L), dtype=torch.int32, device=dev)


def timed(fn, reps=7):
    for _ in range(2):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        fn()
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    return float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))


def check():
    ok = True
    for k in (0, K // 2, K - 1):
        for a in (0, 4096 * 37, L - 4096):
            ok &= bool(np.array_equal(out[k, a:a + 4096].cpu().numpy().view(np.uint32),
                                      O.prg(seeds[k].tobytes(), 4096, a)))
    return ok


acc = torch.empty(L, dtype=torch.int32, device=dev)
configs = [(0, w) for w in (32, 64, 96, 128, 256)]
res = {c: [] for c in configs}
ceil = []
with torch.cuda.stream(s):
    for rnd in range(3):
        eng.seed_table_dev(d_seeds, d_signs, stream=s)
        ceil.append(timed(lambda: eng.aggregate_dev(None, K, acc, L=L, stream=s)))
        for m, w in configs:
            eng.set_tuning("expand_waves", w)
            out.fill_(0x3C3C3C3C)
            ms = timed(lambda: eng.prg_expand_dev(d_seeds, out, L, stream=s))
            ok = check() if rnd == 0 else True
            res[(m, w)].append(ms)
            if not ok:
                print(f"MISMATCH mode {m} waves {w}", flush=True)
words = K * L
c = float(np.median(ceil))
print(f"mask-only summing launch (same seeds, K={K}): {c:.4f} ms = {words / c / 1e6:.1f} G words/s", flush=True)
for (m, w), v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
    ms = float(np.median(v))
    print(f"waves/CU {w:2d}: {ms:.4f} ms  {4 * words / ms / 1e6:7.1f} GB/s written"
          f"  {words / ms / 1e6:6.1f} G words/s = {c / ms:.3f} of the ceiling   runs {[round(x, 4) for x in v]}", flush=True)
