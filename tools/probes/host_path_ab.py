"""Host-pointer entry points, per-call wall time, at the agent run's shapes (c5): one client's
flm_client_mask (N = 1, L = 2^20, x given, 3 seeds), the server's flm_ec_combine (T = 20, D = 1000),
flm_shamir_combine (T = 20, M = 4055) and flm_aggregate_unmask's 4 MiB output path
(flm_mask_accumulate, L = 2^20).  Run once per library build (FLM_LIB_PATH): the pinned-bounce build
against the build before it (tools/gpu.sh hostab).  Median of 30 calls after 5 warm ones."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

eng = MaskEngine(0)
g = np.random.Generator(np.random.PCG64(3))
L = 1 << 20
seeds = g.integers(0, 256, (3, 32), dtype=np.uint8)
signs = np.array([1, -1, 1], np.int8)
x = g.integers(0, 2**32, (1, L), dtype=np.uint32)
pts, _ = eng.hash_to_curve_decimal(0, 2048)
T, D, M = 20, 1000, 4055
shares = np.repeat(pts[None, 1:D + 1], T, axis=0)
lam = g.integers(0, 128, (T, 32), dtype=np.uint8)
sh_ints = [[int(v) for v in g.integers(1, 2**62, M)] for _ in range(T)]
lam_ints = [int(v) for v in g.integers(1, 2**62, T)]
acc = g.integers(0, 2**32, L, dtype=np.uint32)


def med(fn, n=30):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e3)
    return float(np.median(ts))


print(f"lib {os.environ.get('FLM_LIB_PATH', 'default')}", flush=True)
print(f"client_mask N=1 L=2^20 x: {med(lambda: eng.client_mask(np.array([0, 3], np.int64), seeds, signs, L, x=x)):.3f} ms", flush=True)
print(f"ec_combine T=20 D=1000:  {med(lambda: eng.ec_combine_wire(pts[:D], shares, lam)):.3f} ms", flush=True)
print(f"shamir_combine T=20 M=4055 (incl. Python int packing): "
      f"{med(lambda: eng.shamir_combine(sh_ints, lam_ints), 10):.3f} ms", flush=True)
print(f"mask_accumulate L=2^20:  {med(lambda: eng.mask_accumulate(seeds, signs, acc.copy())):.3f} ms", flush=True)
