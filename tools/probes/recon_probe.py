"""Run the c5-shaped server reconstruction (overlapped and sequential schedules) a few times, for
rocprofv3 --kernel-trace: shows whether the EC combine really runs beside the self-mask unmask."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import flamingo_amd.params as P  # noqa: E402
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.reconstruct import ServerReconstruction  # noqa: E402
from flamingo_amd.synthetic import recovery_round  # noqa: E402

N, L = int(os.environ.get("RP_N", "4096")), 1 << 20
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
import bench  # noqa: E402

EC_WAVES = [int(w) for w in os.environ.get("EC_WAVES", "1").split(",")]
EC_CUS = [int(c) for c in os.environ.get("EC_CUS", "16,24,32,40").split(",")]
cases = [(False, 1024, 0, "stride", w) for w in EC_WAVES] + [(True, 1024, 0, "stride", w) for w in EC_WAVES]
cases += [(True, 4096, k, "first", w) for k in EC_CUS for w in EC_WAVES]
for w in EC_WAVES:
    eng.set_tuning("ec_waves", w)
    rec = bench.measure_recovery(eng, torch, D=len(R["c1"]), M=len(on), T=20)
    print(f"ec_waves={w} seed recovery alone: {rec['gpu_ms']:.3f} ms correct={rec['correct']}", flush=True)
for overlap, mi, ec_cus, pick, w in cases:
    eng.set_tuning("ec_waves", w)
    rec = ServerReconstruction(eng, pass1_min_items=mi, ec_cus=ec_cus, cu_pick=pick)
    with torch.cuda.stream(main):
        for _ in range(2):
            rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out,
                    stream=main, overlap=overlap)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        for _ in range(5):
            rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out,
                    stream=main, overlap=overlap)
        e1.record(main)
    torch.cuda.synchronize()
    rec.close()
    print(f"ec_waves={w} overlap={overlap} min_items={mi} ec_cus={ec_cus} pick={pick} ms={e0.elapsed_time(e1) / 5:.3f} correct={bool(torch.all(out == len(on)).item())}",
          flush=True)
