"""Sharded c5-style reconstruction (flamingo_amd.dist_recon) across ranks, checked out == |U|.

Launched by tests/test_distributed_gpu.py with torch.distributed.run on one GPU: gloo ranks sharing
the card (RCCL refuses duplicate devices) exercise the sharding, the pair-chunk all-gather and the
reduce-scatter bookkeeping.  A one-rank nccl run attaches the library's RCCL communicator and runs
every case twice: as world 1 normally runs (the exchanges are device copies) and with
force_collective=True, where both exchanges go through flm_all_gather_dev / flm_reduce_scatter_dev
(ncclAllGather, ncclReduceScatter on a one-rank communicator) -- the branches the G-GPU run takes.
Every rank checks its own output shard."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd import params as P  # noqa: E402
from flamingo_amd.dist_recon import ShardedReconstruction, pair_chunk  # noqa: E402
from flamingo_amd.distributed import client_bounds, init_rccl  # noqa: E402
from flamingo_amd.synthetic import recovery_round  # noqa: E402

backend = sys.argv[1] if len(sys.argv) > 1 else "gloo"
torch.cuda.set_device(0)
if backend == "nccl":
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
else:
    dist.init_process_group("gloo")
G, r = dist.get_world_size(), dist.get_rank()
eng = MaskEngine(0)
if backend == "nccl":
    init_rccl(eng)
dev = torch.device("cuda", 0)
ok = True
forces = (False, True) if backend == "nccl" and G == 1 else (False,)
cases = [(N, L, n_off, T, f) for N, L, n_off, T in ((256, 20000, 7, 5), (512, 1 << 16, 9, 20), (64, 5000, 0, 4))
         for f in forces]
for N, L, n_off, T, force in cases:
    m = np.frombuffer(b"".join(P.bench_seed("dr", i) for i in range(N)), np.uint8).reshape(N, 32)
    nbrs = P.synthetic_neighbors(N, degree=8, seed=N)
    off = np.sort(np.random.Generator(np.random.PCG64(N)).choice(N, n_off, replace=False)) if n_off else \
        np.zeros(0, np.int64)
    on = np.setdiff1d(np.arange(N), off)
    R = recovery_round(eng, m, nbrs, on, off, T=T, committee=3 * T, seed=N)
    pitch = (L + 63) // 64 * 64
    rows = torch.empty((N, pitch), dtype=torch.int32, device=dev)
    eng.client_mask_dev(R["seg"], torch.from_numpy(R["client_seeds"]).to(dev), R["client_signs"], rows, L)
    c0, c1 = client_bounds(len(on), G, r)
    mine = torch.from_numpy(on[c0:c1]).to(dev)
    r_rows = rows[mine].contiguous()
    D = R["D"]
    a, b, _ = pair_chunk(D, G, r)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    rec = ShardedReconstruction(eng, L, force_collective=force)
    if backend == "nccl" and (G > 1 or force) and rec.comm != "rccl":
        print(f"rank {r}: expected the library RCCL communicator, got comm={rec.comm}", flush=True)
        ok = False
    tag = f"force_collective={force} comm={rec.comm}"
    out = torch.full((rec.S,), 7, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for rep in range(2):
        rec.run(r_rows, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]), t(R["pair_shares"][:, a:b]),
                t(R["pair_signs"]), D, out)
        torch.cuda.synchronize()
        got = out[: rec.hi - rec.lo].cpu().numpy().view(np.uint32)
        good = bool(np.all(got == len(on)))
        print(f"rank {r}/{G} N={N} L={L} D={D} {tag} rep {rep}: shard [{rec.lo},{rec.hi}) out==|U| {good}",
              flush=True)
        ok &= good
    # the reference's split: S shards at report, masks over them at reconstruction
    S_shard = torch.full((rec.S,), 5, dtype=torch.int32, device=dev)
    rec.report(r_rows, S_shard)
    torch.cuda.synchronize()
    want_S = rows[torch.from_numpy(on).to(dev)][:, :L].sum(0, dtype=torch.int64).remainder(2**32)
    got_S = S_shard[: rec.hi - rec.lo].cpu().numpy().view(np.uint32).astype(np.int64)
    good = bool(np.array_equal(got_S, want_S[rec.lo:rec.hi].cpu().numpy()))
    out.fill_(7)
    rec.run_from_partial(S_shard, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]), t(R["pair_shares"][:, a:b]),
                         t(R["pair_signs"]), D, out)
    torch.cuda.synchronize()
    good &= bool(np.all(out[: rec.hi - rec.lo].cpu().numpy().view(np.uint32) == len(on)))
    print(f"rank {r}/{G} N={N} L={L} D={D} {tag} from report partial: S shard and out==|U| {good}", flush=True)
    ok &= good
    # the CU-partitioned schedule: combine on its own CUs, Shamir + self masks on the rest
    rec_cu = ShardedReconstruction(eng, L, ec_cus=max(8, eng.cu_count() // 4 // 8 * 8), force_collective=force)
    for name, fn in (("run", lambda: rec_cu.run(r_rows, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]),
                                                t(R["pair_shares"][:, a:b]), t(R["pair_signs"]), D, out)),
                     ("from report partial", lambda: rec_cu.run_from_partial(
                         S_shard, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]), t(R["pair_shares"][:, a:b]),
                         t(R["pair_signs"]), D, out))):
        out.fill_(7)
        fn()
        torch.cuda.synchronize()
        good = bool(np.all(out[: rec.hi - rec.lo].cpu().numpy().view(np.uint32) == len(on)))
        print(f"rank {r}/{G} N={N} L={L} D={D} {tag} ec_cus={rec_cu.ec_cus} {name}: out==|U| {good}", flush=True)
        ok &= good
okt = torch.tensor([1 if ok else 0])
if backend == "nccl":
    okt = okt.to(dev)
dist.all_reduce(okt, op=dist.ReduceOp.MIN)
print(f"sharded reconstruction ok={bool(okt.item())}", flush=True)
from flamingo_amd.distributed import shutdown  # noqa: E402
shutdown(eng)                   # library communicator, then torch's process group, then the context
sys.exit(0 if okt.item() else 1)
