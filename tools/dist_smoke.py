"""G-rank smoke of the sharded round with RCCL: every rank on device LOCAL_RANK % visible GPUs.
Checks the reduce-scattered shard against |U| (valid masked rows)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flamingo_amd import MaskEngine, params as P  # noqa: E402
from flamingo_amd.distributed import ShardedRound, client_bounds  # noqa: E402

rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
dev_id = local % torch.cuda.device_count()
torch.cuda.set_device(dev_id)
backend = os.environ.get("FLM_DIST_BACKEND", "nccl")
if backend == "nccl":
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev_id))
else:
    dist.init_process_group(backend)
eng = MaskEngine(dev_id)
N, L = 256, 1 << 16
m = np.frombuffer(b"".join(P.bench_seed("dist", i) for i in range(N)), np.uint8).reshape(N, 32)
nbrs = P.neighbor_graph(bytes(32), 1, N, 1, encrypt=eng.chacha20_encrypt)
c0, c1 = client_bounds(N, world, rank)
seg, cs, csg = P.client_seed_table(m, nbrs, P.synthetic_pair_seed)
rows = torch.empty((N, L), dtype=torch.int32, device="cuda")
eng.client_mask_dev(seg, torch.from_numpy(cs).cuda(), csg, rows, L)
off = np.array([5, 77])
on = np.setdiff1d(np.arange(N), off)
ss, sg = P.server_seed_table(m, nbrs, on, off, P.synthetic_pair_seed)
mine = on[(on >= c0) & (on < c1)]
r = rows[torch.from_numpy(mine).cuda()].contiguous()
rnd = ShardedRound(eng, L)
out = rnd.step(r, torch.from_numpy(ss).cuda(), torch.from_numpy(sg).cuda())
torch.cuda.synchronize()
ok = bool(torch.all(out == len(on)).item())
print(f"rank {rank}/{world} shard [{rnd.lo},{rnd.hi}) ok={ok}", flush=True)
okt = torch.tensor([int(ok)], device="cuda" if backend == "nccl" else "cpu")
dist.all_reduce(okt, op=dist.ReduceOp.MIN)
dist.destroy_process_group()
sys.exit(0 if okt.item() == 1 else 1)
