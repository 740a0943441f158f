"""Every RCCL branch of the multi-GPU path, run on a one-GPU box (the kernel trace of this script
under rocprofv3 is the evidence that they execute; tools/gpu.sh step `rccl`).

* flm_group with FLM_GROUP_RCCL: ncclCommInitAll over the one device, the grouped
  ncclGroupStart / ncclReduceScatter / ncclGroupEnd exchange (flm_comm.hip exchange()), host and
  device-resident rounds, and a VectorStore whose partial sum goes through it;
* the library communicator of one process per GPU (init_rccl -> flm_comm_init_rank) at world 1
  with force_collective: ShardedRound's flm_reduce_scatter_dev (synchronous and pipelined) and
  ShardedReconstruction's flm_all_gather_dev + flm_reduce_scatter_dev.
Every result is checked against the C oracle or the |U| invariant; exits non-zero on a mismatch.
Argument: the torch.distributed backend of the world-1 group (nccl, default, or gloo).  The
collectives under test are the library's own RCCL communicator either way.  Teardown is
distributed.shutdown: library communicator (finalize + destroy) before torch's process group --
the round-4 order (torch's group first) crashed at exit under rocprofv3 with the nccl backend.
FLM_EXIT_MAPS=path saves /proc/self/maps at interpreter exit (to attribute any exit-time crash)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (checker)
from flamingo_amd import DeviceGroup, MaskEngine  # noqa: E402
from flamingo_amd import params as P  # noqa: E402
from flamingo_amd.dist_recon import ShardedReconstruction, pair_chunk  # noqa: E402
from flamingo_amd.distributed import ShardedRound, init_rccl  # noqa: E402
from flamingo_amd.engine import shard_bounds  # noqa: E402
from flamingo_amd.ingest import VectorStore  # noqa: E402
from flamingo_amd.synthetic import recovery_round  # noqa: E402

ok = True

if os.environ.get("FLM_EXIT_MAPS"):
    # the process's mappings just before the C-level exit handlers run, so that the frames of a
    # crash in __cxa_finalize (the round-4 failure mode) can be attributed to a library
    import atexit
    import shutil
    atexit.register(lambda: shutil.copyfile("/proc/self/maps", os.environ["FLM_EXIT_MAPS"]))


def check(name, good):
    global ok
    ok &= bool(good)
    print(f"{name}: {'ok' if good else 'MISMATCH'}", flush=True)


def case(N, K, L, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    rows = g.integers(0, 2**32, size=(N, L), dtype=np.uint32)
    seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    return rows, seeds, signs


torch.cuda.set_device(0)
dev = torch.device("cuda", 0)

# ---- single-process device group with a one-device RCCL clique
grp = DeviceGroup([0], force_rccl=True)
check("group has an RCCL clique", grp.rccl and not grp.loopback)
for N, K, L in ((64, 33, 1 << 18), (5, 0, 70001), (0, 9, 4100)):
    rows, seeds, signs = case(N, K, L, N + K)
    want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
    got = grp.aggregate_unmask(list(rows) if N else [], seeds, signs, L=L)
    check(f"group host round N={N} K={K} L={L}", np.array_equal(got, want))
    S = shard_bounds(L, 1, 0)[2]
    sh = torch.full((S,), 5, dtype=torch.int32, device=dev)
    d_rows = None
    if N:                                   # device rows at a pitch that is a multiple of 4 words
        d_rows = torch.zeros((N, (L + 63) // 64 * 64), dtype=torch.int32, device=dev)
        d_rows[:, :L] = torch.from_numpy(rows.view(np.int32)).to(dev)
    grp.aggregate_unmask_dev([d_rows], [torch.from_numpy(seeds).to(dev)], [torch.from_numpy(signs).to(dev)], [sh], L)
    grp.sync()
    check(f"group device round N={N} K={K} L={L}", np.array_equal(sh[:L].cpu().numpy().view(np.uint32), want))
st = VectorStore(grp, 100000, 8)
rows, seeds, signs = case(12, 20, 100000, 7)
for i in range(12):
    st.add(i, rows[i])
st.partial_sum()
st.wait_partial()
check("store partial through the clique", np.array_equal(st.host_partial(), rows.sum(0, dtype=np.uint64).astype(np.uint32)))
check("store unmask", np.array_equal(st.unmask(seeds, signs), O.aggregate_unmask(rows, seeds, signs, threads=8)))
st.close()
grp.close()

# ---- one process per GPU at world 1, forced through the collectives
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29573")
backend = sys.argv[1] if len(sys.argv) > 1 else "nccl"
if backend == "nccl":
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
else:
    dist.init_process_group("gloo", rank=0, world_size=1)
eng = MaskEngine(0)
init_rccl(eng)
check("library communicator attached", eng.has_comm() and eng.comm_size() == (1, 0))
N, K, L = 48, 40, 1 << 17
rows, seeds, signs = case(N, K, L, 11)
want = O.aggregate_unmask(rows, seeds, signs, threads=8)
d_rows = torch.from_numpy(rows.view(np.int32)).to(dev)
d_seeds, d_signs = torch.from_numpy(seeds).to(dev), torch.from_numpy(signs).to(dev)
stream = torch.cuda.Stream()
for buffers in (1, 2):
    rnd = ShardedRound(eng, L, buffers=buffers, force_collective=True)
    check(f"ShardedRound buffers={buffers} uses the library communicator", rnd.comm == "rccl")
    for _ in range(3):
        b = rnd.launch(d_rows, d_seeds, d_signs, stream)
    got = rnd.result(b)
    torch.cuda.synchronize()
    check(f"ShardedRound buffers={buffers} forced reduce-scatter", np.array_equal(got.cpu().numpy().view(np.uint32), want))
N, L = 256, 20000
m = np.frombuffer(b"".join(P.bench_seed("rc", i) for i in range(N)), np.uint8).reshape(N, 32)
nbrs = P.synthetic_neighbors(N, degree=8, seed=N)
off = np.sort(np.random.Generator(np.random.PCG64(N)).choice(N, 7, replace=False))
on = np.setdiff1d(np.arange(N), off)
R = recovery_round(eng, m, nbrs, on, off, T=5, committee=15, seed=N)
full = torch.empty((N, L), dtype=torch.int32, device=dev)
eng.client_mask_dev(R["seg"], torch.from_numpy(R["client_seeds"]).to(dev), R["client_signs"], full, L)
r_rows = full[torch.from_numpy(on).to(dev)].contiguous()
D = R["D"]
a, b, _ = pair_chunk(D, 1, 0)
t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
rec = ShardedReconstruction(eng, L, force_collective=True)
check("ShardedReconstruction uses the library communicator", rec.comm == "rccl")
out = torch.full((rec.S,), 7, dtype=torch.int32, device=dev)
rec.run(r_rows, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]), t(R["pair_shares"][:, a:b]), t(R["pair_signs"]),
        D, out)
torch.cuda.synchronize()
check(f"ShardedReconstruction.run D={D}: all-gather + reduce-scatter", bool(torch.all(out[:L] == len(on)).item()))
S_shard = torch.full((rec.S,), 5, dtype=torch.int32, device=dev)
rec.report(r_rows, S_shard)
out.fill_(7)
rec.run_from_partial(S_shard, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]), t(R["pair_shares"][:, a:b]),
                     t(R["pair_signs"]), D, out)
torch.cuda.synchronize()
check("ShardedReconstruction report + run_from_partial", bool(torch.all(out[:L] == len(on)).item()))
from flamingo_amd.distributed import shutdown  # noqa: E402
shutdown(eng)                   # library communicator, then torch's process group, then the context
print(f"rccl clique smoke ok={ok}", flush=True)
sys.exit(0 if ok else 1)
