"""One-rank RCCL run of ShardedRound's pipelined path (buffers=2, async reduce-scatter, stream-side
waits) on a one-GPU box, with force_collective=True so world 1 takes the multi-GPU branches: the
collective is a copy on one rank, but the Work/stream handling is exactly the multi-GPU code.
Checks every round's shard against the plain world-1 round (no collective), for both exchanges:
torch.distributed's reduce-scatter and the library's own communicator (init_rccl ->
flm_comm_init_rank, flm_reduce_scatter_dev with ncclUint32 on a comm stream); the synchronous
forced round (buffers=1) too."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flamingo_amd import MaskEngine  # noqa: E402
from flamingo_amd.distributed import ShardedRound, init_rccl  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
eng = MaskEngine(0)
print("library communicator:", init_rccl(eng), flush=True)
N, K, L = 64, 48, 1 << 16
g = torch.Generator(device="cuda")
g.manual_seed(3)
rows = [torch.randint(-2**31, 2**31 - 1, (N, L), dtype=torch.int32, device="cuda", generator=g) for _ in range(3)]
seeds = torch.randint(0, 256, (K, 32), dtype=torch.uint8, device="cuda", generator=g)
signs = (torch.randint(0, 2, (K,), device="cuda", generator=g) * 2 - 1).to(torch.int8)
stream = torch.cuda.Stream()
ref = ShardedRound(eng, L)
want = []
for r in rows:
    res = ref.step(r, seeds, signs, stream)
    torch.cuda.synchronize()
    want.append(res.clone())
torch.cuda.synchronize()
ok = True
for comm in ("torch", "rccl"):
    sync = ShardedRound(eng, L, comm=comm, force_collective=True)
    for i, r in enumerate(rows):
        got = sync.step(r, seeds, signs, stream)
        torch.cuda.synchronize()
        e = bool(torch.equal(got[:L], want[i]))
        print(f"{comm} synchronous forced collective round {i}: out==want {e}", flush=True)
        ok &= e
    pipe = ShardedRound(eng, L, buffers=2, comm=comm, force_collective=True)
    assert pipe._async_ok() and pipe.comm == comm
    with torch.cuda.stream(stream):
        for rep in range(4):
            bufs = [pipe.launch(r, seeds, signs, stream) for r in rows]
            torch.cuda.synchronize()
            got = [pipe._outs[b][:L] for b in bufs[-2:]]
            parts = [pipe._partials[b][:L] for b in bufs[-2:]]
            for i, (o, p_, w) in enumerate(zip(got, parts, want[1:])):
                e = bool(torch.equal(o, w))
                print(f"{comm} rep {rep} round {i + 1}: out==want {e}  partial==want {bool(torch.equal(p_, w))} "
                      f"mismatches {int((o != w).sum())}", flush=True)
                ok &= e
# launch() with a stream that is NOT torch's current stream (the kernel, the collective and the
# buffer reuse must all order against `stream`, not the current one): a long kernel is queued on
# `stream` first so an unordered collective would read a partial before it is written
side = torch.cuda.Stream()
for comm in ("torch", "rccl"):
    pipe = ShardedRound(eng, L, buffers=2, comm=comm, force_collective=True)
    big = torch.randint(0, 100, (4096, 4096), device="cuda", dtype=torch.float32, generator=g)
    with torch.cuda.stream(side):            # current stream: `side`; the round runs on `stream`
        for rep in range(2):
            with torch.cuda.stream(stream):
                for _ in range(8):
                    big = big @ big * 1e-4   # ~ms of work ahead of the round on `stream`
            bufs = [pipe.launch(r, seeds, signs, stream) for r in rows]
            torch.cuda.synchronize()
            got = [pipe._outs[b][:L] for b in bufs[-2:]]
            for i, (o, w) in enumerate(zip(got, want[1:])):
                e = bool(torch.equal(o, w))
                print(f"{comm} non-current stream rep {rep} round {i + 1}: out==want {e}", flush=True)
                ok &= e
print(f"rccl async pipelined rounds ok={ok}", flush=True)
from flamingo_amd.distributed import shutdown  # noqa: E402
shutdown(eng)                   # library communicator, then torch's process group, then the context
sys.exit(0 if ok else 1)
