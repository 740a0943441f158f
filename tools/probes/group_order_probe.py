"""Debug probe: DeviceGroup.aggregate_unmask_dev ordering against torch's current stream
(tests/test_streams_gpu.py::test_group_dev_orders_after_current_stream).  Runs the same loopback
round (a) with a host sync before the call, (b) behind a long kernel with after_current, and
(c) with the shards read after sync() instead of wait(); prints the mismatching slot ranges."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "oracle"))
import oracle as O  # noqa: E402
from flamingo_amd import DeviceGroup  # noqa: E402
from flamingo_amd.engine import client_bounds, shard_bounds  # noqa: E402


def long_kernel(dev, n=8192, reps=12):
    a = torch.ones((n, n), device=dev)
    for _ in range(reps):
        a = a @ a * 1e-4
    return a


def ranges(bad):
    idx = np.flatnonzero(bad)
    if not idx.size:
        return "none"
    cuts = np.flatnonzero(np.diff(idx) > 1)
    starts = np.concatenate([[idx[0]], idx[cuts + 1]])
    ends = np.concatenate([idx[cuts], [idx[-1]]])
    return f"{idx.size} slots in {len(starts)} runs: " + ", ".join(f"[{a},{b}]" for a, b in list(zip(starts, ends))[:8])


G, N, K, L = 3, 30, 17, 200000
dev = torch.device("cuda", 0)
g = np.random.Generator(np.random.PCG64(21))
rows = g.integers(0, 2**32, (N, L), dtype=np.uint32)
seeds = g.integers(0, 256, (K, 32), dtype=np.uint8)
signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
want = O.aggregate_unmask(rows, seeds, signs, threads=8)
print("shards", [shard_bounds(L, G, r) for r in range(G)], flush=True)
for mode in ("sync_first", "long_wait", "long_sync", "sync_first", "long_wait"):
    with DeviceGroup([0] * G) as grp:
        src = torch.from_numpy(rows.view(np.int32)).to(dev)
        d_rows = [torch.zeros((c1 - c0, L), dtype=torch.int32, device=dev)
                  for c0, c1 in (client_bounds(N, G, r) for r in range(G))]
        shards = [torch.zeros(shard_bounds(L, G, r)[2], dtype=torch.int32, device=dev) for r in range(G)]
        d_seeds = [torch.from_numpy(seeds).to(dev)] * G
        d_signs = [torch.from_numpy(signs).to(dev)] * G
        torch.cuda.synchronize()
        keep = None
        if mode != "sync_first":
            keep = long_kernel(dev)
        for r in range(G):
            c0, c1 = client_bounds(N, G, r)
            d_rows[r].copy_(src[c0:c1])
        if mode == "sync_first":
            torch.cuda.synchronize()
        grp.aggregate_unmask_dev(d_rows, d_seeds, d_signs, shards, L)
        if mode == "long_sync":
            grp.sync()
        else:
            grp.wait()
        got = torch.cat([shards[r][: shard_bounds(L, G, r)[1] - shard_bounds(L, G, r)[0]] for r in range(G)])
        got = got.cpu().numpy().view(np.uint32)
        print(mode, "mismatch:", ranges(got != want), flush=True)
        del keep
