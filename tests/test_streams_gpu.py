"""Stream contract of the *_dev entry points (include/flamingo_hip.h): they enqueue on the
caller's stream and return without waiting for earlier work, and NULL means the HIP null
stream everywhere (the collectives included).

A "long kernel" (a chain of large matmuls, tens of ms) is queued first on the caller's stream;
each call under test must return while it is still running (its event not yet complete), and
the results, read afterwards in stream order, must still match the oracle."""
from __future__ import annotations

import numpy as np
import pytest

import oracle as O
from flamingo_amd import params as P

pytestmark = pytest.mark.gpu


def _long_kernel(dev, n=8192, reps=12):
    import torch
    a = torch.ones((n, n), device=dev)
    for _ in range(reps):
        a = a @ a * 1e-4
    ev = torch.cuda.Event()
    ev.record()
    return a, ev


def _client_table(N, deg, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    seg, seeds, signs = [0], [], []
    for i in range(N):
        for _ in range(1 + int(g.integers(0, deg + 1))):
            seeds.append(g.integers(0, 256, 32, dtype=np.uint8))
            signs.append(1 if g.random() < 0.5 else -1)
        seg.append(len(seeds))
    return np.array(seg, np.int64), np.stack(seeds), np.array(signs, np.int8)


@pytest.fixture(scope="module")
def eng():
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    yield e
    e.close()


@pytest.mark.parametrize("N,L", [(64, 16384), (48, 600000)])   # small-round path, items path (K*L > 2^26)
def test_client_mask_dev_does_not_block(eng, N, L):
    import torch
    dev = torch.device("cuda", 0)
    seg, seeds, signs = _client_table(N, 6, N + L)
    d_seeds = torch.from_numpy(seeds).to(dev)
    outs = [torch.empty((N, L), dtype=torch.int32, device=dev) for _ in range(4)]
    eng.client_mask_dev(seg, d_seeds, signs, outs[0], L)          # warm: plans, staging slots
    torch.cuda.synchronize()
    _, busy = _long_kernel(dev)
    for o in outs:                                                # several calls behind the long kernel
        eng.client_mask_dev(seg, d_seeds, signs, o, L)
    assert not busy.query(), "flm_client_mask_dev waited for earlier work on its stream"
    torch.cuda.synchronize()
    want = eng.client_mask(seg, seeds, signs, L)
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want)


def test_client_mask_dev_shape_changes_behind_a_long_kernel(eng):
    """Different seg tables back to back (each call's own staged seg/signs and work items)."""
    import torch
    dev = torch.device("cuda", 0)
    L = 200000
    cases = [_client_table(N, 5, 10 + N) for N in (9, 17, 33)]
    outs = [torch.empty((len(c[0]) - 1, L), dtype=torch.int32, device=dev) for c in cases]
    d = [torch.from_numpy(c[1]).to(dev) for c in cases]
    torch.cuda.synchronize()
    _long_kernel(dev)
    for (seg, _, signs), ds, o in zip(cases, d, outs):
        eng.client_mask_dev(seg, ds, signs, o, L)
    torch.cuda.synchronize()
    for (seg, seeds, signs), o in zip(cases, outs):
        assert np.array_equal(o.cpu().numpy().view(np.uint32), eng.client_mask(seg, seeds, signs, L))


def test_prg_expand_dev_does_not_block(eng):
    import torch
    dev = torch.device("cuda", 0)
    K, L, slot0 = 23, 70000, 4096
    seeds = np.random.Generator(np.random.PCG64(5)).integers(0, 256, (K, 32), dtype=np.uint8)
    d_seeds = torch.from_numpy(seeds).to(dev)
    out = torch.empty((K, L), dtype=torch.int32, device=dev)
    eng.prg_expand_dev(d_seeds, out, L, slot0=slot0)
    torch.cuda.synchronize()
    out.zero_()
    _, busy = _long_kernel(dev)
    eng.prg_expand_dev(d_seeds, out, L, slot0=slot0)
    assert not busy.query(), "flm_prg_expand_dev waited for earlier work on its stream"
    torch.cuda.synchronize()
    want = np.stack([O.prg(s.tobytes(), L, slot0) for s in seeds[:3]])
    assert np.array_equal(out[:3].cpu().numpy().view(np.uint32), want)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), eng.prg_expand(seeds, L, slot0))


def test_aggregate_dev_new_plan_on_another_stream(eng):
    """A plan first built (items copied in) on stream A and first launched on stream B: the
    launch on B waits for the copy on A (Plan.ready)."""
    import torch
    dev = torch.device("cuda", 0)
    N, K, L = 40, 33, 123456
    g = np.random.Generator(np.random.PCG64(8))
    rows = g.integers(0, 2**32, (N, L), dtype=np.uint32)
    seeds = g.integers(0, 256, (K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    d_rows = torch.from_numpy(rows.view(np.int32)).to(dev)
    d_seeds, d_signs = torch.from_numpy(seeds).to(dev), torch.from_numpy(signs).to(dev)
    out_a = torch.empty(L, dtype=torch.int32, device=dev)
    out_b = torch.empty(L, dtype=torch.int32, device=dev)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(sa):
        _, busy = _long_kernel(dev)
        eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out_a, L=L, stream=sa)   # builds the plan on sa
        assert not busy.query()
    eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out_b, L=L, stream=sb)       # same plan, on sb
    torch.cuda.synchronize()
    want = O.aggregate_unmask(rows, seeds, signs, threads=8)
    assert np.array_equal(out_a.cpu().numpy().view(np.uint32), want)
    assert np.array_equal(out_b.cpu().numpy().view(np.uint32), want)


def test_reduce_scatter_null_stream_orders_with_torch_default_stream(eng):
    """stream=None on the collectives is torch's current stream (default: the null stream), as
    for every other *_dev call: the collective runs after the kernel that wrote the partial and
    before the read of its output (it used to run on the context's private stream)."""
    import torch
    from flamingo_amd.engine import MaskEngine, comm_unique_id
    dev = torch.device("cuda", 0)
    e1 = MaskEngine(0)
    try:
        e1.comm_init(1, 0, comm_unique_id())
        assert e1.comm_size() == (1, 0)
        n = 1 << 22
        part = torch.zeros(n, dtype=torch.int32, device=dev)
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        gath = torch.zeros(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        for k in (3, 11):
            a, _ = _long_kernel(dev)
            part.fill_(k)                     # written after the long kernel, on the default stream
            e1.reduce_scatter_dev(part, out)  # stream None
            e1.all_gather_dev(out, gath)
            assert int(out.sum().item()) == k * n
            assert int(gath.sum().item()) == k * n
    finally:
        e1.close()


def test_group_dev_orders_after_current_stream():
    """DeviceGroup.aggregate_unmask_dev waits for torch's current stream (where the inputs were
    made) and wait() orders the reads after the ranks' rounds -- no host synchronisation."""
    import torch
    from flamingo_amd import DeviceGroup
    from flamingo_amd.engine import client_bounds, shard_bounds
    G, N, K, L = 3, 30, 17, 200000
    dev = torch.device("cuda", 0)
    g = np.random.Generator(np.random.PCG64(21))
    rows = g.integers(0, 2**32, (N, L), dtype=np.uint32)
    seeds = g.integers(0, 256, (K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    want = O.aggregate_unmask(rows, seeds, signs, threads=8)
    with DeviceGroup([0] * G) as grp:
        src = torch.from_numpy(rows.view(np.int32)).to(dev)
        d_rows = [torch.zeros((c1 - c0, L), dtype=torch.int32, device=dev)
                  for c0, c1 in (client_bounds(N, G, r) for r in range(G))]
        shards = [torch.zeros(shard_bounds(L, G, r)[2], dtype=torch.int32, device=dev) for r in range(G)]
        d_seeds = [torch.from_numpy(seeds).to(dev)] * G
        d_signs = [torch.from_numpy(signs).to(dev)] * G
        torch.cuda.synchronize()
        _long_kernel(dev)
        for r in range(G):                    # the rows are produced after the long kernel
            c0, c1 = client_bounds(N, G, r)
            d_rows[r].copy_(src[c0:c1])
        grp.aggregate_unmask_dev(d_rows, d_seeds, d_signs, shards, L)
        grp.wait()
        got = torch.cat([shards[r][: shard_bounds(L, G, r)[1] - shard_bounds(L, G, r)[0]] for r in range(G)])
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want)


def test_group_smaller_round_leaves_zero_padding():
    """After a round of larger L, a smaller round's shards carry zeros past its last slot (the
    partials' stale tail is cleared)."""
    import torch
    from flamingo_amd import DeviceGroup
    from flamingo_amd.engine import shard_bounds
    G = 3
    dev = torch.device("cuda", 0)
    g = np.random.Generator(np.random.PCG64(4))
    with DeviceGroup([0] * G) as grp:
        for L in (300000, 70000):
            rows = g.integers(1, 2**32, (6, L), dtype=np.uint32)
            d_rows = [torch.from_numpy(rows[2 * r:2 * r + 2].view(np.int32)).to(dev) for r in range(G)]
            shards = [torch.full((shard_bounds(L, G, r)[2],), 99, dtype=torch.int32, device=dev) for r in range(G)]
            grp.aggregate_unmask_dev(d_rows, [None] * G, [None] * G, shards, L)
            grp.sync()
            want = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8), threads=8)
            for r in range(G):
                lo, hi, S = shard_bounds(L, G, r)
                sh = shards[r].cpu().numpy().view(np.uint32)
                assert np.array_equal(sh[: hi - lo], want[lo:hi])
                assert not sh[hi - lo:].any(), (L, r)


def test_single_device_group_needs_no_communicator():
    from flamingo_amd import DeviceGroup
    with DeviceGroup([0]) as grp:
        assert not grp.loopback
        assert grp.engines[0].comm_size() == (1, 0)
        L = 5000
        rows = np.arange(3 * L, dtype=np.uint32).reshape(3, L)
        s = np.frombuffer(P.synthetic_pair_seed(1, 2), np.uint8).reshape(1, 32)
        got = grp.aggregate_unmask(list(rows), s, np.array([-1], np.int8), L=L)
        assert np.array_equal(got, O.aggregate_unmask(rows, s, np.array([-1], np.int8), threads=4))
