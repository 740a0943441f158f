"""The single-process multi-GPU round (flm_group, include/flamingo_hip.h) on the GPU.

The drop-in server is one DES process (Kernel.py:190-271); DeviceGroup gives its round every
device: client-sharded upload, slot-sharded unmask, one reduce-scatter (RCCL, ncclUint32) and
the shards back.  On a one-GPU box G = 2..8 ranks run in loopback on the one GPU (each rank its
own context and stream; the exchange is a device kernel instead of RCCL), so the sharding,
per-device threads and shard bookkeeping are checked bit-exactly against the oracle at every G,
wrap-around included.  "1rccl" is a one-device group forced onto the multi-GPU path
(flm_group_init_flags(FLM_GROUP_RCCL)): ncclCommInitAll over the one device, the partial buffer,
the grouped ncclGroupStart / ncclReduceScatter / ncclGroupEnd exchange -- the branches the 8-GPU
node runs, executed here.
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle as O
from refgold import client_inputs, client_table, digest, iterations, ref, refnpz, server_table  # noqa: F401

pytestmark = pytest.mark.gpu


def case(N, K, L, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    rows = g.integers(0, 2**32, size=(N, L), dtype=np.uint32)
    if N:
        rows[:, :7] = 0xFFFFFFFF                  # wraps mod 2^32 inside the exchange
    seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    return rows, seeds, signs


def make_group(G):
    """G ranks on the one GPU: an int (loopback for G > 1) or "1rccl" (one device, RCCL clique)."""
    from flamingo_amd import DeviceGroup
    if G == "1rccl":
        grp = DeviceGroup([0], force_rccl=True)
        assert grp.rccl and not grp.loopback
        return grp, 1
    grp = DeviceGroup([0] * G)
    assert grp.loopback == (G > 1) and not grp.rccl
    return grp, G


@pytest.mark.parametrize("G", [1, "1rccl", 2, 3, 4, 8])
@pytest.mark.parametrize("N,K,L", [(16, 9, 16384), (5, 0, 5000), (3, 11, 70000), (0, 6, 4100), (40, 40, 1 << 18)])
def test_group_round_vs_oracle(G, N, K, L):
    grp, G = make_group(G)
    rows, seeds, signs = case(N, K, L, G * 1000 + N + K)
    want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
    with grp:
        got = grp.aggregate_unmask(list(rows) if N else [], seeds, signs, L=L)
        assert np.array_equal(got, want), (G, N, K, L, np.flatnonzero(got != want)[:8])
        got2 = grp.aggregate_unmask(list(rows) if N else [], seeds, signs, L=L)     # buffers reused
        assert np.array_equal(got2, want)


@pytest.mark.parametrize("G", [1, "1rccl", 4])
def test_group_device_round_vs_oracle(G):
    import torch
    from flamingo_amd.engine import client_bounds, shard_bounds
    grp, G = make_group(G)
    N, K, L = 37, 21, 100000
    rows, seeds, signs = case(N, K, L, 77 + G)
    want = O.aggregate_unmask(rows, seeds, signs, threads=8)
    pitch = (L + 63) // 64 * 64
    dev = torch.device("cuda", 0)
    with grp:
        d_rows, shards = [], []
        for r in range(G):
            c0, c1 = client_bounds(N, G, r)
            t = torch.zeros((c1 - c0, pitch), dtype=torch.int32, device=dev)
            t[:, :L] = torch.from_numpy(rows[c0:c1].view(np.int32)).to(dev)
            d_rows.append(t)
            shards.append(torch.full((shard_bounds(L, G, r)[2],), 7, dtype=torch.int32, device=dev))
        d_seeds = [torch.from_numpy(seeds).to(dev) for _ in range(G)]
        d_signs = [torch.from_numpy(signs).to(dev) for _ in range(G)]
        torch.cuda.synchronize()
        grp.aggregate_unmask_dev(d_rows, d_seeds, d_signs, shards, L)
        grp.sync()
        got = np.concatenate([shards[r][: shard_bounds(L, G, r)[1] - shard_bounds(L, G, r)[0]].cpu().numpy()
                              for r in range(G)]).view(np.uint32)
        assert np.array_equal(got, want)


def test_group_device_rounds_back_to_back():
    """Two loopback device rounds enqueued without a sync between them: round B's kernels rewrite
    the partials that round A's exchange reads on the other ranks' streams (the group orders them)."""
    import torch
    from flamingo_amd import DeviceGroup
    from flamingo_amd.engine import client_bounds, shard_bounds
    G, N, K, L = 4, 24, 30, 1 << 18
    dev = torch.device("cuda", 0)
    cases = [case(N, K, L, 901), case(N, K, L, 902)]
    with DeviceGroup([0] * G) as grp:
        ins, outs = [], []
        for rows, seeds, signs in cases:
            d_rows = [torch.from_numpy(rows[slice(*client_bounds(N, G, r))].view(np.int32)).to(dev) for r in range(G)]
            ins.append((d_rows, [torch.from_numpy(seeds).to(dev)] * G, [torch.from_numpy(signs).to(dev)] * G))
            outs.append([torch.zeros((shard_bounds(L, G, r)[2],), dtype=torch.int32, device=dev) for r in range(G)])
        torch.cuda.synchronize()
        for (d_rows, d_seeds, d_signs), shards in zip(ins, outs):
            grp.aggregate_unmask_dev(d_rows, d_seeds, d_signs, shards, L)
        grp.sync()
        for (rows, seeds, signs), shards in zip(cases, outs):
            got = np.concatenate([shards[r][: shard_bounds(L, G, r)[1] - shard_bounds(L, G, r)[0]].cpu().numpy()
                                  for r in range(G)]).view(np.uint32)
            assert np.array_equal(got, O.aggregate_unmask(rows, seeds, signs, threads=8))


@pytest.mark.parametrize("G", [4, "1rccl"])
def test_group_reproduces_reference_round(ref, refnpz, G):
    """The reference's own round (tests/golden/make_ref_golden.py) through a 4-rank loopback group
    and through the one-device RCCL clique."""
    from flamingo_amd import MaskEngine
    grp, _ = make_group(G)
    with MaskEngine(0) as eng, grp:
        for run, it in iterations(ref):
            seg, seeds, signs = client_table(run, it, refnpz)
            rows = eng.client_mask(seg, seeds, signs, run["L"], x=client_inputs(run, it))
            _, _, sseeds, ssigns = server_table(it, refnpz, run)
            out = grp.aggregate_unmask([rows[i] for i in it["arrival"]], sseeds, ssigns)
            assert digest(out) == it["final_sha256"], (run["name"], it["iteration"])


def test_group_rejects_mixed_devices_and_bad_args():
    from flamingo_amd import DeviceGroup
    with pytest.raises(RuntimeError, match="distinct"):
        DeviceGroup([0, 0, 1])
    with pytest.raises(RuntimeError, match="distinct devices"):
        DeviceGroup([0, 0], force_rccl=True)                  # RCCL refuses two ranks on one GPU
    with DeviceGroup([0, 0]) as grp:
        with pytest.raises(RuntimeError):
            grp.aggregate_unmask([np.zeros(10, np.uint32)], np.zeros((1, 32), np.uint8), np.array([3], np.int8))


def test_group_rccl_rounds_back_to_back_and_shorter():
    """The forced one-device clique over several device rounds without a sync between them, the
    second one shorter than the first: the partial's stale tail [L, Lp) must not reach the shard."""
    import torch
    from flamingo_amd.engine import shard_bounds
    grp, _ = make_group("1rccl")
    dev = torch.device("cuda", 0)
    with grp:
        outs, wants = [], []
        for L, seed in ((70000, 1), (5000, 2), (4100, 3)):
            rows, seeds, signs = case(9, 5, L, seed)
            wants.append(O.aggregate_unmask(rows, seeds, signs, threads=8))
            S = shard_bounds(L, 1, 0)[2]
            assert S % 1024 == 0 and S >= L
            sh = torch.full((S,), 3, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            grp.aggregate_unmask_dev([torch.from_numpy(rows.view(np.int32)).to(dev)],
                                     [torch.from_numpy(seeds).to(dev)], [torch.from_numpy(signs).to(dev)], [sh], L)
            outs.append((sh, L))
        grp.sync()
        for (sh, L), want in zip(outs, wants):
            assert np.array_equal(sh[:L].cpu().numpy().view(np.uint32), want)
            assert not sh[L:].any()                        # the reduce-scatter's padding is zero
