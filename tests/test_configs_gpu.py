"""BASELINE configs c3 and c5 at full size on the GPU (not only in bench.py).

c3: n=1024 clients, L=2^18, neighbourhood -o 2 (config/flamingo.py:37-38), the real
    findNeighbors graph (params.neighbor_graph), valid masked rows from the client kernel, the
    server round; out == |U| everywhere, and three slot windows against the oracle bit for bit.
c5: n=4096, L=2^20, 1 % dropouts, two iterations: the server gets m_i and s_ij only as Shamir /
    threshold-ElGamal decryption shares (flamingo_amd.synthetic) and ServerReconstruction
    (pair-queue schedule on 24 EC CUs with two combine terms per lane, the bench's) recovers them and unmasks on the GPU; out == |U|
    everywhere and windows against the oracle, which is given the recovered seeds' expected
    values (the round's own server seed table).
"""
from __future__ import annotations

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    yield e
    e.close()


def oracle_windows(rows_dev, seeds, signs, L, windows):
    """(window, oracle out) for slot windows [a, a + n) of the round (rows on the device)."""
    res = []
    for a, n in windows:
        host = rows_dev[:, a:a + n].cpu().numpy().view(np.uint32)
        res.append(((a, n), O.aggregate_unmask(host, seeds, signs, L=n, slot0=a, threads=8)))
    return res


def test_c3_full_size(eng):
    import torch
    from flamingo_amd import params as P
    N, L, o = 1024, 1 << 18, 2
    dev = torch.device("cuda", 0)
    m = np.frombuffer(b"".join(P.bench_seed("c3", i) for i in range(N)), np.uint8).reshape(N, 32)
    nbrs = P.neighbor_graph(bytes(32), 1, N, o, encrypt=eng.chacha20_encrypt)
    assert 30 < np.mean([len(s) for s in nbrs]) < 50           # deg ~39 at o=2
    seg, cs, csg = P.client_seed_table(m, nbrs, P.synthetic_pair_seed)
    rows = torch.empty((N, L), dtype=torch.int32, device=dev)
    eng.client_mask_dev(seg, torch.from_numpy(cs).to(dev), csg, rows, L)
    ss, sg = P.server_seed_table(m, nbrs, range(N), [], P.synthetic_pair_seed)
    out = torch.empty(L, dtype=torch.int32, device=dev)
    eng.aggregate_unmask_dev(rows, torch.from_numpy(ss).to(dev), torch.from_numpy(sg).to(dev), out, L=L)
    torch.cuda.synchronize()
    o_ = out.cpu().numpy().view(np.uint32)
    assert np.all(o_ == N), np.flatnonzero(o_ != N)[:8]
    plan = eng.last_plan()
    # planner rule: 256 tiles split into 8 row/seed parts, same-tile merged items with atomics
    assert plan["atomics"] == 1 and plan["items"] == 2048 and plan["variant"] == 2
    for (a, n), want in oracle_windows(rows, ss, sg, L, [(0, 2048), (L // 2 + 1024, 1024), (L - 4096, 4096)]):
        assert np.array_equal(o_[a:a + n], want), a


@pytest.mark.timeout(300)
def test_c5_full_size_reconstruction(eng):
    import torch
    from flamingo_amd import params as P
    from flamingo_amd.reconstruct import ServerReconstruction
    from flamingo_amd.synthetic import recovery_round
    N, L = 4096, 1 << 20
    dev = torch.device("cuda", 0)
    m = np.frombuffer(b"".join(P.bench_seed("c5", i) for i in range(N)), np.uint8).reshape(N, 32)
    rows = torch.empty((N, L), dtype=torch.int32, device=dev)
    out = torch.empty(L, dtype=torch.int32, device=dev)
    rec = ServerReconstruction(eng, ec_cus=24, cu_pick="first", pass1_min_items=4096, pair_queue=True, ec_terms=2)
    cache = {}
    try:
        for it in (1, 2):
            nbrs = P.neighbor_graph(bytes(32), it, N, 1, encrypt=eng.chacha20_encrypt)
            off = np.sort(np.random.Generator(np.random.PCG64(it)).choice(N, N // 100, replace=False))
            on = np.setdiff1d(np.arange(N), off)
            R = recovery_round(eng, m, nbrs, on, off, T=20, committee=60, seed=it, point_cache=cache)
            assert R["D"] > 500                                     # ~41 offline x ~22.5 neighbours
            eng.client_mask_dev(R["seg"], torch.from_numpy(R["client_seeds"]).to(dev), R["client_signs"], rows, L)
            r_on = rows[torch.from_numpy(on).to(dev)].contiguous()
            t = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares", "c1", "pair_shares",
                                                              "pair_signs")}
            out.fill_(0)
            _, flags = rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"],
                               out)
            torch.cuda.synchronize()
            o_ = out.cpu().numpy().view(np.uint32)
            assert np.all(o_ == len(on)), (it, np.flatnonzero(o_ != len(on))[:8])
            assert int(flags.abs().sum()) == 0
            assert np.array_equal(rec._bufs["seeds"].cpu().numpy(), R["server_seeds"])
            for (a, n), want in oracle_windows(r_on, R["server_seeds"], R["server_signs"], L,
                                               [(0, 1024), (L - 1024, 1024)]):
                assert np.array_equal(o_[a:a + n], want), (it, a)
            del r_on
    finally:
        rec.close()
