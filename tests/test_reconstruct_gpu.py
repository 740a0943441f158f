"""Server reconstruction from decryption shares to the unmasked sum, on the GPU.

flamingo_amd.synthetic builds a round whose pair seeds are SHA-256 of group elements and
whose m_i and s_ij reach the server only as Shamir shares / threshold-ElGamal decryption
shares (SA_ServiceAgent.py:499-605).  ServerReconstruction recovers them on the GPU
(flm_shamir_combine_dev, flm_ec_combine_dev) and unmasks; all-ones inputs must sum to
|U| in every slot (SA_ClientAgent.py:304 + SA_ServiceAgent.py:605), with the recovery
overlapped on a second stream and sequential."""
import numpy as np
import pytest

import flamingo_amd.params as P
from flamingo_amd.synthetic import recovery_round

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    yield e
    e.close()


@pytest.mark.parametrize("N,L,n_off,T,committee", [(256, 20000, 7, 5, 12), (128, 16384, 0, 4, 9),
                                                   (512, 4096 + 48, 40, 20, 60)])
def test_reconstruction_end_to_end(eng, N, L, n_off, T, committee):
    import torch
    from flamingo_amd.reconstruct import ServerReconstruction
    m = np.frombuffer(b"".join(P.bench_seed("recon", i) for i in range(N)), np.uint8).reshape(N, 32)
    nbrs = P.synthetic_neighbors(N, degree=8, seed=N)
    g = np.random.Generator(np.random.PCG64(N + n_off))
    off = np.sort(g.choice(N, n_off, replace=False)) if n_off else np.zeros(0, np.int64)
    on = np.setdiff1d(np.arange(N), off)
    R = recovery_round(eng, m, nbrs, on, off, T=T, committee=committee, seed=3)
    dev = torch.device("cuda:0")
    pitch = (L + 3) // 4 * 4
    rows = torch.empty((N, pitch), dtype=torch.int32, device=dev)
    eng.client_mask_dev(R["seg"], torch.from_numpy(R["client_seeds"]).to(dev), R["client_signs"], rows, L)
    r_on = rows[torch.from_numpy(on).to(dev)].contiguous()
    t = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares", "c1", "pair_shares", "pair_signs")}
    rec = ServerReconstruction(eng)
    split = ServerReconstruction(eng, ec_cus=24, cu_pick="first", pass1_min_items=4096)  # CU-partitioned
    # CU-partitioned, and the EC CUs add the pair masks of the first 40 % of the slots
    pair_split = ServerReconstruction(eng, ec_cus=32, cu_pick="first", pass1_min_items=4096, pair_split=0.4)
    # CU-partitioned, the EC CUs claim pair-mask units from a queue until the self-mask pass ends
    queue = ServerReconstruction(eng, ec_cus=32, pass1_min_items=4096, pair_queue=True)
    # the bench's schedule: the queue on 24 EC CUs with two combine terms per lane (Straus)
    queue2 = ServerReconstruction(eng, ec_cus=24, cu_pick="first", pass1_min_items=4096, pair_queue=True, ec_terms=2)
    for overlap, rec in ((True, rec), (False, rec), (True, split), (True, pair_split), (True, queue),
                         (True, queue2)):
        out = torch.empty(L, dtype=torch.int32, device=dev)
        _, flags = rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out,
                           overlap=overlap)
        torch.cuda.synchronize()
        o = out.cpu().numpy().view(np.uint32)
        assert np.all(o == len(on)), (overlap, np.flatnonzero(o != len(on))[:8])
        assert int(flags.abs().sum()) == 0
        # the recovered seeds are exactly the round's server seeds, in recon order
        assert np.array_equal(rec._bufs["seeds"].cpu().numpy(), R["server_seeds"])
    split.close()
    pair_split.close()
    queue.close()
    queue2.close()
    if n_off:
        assert R["D"] > 0


def test_reconstruction_first_run_behind_a_long_kernel(eng):
    """A fresh ServerReconstruction's FIRST run() (its buffers, and the fills of the self-mask
    signs and the queue counters, made then) with a long kernel already queued on the caller's
    stream: the CU-partitioned streams wait on the caller's `ready` event, so they must not read
    a buffer whose fill is still queued behind that kernel."""
    import torch
    from flamingo_amd.reconstruct import ServerReconstruction
    N, L = 256, 20000
    m = np.frombuffer(b"".join(P.bench_seed("recon1", i) for i in range(N)), np.uint8).reshape(N, 32)
    nbrs = P.synthetic_neighbors(N, degree=8, seed=5)
    off = np.arange(3, N, 37)
    on = np.setdiff1d(np.arange(N), off)
    R = recovery_round(eng, m, nbrs, on, off, T=5, committee=12, seed=4)
    dev = torch.device("cuda:0")
    rows = torch.empty((N, L), dtype=torch.int32, device=dev)
    eng.client_mask_dev(R["seg"], torch.from_numpy(R["client_seeds"]).to(dev), R["client_signs"], rows, L)
    r_on = rows[torch.from_numpy(on).to(dev)].contiguous()
    t = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares", "c1", "pair_shares", "pair_signs")}
    caller = torch.cuda.Stream()
    for kw in (dict(ec_cus=24, cu_pick="first", pass1_min_items=4096, pair_queue=True, ec_terms=2),
               dict(ec_cus=24, cu_pick="first", pass1_min_items=4096)):
        torch.cuda.synchronize()
        rec = ServerReconstruction(eng, **kw)
        out = torch.empty(L, dtype=torch.int32, device=dev)
        with torch.cuda.stream(caller):
            big = torch.ones((4096, 4096), device=dev)
            for _ in range(8):
                big = big @ big * 1e-4       # a few ms queued ahead of the run on the caller's stream
            rec.run(r_on, L, t["lambdas"], t["mi_shares"], t["c1"], t["pair_shares"], t["pair_signs"], out,
                    stream=caller)
        torch.cuda.synchronize()
        o = out.cpu().numpy().view(np.uint32)
        assert np.all(o == len(on)), (kw, np.flatnonzero(o != len(on))[:8])
        rec.close()


@pytest.mark.parametrize("K,L", [(37, 5000), (100, 1 << 16), (1, 1024), (16, 17)])
@pytest.mark.parametrize("stop", ["never", "at_once"])
def test_pair_units_queue_vs_oracle(eng, K, L, stop):
    """flm_pair_units_dev: a side pass then a final pass over the same counter add every
    (1024-slot, 16-seed) unit exactly once, whichever pass claims it: with the stop flag never
    set the side pass takes all units, set beforehand it takes none."""
    import torch
    import oracle as O
    g = np.random.Generator(np.random.PCG64(K * 7 + L))
    seeds = g.integers(0, 256, (K, 32), dtype=np.uint8)
    signs = np.where(g.integers(0, 2, K) == 1, 1, -1).astype(np.int8)
    p0 = g.integers(0, 1 << 32, L, dtype=np.uint64).astype(np.uint32)
    dev = torch.device("cuda:0")
    ds, dg = torch.from_numpy(seeds).to(dev), torch.from_numpy(signs).to(dev)
    pitch = (L + 3) // 4 * 4
    part = torch.zeros((2, pitch), dtype=torch.int32, device=dev)
    part[0, :L] = torch.from_numpy(p0.view(np.int32)).to(dev)
    ws = torch.zeros(4, dtype=torch.int32, device=dev)
    if stop == "at_once":
        eng.flag_set_dev(ws)
    eng.pair_units_dev(ds, dg, part[1], L, ws, groups=8)
    out = torch.empty(pitch, dtype=torch.int32, device=dev)
    eng.pair_units_dev(ds, dg, out, L, ws, groups=64, p0=part[0], p1=part[1], final=True)
    torch.cuda.synchronize()
    n_units = ((L + 1023) // 1024) * ((K + 15) // 16)
    claimed = int(ws[0].item())
    if stop == "never":
        assert int(part[1, :L].ne(0).sum()) > 0
    else:
        assert int(part[1].abs().sum()) == 0
    assert claimed >= n_units
    want = O.aggregate_unmask(p0[None, :], seeds, signs, L)
    got = out[:L].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:8]


def test_pair_units_bad_arguments(eng):
    import torch
    dev = torch.device("cuda:0")
    ws = torch.zeros(4, dtype=torch.int32, device=dev)
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    seeds = torch.zeros((4, 32), dtype=torch.uint8, device=dev)
    signs = torch.ones(4, dtype=torch.int8, device=dev)
    with pytest.raises(RuntimeError):
        eng.pair_units_dev(seeds, signs, out, 1024, ws, groups=0)
    with pytest.raises(RuntimeError):       # the final pass needs both partial rows
        eng.pair_units_dev(seeds, signs, out, 1024, ws, groups=4, final=True)
    with pytest.raises(RuntimeError):       # 16-byte alignment of the final pass's rows
        eng.pair_units_dev(seeds, signs, out[1:], 1000, ws, groups=4, p0=out[:1000], p1=out[:1000], final=True)
