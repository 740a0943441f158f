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
    for overlap, rec in ((True, rec), (False, rec), (True, split), (True, pair_split)):
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
    if n_off:
        assert R["D"] > 0
