"""The HIP path against fixtures produced by the reference's own agents (tests/golden/make_ref_golden.py).

Every check goes through libflamingo_hip.so's C ABI on the GPU and compares with
values eniac/flamingo's SA_ClientAgent / SA_ServiceAgent computed on the same
seeds and inputs: the clients' masked vectors (SA_ClientAgent.py:304-324), the
server's vec_sum_partial, mi_vec, cancel_vec and final_sum
(SA_ServiceAgent.py:346-350, 529-605), and the seeds the server recovered from
the decryptors' shares (:506-526 Shamir, :542-585 threshold ElGamal).
"""
from __future__ import annotations

import numpy as np
import pytest

from refgold import client_inputs, client_table, digest, iterations, ref, refnpz, server_table  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    yield e
    e.close()


def test_client_vectors_match_reference(eng, ref, refnpz):
    for run, it in iterations(ref):
        seg, seeds, signs = client_table(run, it, refnpz)
        rows = eng.client_mask(seg, seeds, signs, run["L"], x=client_inputs(run, it))
        assert [digest(r) for r in rows] == [c["y_sha256"] for c in it["clients"]], (run["name"], it["iteration"])


def test_server_round_matches_reference(eng, ref, refnpz):
    for run, it in iterations(ref):
        L = run["L"]
        seg, seeds, signs = client_table(run, it, refnpz)
        rows = eng.client_mask(seg, seeds, signs, L, x=client_inputs(run, it))
        U = [rows[i] for i in it["arrival"]]          # the server's dict order (arrival)
        sm, sp, sseeds, ssigns = server_table(it, refnpz, run)
        none = np.zeros((0, 32), np.uint8)
        assert digest(eng.aggregate_unmask(U, none, np.zeros(0, np.int8))) == it["S_sha256"]
        assert digest(eng.aggregate_unmask([], sm, -np.ones(sm.shape[0], np.int8), L=L)) == it["M_sha256"]
        assert digest(eng.aggregate_unmask([], sp, ssigns[sm.shape[0]:], L=L)) == it["C_sha256"]
        out = eng.aggregate_unmask(U, sseeds, ssigns)
        assert digest(out) == it["final_sha256"], (run["name"], it["iteration"])
        assert out[:8].tolist() == it["final_head"]


def test_device_round_matches_reference(eng, ref, refnpz):
    """The same rounds through the device-resident entry points (rows in HBM, pitch > L)."""
    import torch
    dev = torch.device("cuda", 0)
    for run, it in iterations(ref):
        L = run["L"]
        seg, seeds, signs = client_table(run, it, refnpz)
        rows = eng.client_mask(seg, seeds, signs, L, x=client_inputs(run, it))[it["arrival"]]
        pitch = (L + 63) // 64 * 64 + 64
        d_rows = torch.zeros((rows.shape[0], pitch), dtype=torch.int32, device=dev)
        d_rows[:, :L] = torch.from_numpy(rows.view(np.int32)).to(dev)
        _, _, sseeds, ssigns = server_table(it, refnpz, run)
        d_seeds = torch.from_numpy(sseeds).to(dev)
        d_signs = torch.from_numpy(ssigns).to(dev)
        out = torch.empty(pitch, dtype=torch.int32, device=dev)
        eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L)
        torch.cuda.synchronize()
        assert digest(out[:L].cpu().numpy().view(np.uint32)) == it["final_sha256"]


def test_gpu_seed_recovery_from_reference_shares(eng, ref, refnpz):
    """flm_shamir_combine / flm_ec_combine on the decryptors' own shares give the reference's keys."""
    run = ref["runs"][0]
    it = run["iterations"][0]
    pre = f"{run['name']}_it1_"
    lam = np.frombuffer(b"".join(int(v, 16).to_bytes(32, "big") for v in it["lagrange"]), np.uint8).reshape(-1, 32)
    T = lam.shape[0]
    mi = refnpz[pre + "mi_shares"]
    got_m = eng.shamir_combine([[int.from_bytes(bytes(mi[t, i]), "big") for i in range(mi.shape[1])]
                                for t in range(T)], [int(v, 16) for v in it["lagrange"]])
    assert np.array_equal(np.frombuffer(b"".join(got_m), np.uint8).reshape(-1, 32), refnpz[pre + "server_m"])
    _, seeds, flags = eng.ec_combine_wire(refnpz[pre + "c1"], refnpz[pre + "pair_shares"], lam)
    assert not flags.any()
    assert np.array_equal(seeds, refnpz[pre + "server_pairs"])


def test_reconstruction_from_reference_shares(eng, ref, refnpz):
    """ServerReconstruction (shares -> seeds -> unmask, all on the GPU) reproduces final_sum."""
    import torch
    from flamingo_amd.reconstruct import ServerReconstruction
    dev = torch.device("cuda", 0)
    run = ref["runs"][0]
    it = run["iterations"][0]
    pre = f"{run['name']}_it1_"
    L = run["L"]
    seg, seeds, signs = client_table(run, it, refnpz)
    rows = eng.client_mask(seg, seeds, signs, L)[it["arrival"]]
    pitch = (L + 63) // 64 * 64
    d_rows = torch.zeros((rows.shape[0], pitch), dtype=torch.int32, device=dev)
    d_rows[:, :L] = torch.from_numpy(rows.view(np.int32)).to(dev)
    lam = np.frombuffer(b"".join(int(v, 16).to_bytes(32, "big") for v in it["lagrange"]), np.uint8).reshape(-1, 32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    psigns = np.array([r[2] for r in it["recon_symbol"]], np.int8)
    for kw in (dict(), dict(ec_cus=32, pair_queue=True)):
        rec = ServerReconstruction(eng, **kw)
        out = torch.empty(pitch, dtype=torch.int32, device=dev)
        rec.run(d_rows, L, t(lam), t(refnpz[pre + "mi_shares"]), t(refnpz[pre + "c1"]),
                t(refnpz[pre + "pair_shares"]), t(psigns), out)
        torch.cuda.synchronize()
        rec.close()
        assert digest(out[:L].cpu().numpy().view(np.uint32)) == it["final_sha256"], kw
