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


@pytest.mark.parametrize("run_idx", [0, 3])
def test_gpu_ecdh_pair_seeds_match_reference(eng, ref, refnpz, run_idx):
    """The whole pair-seed pipeline (SA_ClientAgent.py:256-292) on the GPU, every pair of every
    client in every iteration: public keys b_j G and the ECDH points a_i (b_j G) by the batched
    flm_ec_mul the protocol uses (protocol._ecdh_batch), r_ij = SHA-256 of the point
    (flm_ec_combine with no shares: point = c1, seed = SHA-256(c1)), h_ijt from ChaCha20 (and by
    the client agent's batched pair_prf), H = hash-to-curve from the one-launch table of all 2^16
    h values (flm_hash_to_curve_decimal), s_ij = SHA-256(H) -- against the r_ij, h_ijt, H and s_ij
    the reference's clients derived from refshim's deterministic pki keys.  Run D is N = 1024,
    -o 2: ~40k pairs per iteration."""
    from flamingo_amd import crypto as C
    from flamingo_amd.abides.flamingo.client_agent import pair_prf
    from refgold import key_scalar
    run = ref["runs"][run_idx]
    N = run["N"]
    keys = [key_scalar(f"pki_files/client{i}.pem") for i in range(N)]
    g = np.tile(np.frombuffer(C.point_bytes(C.G), np.uint8), (N, 1))
    pub, fl = eng.ec_mul_wire(g, C.scalars_to_wire(keys))               # A_j = b_j G, on the GPU
    assert not fl.any()
    table, tfl = eng.hash_to_curve_decimal(0, 1 << 16)
    assert not tfl.any()
    none_sh, none_l = np.zeros((0, 1, 64), np.uint8), np.zeros((0, 32), np.uint8)
    for it in run["iterations"]:
        pre = f"{run['name']}_it{it['iteration']}_"
        pairs = [(c["id"], j) for c in it["clients"] for j in c["neighbors"]]
        pts, fl = eng.ec_mul_wire(pub[[j for _, j in pairs]], C.scalars_to_wire([keys[i] for i, _ in pairs]))
        assert not fl.any()
        _, r, _ = eng.ec_combine_wire(pts, none_sh.reshape(0, len(pairs), 64), none_l, negate=False)
        assert np.array_equal(r, refnpz[pre + "r"]), it["iteration"]
        hs = pair_prf(eng, [bytes(x) for x in r], it["iteration"])      # PRG word 0 of every r_ij, one launch
        assert hs == [h for c in it["clients"] for h in c["h"]]
        if run_idx == 0:                                                 # the per-key ChaCha20 form too
            assert hs == [str(int.from_bytes(eng.chacha20_encrypt(bytes(x), it["iteration"].to_bytes(16, "big"))[:4],
                                             "big") & 0xFFFF) for x in r]
        H = table[np.array([int(h) for h in hs])]
        assert np.array_equal(H, refnpz[pre + "h2c_point"]), it["iteration"]
        _, s, _ = eng.ec_combine_wire(H, none_sh.reshape(0, len(hs), 64), none_l, negate=False)
        assert np.array_equal(s, refnpz[pre + "s"]), it["iteration"]


def test_device_resident_server_matches_reference(eng, ref, refnpz):
    """The drop-in server's device path (flamingo_amd.ingest.VectorStore: rows stored at arrival,
    S kept on the GPU, masks added over it) reproduces the reference's S and final_sum."""
    from flamingo_amd.ingest import VectorStore
    for run, it in iterations(ref):
        L = run["L"]
        seg, seeds, signs = client_table(run, it, refnpz)
        rows = eng.client_mask(seg, seeds, signs, L, x=client_inputs(run, it))
        st = VectorStore(eng, L, len(it["arrival"]))
        for i in it["arrival"]:
            st.add(i, rows[i])
        st.partial_sum()
        st.wait_partial()
        assert digest(st.host_partial()) == it["S_sha256"]
        _, _, sseeds, ssigns = server_table(it, refnpz, run)
        assert digest(st.unmask(sseeds, ssigns)) == it["final_sha256"], (run["name"], it["iteration"])
