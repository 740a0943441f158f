"""Parity against fixtures produced by the REFERENCE'S OWN CODE (tests/golden/make_ref_golden.py).

These pin (1) the oracle -- the C/numpy restatement every GPU parity test
compares against -- and (2) the host-side product logic (graph and committee
order, dropout-pair order, the pair-seed pipeline, Lagrange coefficients, the
JSON wire formats) to what eniac/flamingo's util/param.py, util/util.py,
util/crypto and agent/flamingo/SA_*Agent.py computed on identical seeds and
inputs.  The HIP path is pinned to the same fixtures in
tests/test_ref_golden_gpu.py.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
import ec_oracle as E
from flamingo_amd import crypto as C
from flamingo_amd import params as P
from flamingo_amd.abides.flamingo import seeds as S
from flamingo_amd.abides.flamingo import wire as W

from refgold import (client_inputs, client_table, digest, iterations, key_scalar,  # noqa: F401
                     ref, refnpz, server_table)

P256_N = E.N


# ------------------------------------------------------------- util/param.py
def test_fixture_comes_from_the_reference(ref):
    assert "/root/reference" in ref["generator"] and "SA_" in ref["generator"]


@pytest.mark.parametrize("n", [128, 1024, 4096])
def test_committee_order_matches_reference(ref, n):
    want = next(c["iter_order"] for c in ref["committee"] if c["num_clients"] == n)
    got = P.choose_committee(bytes(32), 60, n, encrypt=O.chacha20_encrypt)
    assert list(got) == want                     # same members, same set iteration order


def test_graphs_match_reference_in_set_order(ref):
    for g in ref["graphs"]:
        n, o, it = g["num_clients"], g["neighborhood_size"], g["iteration"]
        nb = [list(s) for s in P.neighbor_graph(bytes(32), it, n, o, encrypt=O.chacha20_encrypt)]
        assert hashlib.sha256(json.dumps([sorted(s) for s in nb]).encode()).hexdigest() == g["sorted_sha256"]
        assert hashlib.sha256(json.dumps(nb).encode()).hexdigest() == g["iter_order_sha256"]
        if "neighbors" in g:
            assert nb == g["neighbors"]


def test_client_neighbour_order_matches_sendvectors(ref):
    for run, it in iterations(ref):
        nb = P.neighbor_graph(bytes(32), it["iteration"], run["N"], run["neighborhood_size"],
                              encrypt=O.chacha20_encrypt)
        for c in it["clients"]:
            assert list(nb[c["id"]]) == c["neighbors"]


def test_dropout_pairs_match_recon_symbol_order(ref):
    """SA_ServiceAgent.report_process (:341-380): the product's pairs, in the reference's order."""
    for run, it in iterations(ref):
        N = run["N"]
        nb = P.neighbor_graph(bytes(32), it["iteration"], N, run["neighborhood_size"], encrypt=O.chacha20_encrypt)
        online = [i for i in range(N) if i not in it["offline"]]
        pairs, signs = P.dropout_pairs(nb, online, it["offline"])
        assert [[a, b, s] for (a, b), s in zip(pairs, signs)] == it["recon_symbol"]
        opairs, osigns = O.dropout_pairs(bytes(32), it["iteration"], N, run["neighborhood_size"], set(online))
        assert [[a, b, s] for (a, b), s in zip(opairs, osigns)] == it["recon_symbol"]


# --------------------------------------------------------- oracle vs reference
def test_oracle_client_vectors_match_reference(ref, refnpz):
    """Every client's masked vector y_i (SA_ClientAgent.py:304-324) from the oracle == the reference's."""
    for run, it in iterations(ref):
        seg, seeds, signs = client_table(run, it, refnpz)
        rows = O.client_mask(seg, seeds, signs, run["L"], x=client_inputs(run, it), threads=8)
        assert [digest(r) for r in rows] == [c["y_sha256"] for c in it["clients"]]


def test_oracle_server_round_matches_reference(ref, refnpz):
    """vec_sum_partial, mi_vec, cancel_vec and final_sum of report/reconstruction_process."""
    for run, it in iterations(ref):
        seg, seeds, signs = client_table(run, it, refnpz)
        rows = O.client_mask(seg, seeds, signs, run["L"], x=client_inputs(run, it), threads=8)
        sm, sp, sseeds, ssigns = server_table(it, refnpz, run)
        U = rows[it["arrival"]]
        assert digest(O.aggregate_unmask(U, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8))) == it["S_sha256"]
        M = O.aggregate_unmask(np.zeros((0, run["L"]), np.uint32), sm, -np.ones(sm.shape[0], np.int8), L=run["L"])
        assert digest(M) == it["M_sha256"]
        Cv = O.aggregate_unmask(np.zeros((0, run["L"]), np.uint32), sp, ssigns[sm.shape[0]:], L=run["L"])
        assert digest(Cv) == it["C_sha256"]
        final = O.aggregate_unmask(U, sseeds, ssigns, threads=8)
        assert digest(final) == it["final_sha256"]
        assert final[:8].tolist() == it["final_head"]


def test_server_keys_are_the_clients_seeds(ref, refnpz):
    """The m_i / s_ij the server recovered from shares (:506-526, :542-585) are the clients' own seeds."""
    for run, it in iterations(ref):
        pre = f"{run['name']}_it{it['iteration']}_"
        m = refnpz[pre + "m"]
        assert np.array_equal(refnpz[pre + "server_m"], m[it["arrival"]])
        s, seg = refnpz[pre + "s"], refnpz[pre + "pair_seg"]
        for k, (i, j, _) in enumerate(it["recon_symbol"]):
            c = it["clients"][i]
            assert np.array_equal(refnpz[pre + "server_pairs"][k], s[seg[i] + c["neighbors"].index(j)])


# ------------------------------------------------ seed recovery vs reference
def test_lagrange_coefficients_match_reference(ref):
    for run, it in iterations(ref):
        assert [hex(v) for v in S.lagrange_at_zero(it["decryptor_x"])] == it["lagrange"]


def test_ec_oracle_recovers_reference_seeds(ref, refnpz):
    """ec_oracle's combine on the decryptors' own shares == the s_ij reconstruction_process derived."""
    run = ref["runs"][0]
    it = run["iterations"][0]
    pre = f"{run['name']}_it1_"
    lam = [int(v, 16) for v in it["lagrange"]]
    sh = refnpz[pre + "pair_shares"]
    c1 = refnpz[pre + "c1"]
    pt = lambda w: (int.from_bytes(bytes(w[:32]), "big"), int.from_bytes(bytes(w[32:]), "big"))
    got = []
    for d in range(c1.shape[0]):
        acc = None
        for t in range(sh.shape[0]):
            acc = E.add(acc, E.mul(lam[t], pt(sh[t, d])))
        h = E.add(pt(c1[d]), E.neg(acc))
        got.append(hashlib.sha256(h[0].to_bytes(32, "big") + h[1].to_bytes(32, "big")).digest())
    assert np.array_equal(np.frombuffer(b"".join(got), np.uint8).reshape(-1, 32), refnpz[pre + "server_pairs"])
    mi = refnpz[pre + "mi_shares"]
    ms = [sum(lam[t] * int.from_bytes(bytes(mi[t, i]), "big") for t in range(len(lam))) % P256_N
          for i in range(mi.shape[1])]
    assert np.array_equal(np.frombuffer(b"".join(v.to_bytes(32, "big") for v in ms), np.uint8).reshape(-1, 32),
                          refnpz[pre + "server_m"])


# --------------------------------------------- pair-seed pipeline (f3) vs reference
def test_pair_seed_pipeline_matches_reference(ref, refnpz):
    """ECDH -> SHA-256 -> h_ijt -> hash-to-curve -> SHA-256 (SA_ClientAgent.py:256-292) through
    flamingo_amd.crypto, against the r_ij, h_ijt, points and s_ij the reference produced."""
    run = ref["runs"][0]
    keys = {}
    for it in run["iterations"]:
        pre = f"{run['name']}_it{it['iteration']}_"
        r, s, pts = refnpz[pre + "r"], refnpz[pre + "s"], refnpz[pre + "h2c_point"]
        for c in it["clients"][:24]:
            i = c["id"]
            for j, h_ref in zip(c["neighbors"], c["h"]):
                a = keys.setdefault(i, key_scalar(f"pki_files/client{i}.pem"))
                b = keys.setdefault(j, key_scalar(f"pki_files/client{j}.pem"))
                k = refnpz[pre + "pair_seg"][i] + c["neighbors"].index(j)
                rij = hashlib.sha256(C.point_bytes(C.mul(a, C.mul(b)))).digest()
                assert rij == bytes(r[k])
                hb = O.chacha20_encrypt(rij, it["iteration"].to_bytes(16, "big"))
                h = str(int.from_bytes(hb[:4], "big") & 0xFFFF)
                assert h == h_ref
                H = C.hash_str_to_curve(h)
                assert C.point_bytes(H) == bytes(pts[k])
                assert hashlib.sha256(C.point_bytes(H)).digest() == bytes(s[k])


# ------------------------------------------------------ wire formats (f4)
def test_wire_formats_match_reference_json(ref):
    """flamingo_amd wire.py re-serialises util/util.py:179-252 JSON of real messages byte for byte."""
    w = ref["runs"][0]["iterations"][0]["wire"]
    assert W.serialize_tuples_bytes(W.deserialize_tuples_bytes(w["enc_mi_shares"])) == w["enc_mi_shares"]
    assert W.serialize_dim1_elgamal(W.deserialize_dim1_elgamal(w["enc_pairwise"])) == w["enc_pairwise"]
    assert W.serialize_dim1_ecp(W.deserialize_dim1_ecp(w["shared_result_pairwise"])) == w["shared_result_pairwise"]
    assert W.serialize_dim1_list(W.deserialize_dim1_list(w["shared_result_mi"])) == w["shared_result_mi"]
    assert W.serialize_dim2_ecp(W.deserialize_dim2_ecp(w["dim2_ecp"])) == w["dim2_ecp"]
    # and the GPU wire-array forms agree with the parsed points
    keys, c0, c1 = W.elgamal_json_to_wire(w["enc_pairwise"])
    d = W.deserialize_dim1_elgamal(w["enc_pairwise"])
    assert keys == list(d.keys())
    assert [C.point_bytes(v[0]) for v in d.values()] == [bytes(r) for r in c0]
    assert W.wire_to_ecp_json(W.ecp_json_to_wire(w["shared_result_pairwise"])) == w["shared_result_pairwise"]


def test_pair_prf_matches_reference_h(ref, refnpz):
    """The client agent's h_ijt (client_agent.pair_prf: PRG word 0 of each r_ij, one batch, XOR t)
    against the h_ijt the reference's clients printed (SA_ClientAgent.py:276-283), every pair of
    run A's two iterations; the PRG here is the C oracle standing in for the GPU."""
    from flamingo_amd.abides.flamingo.client_agent import pair_prf

    class OraclePRG:
        def prg_expand(self, seeds, L, slot0=0):
            return np.stack([O.prg(bytes(x), L, slot0) for x in seeds])

    run = ref["runs"][0]
    for it in run["iterations"]:
        r = refnpz[f"{run['name']}_it{it['iteration']}_r"]
        got = pair_prf(OraclePRG(), [bytes(x) for x in r], it["iteration"])
        assert got == [h for c in it["clients"] for h in c["h"]], it["iteration"]
