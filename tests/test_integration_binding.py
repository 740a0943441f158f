"""integration/util_flm.py -- the reference-side binding (util/flm.py) -- against the library and
against the reference's own round (tests/golden/make_ref_golden.py fixtures).

CPU: the file loads libflamingo_hip.so by path and binds every symbol it uses.
GPU: each helper, called the way the edited SA_ServiceAgent / SA_ClientAgent call it, gives the
reference's y_i, recovered keys and final_sum."""
from __future__ import annotations

import collections
import importlib.util
import os

import numpy as np
import pytest

from refgold import client_inputs, client_table, digest, iterations, ref, refnpz, server_table  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
Pt = collections.namedtuple("Pt", "x y")


def load_binding(monkeypatch, gpus=None):
    monkeypatch.setenv("FLM_LIB", os.path.join(ROOT, "flamingo_amd", "lib", "libflamingo_hip.so"))
    if gpus is not None:
        monkeypatch.setenv("FLM_GPUS", str(gpus))
    import torch  # noqa: F401  (one HIP runtime per process: torch's, loaded first)
    spec = importlib.util.spec_from_file_location("util_flm", os.path.join(ROOT, "integration", "util_flm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_binding_loads_and_binds(monkeypatch):
    flm = load_binding(monkeypatch)
    for name in ("flm_aggregate_unmask", "flm_client_mask", "flm_shamir_combine", "flm_ec_combine",
                 "flm_group_aggregate_unmask", "flm_store_create", "flm_store_add", "flm_store_partial",
                 "flm_store_unmask", "flm_store_reset", "flm_store_free", "flm_hash_to_curve",
                 "flm_hash_to_curve_decimal"):
        assert getattr(flm._lib, name).argtypes


def test_binding_body_guard(monkeypatch):
    """util_flm's VECTOR-body guard (no GPU call): 32-bit integer vectors of length L pass as uint32
    views; float, 64-bit, 2-D and wrong-length bodies are refused (the reference's uint32 += raises)."""
    flm = load_binding(monkeypatch)
    L = 8
    assert flm._u32_body(np.arange(L, dtype=np.int32), L).dtype == np.uint32
    assert flm._u32_body(np.arange(L, dtype=np.uint32), L) is not None
    for bad in (np.arange(L, dtype=np.float32), np.arange(L, dtype=np.int64), np.zeros((2, L), np.uint32),
                np.arange(L - 1, dtype=np.uint32)):
        assert flm._u32_body(bad, L) is None


@pytest.mark.gpu
def test_binding_reproduces_reference_round(monkeypatch, ref, refnpz):
    flm = load_binding(monkeypatch)
    run = ref["runs"][0]
    it = run["iterations"][0]
    L = run["L"]
    seg, seeds, signs = client_table(run, it, refnpz)
    # SA_ClientAgent.sendVectors with the edit: one client_mask call per client
    rows = {}
    for c in it["clients"][:32]:
        i = c["id"]
        v = flm.client_mask([bytes(s) for s in seeds[seg[i]:seg[i + 1]]], signs[seg[i]:seg[i + 1]], L)
        assert digest(v) == c["y_sha256"]
    eng_rows = None
    from flamingo_amd import MaskEngine
    with MaskEngine(0) as eng:
        eng_rows = eng.client_mask(seg, seeds, signs, L)
    rows = [eng_rows[i] for i in it["arrival"]]
    # SA_ServiceAgent.reconstruction_process with the edit: keys recovered from the decryptors' shares
    pre = "A_it1_"
    lam = [int(v, 16) for v in it["lagrange"]]
    mi = refnpz[pre + "mi_shares"]
    m_keys = flm.shamir_combine([[int.from_bytes(bytes(mi[t, i]), "big") for i in range(mi.shape[1])]
                                 for t in range(len(lam))], lam)
    assert b"".join(m_keys) == refnpz[pre + "server_m"].tobytes()
    pt = lambda w: Pt(int.from_bytes(bytes(w[:32]), "big"), int.from_bytes(bytes(w[32:]), "big"))
    sh = refnpz[pre + "pair_shares"]
    p_keys = flm.ec_combine([pt(w) for w in refnpz[pre + "c1"]],
                            [[pt(w) for w in sh[t]] for t in range(sh.shape[0])], lam)
    assert b"".join(p_keys) == refnpz[pre + "server_pairs"].tobytes()
    out = flm.aggregate_unmask(rows, m_keys + p_keys, [-1] * len(m_keys) + [r[2] for r in it["recon_symbol"]], L)
    assert digest(out) == it["final_sha256"]
    # the device-resident form of the same server edit: bodies stored at receiveMessage, S at
    # report_process, masks added at reconstruction_process
    st = flm.VectorStore(L, len(rows))
    for sender, v in zip(it["arrival"], rows):
        st.add(sender, v)
    st.partial()
    out2 = st.unmask(m_keys + p_keys, [-1] * len(m_keys) + [r[2] for r in it["recon_symbol"]])
    assert digest(out2) == it["final_sha256"]
    st.reset()
    st.add(0, rows[0][:-1])
    with pytest.raises(RuntimeError, match="incorrect length"):
        st.partial()
    st.reset()
    st.add(0, rows[0].astype(np.float64))      # the reference's uint32 += refuses it: never truncated
    with pytest.raises(RuntimeError, match="incorrect length"):
        st.partial()
    with pytest.raises(RuntimeError, match="incorrect length"):
        flm.aggregate_unmask([rows[0].astype(np.float32)], [], [], L)
    st.close()
    assert st.h is None


@pytest.mark.gpu
def test_binding_hash_to_curve_matches_reference(monkeypatch, ref, refnpz):
    """The client edit at SA_ClientAgent.py:283-286: flm.hash_str_to_curve(h_ijt) gives the points the
    reference's own ecchash produced in run A (.x / .y as the EccPoint it replaces)."""
    flm = load_binding(monkeypatch)
    run = ref["runs"][0]
    it = run["iterations"][0]
    pts = refnpz[f"{run['name']}_it{it['iteration']}_h2c_point"]
    hs = [h for c in it["clients"] for h in c["h"]]
    for k in range(0, len(hs), 7):
        p = flm.hash_str_to_curve(hs[k])
        assert p.x.to_bytes(32, "big") + p.y.to_bytes(32, "big") == bytes(pts[k])
    import ec_oracle as E
    q = flm.hash_str_to_curve("abcdeefekf")                 # the ecchash.py:303 demo message (not a table key)
    assert (q.x, q.y) == E.hash_str_to_curve("abcdeefekf")
