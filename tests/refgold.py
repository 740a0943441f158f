"""Shared loaders for the reference-produced fixtures (tests/golden/make_ref_golden.py)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
P256_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(HERE, "golden", "ref_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def refnpz():
    return dict(np.load(os.path.join(HERE, "golden", "ref_golden.npz")))


def digest(v) -> str:
    return hashlib.sha256(np.ascontiguousarray(v, dtype="<u4").tobytes()).hexdigest()


def x_input(seed: int, it: int, cid: int, L: int) -> np.ndarray:
    """Same recipe as make_ref_golden.x_input (recorded in the fixture's `input` field)."""
    return np.random.Generator(np.random.PCG64([seed, it, cid])).integers(0, 2**32, size=L, dtype=np.uint32)


def key_scalar(name: str) -> int:
    """tests/golden/refshim.key_scalar: the deterministic private key per pki_files/ name."""
    return int.from_bytes(hashlib.sha512(b"refgolden-pki-" + name.encode()).digest(), "big") % (P256_N - 1) + 1


def iterations(ref):
    for run in ref["runs"]:
        for it in run["iterations"]:
            yield run, it


def client_table(run, it, npz):
    """CSR seed table of every client's y_i in the reference's own neighbour order (SA_ClientAgent.py:304-324)."""
    pre = f"{run['name']}_it{it['iteration']}_"
    m, s = npz[pre + "m"], npz[pre + "s"]
    seeds, signs, seg = [], [], [0]
    k = 0
    for c in it["clients"]:
        seeds.append(m[c["id"]])
        signs.append(1)
        for j in c["neighbors"]:
            seeds.append(s[k])
            signs.append(1 if c["id"] < j else -1)
            k += 1
        seg.append(len(seeds))
    assert k == s.shape[0]
    return np.array(seg, np.int64), np.stack(seeds), np.array(signs, np.int8)


def client_inputs(run, it):
    if run["input"].startswith("ones"):
        return None
    seed = int(run["input"].split("(")[1].split(",")[0])
    return np.stack([x_input(seed, it["iteration"], i, run["L"]) for i in range(run["N"])])


def server_table(it, npz, run):
    pre = f"{run['name']}_it{it['iteration']}_"
    sm, sp = npz[pre + "server_m"], npz[pre + "server_pairs"]
    seeds = np.concatenate([sm, sp]) if sp.size else sm
    signs = np.array([-1] * sm.shape[0] + [r[2] for r in it["recon_symbol"]], np.int8)
    return sm, sp, seeds, signs


