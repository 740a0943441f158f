"""The hash-to-curve checker (oracle/ec_oracle.py) pinned to the reference, on CPU.

ec_oracle.hash_str_to_curve is what the GPU table (flm_hash_to_curve_decimal) is compared with.
Pins: the reference's own ecchash.hash_str_to_curve output for every v < 2^16 (table digest and
sampled points, tests/golden/make_h2c_golden.py) and the h2c points logged inside the reference
agents' runs (tests/golden/ref_golden.npz, make_ref_golden.py)."""
import json
import os
from multiprocessing import Pool

import numpy as np

import ec_oracle as E
from refgold import ref, refnpz  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))


def _golden():
    with open(os.path.join(HERE, "golden", "h2c_golden.json")) as f:
        return json.load(f)


def test_h2c_oracle_matches_reference_sample_points():
    g = _golden()
    assert g["dst"] == E.DST.decode() and g["count"] == 1 << 16
    for v, hx in g["points"].items():
        assert E.wire(E.hash_str_to_curve(v)).hex() == hx, v


def _rows(bounds):
    return b"".join(E.wire(E.hash_str_to_curve(str(v))) for v in range(*bounds))


def test_h2c_oracle_full_table_matches_reference_digest():
    """All 65,536 inputs (about 10 s on 8 processes)."""
    import hashlib
    with Pool(8) as p:
        parts = p.map(_rows, [(a, a + 4096) for a in range(0, 1 << 16, 4096)])
    assert hashlib.sha256(b"".join(parts)).hexdigest() == _golden()["table_sha256"]


def test_h2c_oracle_matches_points_inside_reference_runs(ref, refnpz):
    n = 0
    for run in ref["runs"]:
        for it in run["iterations"]:
            pre = f"{run['name']}_it{it['iteration']}_"
            pts = refnpz[pre + "h2c_point"]
            hs = [h for c in it["clients"] for h in c["h"]]
            for k in range(0, len(hs), max(1, len(hs) // 50)):
                assert E.wire(E.hash_str_to_curve(hs[k])) == bytes(pts[k])
                n += 1
    assert n > 100


def test_h2c_oracle_arbitrary_messages_agree_with_host_crypto():
    """Messages other than h_ijt (non-decimal, 0..64 bytes) against flamingo_amd.crypto's
    independent form (OpenSSL point addition)."""
    from flamingo_amd import crypto as C
    rng = np.random.default_rng(7)
    for ln in (0, 1, 5, 17, 55, 56, 63, 64):
        m = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
        u0, u1 = C.hash_to_field(m, 2, C.N)
        assert E.hash_str_to_curve(m) == C.add(C.map_to_curve(u0), C.map_to_curve(u1)), ln
