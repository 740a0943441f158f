"""Golden hash-to-curve table produced BY THE REFERENCE'S OWN CODE (build container only).

Imports util/crypto/ecchash.py read-only from /root/reference, with the absent third-party
modules (pycryptodomex's ECC point, libnum) replaced by tests/golden/refshim.py, and runs
ecchash.hash_str_to_curve exactly as the client calls it (SA_ClientAgent.py:283-286):

    hash_str_to_curve(msg=h_ijt, count=2, modulus=n (the client's self.prime), degree=ecchash.m,
                      blen=ecchash.L, expander=XMDExpander(test_dst("P256_XMD:SHA-256_SSWU_RO_"),
                                                           hashlib.sha256, ecchash.k))

for every h_ijt the client can produce -- str(x & 0xFFFF) (:280), i.e. str(v) for v < 2^16 --
and records (tests/golden/h2c_golden.json):
  * table_sha256: SHA-256 over the 65,536 64-byte wire encodings x||y (big endian) in v order;
  * points: the wire encoding (hex) of v = 0..63, every 257th v, and 65535.
The one convention refshim assumes rather than reproduces is libnum's sqrtmod root order (see
refshim.py's header): the table is pinned to the reference's code under that assumption.

Reproduce:  python tests/golden/make_h2c_golden.py   (~1-2 min on 8 cores)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
N_ORDER = 115792089210356248762697446949407573529996955224135760342422259061068512044369  # ecchash.n
ALL = 1 << 16


def _setup():
    sys.path.insert(0, HERE)
    import refshim
    refshim.install()
    sys.path.insert(0, REF)
    from util.crypto import ecchash
    return ecchash


def _chunk(bounds):
    ecchash = _setup()
    dst = ecchash.test_dst("P256_XMD:SHA-256_SSWU_RO_")
    out = []
    for v in range(*bounds):
        pt = ecchash.hash_str_to_curve(msg=str(v), count=2, modulus=N_ORDER, degree=ecchash.m, blen=ecchash.L,
                                       expander=ecchash.XMDExpander(dst, hashlib.sha256, ecchash.k))
        out.append(int(pt.x).to_bytes(32, "big") + int(pt.y).to_bytes(32, "big"))
    return out


def main():
    step = 1024
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        parts = pool.map(_chunk, [(a, min(a + step, ALL)) for a in range(0, ALL, step)])
    rows = [r for p in parts for r in p]
    assert len(rows) == ALL
    sample = sorted(set(range(64)) | set(range(0, ALL, 257)) | {ALL - 1})
    rec = {"what": "ecchash.hash_str_to_curve(str(v), 2, n, 1, 48, XMD SHA-256) for v < 2^16, "
                   "by the reference's own util/crypto/ecchash.py (refshim stand-ins for pycryptodomex/libnum)",
           "dst": ecchash_dst(),
           "count": ALL,
           "table_sha256": hashlib.sha256(b"".join(rows)).hexdigest(),
           "parity": PARITY_NOTE,
           "points": {str(v): rows[v].hex() for v in sample}}
    with open(os.path.join(HERE, "h2c_golden.json"), "w") as f:
        json.dump(rec, f, indent=0, sort_keys=True)
    print("table_sha256", rec["table_sha256"], len(rec["points"]), "sample points")


PARITY_NOTE = ("parity unpinned: libnum's sqrtmod root order (ecchash.py:263-268) -- the table assumes the root a^((p+1)/4) is yielded first; libnum is absent here and no reference-held fixture pins it")


def ecchash_dst():
    return _setup().test_dst("P256_XMD:SHA-256_SSWU_RO_")


if __name__ == "__main__":
    main()
