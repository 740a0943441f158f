"""TEST INFRASTRUCTURE ONLY -- pure-Python P-256 restatement of Flamingo's seed recovery.

Checker for flm_ec_mul / flm_ec_combine (flamingo_amd/csrc/flm_p256.hip); never
imported by the product path.  Restates, in plain affine integer arithmetic:

* the server's threshold-ElGamal combine and key derivation,
  SA_ServiceAgent.py:542-585:
      sum_df = -(sum_j share_j * lambda_j);  sum_df = sum_df + c1
      seed   = SHA256(int(x).to_bytes(32,'big') + int(y).to_bytes(32,'big'))[:32]
* the Lagrange coefficients of points_to_secret_int
  (util/crypto/secretsharing/polynomials.py modular_lagrange_interpolation, at x = 0, mod n);
* ElGamal encryption (SA_ClientAgent.py:434-447): c0 = r*G, c1 = h + r*pk;
* committee decryption shares (SA_ClientAgent.py:397-400): share = sk_j * c0.

Pins: tests/test_ec_cpu.py checks this arithmetic against OpenSSL's
independent P-256 (EC_POINT_mul / EC_POINT_add) and against the group law
(n*G = infinity, (a+b)G = aG + bG), and
tests/test_ref_golden_cpu.py::test_ec_oracle_recovers_reference_seeds checks it
recovers, from the reference's own decryptors' shares, the exact keys the
reference's reconstruction_process derived (tests/golden/make_ref_golden.py).
"""
from __future__ import annotations

import hashlib

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
A = P - 3
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
G = (0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
     0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5)


def on_curve(pt) -> bool:
    return pt is None or (pt[1] ** 2 - pt[0] ** 3 - A * pt[0] - B) % P == 0


def add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = (3 * x1 * x1 + A) * pow(2 * y1, -1, P) % P
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def mul(k: int, pt=G):
    """k * pt by double-and-add over the bits of k (k taken as is, not reduced)."""
    acc = None
    for bit in bin(k)[2:] if k > 0 else "":
        acc = add(acc, acc)
        if bit == "1":
            acc = add(acc, pt)
    return acc


def wire(pt) -> bytes:
    """64-byte x||y big endian; infinity -> 64 zero bytes (pycryptodome's EccPoint(0, 0))."""
    if pt is None:
        return bytes(64)
    return pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")


def lagrange_at_zero(xs, prime: int = N):
    out = []
    for j, xj in enumerate(xs):
        num, den = 1, 1
        for m, xm in enumerate(xs):
            if m != j:
                num = num * (-xm) % prime
                den = den * (xj - xm) % prime
        out.append(num * pow(den, -1, prime) % prime)
    return out


def combine(c1, shares_by_term, lambdas, negate: bool = True):
    """point_i = c1_i -/+ sum_j lambda_j * shares[j][i]; seed_i = SHA256(wire(point_i))."""
    D = len(c1) if c1 is not None else len(shares_by_term[0])
    points, seeds = [], []
    for i in range(D):
        s = None
        for j, lam in enumerate(lambdas):
            s = add(s, mul(lam, shares_by_term[j][i]))
        if negate:
            s = neg(s)
        pt = add(c1[i], s) if c1 is not None else s
        points.append(pt)
        seeds.append(hashlib.sha256(wire(pt)).digest())
    return points, seeds


def elgamal_encrypt(pk, h, r: int):
    return mul(r), add(h, mul(r, pk))
