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
* committee decryption shares (SA_ClientAgent.py:397-400): share = sk_j * c0;
* hash to curve as the client calls it (SA_ClientAgent.py:283-286):
  util/crypto/ecchash.py expand_message_xmd (:90-133, SHA-256), hash_to_field (:50-61, with
  modulus = n), map_to_curve (:233-275), hash_str_to_curve = Q0 + Q1 (:277-283).  Checker for
  flm_hash_to_curve*; its square root takes a^((p+1)/4) first for libnum's sqrtmod (absent here,
  so that root order is "parity unpinned"; every other step is pinned by the h2c points of the
  reference's own runs in tests/golden/ref_golden.npz and by tests/golden/h2c_golden.json).

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


# ------------------------------------------------------------- hash to curve
DST = b"QUUX-V01-CS02-with-P256_XMD:SHA-256_SSWU_RO_"      # ecchash.test_dst("P256_XMD:SHA-256_SSWU_RO_")


def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    """ecchash.py:90-133 with hashlib.sha256 (b_in_bytes 32, r_in_bytes 64)."""
    ell = (len_in_bytes + 31) // 32
    dst_prime = dst + bytes([len(dst)])
    b0 = hashlib.sha256(bytes(64) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime).digest()
    b = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(1, ell):
        b.append(hashlib.sha256(bytes(x ^ y for x, y in zip(b0, b[-1])) + bytes([i + 1]) + dst_prime).digest())
    return b"".join(b)[:len_in_bytes]


def map_to_curve(u: int):
    """ecchash.py:233-275 (Z = -10); a^((p+1)/4) as the first root of libnum.sqrtmod."""
    den = (100 * pow(u, 4, P) - 10 * pow(u, 2, P)) % P
    tv1 = pow(den, P - 2, P)                       # libnum.invmod; 0 -> 0 takes the :247-248 branch
    x1 = ((-B * pow(A, -1, P)) * (1 + tv1)) % P
    if tv1 == 0:
        x1 = B * pow(30, -1, P) % P
    gx1 = (x1 ** 3 + A * x1 + B) % P
    x2 = (-10 * pow(u, 2, P) * x1) % P
    gx2 = (x2 ** 3 + A * x2 + B) % P
    y = pow(gx1, (P + 1) // 4, P)
    x = x1
    if y * y % P != gx1:
        x, y = x2, pow(gx2, (P + 1) // 4, P)
    if (u <= 0) != (y <= 0):                       # sgn0(u) != sgn0(y), :227-232, :271-272
        y = (-y) % P
    return (x, y)


def hash_str_to_curve(msg) -> tuple | None:
    """ecchash.hash_str_to_curve(msg, 2, n, 1, 48, XMDExpander(DST, sha256, 128))."""
    m = msg.encode() if isinstance(msg, str) else bytes(msg)
    ub = expand_message_xmd(m, DST, 96)
    u0, u1 = (int.from_bytes(ub[48 * i: 48 * i + 48], "big") % N for i in range(2))
    return add(map_to_curve(u0), map_to_curve(u1))


def h2c_table_digest(points) -> str:
    """SHA-256 over the 64-byte wire encodings of a table of points (infinity = 64 zeros)."""
    h = hashlib.sha256()
    for pt in points:
        h.update(wire(pt))
    return h.hexdigest()
