"""Shamir secret sharing over the P-256 group order (util/crypto/secretsharing).

The reference shares two secrets this way:
* each client's self-mask seed m_i, dealt to the committee
  (SA_ClientAgent.py:214-244) and recovered by the server from the first
  `threshold` decrypted shares (SA_ServiceAgent.py:506-526; on the GPU:
  MaskEngine.shamir_combine);
* the system decryption key, dealt by the server at setup
  (SA_ServiceAgent.py:259-279), whose Lagrange coefficients also drive the
  threshold-ElGamal combine (:542-585; on the GPU: MaskEngine.ec_combine_wire).

secret_int_to_points / points_to_secret_int / modular_lagrange_interpolation
(secretsharing/sharing.py:20-57, polynomials.py:31-109) restated: points at
x = 1..num_points, all arithmetic mod n.
"""
from __future__ import annotations

import secrets

# P-256 group order (the `prime` the reference shares over: ecchash.n)
P256_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551


def shamir_share(secret: int, threshold: int, num_points: int, prime: int = P256_N, rng=None):
    """Points (x, f(x)) for x = 1..num_points of a random degree-(threshold-1) polynomial with f(0)=secret."""
    if threshold < 1 or threshold > num_points:
        raise ValueError("need 1 <= threshold <= num_points")
    draw = (lambda: rng.randrange(prime)) if rng is not None else (lambda: secrets.randbelow(prime))
    coeffs = [secret % prime] + [draw() for _ in range(threshold - 1)]
    pts = []
    for x in range(1, num_points + 1):
        y = 0
        for c in reversed(coeffs):
            y = (y * x + c) % prime
        pts.append((x, y))
    return pts


def lagrange_at_zero(xs, prime: int = P256_N):
    """Coefficients l_j with f(0) = sum_j l_j f(x_j) mod prime."""
    out = []
    for j, xj in enumerate(xs):
        num, den = 1, 1
        for m, xm in enumerate(xs):
            if m != j:
                num = num * (-xm) % prime
                den = den * (xj - xm) % prime
        out.append(num * pow(den, -1, prime) % prime)
    return out


def shamir_recover(points, prime: int = P256_N) -> int:
    xs = [x for x, _ in points]
    return sum(l * y for l, (_, y) in zip(lagrange_at_zero(xs, prime), points)) % prime
