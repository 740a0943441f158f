"""Seed transport for the Flamingo agents: real Shamir sharing, stand-in encryption.

The reference protects the two kinds of mask seeds with public-key crypto:
* self-mask seed m_i: Shamir-shared over the P-256 group order n to the
  committee, each share AES-GCM encrypted under an ECDH key
  (SA_ClientAgent.py:214-244); the server Lagrange-interpolates the first
  `threshold` decrypted shares (SA_ServiceAgent.py:506-526).
* pairwise seed s_ij: ECDH -> SHA-256 -> ChaCha20 PRF of the iteration ->
  hash-to-curve -> SHA-256 (SA_ClientAgent.py:256-292), ElGamal-encrypted to
  the committee's threshold key and decrypted only for dropout pairs
  (SA_ServiceAgent.py:542-585).

Those EC/AES steps are outside this repository's hot path.
Here the Shamir sharing and Lagrange recovery of m_i are real (mod n, so the
reference's m_i mod n behaviour is kept), while share "encryption" and the
pairwise-seed derivation are explicit stand-ins: shares travel as integers and
s_ij = SHA-256(b"flm-pair" || root || iteration || min(i,j) || max(i,j)).
"""
from __future__ import annotations

import hashlib
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


def pair_seed(root_seed: bytes, iteration: int, i: int, j: int) -> bytes:
    """Stand-in for the reference's s_ij (symmetric in i, j; new every iteration)."""
    a, b = (i, j) if i < j else (j, i)
    return hashlib.sha256(b"flm-pair" + root_seed + iteration.to_bytes(8, "big") + a.to_bytes(4, "big")
                          + b.to_bytes(4, "big")).digest()
