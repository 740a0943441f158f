"""Synthetic Flamingo rounds whose seed recovery is real (bench.py and tests only).

A round built here has the structure the reference's server sees in
reconstruction_process (SA_ServiceAgent.py:499-605):

* every pair seed is s_ij = SHA-256(x || y) of a group element H_ij
  (SA_ClientAgent.py:283-292).  H_ij = h_ij * G with h_ij taken from
  params.synthetic_pair_seed, which stands in for hash-to-curve of h_ijt;
* each dropout pair's H is ElGamal-encrypted to a system key whose Shamir
  shares are held by T committee members, and those members' decryption
  shares sk_j * c0 are given (SA_ClientAgent.py:397-400, 434-447);
* each online client's m_i is given as T Shamir shares y_{j,i}
  (SA_ClientAgent.py:214-224, decrypted: :402-420) with
  sum_j lambda_j y_{j,i} = m_i mod n.

So recovering the seeds on the GPU and unmasking must give out == |U| for
all-ones inputs, with no stand-in left between shares and sum.  The
scalar multiplications that build the inputs run on the GPU (flm_ec_mul).
"""
from __future__ import annotations

import hashlib
import random

import numpy as np

from . import crypto as C
from . import params as P
from .abides.flamingo.seeds import lagrange_at_zero, shamir_share


def _g_rows(n: int) -> np.ndarray:
    return np.tile(np.frombuffer(C.point_bytes(C.G), np.uint8), (n, 1))


def pair_points(eng, pairs, cache: dict | None = None) -> dict:
    """{(a, b): (H wire row (64,), s_ab 32 bytes)} for unordered pairs a < b, computed in one GPU batch."""
    cache = {} if cache is None else cache
    todo = sorted({(min(i, j), max(i, j)) for i, j in pairs} - set(cache))
    if todo:
        ks = [int.from_bytes(P.synthetic_pair_seed(a, b), "big") % (C.N - 1) + 1 for a, b in todo]
        H, _ = eng.ec_mul_wire(_g_rows(len(todo)), C.scalars_to_wire(ks))
        for k, ab in enumerate(todo):
            cache[ab] = (H[k].copy(), hashlib.sha256(H[k].tobytes()).digest())
    return cache


def recovery_round(eng, m: np.ndarray, nbrs: list, online, offline, T: int = 20, committee: int = 60,
                   seed: int = 0, point_cache: dict | None = None) -> dict:
    """Client seed table, server seeds, and the recovery inputs of one round.

    m: (N, 32) self-mask seeds (each must be < n as a big-endian integer, like the
    reference's m_i, which the server recovers mod n).  Returns host arrays:
      seg, client_seeds, client_signs     -- for flm_client_mask (rows of all clients)
      server_seeds, server_signs          -- the K = |U| + D seeds the recovery must reproduce
      lambdas (T, 32), mi_shares (T, M, 32), c1 (D, 64), pair_shares (T, D, 64), pair_signs (D,)
    """
    rng = random.Random(seed)
    N = m.shape[0]
    edges = [(i, j) for i in range(N) for j in nbrs[i] if i < j]
    pts = pair_points(eng, edges, point_cache)

    def s_of(i, j):
        return pts[(min(i, j), max(i, j))][1]

    seg, cs, csg = P.client_seed_table(m, nbrs, s_of)
    online = [int(i) for i in online]
    ss, sg = P.server_seed_table(m, nbrs, online, offline, s_of)
    pairs, psigns = P.dropout_pairs(nbrs, online, offline)
    M, D = len(online), len(pairs)

    # committee key, its Shamir shares, T decryptors and their Lagrange coefficients
    sk = rng.randrange(1, C.N)
    members = sorted(rng.sample(range(1, committee + 1), T))
    sk_share = dict(shamir_share(sk, T, committee, rng=rng))
    lam = lagrange_at_zero(members)

    # m_i as T shares: T-1 random, the last solved so that sum_j lambda_j y_j = m_i (mod n)
    inv_last = pow(lam[-1], -1, C.N)
    ys = np.zeros((T, M, 32), np.uint8)
    for col, i in enumerate(online):
        mi = int.from_bytes(m[i].tobytes(), "big")
        if mi >= C.N:
            raise ValueError(f"m_{i} >= n: the reference would recover m_i mod n and not cancel the mask")
        vals = [rng.randrange(0, C.N) for _ in range(T - 1)]
        acc = sum(l * v for l, v in zip(lam, vals)) % C.N
        vals.append((mi - acc) * inv_last % C.N)
        ys[:, col, :] = C.scalars_to_wire(vals)

    c1 = np.zeros((D, 64), np.uint8)
    dec = np.zeros((T, D, 64), np.uint8)
    if D:
        pk, _ = eng.ec_mul_wire(_g_rows(1), C.scalars_to_wire([sk]))
        rs = [rng.randrange(1, C.N) for _ in range(D)]
        c0, _ = eng.ec_mul_wire(_g_rows(D), C.scalars_to_wire(rs))
        rpk, _ = eng.ec_mul_wire(np.tile(pk, (D, 1)), C.scalars_to_wire(rs))
        H = np.stack([pts[(min(i, j), max(i, j))][0] for i, j in pairs])
        c1, _, _ = eng.ec_combine_wire(H, rpk[None], C.scalars_to_wire([1]), negate=False)   # H + r pk
        d, _ = eng.ec_mul_wire(np.tile(c0, (T, 1)),
                               C.scalars_to_wire([sk_share[x] for x in members for _ in range(D)]))
        dec = d.reshape(T, D, 64)
    return {"seg": seg, "client_seeds": cs, "client_signs": csg, "server_seeds": ss, "server_signs": sg,
            "lambdas": C.scalars_to_wire(lam), "mi_shares": ys, "c1": c1, "pair_shares": dec,
            "pair_signs": np.array(psigns, np.int8), "online": np.array(online, np.int64), "D": D, "M": M}
