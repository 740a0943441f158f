"""Parity of the P-256 seed-recovery kernels (flm_ec_mul, flm_ec_combine) through the C ABI.

Checked against the pure-Python oracle (oracle/ec_oracle.py) on small batches
and, at the c5 dropout size (D ~ 1000 pairs x T = 20 committee shares,
SA_ServiceAgent.py:542-585), through the protocol identity
c1 - sum_j lambda_j (sk_j c0) == h with inputs built by OpenSSL.  Bit-exact:
points are integers and seeds are SHA-256 digests.
"""
import hashlib
import random

import numpy as np
import pytest

import ec_oracle as E

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=[(0, 1), (1, 1), (2, 1), (0, 2), (0, 4)],
                ids=["per_lane", "coop", "row", "straus2", "straus4"])
def eng(request):
    """Every test runs with each scalar-multiplication kernel: one lane per product (ec_mul_kernel),
    four cooperating waves per 64 products (ec_mul_coop_kernel), the same with every field element
    on a 16-lane row (ec_mul_row_kernel, flm_fe_row.h), and 2 / 4 combine terms per lane sharing
    one chain of doublings (ec_mul_straus_kernel; the combine only, T = 3 leaves a partial group)."""
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    e.set_tuning("ec_coop", request.param[0])
    e.set_tuning("ec_terms", request.param[1])
    yield e
    e.close()


def test_ec_mul_matches_oracle(eng):
    rng = random.Random(5)
    pts = [E.mul(rng.randrange(1, E.N)) for _ in range(40)] + [E.G] * 12
    ks = [rng.randrange(0, 2**256) for _ in range(40)] + [0, 1, 2, 15, 16, 17, E.N - 1, E.N, E.N + 1,
                                                            2**256 - 1, 2**255, 0xF0F0F0F0]
    got = eng.ec_mul(pts, ks)
    want = [E.mul(k, p) for k, p in zip(ks, pts)]
    assert got == want
    assert got[40] is None and got[47] is None      # 0*G, n*G


def test_ec_mul_rejects_off_curve(eng):
    bad = (E.G[0], (E.G[1] + 1) % E.P)
    with pytest.raises(RuntimeError, match="not a point on P-256"):
        eng.ec_mul([E.G, bad], [3, 3])
    with pytest.raises(RuntimeError, match="not a point on P-256"):
        eng.ec_mul([(E.P, 0)], [3])                 # coordinate >= p


def _threshold_case(D, T, committee, seed, builder):
    """Real threshold ElGamal: pk = sk*G, Shamir shares of sk, c = (rG, h + r pk),
    member j's decryption share sk_j * c0.  builder: ec module used to make inputs."""
    from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero, shamir_share
    rng = random.Random(seed)
    sk = rng.randrange(1, E.N)
    pk = builder.mul(sk)
    chosen = rng.sample(shamir_share(sk, T, committee, rng=rng), T)
    lam = lagrange_at_zero([x for x, _ in chosen])
    hs = [builder.mul(rng.randrange(1, E.N)) for _ in range(D)]
    rs = [rng.randrange(1, E.N) for _ in range(D)]
    c0 = [builder.mul(r) for r in rs]
    c1 = [builder.add(h, builder.mul(r, pk)) for h, r in zip(hs, rs)]
    dec = [[builder.mul(y, c) for c in c0] for _, y in chosen]
    return c1, dec, lam, hs


def test_ec_combine_matches_oracle(eng):
    c1, dec, lam, hs = _threshold_case(D=7, T=3, committee=8, seed=11, builder=E)
    pts, seeds = eng.ec_combine(c1, dec, lam)
    want_pts, want_seeds = E.combine(c1, dec, lam)
    assert pts == want_pts == hs
    assert seeds == want_seeds
    # negate = False, no c1: plain multi-scalar sum
    pts2, _ = eng.ec_combine(None, dec, lam, negate=False)
    assert pts2 == E.combine(None, dec, lam, negate=False)[0]


def test_ec_combine_with_lds_spread(eng):
    """ec_spread reserves LDS per workgroup of the per-lane kernels (fewer workgroups per CU): same result."""
    c1, dec, lam, hs = _threshold_case(D=70, T=5, committee=9, seed=17, builder=E)
    want = E.combine(c1, dec, lam)
    eng.set_tuning("ec_spread", 40)
    try:
        assert eng.ec_combine(c1, dec, lam) == want
    finally:
        eng.set_tuning("ec_spread", 0)
    with pytest.raises(RuntimeError):
        eng.set_tuning("ec_spread", 65)


def test_ec_combine_edge_cases(eng):
    # T = 0: the point is c1 itself; a result at infinity hashes 64 zero bytes (EccPoint(0,0))
    c1 = [E.G, E.mul(5)]
    pts, seeds = eng.ec_combine(c1, [], [])
    assert pts == c1 and seeds[0] == hashlib.sha256(E.wire(E.G)).digest()
    pts, seeds = eng.ec_combine([E.G], [[E.G]], [1])          # G - 1*G
    assert pts == [None] and seeds == [hashlib.sha256(bytes(64)).digest()]
    with pytest.raises(RuntimeError, match="ciphertext c1"):
        eng.ec_combine([(1, 1)], [[E.G]], [1])
    with pytest.raises(RuntimeError, match="decryption share"):
        eng.ec_combine([E.G], [[(1, 1)]], [1])
    assert eng.ec_combine([], [[]], [1]) == ([], [])


def test_ec_combine_c5_size(eng):
    """c5: 10000 clients, ~10% of pairs dropped -> D ~ 1000 recoveries over T = 20 shares."""
    from flamingo_amd import crypto as C
    c1, dec, lam, hs = _threshold_case(D=1000, T=20, committee=60, seed=3, builder=C)
    pts, seeds = eng.ec_combine(c1, dec, lam)
    assert pts == hs
    assert seeds == [hashlib.sha256(C.point_bytes(h)).digest() for h in hs]


def test_ec_combine_dev_feeds_seed_table(eng):
    """Device seed recovery -> seed table -> unmask, no host round trip for the seeds."""
    import torch
    import oracle as O
    from flamingo_amd import crypto as C
    c1, dec, lam, hs = _threshold_case(D=33, T=4, committee=12, seed=9, builder=C)
    dev = torch.device("cuda:0")
    c1_t = torch.from_numpy(C.points_to_wire(c1)).to(dev)
    sh_t = torch.from_numpy(np.stack([C.points_to_wire(d) for d in dec])).to(dev)
    lam_t = torch.from_numpy(C.scalars_to_wire(lam)).to(dev)
    seeds_t = torch.empty((33, 32), dtype=torch.uint8, device=dev)
    flags_t = torch.empty(33, dtype=torch.int32, device=dev)
    eng.ec_combine_dev(c1_t, sh_t, lam_t, seeds_t, flags_t)
    L = 5000
    rng = np.random.Generator(np.random.PCG64(1))
    rows = rng.integers(0, 2**32, size=(5, L), dtype=np.uint32)
    signs = rng.choice(np.array([1, -1], np.int8), 33)
    rows_t = torch.from_numpy(rows.view(np.int32)).to(dev)
    pitch = (L + 3) // 4 * 4
    rows_p = torch.zeros((5, pitch), dtype=torch.int32, device=dev)
    rows_p[:, :L] = rows_t
    out = torch.empty(L, dtype=torch.int32, device=dev)
    eng.aggregate_unmask_dev(rows_p, seeds_t, torch.from_numpy(signs).to(dev), out, L=L)
    torch.cuda.synchronize()
    assert int(flags_t.abs().sum()) == 0
    want_seeds = np.frombuffer(b"".join(hashlib.sha256(C.point_bytes(h)).digest() for h in hs),
                               np.uint8).reshape(33, 32)
    assert np.array_equal(seeds_t.cpu().numpy(), want_seeds)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.aggregate_unmask(rows, want_seeds, signs))


def test_shamir_combine_matches_bigint(eng):
    """m_i = sum_j lambda_j y_{j,i} mod n (SA_ServiceAgent.py:506-526) against Python big ints."""
    from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero, shamir_share
    rng = random.Random(17)
    T, M = 20, 300
    secrets_ = [rng.randrange(0, 2**256) for _ in range(M)]
    pts = [shamir_share(s, T, 60, rng=rng) for s in secrets_]
    chosen = sorted(rng.sample(range(60), T))
    lam = lagrange_at_zero([c + 1 for c in chosen])
    shares = [[pts[i][c][1] for i in range(M)] for c in chosen]
    got = eng.shamir_combine(shares, lam)
    assert got == [(s % E.N).to_bytes(32, "big") for s in secrets_]
    # edge values: y >= n, y = 2^256 - 1, lambda in {0, 1, n - 1}
    ys = [[E.N, E.N + 5, 2**256 - 1, 0, 1], [E.N - 1, 2**255, 7, 2**256 - 1, 0], [3, 3, 3, 3, 3]]
    ls = [0, 1, E.N - 1]
    want = [(sum(l * y[i] for l, y in zip(ls, ys)) % E.N).to_bytes(32, "big") for i in range(5)]
    assert eng.shamir_combine(ys, ls) == want
    assert eng.shamir_combine([], []) == []
