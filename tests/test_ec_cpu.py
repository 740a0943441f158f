"""CPU checks for the seed-recovery layer (no GPU).

1. Pin the pure-Python EC oracle (oracle/ec_oracle.py) against OpenSSL's
   independent P-256 (through flamingo_amd.crypto) and the group law.
2. The threshold-ElGamal algebra the server relies on
   (SA_ServiceAgent.py:542-585): c1 - sum_j lambda_j (sk_j c0) == h.
3. Host crypto helpers: hash-to-curve lands on the curve, AES-GCM round trip
   with the reference's 16-byte nonces, ECDSA sign/verify.
"""
import hashlib
import random

import pytest

import ec_oracle as E
from flamingo_amd import crypto as C
from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero, shamir_share

rng = random.Random(1234)


def test_generator_and_order():
    assert E.on_curve(E.G) and C.G == E.G
    assert E.mul(E.N) is None and C.mul(E.N) is None
    assert E.mul(E.N - 1) == E.neg(E.G)
    assert C.mul(2) == E.add(E.G, E.G)


@pytest.mark.parametrize("k", [1, 2, 3, 15, 16, 17, 2**255 + 11, E.N - 2, E.N + 5, 2**256 - 1])
def test_oracle_mul_matches_openssl(k):
    pt = C.mul(rng.randrange(1, E.N))
    assert E.mul(k, pt) == C.mul(k, pt)


def test_oracle_add_matches_openssl():
    for _ in range(10):
        a, b = C.mul(rng.randrange(1, E.N)), C.mul(rng.randrange(1, E.N))
        assert E.add(a, b) == C.add(a, b)
    a = C.mul(77)
    assert E.add(a, a) == C.add(a, a) == C.mul(154)
    assert E.add(a, E.neg(a)) is None and C.add(a, C.neg(a)) is None


def test_threshold_elgamal_combine_recovers_plaintext():
    sk = rng.randrange(1, E.N)
    pk = E.mul(sk)
    committee, T = 9, 3
    shares = shamir_share(sk, T, committee, rng=rng)
    chosen = rng.sample(shares, T)
    lam = lagrange_at_zero([x for x, _ in chosen])
    hs = [C.hash_str_to_curve(f"pair-{i}") for i in range(3)]
    cts = [E.elgamal_encrypt(pk, h, rng.randrange(1, E.N)) for h in hs]
    dec = [[E.mul(y, c0) for c0, _ in cts] for _, y in chosen]       # member shares sk_j * c0
    pts, seeds = E.combine([c1 for _, c1 in cts], dec, lam)
    assert pts == hs
    assert seeds == [hashlib.sha256(E.wire(h)).digest() for h in hs]


def test_hash_to_curve_points_on_curve_and_deterministic():
    for m in ["", "a", "x" * 300, "h_ijt-0123"]:
        pt = C.hash_str_to_curve(m)
        assert E.on_curve(pt)
        assert pt == C.hash_str_to_curve(m)
    assert C.hash_str_to_curve("a") != C.hash_str_to_curve("b")


def test_expand_message_xmd_rfc9380_vector():
    # RFC 9380 K.1 expand_message_xmd(SHA-256), DST "QUUX-V01-CS02-with-expander-SHA256-128", msg "", 0x20 bytes
    out = C.expand_message_xmd(b"", b"QUUX-V01-CS02-with-expander-SHA256-128", 0x20)
    assert out.hex() == "68a985b87eb6b46952128911f2a4412bbc302a9d759667f87f7a21d803f07235"


def test_aes_gcm_and_ecdsa():
    key = bytes(range(16))
    ct, nonce = C.aes_gcm_encrypt(key, b"share-bytes" * 3)
    assert len(nonce) == 16 and C.aes_gcm_decrypt(key, ct, nonce) == b"share-bytes" * 3
    d, Q = C.keygen(b"client-1")
    sig = C.ecdsa_sign(d, Q, b"msg")
    assert len(sig) == 64 and C.ecdsa_verify(Q, b"msg", sig) and not C.ecdsa_verify(Q, b"msg2", sig)


def test_wire_helpers_roundtrip():
    pts = [C.mul(5), None, E.G]
    w = C.points_to_wire(pts)
    assert bytes(w[1]) == bytes(64) and bytes(w[0]) == E.wire(pts[0])
    back = C.points_from_wire(w, [0, 4, 0])
    assert back == pts


def test_hash_to_field_and_map_rfc9380_vector():
    # RFC 9380 J.1.1 P256_XMD:SHA-256_SSWU_RO_, msg "": u[0], u[1] and Q0.x.  The reference
    # reduces mod n rather than p (SA_ClientAgent.py:285) and picks y by its own sgn0, so
    # only the modulus-p field elements and the x coordinate are comparable.
    u = C.hash_to_field(b"", 2, C.P)
    assert u == [0xad5342c66a6dd0ff080df1da0ea1c04b96e0330dd89406465eeba11582515009,
                 0x8c0f1d43204bd6f6ea70ae8013070a1518b43873bcd850aafa0a9e220e2eea5a]
    assert C.map_to_curve(u[0])[0] == 0xab640a12220d3ff283510ff3f4b1953d09fad35795140b1c5d64f313967934d5
