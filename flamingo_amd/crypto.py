"""Host-side public-key crypto of the Flamingo protocol (not the vector hot path).

The reference gets these from pycryptodomex (ECC P-256, AES-GCM, DSS) and
libnum (util/crypto/ecchash.py); neither is installed here, so this module
binds the same primitives from OpenSSL's libcrypto through ctypes:

* P-256 point arithmetic (affine (x, y) integer pairs, None = infinity)
  -- ECC.EccPoint +, *, used for ECDH (SA_ClientAgent.py:256-263), ElGamal
  (:434-447) and the threshold combine (SA_ServiceAgent.py:542-585);
* hash-to-curve restated from util/crypto/ecchash.py:50-283 (XMD SHA-256
  expander, hash_to_field -- with the reference's modulus = group order n
  quirk, SA_ClientAgent.py:285 -- and its map_to_curve);
* AES-GCM encrypt/decrypt with 16-byte nonces, tag discarded as in
  SA_ClientAgent.py:236-241 / :423-425;
* ECDSA-SHA256 signatures (DSS 'fips-186-3', SA_ServiceAgent.py:382-386).

PARITY NOTE: map_to_curve takes `next(libnum.sqrtmod(...))` (ecchash.py:263-268).
libnum is absent, so its root order cannot be observed; this module takes the
direct root a^((p+1)/4) mod p first (p = 3 mod 4), which is what libnum's
sqrtmod_prime_power computes before yielding p - root.  With that one
convention assumed, the whole pair-seed pipeline (ECDH -> SHA-256 -> h_ijt ->
hash-to-curve -> SHA-256) reproduces the s_ij the reference's own
SA_ClientAgent.sendVectors produced (tests/test_ref_golden_cpu.py).
"""
from __future__ import annotations

import ctypes
import hashlib
import os

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
A = P - 3
B = 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B
GX = 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296
GY = 0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5
G = (GX, GY)
NID_P256 = 415

_c = None


def _lib():
    global _c
    if _c is not None:
        return _c
    c = ctypes.CDLL("libcrypto.so.3")
    vp, ip = ctypes.c_void_p, ctypes.c_int
    sig = {
        "EC_GROUP_new_by_curve_name": (vp, [ip]),
        "EC_POINT_new": (vp, [vp]), "EC_POINT_free": (None, [vp]),
        "EC_POINT_set_affine_coordinates": (ip, [vp, vp, vp, vp, vp]),
        "EC_POINT_get_affine_coordinates": (ip, [vp, vp, vp, vp, vp]),
        "EC_POINT_add": (ip, [vp, vp, vp, vp, vp]), "EC_POINT_mul": (ip, [vp, vp, vp, vp, vp, vp]),
        "EC_POINT_is_at_infinity": (ip, [vp, vp]), "EC_POINT_set_to_infinity": (ip, [vp, vp]),
        "EC_POINT_is_on_curve": (ip, [vp, vp, vp]), "EC_POINT_invert": (ip, [vp, vp, vp]),
        "BN_new": (vp, []), "BN_free": (None, [vp]), "BN_CTX_new": (vp, []),
        "BN_bin2bn": (vp, [ctypes.c_char_p, ip, vp]), "BN_bn2binpad": (ip, [vp, ctypes.c_char_p, ip]),
        "EVP_CIPHER_CTX_new": (vp, []), "EVP_CIPHER_CTX_free": (None, [vp]),
        "EVP_aes_128_gcm": (vp, []), "EVP_CIPHER_CTX_ctrl": (ip, [vp, ip, ip, vp]),
        "EVP_EncryptInit_ex": (ip, [vp, vp, vp, ctypes.c_char_p, ctypes.c_char_p]),
        "EVP_EncryptUpdate": (ip, [vp, ctypes.c_char_p, ctypes.POINTER(ip), ctypes.c_char_p, ip]),
        "EVP_DecryptInit_ex": (ip, [vp, vp, vp, ctypes.c_char_p, ctypes.c_char_p]),
        "EVP_DecryptUpdate": (ip, [vp, ctypes.c_char_p, ctypes.POINTER(ip), ctypes.c_char_p, ip]),
        "ECDSA_do_sign": (vp, [ctypes.c_char_p, ip, vp]), "ECDSA_do_verify": (ip, [ctypes.c_char_p, ip, vp, vp]),
        "ECDSA_SIG_get0": (None, [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]), "ECDSA_SIG_free": (None, [vp]),
        "ECDSA_SIG_new": (vp, []), "ECDSA_SIG_set0": (ip, [vp, vp, vp]),
        "EC_KEY_new_by_curve_name": (vp, [ip]), "EC_KEY_set_private_key": (ip, [vp, vp]),
        "EC_KEY_set_public_key": (ip, [vp, vp]), "EC_KEY_free": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(c, name)
        f.restype, f.argtypes = res, args
    _c = c
    return c


class _Curve:
    def __init__(self):
        c = _lib()
        self.c = c
        self.g = c.EC_GROUP_new_by_curve_name(NID_P256)
        self.ctx = c.BN_CTX_new()
        self.bx, self.by, self.bk, self.bk2 = c.BN_new(), c.BN_new(), c.BN_new(), c.BN_new()

    def _bn(self, v: int, bn):
        return self.c.BN_bin2bn(int(v).to_bytes(32, "big"), 32, bn)

    def _int(self, bn) -> int:
        buf = ctypes.create_string_buffer(32)
        self.c.BN_bn2binpad(bn, buf, 32)
        return int.from_bytes(buf.raw, "big")

    def _pt(self, pt):
        e = self.c.EC_POINT_new(self.g)
        if pt is None:
            self.c.EC_POINT_set_to_infinity(self.g, e)
        elif not self.c.EC_POINT_set_affine_coordinates(self.g, e, self._bn(pt[0], self.bx), self._bn(pt[1], self.by),
                                                        self.ctx):
            self.c.EC_POINT_free(e)
            raise ValueError("point is not on P-256")
        return e

    def _out(self, e):
        try:
            if self.c.EC_POINT_is_at_infinity(self.g, e):
                return None
            assert self.c.EC_POINT_get_affine_coordinates(self.g, e, self.bx, self.by, self.ctx) == 1
            return (self._int(self.bx), self._int(self.by))
        finally:
            self.c.EC_POINT_free(e)

    def mul(self, k: int, pt=None):
        """k * pt (pt=None: the generator)."""
        k %= N
        r = self.c.EC_POINT_new(self.g)
        if pt is None:
            assert self.c.EC_POINT_mul(self.g, r, self._bn(k, self.bk), None, None, self.ctx) == 1
        else:
            q = self._pt(pt)
            assert self.c.EC_POINT_mul(self.g, r, None, q, self._bn(k, self.bk), self.ctx) == 1
            self.c.EC_POINT_free(q)
        return self._out(r)

    def add(self, p1, p2):
        a, b, r = self._pt(p1), self._pt(p2), self.c.EC_POINT_new(self.g)
        assert self.c.EC_POINT_add(self.g, r, a, b, self.ctx) == 1
        self.c.EC_POINT_free(a)
        self.c.EC_POINT_free(b)
        return self._out(r)


_curve = None


def curve() -> _Curve:
    global _curve
    if _curve is None:
        _curve = _Curve()
    return _curve


def mul(k: int, pt=None):
    return curve().mul(k, pt)


def add(p1, p2):
    return curve().add(p1, p2)


def neg(pt):
    return None if pt is None else (pt[0], (-pt[1]) % P)


def on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - (x * x * x + A * x + B)) % P == 0


def point_bytes(pt) -> bytes:
    """int(x).to_bytes(32,'big') + int(y).to_bytes(32,'big') (SA_ClientAgent.py:260-261, :288-289)."""
    return pt[0].to_bytes(32, "big") + pt[1].to_bytes(32, "big")


def points_to_wire(points) -> "np.ndarray":
    """(n, 64) uint8: x||y big endian per point; None (infinity) -> zeros."""
    import numpy as np
    out = np.zeros((len(points), 64), np.uint8)
    for i, pt in enumerate(points):
        if pt is not None:
            out[i] = np.frombuffer(point_bytes(pt), np.uint8)
    return out


def scalars_to_wire(scalars) -> "np.ndarray":
    import numpy as np
    return np.frombuffer(b"".join(int(k).to_bytes(32, "big") for k in scalars), np.uint8).reshape(-1, 32).copy()


def points_from_wire(buf, flags=None) -> list:
    out = []
    for i, row in enumerate(buf):
        if flags is not None and int(flags[i]) & 4:
            out.append(None)
            continue
        b = bytes(row)
        out.append((int.from_bytes(b[:32], "big"), int.from_bytes(b[32:], "big")))
    return out


def keygen(seed: bytes):
    """Deterministic P-256 key pair from a seed (stand-in for pki_files/setup_pki.py)."""
    d = int.from_bytes(hashlib.sha512(b"flm-key" + seed).digest(), "big") % (N - 1) + 1
    return d, mul(d)


# ---------------------------------------------------------------- hash to curve
# util/crypto/ecchash.py: XMD expander (:90-133), hash_to_field (:50-61),
# map_to_curve (:233-275), hash_str_to_curve = Q0 + Q1 (:277-283).
DST = b"QUUX-V01-CS02-with-P256_XMD:SHA-256_SSWU_RO_"      # ecchash.test_dst(...)


def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in, r_in = 32, 64
    ell = (len_in_bytes + b_in - 1) // b_in
    if ell > 255 or len(dst) > 255:
        raise ValueError("bad expand_message_xmd call")
    dst_prime = dst + bytes([len(dst)])
    b0 = hashlib.sha256(bytes(r_in) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime).digest()
    out = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(1, ell):
        out.append(hashlib.sha256(bytes(x ^ y for x, y in zip(b0, out[-1])) + bytes([i + 1]) + dst_prime).digest())
    return b"".join(out)[:len_in_bytes]


def hash_to_field(msg: bytes, count: int, modulus: int, blen: int = 48):
    u = expand_message_xmd(msg, DST, count * blen)
    return [int.from_bytes(u[blen * i: blen * (i + 1)], "big") % modulus for i in range(count)]


def _sqrt(v: int):
    r = pow(v, (P + 1) // 4, P)          # P = 3 mod 4: the root libnum yields first
    if r * r % P != v % P:
        return None
    return r


def map_to_curve(u: int):
    z_minus_10 = -10
    tv1_den = (100 * pow(u, 4, P) + z_minus_10 * pow(u, 2, P)) % P
    tv1 = pow(tv1_den, -1, P) if tv1_den else 0
    x1 = ((-B * pow(A, -1, P)) * (1 + tv1)) % P
    if tv1 == 0:
        x1 = (B * pow(30, -1, P)) % P
    gx1 = (x1 ** 3 + A * x1 + B) % P
    x2 = (z_minus_10 * pow(u, 2, P) * x1) % P
    gx2 = (x2 ** 3 + A * x2 + B) % P
    y = _sqrt(gx1)
    if y is not None:
        x = x1
    else:
        x, y = x2, _sqrt(gx2)
    # sgn0 of ecchash.py:228-232 is 1 only for x <= 0; u == 0 flips y
    if (1 if u <= 0 else 0) != (1 if y <= 0 else 0):
        y = (-y) % P
    return (x, y)


def hash_str_to_curve(msg: str, modulus: int = N):
    """ecchash.hash_str_to_curve(msg, count=2, modulus=n, degree=1, blen=48, XMD SHA-256) as the client calls it."""
    u0, u1 = hash_to_field(msg.encode(), 2, modulus)
    return add(map_to_curve(u0), map_to_curve(u1))


# --------------------------------------------------------------------- AES-GCM
EVP_CTRL_GCM_SET_IVLEN = 0x9


def aes_gcm_encrypt(key16: bytes, data: bytes, nonce: bytes | None = None):
    """AES.new(key, AES.MODE_GCM).encrypt_and_digest(data)[0] with its 16-byte nonce (tag discarded, :240-241)."""
    c = _lib()
    nonce = nonce or os.urandom(16)
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_EncryptInit_ex(ctx, c.EVP_aes_128_gcm(), None, None, None) == 1
        assert c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, len(nonce), None) == 1
        assert c.EVP_EncryptInit_ex(ctx, None, None, key16, nonce) == 1
        out = ctypes.create_string_buffer(len(data) + 16)
        n = ctypes.c_int(0)
        assert c.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), data, len(data)) == 1
        return out.raw[: n.value], nonce
    finally:
        c.EVP_CIPHER_CTX_free(ctx)


def aes_gcm_decrypt(key16: bytes, ct: bytes, nonce: bytes) -> bytes:
    """AES.new(key, AES.MODE_GCM, nonce=nonce).decrypt(ct) (no tag check, as :423-425)."""
    c = _lib()
    ctx = c.EVP_CIPHER_CTX_new()
    try:
        assert c.EVP_DecryptInit_ex(ctx, c.EVP_aes_128_gcm(), None, None, None) == 1
        assert c.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, len(nonce), None) == 1
        assert c.EVP_DecryptInit_ex(ctx, None, None, key16, nonce) == 1
        out = ctypes.create_string_buffer(len(ct) + 16)
        n = ctypes.c_int(0)
        assert c.EVP_DecryptUpdate(ctx, out, ctypes.byref(n), ct, len(ct)) == 1
        return out.raw[: n.value]
    finally:
        c.EVP_CIPHER_CTX_free(ctx)


# ----------------------------------------------------------------------- ECDSA
def _eckey(d: int, pub):
    c, cv = _lib(), curve()
    k = c.EC_KEY_new_by_curve_name(NID_P256)
    bn = c.BN_bin2bn(d.to_bytes(32, "big"), 32, None) if d else None
    if bn:
        assert c.EC_KEY_set_private_key(k, bn) == 1
        c.BN_free(bn)
    q = cv._pt(pub)
    assert c.EC_KEY_set_public_key(k, q) == 1
    c.EC_POINT_free(q)
    return k


def ecdsa_sign(d: int, pub, msg: bytes) -> bytes:
    """DSS.new(key, 'fips-186-3').sign(SHA256.new(msg)): r || s, 64 bytes."""
    c = _lib()
    k = _eckey(d, pub)
    dg = hashlib.sha256(msg).digest()
    sig = c.ECDSA_do_sign(dg, 32, k)
    r, s = ctypes.c_void_p(), ctypes.c_void_p()
    c.ECDSA_SIG_get0(sig, ctypes.byref(r), ctypes.byref(s))
    out = curve()._int(r) .to_bytes(32, "big") + curve()._int(s).to_bytes(32, "big")
    c.ECDSA_SIG_free(sig)
    c.EC_KEY_free(k)
    return out


def ecdsa_verify(pub, msg: bytes, signature: bytes) -> bool:
    c = _lib()
    k = _eckey(0, pub)
    sig = c.ECDSA_SIG_new()
    r = c.BN_bin2bn(signature[:32], 32, None)
    s = c.BN_bin2bn(signature[32:], 32, None)
    c.ECDSA_SIG_set0(sig, r, s)
    ok = c.ECDSA_do_verify(hashlib.sha256(msg).digest(), 32, sig, k)
    c.ECDSA_SIG_free(sig)
    c.EC_KEY_free(k)
    return ok == 1
