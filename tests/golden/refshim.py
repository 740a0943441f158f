"""TEST INFRASTRUCTURE ONLY -- stand-ins for the reference's absent third-party modules.

The reference (eniac/flamingo, pure Python) imports pycryptodomex 3.19.1
(``Cryptodome``), ``libnum`` and ``utilitybelt`` at module top
(requirements.txt:10-25); none is installed here and none can be.  This module
installs in-memory ``sys.modules`` entries that provide exactly the calls the
reference makes, so that its OWN code (util/param.py, util/util.py,
util/crypto/*, agent/flamingo/*) imports and runs unmodified, read-only, from
/root/reference.  Only ``tests/golden/make_ref_golden.py`` uses it, in the build
container; nothing here travels to the GPU box or is imported by the product.

What each stand-in is, and how faithful:

* ``Cryptodome.Cipher.ChaCha20`` -- OpenSSL ``EVP_chacha20`` with IV =
  8 zero counter bytes || the 8-byte nonce.  That is the DJB layout
  pycryptodome uses for 8-byte nonces (64-bit block counter, 64-bit nonce),
  bit-exact for every block < 2^32 (RFC 7539 vectors in tests/test_oracle.py).
  Stateful like pycryptodome: successive ``encrypt`` calls continue the stream.
* ``Cryptodome.Cipher.AES`` (MODE_GCM) -- OpenSSL AES-128-GCM with
  pycryptodome's default 16-byte random nonce; encrypt_and_digest / decrypt.
* ``Cryptodome.PublicKey.ECC.EccPoint`` -- NIST P-256 through OpenSSL
  ``EC_POINT_add`` / ``EC_POINT_mul``; x, y as Python ints; infinity is (0, 0)
  as in pycryptodome.
* ``Cryptodome.Hash.SHA256`` -- hashlib.
* ``Cryptodome.Signature.DSS`` -- a deterministic placeholder signature
  (signatures are not on the vector path; nothing checks them,
  SA_ClientAgent.py:387 "CHECK SIGNATURES" is a comment).
* ``Cryptodome.Random.get_random_bytes`` and ``utilitybelt.secure_randint`` --
  a seeded SHA-256 counter DRBG, so m_i, ElGamal randomness and Shamir
  polynomials are reproducible and recorded.
* ``libnum.invmod / has_sqrtmod / sqrtmod`` -- modular inverse, Euler's
  criterion, and for p = 3 (mod 4) the roots a^((p+1)/4) then p - a^((p+1)/4).
  ASSUMPTION (the one convention not pinned -- parity unpinned): that libnum
  1.7's sqrtmod_prime_power yields the direct root first.  It decides which of
  the two hash-to-curve points (x, +-y) a pair seed s_ij is hashed from
  (ecchash.py:263-268; sgn0 at :227-231,271-272 flips y only when u or y is 0),
  so s_ij = SHA-256(x||y) and every pairwise PRG mask depend on it.  Only the
  cancellation of the masks within one simulation (every party uses the same
  convention) is independent of it.
"""
from __future__ import annotations

import ctypes
import hashlib
import random
import sys
import types

P256_P = 2**256 - 2**224 + 2**192 + 2**96 - 1
P256_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551

_c = ctypes.CDLL("libcrypto.so.3")
_vp, _ip = ctypes.c_void_p, ctypes.c_int
for _name, _res, _args in (
        ("EVP_CIPHER_CTX_new", _vp, []), ("EVP_CIPHER_CTX_free", None, [_vp]),
        ("EVP_chacha20", _vp, []), ("EVP_aes_128_gcm", _vp, []),
        ("EVP_CIPHER_CTX_ctrl", _ip, [_vp, _ip, _ip, _vp]),
        ("EVP_EncryptInit_ex", _ip, [_vp, _vp, _vp, ctypes.c_char_p, ctypes.c_char_p]),
        ("EVP_EncryptUpdate", _ip, [_vp, ctypes.c_char_p, ctypes.POINTER(_ip), ctypes.c_char_p, _ip]),
        ("EVP_EncryptFinal_ex", _ip, [_vp, ctypes.c_char_p, ctypes.POINTER(_ip)]),
        ("EVP_DecryptInit_ex", _ip, [_vp, _vp, _vp, ctypes.c_char_p, ctypes.c_char_p]),
        ("EVP_DecryptUpdate", _ip, [_vp, ctypes.c_char_p, ctypes.POINTER(_ip), ctypes.c_char_p, _ip]),
        ("EC_GROUP_new_by_curve_name", _vp, [_ip]),
        ("EC_POINT_new", _vp, [_vp]), ("EC_POINT_free", None, [_vp]),
        ("EC_POINT_set_affine_coordinates", _ip, [_vp, _vp, _vp, _vp, _vp]),
        ("EC_POINT_get_affine_coordinates", _ip, [_vp, _vp, _vp, _vp, _vp]),
        ("EC_POINT_add", _ip, [_vp, _vp, _vp, _vp, _vp]),
        ("EC_POINT_mul", _ip, [_vp, _vp, _vp, _vp, _vp, _vp]),
        ("EC_POINT_is_at_infinity", _ip, [_vp, _vp]), ("EC_POINT_set_to_infinity", _ip, [_vp, _vp]),
        ("BN_new", _vp, []), ("BN_free", None, [_vp]), ("BN_CTX_new", _vp, []),
        ("BN_bin2bn", _vp, [ctypes.c_char_p, _ip, _vp]), ("BN_bn2binpad", _ip, [_vp, ctypes.c_char_p, _ip])):
    _f = getattr(_c, _name)
    _f.restype, _f.argtypes = _res, _args

_GROUP = _c.EC_GROUP_new_by_curve_name(415)      # NID_X9_62_prime256v1
_BNCTX = _c.BN_CTX_new()

# Every ChaCha20 stream the reference opens: (tag, key, plaintext length); the driver
# sets TAG before each protocol step so the log says which agent and step used a key.
CHACHA_LOG: list = []
TAG = [None]


# ------------------------------------------------------------------ DRBG
class _Drbg:
    def __init__(self, seed: bytes = b""):
        self.reset(seed)

    def reset(self, seed: bytes):
        self.seed, self.ctr = seed, 0
        self.rng = random.Random(hashlib.sha256(b"refshim-randint" + seed).digest())

    def bytes(self, n: int) -> bytes:
        out = b""
        while len(out) < n:
            out += hashlib.sha256(b"refshim" + self.seed + self.ctr.to_bytes(8, "big")).digest()
            self.ctr += 1
        return out[:n]


DRBG = _Drbg()


# ---------------------------------------------------------------- ChaCha20
class _ChaChaCipher:
    def __init__(self, key: bytes, nonce: bytes):
        if len(key) != 32 or len(nonce) != 8:
            raise ValueError("stand-in supports the reference's 32-byte key / 8-byte nonce only")
        self.key = bytes(key)
        self.nonce = bytes(nonce)
        self._ctx = _c.EVP_CIPHER_CTX_new()
        assert _c.EVP_EncryptInit_ex(self._ctx, _c.EVP_chacha20(), None, self.key, bytes(8) + self.nonce) == 1

    def encrypt(self, data: bytes) -> bytes:
        CHACHA_LOG.append((TAG[0], self.key, len(data)))
        if not data:
            return b""
        out = ctypes.create_string_buffer(len(data) + 64)
        n = _ip(0)
        assert _c.EVP_EncryptUpdate(self._ctx, out, ctypes.byref(n), bytes(data), len(data)) == 1
        assert n.value == len(data)
        return out.raw[:len(data)]

    def __del__(self):
        try:
            _c.EVP_CIPHER_CTX_free(self._ctx)
        except Exception:
            pass


def _chacha_new(key=None, nonce=None):
    return _ChaChaCipher(key, nonce if nonce is not None else bytes(8))


# --------------------------------------------------------------------- AES
_GCM_SET_IVLEN = 0x9


class _AesGcm:
    def __init__(self, key: bytes, nonce: bytes | None):
        self.key = bytes(key)
        self.nonce = DRBG.bytes(16) if nonce is None else bytes(nonce)

    def _run(self, data: bytes, enc: bool) -> bytes:
        ctx = _c.EVP_CIPHER_CTX_new()
        try:
            init, upd = (_c.EVP_EncryptInit_ex, _c.EVP_EncryptUpdate) if enc else \
                (_c.EVP_DecryptInit_ex, _c.EVP_DecryptUpdate)
            assert init(ctx, _c.EVP_aes_128_gcm(), None, None, None) == 1
            assert _c.EVP_CIPHER_CTX_ctrl(ctx, _GCM_SET_IVLEN, len(self.nonce), None) == 1
            assert init(ctx, None, None, self.key, self.nonce) == 1
            out = ctypes.create_string_buffer(len(data) + 16)
            n = _ip(0)
            assert upd(ctx, out, ctypes.byref(n), bytes(data), len(data)) == 1
            return out.raw[:n.value]
        finally:
            _c.EVP_CIPHER_CTX_free(ctx)

    def encrypt_and_digest(self, data: bytes):
        return self._run(data, True), hashlib.sha256(b"tag" + self.key + self.nonce).digest()[:16]

    def decrypt(self, ct: bytes) -> bytes:
        return self._run(ct, False)


def _aes_new(key, mode, nonce=None):
    if mode != 11:
        raise ValueError("stand-in supports MODE_GCM only")
    return _AesGcm(key, nonce)


# ---------------------------------------------------------------- P-256
def _bn(v: int):
    b = int(v).to_bytes(32, "big")
    return _c.BN_bin2bn(b, 32, None)


def _bn_int(bn) -> int:
    buf = ctypes.create_string_buffer(32)
    assert _c.BN_bn2binpad(bn, buf, 32) == 32
    return int.from_bytes(buf.raw, "big")


class EccPoint:
    """pycryptodome's ECC.EccPoint on P-256, as the reference uses it: +, int*P, P*int, -P."""

    __slots__ = ("_x", "_y")

    def __init__(self, x, y, curve="p256"):
        self._x, self._y = int(x), int(y)

    @property
    def x(self) -> int:
        return self._x

    @property
    def y(self) -> int:
        return self._y

    def is_point_at_infinity(self) -> bool:
        return self._x == 0 and self._y == 0

    def _to_ossl(self):
        pt = _c.EC_POINT_new(_GROUP)
        if self.is_point_at_infinity():
            assert _c.EC_POINT_set_to_infinity(_GROUP, pt) == 1
        else:
            bx, by = _bn(self._x), _bn(self._y)
            ok = _c.EC_POINT_set_affine_coordinates(_GROUP, pt, bx, by, _BNCTX)
            _c.BN_free(bx)
            _c.BN_free(by)
            if ok != 1:
                _c.EC_POINT_free(pt)
                raise ValueError("The EC point does not belong to the curve")
        return pt

    @staticmethod
    def _from_ossl(pt) -> "EccPoint":
        if _c.EC_POINT_is_at_infinity(_GROUP, pt):
            r = EccPoint(0, 0)
        else:
            bx, by = _c.BN_new(), _c.BN_new()
            assert _c.EC_POINT_get_affine_coordinates(_GROUP, pt, bx, by, _BNCTX) == 1
            r = EccPoint(_bn_int(bx), _bn_int(by))
            _c.BN_free(bx)
            _c.BN_free(by)
        _c.EC_POINT_free(pt)
        return r

    def __add__(self, other):
        if isinstance(other, int) and other == 0:      # sum() / pandas reductions start at 0
            return self
        a, b, r = self._to_ossl(), other._to_ossl(), _c.EC_POINT_new(_GROUP)
        assert _c.EC_POINT_add(_GROUP, r, a, b, _BNCTX) == 1
        _c.EC_POINT_free(a)
        _c.EC_POINT_free(b)
        return EccPoint._from_ossl(r)

    __radd__ = __add__

    def __mul__(self, k):
        k = int(k)
        if k < 0:
            raise ValueError("Scalar multiplication is only defined for non-negative integers")
        k %= P256_N
        if k == 0 or self.is_point_at_infinity():
            return EccPoint(0, 0)
        a, r = self._to_ossl(), _c.EC_POINT_new(_GROUP)
        bk = _bn(k)
        assert _c.EC_POINT_mul(_GROUP, r, None, a, bk, _BNCTX) == 1
        _c.BN_free(bk)
        _c.EC_POINT_free(a)
        return EccPoint._from_ossl(r)

    __rmul__ = __mul__

    def __neg__(self):
        if self.is_point_at_infinity():
            return EccPoint(0, 0)
        return EccPoint(self._x, (-self._y) % P256_P)

    def __eq__(self, other):
        return isinstance(other, EccPoint) and (self._x, self._y) == (other._x, other._y)

    def __hash__(self):
        return hash((self._x, self._y))

    def __repr__(self):
        return f"EccPoint({self._x:#x}, {self._y:#x})"

    def __getstate__(self):
        return (self._x, self._y)

    def __setstate__(self, st):
        self._x, self._y = st


class EccKey:
    def __init__(self, d: int):
        self.d = int(d)
        self.pointQ = EccPoint(0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
                               0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5) * self.d


def key_scalar(name: str) -> int:
    """Deterministic private key for a pki_files/ name (stands in for setup_pki.py's random keys)."""
    return int.from_bytes(hashlib.sha512(b"refgolden-pki-" + name.encode()).digest(), "big") % (P256_N - 1) + 1


_KEYS: dict = {}


def read_key(file_name: str) -> EccKey:
    """util.read_key stand-in: a deterministic key per PEM file name (no files on disk)."""
    if file_name not in _KEYS:
        _KEYS[file_name] = EccKey(key_scalar(file_name))
    return _KEYS[file_name]


# ------------------------------------------------------------- SHA256 / DSS
class _Sha256:
    digest_size = 32

    def __init__(self, data=None):
        self._h = hashlib.sha256()
        if data is not None:
            self._h.update(data)

    def update(self, data):
        self._h.update(data)
        return self

    def digest(self):
        return self._h.digest()

    def hexdigest(self):
        return self._h.hexdigest()


class _Signer:
    def __init__(self, key, mode):
        self.key = key

    def sign(self, h):
        return hashlib.sha512(b"sig" + h.digest()).digest()[:64]


# ------------------------------------------------------------------ libnum
def _invmod(a: int, m: int) -> int:
    return pow(int(a), -1, int(m))


def _has_sqrtmod(a: int, factors: dict) -> bool:
    (p, k), = factors.items()
    assert k == 1
    a %= p
    return a == 0 or pow(a, (p - 1) // 2, p) == 1


def _sqrtmod(a: int, factors: dict):
    (p, k), = factors.items()
    assert k == 1 and p % 4 == 3
    a %= p
    if not _has_sqrtmod(a, factors):
        raise ValueError("No square root for given value")
    r = pow(a, (p + 1) // 4, p)
    yield r
    if r != p - r:
        yield p - r


# ---------------------------------------------------------------- install
def install():
    """Register the stand-ins in sys.modules (idempotent)."""
    if "Cryptodome" in sys.modules and getattr(sys.modules["Cryptodome"], "_refshim", False):
        return
    m = {}
    for name in ("Cryptodome", "Cryptodome.Cipher", "Cryptodome.Random", "Cryptodome.Hash",
                 "Cryptodome.Signature", "Cryptodome.PublicKey", "libnum", "utilitybelt"):
        m[name] = types.ModuleType(name)
    m["Cryptodome"]._refshim = True
    chacha = types.SimpleNamespace(new=_chacha_new)
    aes = types.SimpleNamespace(new=_aes_new, MODE_GCM=11)
    m["Cryptodome.Cipher"].ChaCha20 = chacha
    m["Cryptodome.Cipher"].AES = aes
    m["Cryptodome.Random"].get_random_bytes = DRBG.bytes
    m["Cryptodome.Hash"].SHA256 = types.SimpleNamespace(new=_Sha256)
    m["Cryptodome.Signature"].DSS = types.SimpleNamespace(new=_Signer)

    def _import_key(*a, **k):
        raise RuntimeError("refshim: PEM files are replaced by refshim.read_key")
    m["Cryptodome.PublicKey"].ECC = types.SimpleNamespace(EccPoint=EccPoint, EccKey=EccKey, import_key=_import_key)
    for sub in ("Cipher", "Random", "Hash", "Signature", "PublicKey"):
        setattr(m["Cryptodome"], sub, m[f"Cryptodome.{sub}"])
    m["libnum"].invmod = _invmod
    m["libnum"].has_sqrtmod = _has_sqrtmod
    m["libnum"].sqrtmod = _sqrtmod
    ub = m["utilitybelt"]
    ub.secure_randint = lambda lo, hi: DRBG.rng.randint(lo, hi)
    ub.int_to_charset = ub.charset_to_int = None
    ub.base58_chars = ub.base32_chars = ub.zbase32_chars = ""
    sys.modules.update(m)
