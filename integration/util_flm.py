"""util/flm.py for the reference tree: the ctypes binding a maintainer adds to eniac/flamingo.

Save as ``util/flm.py`` in the reference, then edit the call sites as INTEGRATION.md shows
(agent/flamingo/SA_ServiceAgent.py:346-350, 506-605; SA_ClientAgent.py:246-324).  It binds
libflamingo_hip.so directly -- no dependency on the flamingo_amd package -- and mirrors the
reference's own conventions: uint32 numpy vectors, 32-byte seeds, +-1 signs, EccPoint-like
objects with .x/.y for the ElGamal and decryption-share points, RuntimeError on failure
(as SA_ServiceAgent.py:349,502,579,592 raise).

Environment:
  FLM_LIB      path of libflamingo_hip.so (default: found by the dynamic loader)
  FLM_DEVICE   the GPU of the single-device context (default 0)
  FLM_GPUS     > 1: the server's aggregate_unmask runs on devices 0..FLM_GPUS-1 of this one
               process (flm_group: client-sharded rows, slot-sharded masks, one RCCL
               reduce-scatter, ncclUint32) -- the reference server is a single DES process
               (Kernel.py:190-271), so this is how it uses all GPUs of the node.
The contexts are created lazily, on first use: after SA_ServiceAgent.py:562 forks its
multiprocessing.Pool, never before.
"""
import ctypes
import os

import numpy as np

_lib = ctypes.CDLL(os.environ.get("FLM_LIB", "libflamingo_hip.so"))
_vp, _int, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
_u8p, _i8p, _u32p, _i64p = (ctypes.POINTER(t) for t in (ctypes.c_uint8, ctypes.c_int8, ctypes.c_uint32,
                                                         ctypes.c_int64))
for _name, _res, _args in (
        ("flm_init", _int, [ctypes.POINTER(_vp), _int]),
        ("flm_last_error", ctypes.c_char_p, [_vp]),
        ("flm_aggregate_unmask", _int, [_vp, ctypes.POINTER(_u32p), _int, _u8p, _i8p, _int, _sz, _u32p]),
        ("flm_client_mask", _int, [_vp, _u32p, _int, _i64p, _u8p, _i8p, _sz, _u32p]),
        ("flm_shamir_combine", _int, [_vp, _u8p, _u8p, _int, _int, _u8p]),
        ("flm_ec_combine", _int, [_vp, _u8p, _u8p, _u8p, _int, _int, _int, _u8p, _u8p, ctypes.POINTER(ctypes.c_uint32)]),
        ("flm_group_init", _int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(_int)]),
        ("flm_group_last_error", ctypes.c_char_p, [_vp]),
        ("flm_group_aggregate_unmask", _int, [_vp, ctypes.POINTER(_u32p), _int, _u8p, _i8p, _int, _sz, _u32p]),
        ("flm_store_create", _int, [ctypes.POINTER(_vp), _vp, _vp, _sz, _int]),
        ("flm_store_free", None, [_vp]),
        ("flm_store_last_error", ctypes.c_char_p, [_vp]),
        ("flm_store_add", _int, [_vp, ctypes.c_int64, _vp, _sz]),
        ("flm_store_partial", _int, [_vp]),
        ("flm_store_unmask", _int, [_vp, _u8p, _i8p, _int, _u32p]),
        ("flm_store_reset", _int, [_vp]),
        ("flm_hash_to_curve", _int, [_vp, _u8p, _u32p, _int, _u8p, _u32p]),
        ("flm_hash_to_curve_decimal", _int, [_vp, ctypes.c_uint32, _int, _u8p, _u32p])):
    _f = getattr(_lib, _name)
    _f.restype, _f.argtypes = _res, _args

_ctx = None
_group = None


def _context():
    global _ctx
    if _ctx is None:
        c = _vp()
        if _lib.flm_init(ctypes.byref(c), int(os.environ.get("FLM_DEVICE", "0"))):
            raise RuntimeError(_lib.flm_last_error(None).decode())
        _ctx = c
    return _ctx


def _server_group():
    """The process's device group when FLM_GPUS > 1, else None."""
    global _group
    n = int(os.environ.get("FLM_GPUS", "1"))
    if n <= 1:
        return None
    if _group is None:
        g = _vp()
        if _lib.flm_group_init(ctypes.byref(g), n, None):
            raise RuntimeError(_lib.flm_group_last_error(None).decode())
        _group = g
    return _group


def _check(rc, group=None):
    if rc:
        msg = _lib.flm_group_last_error(group) if group is not None else _lib.flm_last_error(_ctx)
        raise RuntimeError(msg.decode())


def _u32_body(vec, L):
    """A VECTOR body as contiguous uint32[L], or None when it is not a 1-D 32-bit integer vector of
    length L: the reference's `vec_sum_partial += v` (SA_ServiceAgent.py:346-350) raises on such a
    body (wrong length at :348-349; numpy's same-kind cast refuses float and 64-bit bodies), so it
    is never silently truncated into one."""
    v = np.asarray(vec)
    if v.ndim != 1 or v.shape[0] != L or v.dtype.kind not in "ui" or v.dtype.itemsize != 4:
        return None
    return np.ascontiguousarray(v).view(np.uint32)


def _seed_arrays(seeds, signs):
    K = len(seeds)
    sd = np.frombuffer(b"".join(bytes(s) for s in seeds), np.uint8) if K else np.zeros(32, np.uint8)
    sg = np.asarray(signs, np.int8) if K else np.ones(1, np.int8)
    if sd.size != 32 * K or sg.size != max(K, 1):
        raise RuntimeError("seeds must be 32 bytes each, one sign per seed")
    return sd, sg, K


def aggregate_unmask(vectors, seeds, signs, L):
    """sum(vectors) + sum_k signs[k] * PRG(seeds[k]) mod 2^32, as uint32[L]
    (vec_sum_partial + cancel_vec + mi_vec, SA_ServiceAgent.py:346-350, 529-605)."""
    vecs = [_u32_body(v, L) for v in vectors]
    if any(v is None for v in vecs):
        raise RuntimeError("Client sends vector of incorrect length.")
    rows = (_u32p * max(1, len(vecs)))(*[v.ctypes.data_as(_u32p) for v in vecs])
    sd, sg, K = _seed_arrays(seeds, signs)
    out = np.empty(L, np.uint32)
    g = _server_group()
    if g is not None:
        _check(_lib.flm_group_aggregate_unmask(g, rows, len(vecs), sd.ctypes.data_as(_u8p), sg.ctypes.data_as(_i8p),
                                               K, L, out.ctypes.data_as(_u32p)), g)
    else:
        _check(_lib.flm_aggregate_unmask(_context(), rows, len(vecs), sd.ctypes.data_as(_u8p),
                                         sg.ctypes.data_as(_i8p), K, L, out.ctypes.data_as(_u32p)))
    return out


def _be(ints):
    """Python ints -> n x 32 big-endian bytes."""
    return np.frombuffer(b"".join(int(v).to_bytes(32, "big") for v in ints), np.uint8)


def shamir_combine(shares_by_member, coeffs):
    """[(sum_j coeffs[j] * shares_by_member[j][i]) % n .to_bytes(32, 'big') for each i]
    (the m_i recovery of SA_ServiceAgent.py:517-526)."""
    T, M = len(coeffs), len(shares_by_member[0])
    sh = np.concatenate([_be(s) for s in shares_by_member])
    out = np.empty(M * 32, np.uint8)
    _check(_lib.flm_shamir_combine(_context(), sh.ctypes.data_as(_u8p), _be(coeffs).ctypes.data_as(_u8p), T, M,
                                   out.ctypes.data_as(_u8p)))
    return [out[32 * i:32 * i + 32].tobytes() for i in range(M)]


def ec_combine(c1_points, shares_by_member, coeffs):
    """SHA-256 keys of c1_i - sum_j coeffs[j] * shares_by_member[j][i] (SA_ServiceAgent.py:542-585):
    EccPoint-like objects (.x, .y) in, 32-byte ChaCha20 keys out."""
    xy = lambda pts: _be([c for p in pts for c in (int(p.x), int(p.y))])
    T, D = len(coeffs), len(c1_points)
    if D == 0:
        return []
    sh = np.concatenate([xy(s) for s in shares_by_member])
    seeds = np.empty(D * 32, np.uint8)
    _check(_lib.flm_ec_combine(_context(), xy(c1_points).ctypes.data_as(_u8p), sh.ctypes.data_as(_u8p),
                               _be(coeffs).ctypes.data_as(_u8p), T, D, 1, None, seeds.ctypes.data_as(_u8p), None))
    return [seeds[32 * i:32 * i + 32].tobytes() for i in range(D)]


class Point:
    """The .x / .y of pycryptodome's EccPoint, which is all SA_ClientAgent.py:288-289 and the
    ElGamal encryption (:434-447, via ECC.EccPoint(x, y)) read of a hash-to-curve result."""
    __slots__ = ("x", "y")

    def __init__(self, x, y):
        self.x, self.y = x, y


_h2c_table = None


def hash_str_to_curve(msg):
    """ecchash.hash_str_to_curve(msg, count=2, modulus=n, degree=1, blen=48, XMD SHA-256) as
    SA_ClientAgent.py:283-286 calls it, on the GPU.  The client's h_ijt is str(x & 0xFFFF) (:280):
    the first such call computes all 2^16 points in one launch (flm_hash_to_curve_decimal) and later
    calls index the table; any other message (<= 64 bytes) is one flm_hash_to_curve launch."""
    global _h2c_table
    if isinstance(msg, str) and msg.isdigit() and str(int(msg)) == msg and int(msg) < (1 << 16):
        if _h2c_table is None:
            out = np.empty((1 << 16, 64), np.uint8)
            fl = np.empty(1 << 16, np.uint32)
            _check(_lib.flm_hash_to_curve_decimal(_context(), 0, 1 << 16, out.ctypes.data_as(_u8p),
                                                  fl.ctypes.data_as(_u32p)))
            _h2c_table = (out, fl)
        row, f = _h2c_table[0][int(msg)], int(_h2c_table[1][int(msg)])
    else:
        m = msg.encode() if isinstance(msg, str) else bytes(msg)
        buf = np.zeros(64, np.uint8)
        buf[:len(m)] = np.frombuffer(m, np.uint8)
        out, fl, ln = np.empty(64, np.uint8), np.zeros(1, np.uint32), np.array([len(m)], np.uint32)
        _check(_lib.flm_hash_to_curve(_context(), buf.ctypes.data_as(_u8p), ln.ctypes.data_as(_u32p), 1,
                                      out.ctypes.data_as(_u8p), fl.ctypes.data_as(_u32p)))
        row, f = out, int(fl[0])
    if f & 4:
        return Point(0, 0)                   # the point at infinity, as pycryptodome's EccPoint(0, 0)
    b = row.tobytes()
    return Point(int.from_bytes(b[:32], "big"), int.from_bytes(b[32:], "big"))


def client_mask(seeds, signs, L, x=None):
    """x (default: the all-ones input of SA_ClientAgent.py:304) + sum_k signs[k] * PRG(seeds[k])
    for one client: the composition of SA_ClientAgent.py:246-324."""
    seg = np.array([0, len(seeds)], np.int64)
    sd, sg, K = _seed_arrays(seeds, signs)
    out = np.empty(L, np.uint32)
    xp = None
    if x is not None:
        x = np.ascontiguousarray(x, dtype=np.uint32)
        if x.shape != (L,):
            raise RuntimeError("vector length error")
        xp = x.ctypes.data_as(_u32p)
    _check(_lib.flm_client_mask(_context(), xp, 1, seg.ctypes.data_as(_i64p), sd.ctypes.data_as(_u8p),
                                sg.ctypes.data_as(_i8p), L, out.ctypes.data_as(_u32p)))
    return out


class VectorStore:
    """The server's VECTOR bodies on the GPU(s) from arrival to final_sum (flm_store_*): hand each
    body to add() in receiveMessage (:205-210), call partial() in report_process (:346-350) and
    unmask() in reconstruction_process (:529-605), reset() when the pools are cleared (:488-497).
    On FLM_GPUS > 1 devices the rows are spread over the group and S stays slot-sharded."""

    def __init__(self, L, capacity):
        h = _vp()
        g = _server_group()
        if _lib.flm_store_create(ctypes.byref(h), None if g is not None else _context(), g, L, capacity):
            raise RuntimeError(_lib.flm_store_last_error(None).decode())
        self.h, self.L = h, L

    def _check(self, rc):
        if rc:
            raise RuntimeError(_lib.flm_store_last_error(self.h).decode())

    def close(self):
        """Free the store's device rows and pinned staging ring (flm_store_free)."""
        if getattr(self, "h", None) is not None and self.h.value:
            _lib.flm_store_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, sender, vec):
        """A body that is not a uint32[L]-compatible vector is remembered as bad: partial() then
        raises, as report_process does (:348-349)."""
        v = _u32_body(vec, self.L)
        if v is None:
            self._check(_lib.flm_store_add(self.h, int(sender), None, 0))
            return
        self._check(_lib.flm_store_add(self.h, int(sender), v.ctypes.data, self.L))

    def partial(self):
        """S = sum of the stored vectors, left on the GPU(s); raises on a body of the wrong length
        (:348-349)."""
        self._check(_lib.flm_store_partial(self.h))

    def unmask(self, seeds, signs):
        """final_sum = S + sum_k signs[k] * PRG(seeds[k]) as uint32[L] (:538-540, :605)."""
        sd, sg, K = _seed_arrays(seeds, signs)
        out = np.empty(self.L, np.uint32)
        self._check(_lib.flm_store_unmask(self.h, sd.ctypes.data_as(_u8p), sg.ctypes.data_as(_i8p), K,
                                          out.ctypes.data_as(_u32p)))
        return out

    def reset(self):
        self._check(_lib.flm_store_reset(self.h))
