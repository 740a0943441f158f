"""TEST INFRASTRUCTURE ONLY -- CPU oracle for Flamingo's mask-and-aggregate path.

Only tests/, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
bench.py may import this module; the product package ``flamingo_amd`` never
does.  Two independent restatements live here:

* ``liboracle.so`` (oracle/flamingo_oracle.c) -- scalar C, used for large
  cases and as the CPU baseline;
* numpy restatements (``np_chacha20_blocks`` ...) -- vectorised over blocks,
  used to cross-check the C restatement on small cases.

Reference call sites restated (paths relative to /root/reference):

* PRG: ``ChaCha20.new(key=seed, nonce=param.nonce).encrypt(param.fixed_key*L)``
  + ``np.frombuffer(.., 'uint32')`` -- agent/flamingo/SA_ClientAgent.py:248-250,
  296-298; agent/flamingo/SA_ServiceAgent.py:533-536, 596-603.
* ``choose_committee`` -- util/param.py:38-53.
* ``findNeighbors`` / ``parse_segment_to_list`` -- util/param.py:56-112.
* dropout pairs and ``recon_symbol`` -- agent/flamingo/SA_ServiceAgent.py:341-380.
* client masking -- agent/flamingo/SA_ClientAgent.py:304-324.
* server aggregate + unmask -- agent/flamingo/SA_ServiceAgent.py:346-350,
  529-540, 587-605.

PINNED to the reference itself: tests/test_ref_golden_cpu.py checks these
functions against fixtures the reference's own agents produced
(tests/golden/make_ref_golden.py: util/param.py and agent/flamingo imported from
the reference under a pycryptodomex/libnum stand-in) -- client vectors, the
server's S / M / C / final_sum, committee, graphs and recon_symbol order.  Also
pinned by RFC 7539 vectors, OpenSSL-generated fixtures (tests/golden/) and the
out == |U| protocol invariant; see DESIGN.md section 3.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLM_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")   # env: sanitizer build

ABCD = 0x64636261            # LE32(b"abcd"), util/param.py:12
NONCE = b"\x00" * 8          # util/param.py:32
VECTOR_LEN = 16000           # util/param.py:8
COMMITTEE_SIZE = 60          # util/param.py:10
SIGMA = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)

_lib = None


def build(force: bool = False) -> str:
    """Compile oracle/liboracle.so with gcc (checker only)."""
    if os.environ.get("FLM_ORACLE_LIB"):
        return LIB_PATH
    if force or not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "flamingo_oracle.c"))):
        subprocess.run(["make", "-C", HERE, "-B" if force else "all"], check=True,
                       stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        i8p = ctypes.POINTER(ctypes.c_int8)
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.flmo_chacha20_block.argtypes = [u8p, u8p, ctypes.c_uint64, u32p]
        L.flmo_chacha20_xor.argtypes = [u8p, u8p, ctypes.c_uint64, u8p, u8p, ctypes.c_size_t]
        L.flmo_prg_words.argtypes = [u8p, ctypes.c_uint64, ctypes.c_size_t, u32p]
        L.flmo_aggregate_unmask.argtypes = [u32p, ctypes.c_size_t, ctypes.c_int, u8p, i8p,
                                            ctypes.c_int, ctypes.c_size_t, ctypes.c_uint64, u32p,
                                            ctypes.c_int]
        L.flmo_aggregate_unmask.restype = ctypes.c_int
        L.flmo_client_mask.argtypes = [u32p, ctypes.c_size_t, ctypes.c_int, i64p, u8p, i8p,
                                       ctypes.c_size_t, u32p, ctypes.c_size_t, ctypes.c_int]
        L.flmo_client_mask.restype = ctypes.c_int
        L.flmo_has_openmp.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _bytes_arr(b: bytes) -> np.ndarray:
    return np.frombuffer(bytes(b), dtype=np.uint8).copy()


# ----------------------------------------------------------------- C oracle
def chacha20_block(key: bytes, nonce: bytes, counter: int) -> np.ndarray:
    out = np.zeros(16, dtype=np.uint32)
    lib().flmo_chacha20_block(_p(_bytes_arr(key), ctypes.c_uint8), _p(_bytes_arr(nonce), ctypes.c_uint8),
                              counter, _p(out, ctypes.c_uint32))
    return out


def chacha20_encrypt(key: bytes, data: bytes, nonce: bytes = NONCE, counter: int = 0) -> bytes:
    """ChaCha20.new(key=key, nonce=nonce).encrypt(data) (DJB, 64-bit counter)."""
    src = _bytes_arr(data) if len(data) else np.zeros(1, np.uint8)
    dst = np.zeros_like(src)
    lib().flmo_chacha20_xor(_p(_bytes_arr(key), ctypes.c_uint8), _p(_bytes_arr(nonce), ctypes.c_uint8),
                            counter, _p(src, ctypes.c_uint8), _p(dst, ctypes.c_uint8), len(data))
    return dst[:len(data)].tobytes()


def prg(seed: bytes, L: int, slot0: int = 0) -> np.ndarray:
    """PRG(seed)[slot0:slot0+L] -- the reference's mask vector, uint32."""
    out = np.zeros(max(L, 1), dtype=np.uint32)
    lib().flmo_prg_words(_p(_bytes_arr(seed), ctypes.c_uint8), slot0, L, _p(out, ctypes.c_uint32))
    return out[:L]


def aggregate_unmask(rows: np.ndarray, seeds: np.ndarray, signs: np.ndarray, L: int | None = None,
                     slot0: int = 0, threads: int = 1) -> np.ndarray:
    """out = sum(rows) + sum_k signs[k] * PRG(seeds[k])  (mod 2^32)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    if rows.ndim == 1:
        rows = rows[None, :]
    N = rows.shape[0]
    pitch = rows.shape[1] if rows.size else 0
    if L is None:
        L = pitch
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
    signs = np.ascontiguousarray(signs, dtype=np.int8).reshape(-1)
    assert seeds.shape[0] == signs.shape[0]
    out = np.zeros(max(L, 1), dtype=np.uint32)
    rows_c = rows if rows.size else np.zeros((1, 1), np.uint32)
    seeds_c = seeds if seeds.size else np.zeros((1, 32), np.uint8)
    signs_c = signs if signs.size else np.ones(1, np.int8)
    rc = lib().flmo_aggregate_unmask(_p(rows_c, ctypes.c_uint32), max(pitch, L) if N else L, N,
                                     _p(seeds_c, ctypes.c_uint8), _p(signs_c, ctypes.c_int8),
                                     seeds.shape[0], L, slot0, _p(out, ctypes.c_uint32), threads)
    if rc != 0:
        raise RuntimeError(f"oracle aggregate_unmask failed: {rc}")
    return out[:L]


def client_mask(seg: np.ndarray, seeds: np.ndarray, signs: np.ndarray, L: int,
                x: np.ndarray | None = None, threads: int = 1) -> np.ndarray:
    """y_i = x_i + sum_{k in seg i} signs[k]*PRG(seeds[k]); x=None -> all ones."""
    seg = np.ascontiguousarray(seg, dtype=np.int64)
    N = seg.shape[0] - 1
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
    signs = np.ascontiguousarray(signs, dtype=np.int8).reshape(-1)
    out = np.zeros((N, L), dtype=np.uint32)
    xp = None
    if x is not None:
        x = np.ascontiguousarray(x, dtype=np.uint32)
        xp = _p(x, ctypes.c_uint32)
    lib().flmo_client_mask(xp, L, N, _p(seg, ctypes.c_int64), _p(seeds, ctypes.c_uint8),
                           _p(signs, ctypes.c_int8), L, _p(out, ctypes.c_uint32), L, threads)
    return out


# ------------------------------------------------------- numpy restatement
def _rotl(v: np.ndarray, c: int) -> np.ndarray:
    return (v << np.uint32(c)) | (v >> np.uint32(32 - c))


def np_chacha20_blocks(key: bytes, counters: np.ndarray, nonce: bytes = NONCE) -> np.ndarray:
    """Vectorised ChaCha20 block function over an array of 64-bit counters.

    Returns uint32 array of shape (len(counters), 16)."""
    counters = np.asarray(counters, dtype=np.uint64)
    n = counters.shape[0]
    kw = np.frombuffer(key, dtype="<u4").astype(np.uint32)
    nw = np.frombuffer(nonce, dtype="<u4").astype(np.uint32)
    st = [np.full(n, SIGMA[i], np.uint32) for i in range(4)]
    st += [np.full(n, kw[i], np.uint32) for i in range(8)]
    st += [(counters & np.uint64(0xFFFFFFFF)).astype(np.uint32),
           (counters >> np.uint64(32)).astype(np.uint32),
           np.full(n, nw[0], np.uint32), np.full(n, nw[1], np.uint32)]
    x = [s.copy() for s in st]

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 16)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 12)
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 8)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 7)

    with np.errstate(over="ignore"):
        for _ in range(10):
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
        return np.stack([x[i] + st[i] for i in range(16)], axis=1)


def np_prg(seed: bytes, L: int, slot0: int = 0) -> np.ndarray:
    if L == 0:
        return np.zeros(0, np.uint32)
    b0 = slot0 // 16
    b1 = (slot0 + L + 15) // 16
    ks = np_chacha20_blocks(seed, np.arange(b0, b1, dtype=np.uint64)).reshape(-1)
    off = slot0 - 16 * b0
    return ks[off:off + L] ^ np.uint32(ABCD)


def np_chacha20_encrypt(key: bytes, data: bytes, nonce: bytes = NONCE) -> bytes:
    n = len(data)
    nb = (n + 63) // 16 // 4
    ks = np_chacha20_blocks(key, np.arange(nb, dtype=np.uint64), nonce).astype("<u4").tobytes()
    return (np.frombuffer(data, np.uint8) ^ np.frombuffer(ks[:n], np.uint8)).tobytes()


# ------------------------------------------- host-side protocol restatement
def choose_committee(root_seed: bytes, committee_size: int, num_clients: int, encrypt=None) -> set:
    """util/param.py:38-53."""
    encrypt = encrypt or chacha20_encrypt
    stream = encrypt(root_seed, b"secr" * committee_size * 128)
    nums = np.frombuffer(stream, dtype=np.uint32)
    committee = set()
    cnt = 0
    while len(committee) < committee_size:
        committee.add(int(nums[cnt] % num_clients))
        cnt += 1
    return committee


def _graph_string(root_seed: bytes, iteration: int, num_clients: int, neighborhood_size: int,
                  encrypt=None):
    encrypt = encrypt or chacha20_encrypt
    current_seed = encrypt(root_seed, iteration.to_bytes(32, "big"))                 # :63-64
    num_choose = math.ceil(math.log2(num_clients)) * neighborhood_size               # :70-71
    bytes_per_client = math.ceil(math.log2(num_clients) / 8)                         # :73
    segment_len = num_choose * bytes_per_client
    graph = encrypt(current_seed, b"a" * (segment_len * num_clients))                # :75-76
    return graph, num_choose, bytes_per_client, segment_len


def _segment_ids(seg: bytes, num_choose: int, bytes_per_client: int, bits: int):
    mask = (1 << bits) - 1
    return [int.from_bytes(seg[i * bytes_per_client:(i + 1) * bytes_per_client], "big") & mask
            for i in range(num_choose)]


def find_neighbors(root_seed: bytes, iteration: int, num_clients: int, cid: int,
                   neighborhood_size: int, encrypt=None) -> set:
    """util/param.py:56-103 (the set the reference returns)."""
    graph, num_choose, bpc, seglen = _graph_string(root_seed, iteration, num_clients,
                                                   neighborhood_size, encrypt)
    bits = math.ceil(math.log2(num_clients))
    nbrs = set()
    for t in _segment_ids(graph[cid * seglen:(cid + 1) * seglen], num_choose, bpc, bits):
        if t == cid or t in nbrs:
            continue
        nbrs.add(t)
    for i in range(num_clients):
        if i == cid:
            continue
        if cid in set(_segment_ids(graph[i * seglen:(i + 1) * seglen], num_choose, bpc, bits)):
            nbrs.add(i)
    return nbrs


def dropout_pairs(root_seed: bytes, iteration: int, num_clients: int, neighborhood_size: int,
                  online: set, users=None, encrypt=None):
    """SA_ServiceAgent.report_process (:341-380): ordered (online nb, offline id) pairs and signs.

    Iteration order mirrors the reference: offline ids in set order, then each
    offline id's neighbour set in set order."""
    users = range(num_clients) if users is None else users
    offline = set(users) - set(online)
    pairs, signs = [], []
    for cid in offline:
        for nb in find_neighbors(root_seed, iteration, num_clients, cid, neighborhood_size, encrypt):
            if nb in online:
                if nb == cid:
                    raise RuntimeError("id should not be its own neighbor.")
                pairs.append((nb, cid))
                signs.append(1 if nb > cid else -1)
    return pairs, signs
