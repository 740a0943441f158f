"""Protocol parameters and host-side round logic of Flamingo (util/param.py surface).

Constants mirror util/param.py:8-32.  The neighbour graph and committee are
derived exactly as util/param.py:38-112 derives them, but computed once per
(root, iteration) for all clients instead of once per call (the reference
re-derives the whole graph string in every findNeighbors call, :63-76, and
the server calls it once per offline client, SA_ServiceAgent.py:359-366).
Every ChaCha20 keystream here is produced on the GPU by the engine
(``MaskEngine.chacha20_encrypt``); the package has no CPU ChaCha20 at all (the
clients' h_ijt PRF is a GPU batch too, client_agent.py).  The host ciphers it
does use are OpenSSL's AES-GCM and ECDSA for the m_i shares and signatures
(flamingo_amd/crypto.py), which are not on the mask path.

The seed tables built here are what the HIP kernels consume:
* client side (SA_ClientAgent.py:304-324): seeds [m_i, s_ij for j in N(i)]
  with signs [+1, +1 if i < j else -1];
* server side (SA_ServiceAgent.py:529-536, 359-380, 587-603): seeds
  [m_i for i in U] with sign -1, then s_ij for every (online i, offline j in
  N(i)) with sign +1 if i > j else -1.
"""
from __future__ import annotations

import hashlib
import math

import numpy as np

# util/param.py:8-32
vector_len = 16000
vector_type = "uint32"
committee_size = 60
fraction = 1 / 3
fixed_key = b"abcd"
nonce = b"\x00" * 8
# waiting times (util/param.py:17-19), in nanoseconds of simulated time
wt_flamingo_report_ns = 10_000_000_000
wt_flamingo_crosscheck_ns = 3_000_000_000
wt_flamingo_reconstruction_ns = 3_000_000_000

_default_engine = None


def default_encrypt():
    """ChaCha20(key, nonce=0^8).encrypt on the GPU through a shared engine."""
    global _default_engine
    if _default_engine is None:
        from .engine import MaskEngine
        _default_engine = MaskEngine(0)
    return _default_engine.chacha20_encrypt


def assert_power_of_two(x: int) -> bool:
    """util/param.py:34-35."""
    return math.ceil(math.log2(x)) == math.floor(math.log2(x))


def choose_committee(root_seed: bytes, committee_size: int, num_clients: int, encrypt=None) -> set:
    """util/param.py:38-53: ChaCha20(root).encrypt(b"secr"*size*128) as uint32, mod N, first distinct."""
    encrypt = encrypt or default_encrypt()
    nums = np.frombuffer(encrypt(root_seed, b"secr" * committee_size * 128), dtype="<u4")
    picked = nums % np.uint32(num_clients)
    committee: set = set()
    for v in picked:
        committee.add(int(v))
        if len(committee) == committee_size:
            break
    return committee


def chosen_table(root_seed: bytes, iteration: int, num_clients: int, neighborhood_size: int, encrypt=None):
    """(N, num_choose) array of the ids each client draws (util/param.py:63-90, before de-duplication)."""
    encrypt = encrypt or default_encrypt()
    seed = encrypt(root_seed, iteration.to_bytes(32, "big"))
    bits = math.ceil(math.log2(num_clients))
    num_choose = bits * neighborhood_size
    bpc = math.ceil(math.log2(num_clients) / 8)
    seglen = num_choose * bpc
    graph = np.frombuffer(encrypt(seed, b"a" * (seglen * num_clients)), dtype=np.uint8)
    g = graph.reshape(num_clients, num_choose, bpc).astype(np.int64)
    val = np.zeros((num_clients, num_choose), np.int64)
    for b in range(bpc):                     # big-endian bytes -> int (:87)
        val = (val << 8) | g[:, :, b]
    return val & ((1 << bits) - 1)


def neighbor_graph(root_seed: bytes, iteration: int, num_clients: int, neighborhood_size: int,
                   encrypt=None) -> list:
    """findNeighbors for every client at once: N(i) = chosen(i) \\ {i}  U  {j != i : i in chosen(j)}.

    Each set is built with the reference's insertion sequence -- its own draws in
    draw order (util/param.py:83-91), then the choosers in ascending id (:95-101) --
    so that iterating it gives the reference's set order, which fixes the order of
    dec_target_pairwise / recon_symbol on the server (SA_ServiceAgent.py:360-378)."""
    ch = chosen_table(root_seed, iteration, num_clients, neighborhood_size, encrypt).tolist()
    choosers = [[] for _ in range(num_clients)]
    for i in range(num_clients):
        for t in ch[i]:
            if t != i:
                choosers[t].append(i)       # i chose t: i is in t's list of choosers
    nbrs = []
    for i in range(num_clients):
        s = set()
        for t in ch[i]:
            if t != i:
                s.add(t)
        for j in choosers[i]:               # ascending: appended in increasing i
            s.add(j)
        nbrs.append(s)
    return nbrs


def find_neighbors(root_seed: bytes, current_iteration: int, num_clients: int, id: int,
                   neighborhood_size: int, encrypt=None) -> set:
    """Drop-in for util/param.findNeighbors (:56-103)."""
    return neighbor_graph(root_seed, current_iteration, num_clients, neighborhood_size, encrypt)[id]


def dropout_pairs(nbrs: list, online, offline, users=None):
    """SA_ServiceAgent.report_process (:341-380): (online nb, offline id) pairs and recon_symbol.

    The offline set is formed as the reference forms it, ``set(users) - set(online)``
    (users defaults to range(N), config/flamingo.py:208), and walked in that set's
    iteration order, each offline id's neighbours in the order of their set -- the
    reference's insertion order of dec_target_pairwise.  Pinned against the
    reference's own recon_symbol in tests/test_ref_golden_cpu.py."""
    online_s = set(int(i) for i in online)
    users = range(len(nbrs)) if users is None else users
    want = set(int(j) for j in offline)
    pairs, signs = [], []
    for cid in set(users) - online_s:
        if cid not in want:
            continue
        for nb in nbrs[cid]:
            if nb in online_s:
                if nb == cid:
                    raise RuntimeError("id should not be its own neighbor.")
                pairs.append((nb, cid))
                signs.append(1 if nb > cid else -1)
    return pairs, signs


# ----------------------------------------------------------- seed tables
def client_seed_table(m: np.ndarray, nbrs: list, pair_seed):
    """CSR seed table for batched client masking (SA_ClientAgent.py:304-324).

    m: (N, 32) self-mask seeds; nbrs: neighbour sets; pair_seed(i, j) -> 32 bytes.
    Returns seg (N+1,), seeds (K, 32) uint8, signs (K,) int8."""
    N = m.shape[0]
    seg = [0]
    seeds, signs = [], []
    for i in range(N):
        seeds.append(m[i].tobytes())
        signs.append(1)
        for j in sorted(nbrs[i]):
            if j == i:
                raise RuntimeError("id itself appears in its neighbor list")  # :323-324
            seeds.append(pair_seed(i, j))
            signs.append(1 if i < j else -1)
        seg.append(len(seeds))
    return (np.array(seg, np.int64), np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32).copy(),
            np.array(signs, np.int8))


def server_seed_table(m: np.ndarray, nbrs: list, online, offline, pair_seed):
    """Seeds and signs of one server round: -PRG(m_i) for i in U, sigma*PRG(s_ij) for dropout pairs."""
    online = [int(i) for i in online]
    pairs, psigns = dropout_pairs(nbrs, online, offline)
    seeds = [m[i].tobytes() for i in online] + [pair_seed(i, j) for i, j in pairs]
    signs = [-1] * len(online) + psigns
    if not seeds:
        return np.zeros((0, 32), np.uint8), np.zeros(0, np.int8)
    return np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32).copy(), np.array(signs, np.int8)


def synthetic_pair_seed(i: int, j: int) -> bytes:
    """Explicit stand-in for s_ij (the reference derives it by ECDH + hash-to-curve,
    SA_ClientAgent.py:256-292; out of this path's scope).  Symmetric in (i, j)."""
    a, b = (i, j) if i < j else (j, i)
    return hashlib.sha256(b"flm-pair" + a.to_bytes(4, "big") + b.to_bytes(4, "big")).digest()


def synthetic_neighbors(N: int, degree: int, seed: int = 0) -> list:
    """A symmetric random graph with ~degree neighbours per client (tests and benches only)."""
    g = np.random.Generator(np.random.PCG64(seed))
    nbrs = [set() for _ in range(N)]
    picks = g.integers(0, N, size=(N, max(1, degree // 2)))
    for i in range(N):
        for t in picks[i].tolist():
            if t != i:
                nbrs[i].add(t)
                nbrs[t].add(i)
    return nbrs


def bench_seed(cfg_id: str, k: int) -> bytes:
    """seed_k = SHA-256(b"flm-bench" || cfg_id || k.to_bytes(4, 'big'))."""
    return hashlib.sha256(b"flm-bench" + cfg_id.encode() + k.to_bytes(4, "big")).digest()
