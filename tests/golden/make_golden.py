"""Generate the committed golden fixtures in tests/golden/ (run in the build container).

Independence: every PRG value here comes from OpenSSL's ChaCha20
(``EVP_chacha20`` through ctypes on libcrypto.so.3), NOT from oracle/ or
flamingo_amd/.  With a zero 16-byte IV (RFC 7539 layout: 32-bit counter +
96-bit nonce) OpenSSL's keystream equals the 8-byte-zero-nonce DJB ChaCha20
that pycryptodomex uses in the reference (util/param.py:32, 64-bit counter)
for every block index < 2^32, which covers every length used here.

These vectors are the independent-implementation pin.  The reference's OWN
code produces the other set: tests/golden/make_ref_golden.py imports
util/param.py, util/util.py, util/crypto and agent/flamingo/SA_*Agent.py from
/root/reference under a dependency shim (tests/golden/refshim.py) and records
whole protocol rounds (ref_golden.json / ref_golden.npz), which
tests/test_ref_golden_{cpu,gpu}.py compare against the oracle and the HIP path.

Outputs:
  golden.json      -- PRG heads/tails/digests, graph digests, round fixtures
  round_n128.npz   -- N=128, L=16384 round: seeds, signs, offline set
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ABCD = 0x64636261

_crypto = ctypes.CDLL("libcrypto.so.3")
_crypto.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
_crypto.EVP_chacha20.restype = ctypes.c_void_p
_crypto.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_char_p, ctypes.c_char_p]
_crypto.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, ctypes.c_int]
_crypto.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]


def ossl_encrypt(key: bytes, data: bytes) -> bytes:
    """OpenSSL ChaCha20 with a zero IV == ChaCha20.new(key, nonce=8x00).encrypt(data)."""
    assert len(key) == 32
    ctx = _crypto.EVP_CIPHER_CTX_new()
    try:
        assert _crypto.EVP_EncryptInit_ex(ctx, _crypto.EVP_chacha20(), None, key, b"\x00" * 16) == 1
        out = ctypes.create_string_buffer(len(data) + 64)
        outl = ctypes.c_int(0)
        if data:
            assert _crypto.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), data, len(data)) == 1
            assert outl.value == len(data)
        return out.raw[:len(data)]
    finally:
        _crypto.EVP_CIPHER_CTX_free(ctx)


def ossl_prg(seed: bytes, L: int) -> np.ndarray:
    """The reference idiom: frombuffer(ChaCha20(seed).encrypt(b"abcd"*L), uint32)."""
    return np.frombuffer(ossl_encrypt(seed, b"abcd" * L), dtype="<u4").astype(np.uint32)


def digest(v: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(v, dtype="<u4").tobytes()).hexdigest()


def seed_of(label: str) -> bytes:
    return hashlib.sha256(label.encode()).digest()


# graph restatement over OpenSSL (same statement as util/param.py:56-103)
def graph(root: bytes, it: int, n: int, o: int):
    cur = ossl_encrypt(root, it.to_bytes(32, "big"))
    num_choose = math.ceil(math.log2(n)) * o
    bpc = math.ceil(math.log2(n) / 8)
    seglen = num_choose * bpc
    g = ossl_encrypt(cur, b"a" * (seglen * n))
    bits = math.ceil(math.log2(n))
    chosen = []
    for i in range(n):
        seg = g[i * seglen:(i + 1) * seglen]
        chosen.append([int.from_bytes(seg[t * bpc:(t + 1) * bpc], "big") & ((1 << bits) - 1)
                       for t in range(num_choose)])
    nbrs = []
    for cid in range(n):
        s = set()
        for t in chosen[cid]:
            if t != cid:
                s.add(t)
        for i in range(n):
            if i != cid and cid in chosen[i]:
                s.add(i)
        nbrs.append(s)
    return nbrs


def main():
    out = {"generator": "tests/golden/make_golden.py (OpenSSL EVP_chacha20, zero IV)",
           "abcd": ABCD}

    # 1. PRG vectors: heads, tails and digests over lengths covering partial blocks.
    seeds = {"zero": b"\x00" * 32, "ff": b"\xff" * 32}
    for i in range(6):
        seeds[f"s{i}"] = seed_of(f"flamingo-golden-{i}")
    prg = []
    for name, s in seeds.items():
        for L in (1, 15, 16, 17, 1000, 16000, 16384):
            v = ossl_prg(s, L)
            prg.append({"seed": s.hex(), "name": name, "L": L, "head": v[:32].tolist(),
                        "tail": v[-32:].tolist(), "sha256": digest(v)})
    out["prg"] = prg

    # 2. Slot windows of long streams: PRG(seed)[slot0 : slot0+n].
    win = []
    long_L = (1 << 20) + 64
    for name in ("s0", "s1"):
        full = ossl_prg(seeds[name], long_L)
        for slot0, n in ((16, 1024), (4096, 4096), (1 << 17, 1 << 17), ((1 << 20) - 16, 80),
                         (0, 1 << 20)):
            v = full[slot0:slot0 + n]
            win.append({"seed": seeds[name].hex(), "slot0": slot0, "n": n, "sha256": digest(v),
                        "head": v[:16].tolist()})
    out["prg_windows"] = win

    # 3. Raw keystream bytes (findNeighbors / committee use encrypt on other plaintexts).
    ks = []
    for name in ("zero", "s2"):
        data = bytes(range(256)) * 3
        ks.append({"key": seeds[name].hex(), "data": data.hex(), "ct": ossl_encrypt(seeds[name], data).hex()})
    out["keystream"] = ks

    # 4. Neighbour graph (util/param.py:56-103) restated over OpenSSL.  SURVEY.md 8c
    #    lists a findNeighbors probe said to come from the reference under a
    #    dependency shim; it does not reproduce with any zero-root reading
    #    (checked over every id and iterations 0-4), so it is NOT used as a pin.
    graphs = []
    for n, o, it in ((128, 1, 1), (128, 1, 2), (1024, 1, 1), (1024, 2, 1)):
        nb = graph(b"\x00" * 32, it, n, o)
        graphs.append({"num_clients": n, "neighborhood_size": o, "iteration": it,
                       "degree_sum": int(sum(len(s) for s in nb)),
                       "sha256": hashlib.sha256(json.dumps([sorted(s) for s in nb]).encode()).hexdigest(),
                       "first8": [sorted(nb[i]) for i in range(8)]})
    out["graphs"] = graphs

    # 5. Committee (util/param.py:38-53) for root 0^32.
    nums = np.frombuffer(ossl_encrypt(b"\x00" * 32, b"secr" * 60 * 128), dtype="<u4")
    for n in (128, 1024):
        com, c = set(), 0
        while len(com) < 60:
            com.add(int(nums[c] % n)); c += 1
        out.setdefault("committee", []).append({"num_clients": n, "members": sorted(com)})

    # 6. One full round, N=128, L=16384, root 0^32, iteration 1, o=1.
    N, L = 128, 16384
    nb = graph(b"\x00" * 32, 1, N, 1)
    m = np.stack([np.frombuffer(seed_of(f"m-{i}"), np.uint8) for i in range(N)])
    def pair_seed(i, j):
        a, b = min(i, j), max(i, j)
        return np.frombuffer(seed_of(f"pair-{a}-{b}"), np.uint8)
    offline = sorted(int(x) for x in np.random.Generator(np.random.PCG64(7)).choice(N, 2, replace=False))
    online = [i for i in range(N) if i not in offline]
    # client side (SA_ClientAgent.py:304-324), all-ones input
    rows = np.zeros((N, L), np.uint32)
    seg = [0]; cseeds = []; csigns = []
    for i in range(N):
        v = np.ones(L, np.uint32)
        v += ossl_prg(m[i].tobytes(), L)
        cseeds.append(m[i]); csigns.append(1)
        for j in sorted(nb[i]):
            p = ossl_prg(pair_seed(i, j).tobytes(), L)
            if i < j:
                v += p; csigns.append(1)
            else:
                v -= p; csigns.append(-1)
            cseeds.append(pair_seed(i, j))
        rows[i] = v
        seg.append(len(cseeds))
    # server side (SA_ServiceAgent.py:346-350, 529-536, 587-605)
    S = np.zeros(L, np.uint32)
    for i in online:
        S += rows[i]
    M = np.zeros(L, np.uint32)
    for i in online:
        M = M - ossl_prg(m[i].tobytes(), L)
    pairs, psigns = [], []
    for j in offline:
        for i in sorted(nb[j]):
            if i in online:
                pairs.append((i, j)); psigns.append(1 if i > j else -1)
    C = np.zeros(L, np.uint32)
    for (i, j), s in zip(pairs, psigns):
        p = ossl_prg(pair_seed(i, j).tobytes(), L)
        C = C + p if s == 1 else C - p
    final = S + C + M
    assert np.all(final == len(online)), "protocol invariant out == |U| violated"
    sseeds = np.concatenate([m[online], np.stack([pair_seed(i, j) for i, j in pairs])]) if pairs else m[online]
    ssigns = np.array([-1] * len(online) + psigns, np.int8)
    # random-input variant: uniform u32 client inputs
    x = np.random.Generator(np.random.PCG64(20231015)).integers(0, 2**32, size=(N, L), dtype=np.uint32)
    rows_x = rows - np.uint32(1) + x
    final_x = np.zeros(L, np.uint32)
    for i in online:
        final_x += rows_x[i]
    final_x += C + M
    expect_x = np.zeros(L, np.uint32)
    for i in online:
        expect_x += x[i]
    assert np.array_equal(final_x, expect_x)
    np.savez_compressed(os.path.join(HERE, "round_n128.npz"),
                        client_seeds=np.stack(cseeds), client_signs=np.array(csigns, np.int8),
                        client_seg=np.array(seg, np.int64), server_seeds=sseeds, server_signs=ssigns,
                        online=np.array(online, np.int32), offline=np.array(offline, np.int32),
                        pairs=np.array(pairs, np.int32).reshape(-1, 2))
    out["round_n128"] = {
        "N": N, "L": L, "offline": offline, "num_pairs": len(pairs),
        "rows_sha256": digest(rows), "S_sha256": digest(S), "M_sha256": digest(M),
        "C_sha256": digest(C), "final_value": int(len(online)),
        "rows_x_sha256": digest(rows_x), "final_x_sha256": digest(final_x),
        "x_rng": "PCG64(20231015).integers(0, 2**32, (128, 16384), uint32)",
        "rows_head": rows[:4, :8].tolist(), "C_head": C[:8].tolist(), "M_head": M[:8].tolist(),
    }

    # 7. mod-2^32 edge case: all-0xFFFFFFFF rows.
    ff = np.full((5, 33), 0xFFFFFFFF, np.uint32)
    out["edge_ff"] = {"N": 5, "L": 33, "sum": int(ff.sum(axis=0, dtype=np.uint32)[0])}

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    sys.exit(main())
