"""CPU checks of the launch planner through flm_plan_aggregate (no GPU needed).

For every round shape the work items must cover each output slot with every
row exactly once and every seed exactly once (over the mask window), add the
negative-sign bias exactly once per masked slot, use atomics wherever a slot
has more than one writer (and then zero-fill), and start every mask tile on a
ChaCha block boundary."""
import ctypes

import numpy as np
import pytest

ITEM = np.dtype([("row_in", "<u8"), ("row_out", "<u8"), ("mask_out", "<u8"), ("mask_ctr", "<u8"),
                 ("nrows", "<u4"), ("k0", "<u4"), ("nseeds", "<u4"), ("row_valid", "<u4"),
                 ("mask_valid", "<u4"), ("flags", "<u4"), ("row_bias", "<u4"), ("mask_bias", "<u4")])
HAS_ROWS, HAS_MASK, SAME, ROW_ATOMIC, MASK_ATOMIC, BIAS_NNEG = 1, 2, 4, 8, 16, 32


def plan(N, K, L, lo=0, hi=None, pitch=None, prg_slot0=0, subtiles=0, pairing=1):
    from flamingo_amd import _lib
    lib = _lib.load()
    hi = L if hi is None else hi
    pitch = pitch or (L + 63) // 64 * 64
    n, fl = ctypes.c_int(), ctypes.c_int()
    assert lib.flm_plan_aggregate(subtiles, pairing, pitch, N, K, L, lo, hi, prg_slot0, None, 0,
                                  ctypes.byref(n), ctypes.byref(fl)) == 0
    buf = np.zeros(max(1, n.value), ITEM)
    assert lib.flm_plan_aggregate(subtiles, pairing, pitch, N, K, L, lo, hi, prg_slot0,
                                  buf.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(n),
                                  ctypes.byref(fl)) == 0
    return buf[: n.value], fl.value, pitch


@pytest.mark.parametrize("N,K,L,lo,hi,pairing", [
    (1024, 1024, 1 << 20, 0, None, 1),          # c4, one GPU
    (1024, 1024, 1 << 18, 0, None, 1),          # c3: 256 tiles split into 8 same-tile parts
    (1024, 1000, 1 << 18, 0, None, 1),          # c3 with dropouts (K != N)
    (1024, 204, 1 << 20, 0, None, 1),           # pairs-only
    (1024, 8192, 1 << 20, 3 << 17, 4 << 17, 1),  # rank 3 of 8
    (1024, 8192, 1 << 20, 3 << 17, 4 << 17, 0),  # interleaved items
    (128, 128, 16384, 0, None, 1),              # c2 (split into parts, atomics)
    (128, 156, 16000, 0, None, 1),              # default vector_len, ragged tail
    (0, 7, 1000, 0, None, 1),                   # masks only
    (5, 0, 1000, 0, None, 1),                   # rows only
    (33, 33, 4100, 1024, 3072, 1),              # window inside
    (7, 3, 70000, 69984, 70000, 1),             # last block only
    (128, 1024, 1 << 20, 7 << 17, 8 << 17, 2),  # strong-scaled c4, rank 7 of 8, same-tile window items
    (256, 1024, 1 << 20, 1 << 18, 2 << 18, 2),  # rank 1 of 4
    (512, 1024, 1 << 20, 0, 1 << 19, 2),        # rank 0 of 2
    (1024, 8192, 1 << 20, 3 << 17, 4 << 17, 2),
    (33, 40, 4100, 1024, 3072, 2),              # window inside, ragged
    (7, 3, 70000, 69984, 70000, 2),             # last block only (one part)
    (5, 64, 70000, 4096, 69984, 2),             # fewer rows than parts
])
def test_plan_covers_everything_once(N, K, L, lo, hi, pairing):
    hi = L if hi is None else hi
    items, flags, pitch = plan(N, K, L, lo, hi, pairing=pairing)
    needs_zero, atomics = flags & 1, flags & 2
    rows_cnt = np.zeros(L, np.int64)       # sum of row counts per slot
    rows_lo = np.full(L, -1, np.int64)
    seeds_cnt = np.zeros(L, np.int64)
    bias_cnt = np.zeros(L, np.int64)
    writers = np.zeros(L, np.int64)
    row_ranges, seed_ranges = {}, {}
    for it in items:
        f = int(it["flags"])
        if f & HAS_ROWS:
            o, v = int(it["row_out"]), int(it["row_valid"])
            a = (int(it["row_in"]) - o) // pitch
            assert (int(it["row_in"]) - o) % pitch == 0
            rows_cnt[o:o + v] += int(it["nrows"])
            row_ranges.setdefault(o, []).append((a, a + int(it["nrows"])))
            if not (f & SAME):
                writers[o:o + v] += 1
            if writers[o:o + v].max() > 1 or (f & ROW_ATOMIC):
                pass
        if f & HAS_MASK:
            o, v = int(it["mask_out"]), int(it["mask_valid"])
            assert (o % 16) == 0 and int(it["mask_ctr"]) * 16 == o
            seeds_cnt[o:o + v] += int(it["nseeds"])
            seed_ranges.setdefault(o, []).append((int(it["k0"]), int(it["k0"]) + int(it["nseeds"])))
            writers[o:o + v] += 1
            if f & BIAS_NNEG:
                bias_cnt[o:o + v] += 1
    if N:
        assert np.all(rows_cnt == N)
        for o, rs in row_ranges.items():           # row sub-ranges partition [0, N)
            rs.sort()
            assert rs[0][0] == 0 and rs[-1][1] == N
            assert all(b == c for (_, b), (c, _) in zip(rs, rs[1:]))
    if K:
        assert np.all(seeds_cnt[lo:hi] == K) and np.all(seeds_cnt[:lo] == 0) and np.all(seeds_cnt[hi:] == 0)
        assert np.all(bias_cnt[lo:hi] == 1) and bias_cnt.sum() == hi - lo
        for o, rs in seed_ranges.items():
            rs.sort()
            assert rs[0][0] == 0 and rs[-1][1] == K
    multi = writers > 1
    if multi.any():
        assert atomics and needs_zero
        for it in items:
            f = int(it["flags"])
            if f & HAS_MASK:
                o, v = int(it["mask_out"]), int(it["mask_valid"])
                if multi[o:o + v].any():
                    assert f & MASK_ATOMIC
    if N == 0 and (lo > 0 or hi < L or K == 0):
        assert needs_zero
    # enough workgroups to fill the chip for the large shapes
    if N * L >= (1 << 28):
        assert len(items) >= 256


def test_plan_modes():
    _, f, _ = plan(1024, 1024, 1 << 20)
    assert f & 4 and not f & 2 and (f >> 8) == 1          # single tile, stores, 1024-slot tiles
    items, f, _ = plan(1024, 1024, 1 << 18)
    assert f & 4 and f & 2 and f & 1 and len(items) == 2048  # c3: same-tile parts, atomics
    assert all(int(it["flags"]) & SAME for it in items)
    _, f, _ = plan(1024, 204, 1 << 20)
    assert f & 8 and (f >> 8) == 4                         # seed-light: 4096-slot tiles
    _, f, _ = plan(1024, 8192, 1 << 20, 0, 1 << 17)
    assert f & 2 and f & 1 and not f & 4                   # shard: dual-tile, atomics
    items, f, _ = plan(128, 1024, 1 << 20, 7 << 17, 8 << 17, pairing=2)
    assert f & 4 and f & 2 and f & 1 and (f >> 8) == 1      # shard as same-tile parts: merged kernel
    heavy = [(int(it["flags"]) & HAS_MASK) != 0 for it in items]
    assert sum(heavy) == 128 * 8 and len(items) == 128 * 8 + 896
    assert heavy[0] and heavy.index(False) <= 3              # rows-only items spread between the heavy ones
    gaps = np.diff(np.flatnonzero(~np.array(heavy)))
    assert gaps.max() <= 3


def test_pick_cus_balances_xcds():
    """ServerReconstruction's EC CU set: CU-mask bit i selects XCD i % 8 (profiles/r01_cu_map_probe.log),
    so "first k" takes k/8 CUs from every XCD; the complement is what the unmask runs on."""
    from flamingo_amd.reconstruct import pick_cus
    for k in (8, 16, 24, 32):
        ec = pick_cus(256, k, "first")
        assert len(ec) == k and len(set(ec)) == k
        per_xcd = np.bincount(np.array(ec) % 8, minlength=8)
        assert per_xcd.min() == per_xcd.max() == k // 8
    st = pick_cus(256, 24, "stride")
    assert len(st) == 24 and max(st) < 256


@pytest.mark.parametrize("G", [1, 2, 3, 4, 7, 8, 16])
def test_shard_and_client_bounds_partition_the_round(G):
    """flm_shard_bounds / flm_client_bounds (the library's multi-GPU geometry, host-only): the
    shards tile [0, L) in order with 16-slot-aligned starts, each S = round_up(L, 1024 G)/G long
    at most; clients tile [0, N); and distributed.py's Python view agrees."""
    from flamingo_amd import distributed as D
    from flamingo_amd.engine import client_bounds, shard_bounds
    for L in (1, 15, 1000, 16000, 16384, 70000, 1 << 18, (1 << 20) + 48):
        prev = 0
        for r in range(G):
            lo, hi, S = shard_bounds(L, G, r)
            assert (lo, hi) == D.shard_bounds(L, G, r)
            assert S * G == D.padded_length(L, G) and S % 1024 == 0
            assert lo == prev and lo <= hi and hi - lo <= S and (lo % 16 == 0 or lo == hi == L)
            prev = hi
        assert prev == L
    for N in (0, 1, 5, 128, 1024, 4096):
        prev = 0
        for r in range(G):
            c0, c1 = client_bounds(N, G, r)
            assert (c0, c1) == D.client_bounds(N, G, r) and c0 == prev and c0 <= c1
            prev = c1
        assert prev == N
