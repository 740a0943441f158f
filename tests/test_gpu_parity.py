"""Parity of the HIP path (through the C ABI) against the CPU oracle and the
OpenSSL-generated golden fixtures.  Bit-exact: this is uint32 arithmetic.

Edge cases follow what the reference's path can see: lengths that are not
multiples of a ChaCha block (default vector_len 16000, util/param.py:8), no
dropouts (K = |U|, SA_ServiceAgent.py:538-540), dropouts with both signs
(:375-378), mod-2^32 wrap, empty sets, and the full benchmark size through
the out == |U| invariant (SA_ClientAgent.py:304 + SA_ServiceAgent.py:605).
"""
import hashlib

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def h(v):
    return hashlib.sha256(np.ascontiguousarray(v, dtype="<u4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def eng():
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    yield e
    e.close()


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def rand_case(seed, N, K, L):
    g = rng(seed)
    rows = g.integers(0, 2**32, size=(N, L), dtype=np.uint32)
    seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    return rows, seeds, signs


# ------------------------------------------------------------------ PRG
def test_prg_golden(eng, golden):
    by_seed = {}
    for e in golden["prg"]:
        by_seed.setdefault(e["seed"], []).append(e)
    for seed_hex, entries in by_seed.items():
        seed = bytes.fromhex(seed_hex)
        for e in entries:
            v = eng.prg(seed, e["L"])
            assert v[:32].tolist() == e["head"], (e["name"], e["L"])
            assert h(v) == e["sha256"], (e["name"], e["L"])


def test_prg_windows_golden(eng, golden):
    for e in golden["prg_windows"]:
        seed = bytes.fromhex(e["seed"])
        if e["slot0"] % 16:
            continue
        v = eng.prg(seed, e["n"], slot0=e["slot0"])
        assert h(v) == e["sha256"], (e["slot0"], e["n"])


def test_prg_expand_batch_vs_oracle(eng):
    g = rng(11)
    seeds = g.integers(0, 256, size=(37, 32), dtype=np.uint8)
    for L in (1, 15, 16, 17, 1000, 1023, 1024, 1025, 16000, 16385, 40000):
        got = eng.prg_expand(seeds, L)
        for k in (0, 1, 17, 36):
            assert np.array_equal(got[k], O.prg(seeds[k].tobytes(), L)), (k, L)


@pytest.mark.parametrize("waves", [1, 64, 256])
def test_prg_expand_dev_kernel(eng, waves):
    """prg_expand_kernel (flm_prg_expand_dev) with grids from far fewer workgroups than units (each
    takes a run of units across several seeds) to more workgroups than units: ragged L (tails inside
    a 16-word block, inside a 1024-slot chunk), PRG windows (slot0), a padded pitch that must stay
    untouched, and the whole output against oracle.prg (SA_ServiceAgent.py:596-603)."""
    import torch
    g = rng(40 + waves)
    eng.set_tuning("expand_waves", waves)
    try:
        for L, slot0, pad in ((1, 0, 4), (17, 16, 0), (1023, 4096, 8), (1025, 0, 4), (5000, 2**20 - 5008, 12),
                              (40000, 2**30, 0)):
            K = int(g.integers(1, 40))
            seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
            pitch = (L + 3) // 4 * 4 + pad
            out = torch.full((K, pitch), 0x3C3C3C3C, dtype=torch.int32, device="cuda")
            eng.prg_expand_dev(torch.from_numpy(seeds).cuda(), out, L, slot0=slot0)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            for k in range(K):
                assert np.array_equal(got[k, :L], O.prg(seeds[k].tobytes(), L, slot0)), (waves, L, slot0, k)
            assert np.all(got[:, L:] == 0x3C3C3C3C), (waves, L, "wrote past L")
            assert eng.last_plan()["variant"] == 101
    finally:
        eng.set_tuning("expand_waves", 128)


def test_keystream_golden(eng, golden):
    for e in golden["keystream"]:
        key, data = bytes.fromhex(e["key"]), bytes.fromhex(e["data"])
        assert eng.chacha20_encrypt(key, data).hex() == e["ct"]
    # arbitrary nonce / counter against the oracle
    key = bytes(range(32))
    data = bytes(rng(5).integers(0, 256, 1000, dtype=np.uint8))
    nonce = bytes.fromhex("0000004a00000000")
    assert eng.chacha20_encrypt(key, data, nonce, counter=7) == O.chacha20_encrypt(key, data, nonce, counter=7)


# ------------------------------------------------------------- client side
def test_client_mask_round_n128(eng, golden, round128):
    g, r = golden["round_n128"], round128
    rows = eng.client_mask(r["client_seg"], r["client_seeds"], r["client_signs"], g["L"])
    assert rows[:4, :8].tolist() == g["rows_head"]
    assert h(rows) == g["rows_sha256"]
    x = rng(20231015).integers(0, 2**32, size=(128, g["L"]), dtype=np.uint32)
    rows_x = eng.client_mask(r["client_seg"], r["client_seeds"], r["client_signs"], g["L"], x=x)
    assert h(rows_x) == g["rows_x_sha256"]


def test_client_mask_ragged_vs_oracle(eng):
    g = rng(3)
    N, L = 9, 2077
    deg = g.integers(0, 5, size=N)          # includes clients with no pairwise seeds
    seg = np.concatenate([[0], np.cumsum(deg + 1)]).astype(np.int64)
    K = int(seg[-1])
    seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    want = O.client_mask(seg, seeds, signs, L)
    assert np.array_equal(eng.client_mask(seg, seeds, signs, L), want)
    x = g.integers(0, 2**32, size=(N, L), dtype=np.uint32)
    assert np.array_equal(eng.client_mask(seg, seeds, signs, L, x=x), O.client_mask(seg, seeds, signs, L, x=x))
    # a client with no seeds at all
    seg0 = np.array([0, 0, 2], np.int64)
    got = eng.client_mask(seg0, seeds[:2], signs[:2], 100)
    assert np.all(got[0] == 1)
    assert np.array_equal(got, O.client_mask(seg0, seeds[:2], signs[:2], 100))


# ------------------------------------------------------------- server side
def test_round_n128_server(eng, golden, round128):
    g, r = golden["round_n128"], round128
    rows = O.client_mask(r["client_seg"], r["client_seeds"], r["client_signs"], g["L"])
    online = r["online"]
    vectors = [rows[i] for i in online]
    out = eng.aggregate_unmask(vectors, r["server_seeds"], r["server_signs"])
    assert np.all(out == g["final_value"])
    x = rng(20231015).integers(0, 2**32, size=(128, g["L"]), dtype=np.uint32)
    rows_x = O.client_mask(r["client_seg"], r["client_seeds"], r["client_signs"], g["L"], x=x)
    out_x = eng.aggregate_unmask(rows_x[online], r["server_seeds"], r["server_signs"])
    assert h(out_x) == g["final_x_sha256"]


@pytest.mark.parametrize("N,K,L", [
    (1, 1, 1), (3, 2, 17), (5, 0, 1000), (0, 7, 1000), (128, 128, 16000), (128, 158, 16384),
    (64, 3, 16385), (17, 300, 4099), (1, 1, 65536), (200, 13, 2**18 + 48), (2, 0, 5), (33, 33, 1024),
])
def test_aggregate_vs_oracle(eng, N, K, L):
    rows, seeds, signs = rand_case(N * 1000 + K * 10 + L, N, K, L)
    want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
    got = eng.aggregate_unmask(list(rows), seeds, signs, L=L)
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:10]


def test_plan_cache_recycles_past_its_capacity():
    """More distinct round shapes than the launch-plan cache holds (64; a server's seed count changes
    every iteration): the least recently used plan's buffers are recycled, never freed under a
    launch, and every round -- new shapes, and shapes seen before and evicted -- stays exact."""
    from flamingo_amd import MaskEngine
    L, N = 4096, 2
    with MaskEngine(0) as e:
        e.set_tuning("small", 0)                     # the planned items_kernel path, not small_round_kernel
        rows, seeds, signs = rand_case(4242, N, 90, L)
        for K in list(range(1, 81)) + [1, 2, 3, 79, 80, 90]:
            got = e.aggregate_unmask(list(rows), seeds[:K], signs[:K], L=L)
            want = O.aggregate_unmask(rows, seeds[:K], signs[:K], L=L, threads=8)
            assert np.array_equal(got, want), K
            assert e.last_plan()["variant"] != 100   # not the small-round kernel


def test_plan_cache_recycling_across_streams():
    """One shape launched on two streams behind long queued work, then more new shapes (mask
    windows of the same seeds; test_seed_table_across_streams_varying_k varies the seeds too)
    than the cache holds, on a third stream, while those launches may still run: the recycled plan's
    item buffer is reused only after every launch of it (its `done` event, the second stream's
    launch ordered after the first's)."""
    import torch
    from flamingo_amd import MaskEngine
    L, N, K = 4096, 2, 100
    with MaskEngine(0) as e:
        e.set_tuning("small", 0)
        rows, seeds, signs = rand_case(5151, N, K, L)
        d_rows = torch.from_numpy(rows.view(np.int32)).cuda()
        d_seeds, d_signs = torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda()
        sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
        outs = []
        for st in (sa, sb):
            with torch.cuda.stream(st):
                a = torch.randn(2048, 2048, device="cuda")
                for _ in range(20):                   # queue work ahead of the launch
                    a = a @ a / 2048.0
                out = torch.empty(L, dtype=torch.int32, device="cuda")
                e.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L, stream=st)
                outs.append(out)
        with torch.cuda.stream(sc):
            for j in range(1, 80):                    # 79 new shapes: recycles the plan of the two launches
                last = torch.empty(L, dtype=torch.int32, device="cuda")
                e.aggregate_unmask_dev(d_rows, d_seeds, d_signs, last, L=L, mask_lo=0, mask_hi=16 * j, stream=sc)
        torch.cuda.synchronize()
        want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
        for out in outs:
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
        hi = 16 * 79
        got = last.cpu().numpy().view(np.uint32)
        assert np.array_equal(got[:hi], want[:hi])
        assert np.array_equal(got[hi:], rows[:, hi:].sum(axis=0, dtype=np.uint64).astype(np.uint32))


def _queue_matmuls(n=20):
    """Queue ~tens of ms of work on the current stream, so what follows it there stays pending."""
    import torch
    a = torch.randn(2048, 2048, device="cuda")
    for _ in range(n):
        a = a @ a / 2048.0
    return a


@pytest.mark.parametrize("third", ["null", "side"])
def test_seed_table_across_streams_varying_k(third):
    """The round-5 red case (gpurun_out/r05ag_pytest_gpu_k.log): two K = 100
    rounds queued behind matmuls on streams sa / sb, then K = 1..79 rounds -- each a NEW seed table
    and a new plan shape -- on a third stream (the null stream, or a side stream) while those two
    still wait.  The context's seed-table ring keeps the tables the queued launches read, so all
    81 outputs equal the oracle bit for bit."""
    import torch
    from flamingo_amd import MaskEngine
    L, N = 4096, 2
    with MaskEngine(0) as e:
        e.set_tuning("small", 0)
        rows, seeds, signs = rand_case(5151, N, 100, L)
        d_rows = torch.from_numpy(rows.view(np.int32)).cuda()
        d_seeds, d_signs = torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda()
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        sc = torch.cuda.Stream() if third == "side" else torch.cuda.default_stream()
        torch.cuda.synchronize()
        outs = []
        for st in (sa, sb):
            with torch.cuda.stream(st):
                _queue_matmuls()
                out = torch.empty(L, dtype=torch.int32, device="cuda")
                e.aggregate_unmask_dev(d_rows, d_seeds[:100], d_signs[:100], out, L=L, stream=st)
                outs.append(out)
        later = []
        with torch.cuda.stream(sc):
            for K in range(1, 80):
                out = torch.empty(L, dtype=torch.int32, device="cuda")
                e.aggregate_unmask_dev(d_rows, d_seeds[:K], d_signs[:K], out, L=L, stream=sc)
                later.append((K, out))
        torch.cuda.synchronize()
        want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
        for out in outs:
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
        for K, out in later:
            want_k = O.aggregate_unmask(rows, seeds[:K], signs[:K], L=L, threads=8)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want_k), K


def test_seed_table_ring_exhausted_across_streams():
    """More streams with a queued round than the ring has tables (8): each stream's round gets its
    own K, so a reused table must wait (on the device) for the queued reads of its previous seeds."""
    import torch
    from flamingo_amd import MaskEngine
    L, N, S = 2048, 3, 11
    with MaskEngine(0) as e:
        e.set_tuning("small", 0)
        rows, seeds, signs = rand_case(6262, N, 64, L)
        d_rows = torch.from_numpy(rows.view(np.int32)).cuda()
        d_seeds, d_signs = torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda()
        streams = [torch.cuda.Stream() for _ in range(S)]
        torch.cuda.synchronize()
        outs = []
        for i, st in enumerate(streams):
            K = 64 - 5 * i
            with torch.cuda.stream(st):
                _queue_matmuls(6)
                out = torch.empty(L, dtype=torch.int32, device="cuda")
                e.aggregate_unmask_dev(d_rows, d_seeds[:K], d_signs[:K], out, L=L, stream=st)
                outs.append((K, out))
        torch.cuda.synchronize()
        for K, out in outs:
            want = O.aggregate_unmask(rows, seeds[:K], signs[:K], L=L, threads=8)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want), K


def test_published_table_read_on_another_stream():
    """flm_seed_table_dev on stream sa behind queued work, flm_aggregate_dev on stream sb at once:
    the read waits for the table's write (its `written` event), with no ordering by the caller."""
    import torch
    from flamingo_amd import MaskEngine
    L, N, K = 4096, 4, 40
    with MaskEngine(0) as e:
        rows, seeds, signs = rand_case(7373, N, K, L)
        d_rows = torch.from_numpy(rows.view(np.int32)).cuda()
        d_seeds, d_signs = torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda()
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(sa):
            _queue_matmuls()
            e.seed_table_dev(d_seeds, d_signs, stream=sa)
        out = torch.empty(L, dtype=torch.int32, device="cuda")
        with torch.cuda.stream(sb):
            e.aggregate_dev(d_rows, K, out, L=L, stream=sb)
        torch.cuda.synchronize()
        want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_get_tuning_reads_the_context(eng):
    """get_tuning reads the library (flm_get_tuning), so a value set through another wrapper of the
    same context -- here a direct flm_set_tuning call -- is what it returns."""
    assert eng.get_tuning("min_items") == 1024
    assert eng.lib.flm_set_tuning(eng.ctx, b"min_items", 2048) == 0
    try:
        assert eng.get_tuning("min_items") == 2048
    finally:
        eng.set_tuning("min_items", 1024)
    assert eng.get_tuning("pairing") == 1 and eng.get_tuning("ec_coop") == -1
    with pytest.raises(RuntimeError, match="unknown tuning key"):
        eng.get_tuning("ec_row_terms")


def test_aggregate_wraps_mod_2_32(eng):
    rows = np.full((7, 333), 0xFFFFFFFF, np.uint32)
    out = eng.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8))
    assert np.all(out == np.uint32((7 * 0xFFFFFFFF) % 2**32))


def test_mask_accumulate_windows(eng):
    g = rng(9)
    seeds = g.integers(0, 256, size=(5, 32), dtype=np.uint8)
    signs = np.array([1, -1, -1, 1, -1], np.int8)
    for slot0, L in ((0, 100), (16, 1024), (4096, 3000), (2**20 - 16, 80)):
        acc = g.integers(0, 2**32, size=L, dtype=np.uint32)
        want = acc.copy()
        for s, sg in zip(seeds, signs):
            p = O.prg(s.tobytes(), L, slot0)
            want = want + p if sg == 1 else want - p
        eng.mask_accumulate(seeds, signs, acc, slot0=slot0)
        assert np.array_equal(acc, want), slot0


def test_bad_arguments_raise(eng):
    rows, seeds, signs = rand_case(1, 2, 2, 64)
    with pytest.raises(RuntimeError):
        eng.aggregate_unmask(list(rows), seeds, np.array([1, 0], np.int8))
    with pytest.raises(RuntimeError):
        eng.aggregate_unmask([rows[0], rows[1][:10]], seeds, signs)
    with pytest.raises(RuntimeError):
        eng.mask_accumulate(seeds, signs, np.zeros(32, np.uint32), slot0=8)
    # device client masking: seg sizes the launch, so a decreasing or offset seg is refused
    import torch
    d_seeds = torch.from_numpy(seeds).cuda()
    out = torch.empty((2, 64), dtype=torch.int32, device="cuda")
    for mode in (0, 2):
        eng.set_tuning("small", mode)
        try:
            for bad in ([0, 2, 1], [1, 1, 2]):
                with pytest.raises(RuntimeError, match="seg"):
                    eng.client_mask_dev(np.array(bad, np.int64), d_seeds, signs, out, 64)
        finally:
            eng.set_tuning("small", 1)


def test_device_wrappers_check_shapes(eng):
    """The *_dev wrappers refuse tensors the kernels would index past (short outputs, ragged pitches)."""
    import torch
    from flamingo_amd import DeviceGroup
    from flamingo_amd.engine import shard_bounds
    dev = torch.device("cuda", 0)
    rows, seeds, signs = rand_case(3, 4, 5, 3000)
    d_rows = torch.from_numpy(rows.view(np.int32)).to(dev)
    d_seeds, d_signs = torch.from_numpy(seeds).to(dev), torch.from_numpy(signs).to(dev)
    with pytest.raises(RuntimeError):
        eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, torch.empty(2999, dtype=torch.int32, device=dev), L=3000)
    eng.seed_table_dev(d_seeds, d_signs)
    with pytest.raises(RuntimeError):
        eng.aggregate_dev(d_rows, 5, torch.empty(100, dtype=torch.int32, device=dev), L=3000)
    T, D, M = 3, 4, 6
    u8 = lambda *s: torch.zeros(s, dtype=torch.uint8, device=dev)  # noqa: E731
    with pytest.raises(RuntimeError):
        eng.shamir_combine_dev(u8(T, M, 32), u8(T, 32), u8(M - 1, 32))
    with pytest.raises(RuntimeError):
        eng.ec_combine_dev(u8(D, 64), u8(T, D, 64), u8(T, 32), u8(D, 32), torch.zeros(D - 1, dtype=torch.int32,
                                                                                      device=dev))
    with pytest.raises(RuntimeError):
        eng.pair_units_dev(d_seeds, d_signs, torch.zeros(10, dtype=torch.int32, device=dev), 3000,
                           torch.zeros(4, dtype=torch.int32, device=dev), 8)
    with DeviceGroup([0, 0]) as grp:
        wide = torch.zeros((2, 3072), dtype=torch.int32, device=dev)
        S = shard_bounds(3000, 2, 0)[2]
        shards = [torch.zeros(S, dtype=torch.int32, device=dev) for _ in range(2)]
        with pytest.raises(RuntimeError, match="pitch"):
            grp.aggregate_unmask_dev([d_rows[:2], wide], [d_seeds] * 2, [d_signs] * 2, shards, 3000)
        with pytest.raises(RuntimeError):
            grp.aggregate_unmask_dev([d_rows[:2], d_rows[2:]], [d_seeds] * 2, [d_signs] * 2,
                                     [shards[0], shards[1][:S - 1]], 3000)


def test_device_round_on_strided_rows(eng):
    """Rows handed over as a column slice of a wider buffer: the wrapper passes the buffer's true pitch."""
    import torch
    N, K, L = 9, 7, 5000
    rows, seeds, signs = rand_case(4, N, K, L)
    wide = torch.zeros((N, L + 200), dtype=torch.int32, device="cuda")
    wide[:, :L] = torch.from_numpy(rows.view(np.int32)).cuda()
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(wide[:, :L], torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda(), out, L=L)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.aggregate_unmask(rows, seeds, signs, L=L, threads=8))


# -------------------------------------------------------- device-resident
def test_device_windows_sum_to_whole(eng):
    """Slot-sharded unmask: per-shard windows reproduce the whole round."""
    import torch
    N, K, L = 96, 200, 3 * 4096 + 512
    rows, seeds, signs = rand_case(77, N, K, L)
    pitch = (L + 63) // 64 * 64
    d_rows = torch.zeros((N, pitch), dtype=torch.int32, device="cuda")
    d_rows[:, :L] = torch.from_numpy(rows.view(np.int32)).cuda()
    d_seeds = torch.from_numpy(seeds).cuda()
    d_signs = torch.from_numpy(signs).cuda()
    want = O.aggregate_unmask(rows, seeds, signs, threads=8)
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    # G shards: rank g sums its client rows over all slots, masks only its slots
    for G in (2, 3, 4):
        bounds = [0] + [((L * (g + 1)) // G) // 16 * 16 for g in range(G - 1)] + [L]
        parts = []
        for g in range(G):
            lo, hi = bounds[g], bounds[g + 1]
            r0, r1 = N * g // G, N * (g + 1) // G
            part = torch.empty(L, dtype=torch.int32, device="cuda")
            eng.aggregate_unmask_dev(d_rows[r0:r1], d_seeds, d_signs, part, L=L, mask_lo=lo, mask_hi=hi)
            parts.append(part)
        torch.cuda.synchronize()
        total = sum(p.cpu().numpy().view(np.uint32).astype(np.uint64) for p in parts) % 2**32
        assert np.array_equal(total.astype(np.uint32), want), G
    assert eng.check_signs() == 0


@pytest.mark.parametrize("N,L", [(1024, 2**20), (4096, 2**18)])
def test_full_size_invariant(eng, N, L):
    """Benchmark-size round: valid masked rows made on the GPU, out == |U| everywhere."""
    import torch
    import flamingo_amd.params as P
    g = rng(N + L)
    m = g.integers(0, 256, size=(N, 32), dtype=np.uint8)
    nbrs = P.synthetic_neighbors(N, degree=8, seed=N)
    offline = np.sort(g.choice(N, max(1, N // 100), replace=False))
    seg, cseeds, csigns = P.client_seed_table(m, nbrs, P.synthetic_pair_seed)
    pitch = L
    d_rows = torch.empty((N, pitch), dtype=torch.int32, device="cuda")
    eng.client_mask_dev(seg, torch.from_numpy(cseeds).cuda(), csigns, d_rows, L)
    online = np.setdiff1d(np.arange(N), offline)
    sseeds, ssigns = P.server_seed_table(m, nbrs, online, offline, P.synthetic_pair_seed)
    d_on = d_rows[torch.from_numpy(online).cuda()].contiguous()
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(d_on, torch.from_numpy(sseeds).cuda(), torch.from_numpy(ssigns).cuda(), out, L=L)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint32)
    assert np.all(o == len(online)), np.flatnonzero(o != len(online))[:8]
    # spot-check a slice of the masked rows against the oracle
    i = int(online[3])
    want = O.client_mask(seg[i:i + 2] - seg[i], cseeds[seg[i]:seg[i + 1]], csigns[seg[i]:seg[i + 1]], 4096)
    assert np.array_equal(d_rows[i, :4096].cpu().numpy().view(np.uint32), want[0])


@pytest.mark.parametrize("variant", [-1, 0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("subtiles", [0, 1, 4, 16])
def test_kernel_variants_bit_identical(eng, variant, subtiles):
    """Every items_kernel variant / tiling gives the oracle's bits (incl. tails, K > 256)."""
    eng.set_tuning("variant", variant)
    eng.set_tuning("subtiles", subtiles)
    try:
        for N, K, L in ((40, 300, 5000), (3, 700, 16000), (64, 5, 70000)):
            rows, seeds, signs = rand_case(N + K + L + subtiles, N, K, L)
            want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
            assert np.array_equal(eng.aggregate_unmask(list(rows), seeds, signs, L=L), want), (N, K, L)
    finally:
        eng.set_tuning("variant", -1)
        eng.set_tuning("subtiles", 0)


def test_sharded_windows_variants(eng):
    """Dual-tile plans (rows and masks on different tiles) for each variant."""
    import torch
    N, K, L = 50, 90, 9000
    rows, seeds, signs = rand_case(5, N, K, L)
    d_rows = torch.from_numpy(rows.view(np.int32)).cuda()
    d_seeds, d_signs = torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda()
    want_rows = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8))
    lo, hi = 2048, 6144
    want = want_rows.copy()
    want[lo:hi] += O.aggregate_unmask(np.zeros((0, 1), np.uint32), seeds, signs, L=hi - lo, slot0=lo)
    for pairing in (0, 1):
        eng.set_tuning("pairing", pairing)
        for v in (-1, 0, 1, 2, 5, 7, 8):
            eng.set_tuning("variant", v)
            out = torch.empty(L, dtype=torch.int32, device="cuda")
            eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L, mask_lo=lo, mask_hi=hi)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want), (pairing, v)
    eng.set_tuning("variant", -1)
    eng.set_tuning("pairing", 1)
    # empty shard (rank owning no slots) with an unaligned clipped bound
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L, mask_lo=L, mask_hi=L)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want_rows)


def test_host_rows_pinned_and_pageable_mix(eng):
    """VECTOR bodies may be pageable numpy arrays or live in the pinned arena; both upload paths
    (staging ring, direct DMA) and their interleaving give the oracle's bits."""
    from flamingo_amd import PinnedArena
    for N, L in ((300, 16000), (9, 3 * 2**20 + 5), (40, 17)):
        rows, seeds, signs = rand_case(N + L, N, 5, L)
        arena = PinnedArena(N * L * 4 + 4096 * N)
        vecs = []
        for i in range(N):
            if i % 3 == 1:
                a = arena.array((L,), np.uint32)
                a[:] = rows[i]
                vecs.append(a)
            else:
                vecs.append(rows[i].copy())
        want = O.aggregate_unmask(rows, seeds, signs, threads=8)
        assert np.array_equal(eng.aggregate_unmask(vecs, seeds, signs, L=L), want), (N, L)
        arena.free()


def test_rows_beyond_2_32_elements(eng):
    """16384 clients x 2^20 slots = 2^34 row elements (64 GiB in HBM): row offsets and the
    planner's item table must be 64-bit.  Masked rows y_i = 1 + PRG(m_i) made on the GPU; the
    server unmask of all m_i must give out == N in every slot."""
    import torch
    N, L = 16384, 1 << 20
    g = rng(16384)
    m = torch.from_numpy(g.integers(0, 256, size=(N, 32), dtype=np.uint8)).cuda()
    rows = torch.empty((N, L), dtype=torch.int32, device="cuda")
    eng.client_mask_dev(np.arange(N + 1, dtype=np.int64), m, np.ones(N, np.int8), rows, L)
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(rows, m, torch.full((N,), -1, dtype=torch.int8, device="cuda"), out, L=L)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint32)
    assert np.all(o == N), np.flatnonzero(o != N)[:8]
    # the last client's row, far past 2^32 elements, against the oracle
    want = O.client_mask(np.array([0, 1], np.int64), m[N - 1:].cpu().numpy(), np.ones(1, np.int8), 2048)
    assert np.array_equal(rows[N - 1, :2048].cpu().numpy().view(np.uint32), want[0])
    del rows
    torch.cuda.empty_cache()


def test_counter_limit_2_36_slots(eng):
    """Slots map to ChaCha blocks slot/16 with a 32-bit block counter: the last block below
    2^36 slots is computed like the oracle's 64-bit counter; one slot further is an error."""
    seed = bytes(range(32))
    top = (1 << 36) - 16
    got = eng.prg_expand([seed], 16, slot0=top)[0]
    assert np.array_equal(got, O.prg(seed, 16, slot0=top))
    with pytest.raises(RuntimeError):
        eng.prg_expand([seed], 32, slot0=top)


def test_device_fuzz_vs_oracle(eng):
    """Random device-resident rounds (rows pitch, mask window, PRG slot offset, empty sets) against
    the oracle: out[l] = sum_i rows[i][l] + [lo <= l < hi] sum_k sign_k PRG(seed_k)[prg_slot0 + l]."""
    import torch
    g = rng(2024)
    for case in range(24):
        N, K, L = int(g.integers(0, 80)), int(g.integers(0, 400)), int(g.integers(1, 40000))
        pitch = (L + 3) // 4 * 4 + 4 * int(g.integers(0, 4))
        lo = int(g.integers(0, L // 16 + 1)) * 16 if g.random() < 0.5 else 0
        hi = L if g.random() < 0.5 else int(g.integers(lo, L + 1))
        slot0 = 16 * int(g.integers(0, 1 << 16)) if g.random() < 0.5 else 0
        rows, seeds, signs = rand_case(case, N, K, L)
        want = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8), L=L, threads=8) \
            if N else np.zeros(L, np.uint32)
        if K and hi > lo:
            want[lo:hi] += O.aggregate_unmask(np.zeros((0, 1), np.uint32), seeds, signs, L=hi - lo,
                                              slot0=slot0 + lo, threads=8)
        d_rows = torch.zeros((max(N, 1), pitch), dtype=torch.int32, device="cuda")[:N]
        if N:
            d_rows[:, :L] = torch.from_numpy(rows.view(np.int32)).cuda()
        d_seeds = torch.from_numpy(seeds).cuda() if K else torch.zeros((0, 32), dtype=torch.uint8, device="cuda")
        d_signs = torch.from_numpy(signs).cuda() if K else torch.zeros(0, dtype=torch.int8, device="cuda")
        out = torch.full((pitch,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L, mask_lo=lo, mask_hi=hi, prg_slot0=slot0)
        torch.cuda.synchronize()
        got = out[:L].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), (case, N, K, L, pitch, lo, hi, slot0, np.flatnonzero(got != want)[:5])
        assert np.all(out[L:].cpu().numpy() == 0x5A5A5A5A), (case, "wrote past L")


def test_client_mask_dev_fuzz_vs_oracle(eng):
    """Random device client-masking batches (SA_ClientAgent.py:304-324): ragged CSR seed lists
    (clients with no seeds included), odd L, padded pitch, with and without explicit inputs x."""
    import torch
    g = rng(77)
    for case in range(12):
        N, L = int(g.integers(1, 40)), int(g.integers(1, 9000))
        pitch = (L + 3) // 4 * 4 + 4 * int(g.integers(0, 3))
        deg = g.integers(0, 9, size=N) * (g.random(N) < 0.85)
        seg = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
        K = int(seg[-1])
        seeds = g.integers(0, 256, size=(max(K, 1), 32), dtype=np.uint8)[:K]
        signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
        use_x = bool(g.random() < 0.5)
        x = g.integers(0, 2**32, size=(N, L), dtype=np.uint32) if use_x else None
        want = O.client_mask(seg, seeds, signs, L, x=x)
        d_seeds = torch.from_numpy(seeds.copy()).cuda() if K else torch.zeros((1, 32), dtype=torch.uint8,
                                                                               device="cuda")
        out = torch.full((N, pitch), 0x3C3C3C3C, dtype=torch.int32, device="cuda")
        d_x = None
        if use_x:
            d_x = torch.zeros((N, pitch), dtype=torch.int32, device="cuda")
            d_x[:, :L] = torch.from_numpy(x.view(np.int32)).cuda()
        eng.client_mask_dev(seg, d_seeds, signs, out, L, x=d_x)
        torch.cuda.synchronize()
        got = out[:, :L].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), (case, N, L, pitch, K, use_x)


@pytest.mark.parametrize("mode", [0, 2])
def test_small_round_path_vs_oracle(eng, mode):
    """The one-launch small-round kernel (flm_set_tuning "small" 2: whenever the window allows it)
    and the seed-schedule + items path ("small" 0) against the oracle on the same random rounds:
    K past one 128/64-seed pass, N past the 128 rows a thread batches, L odd and past 2^16
    (64-slot tiles), windows, PRG slot offsets, unaligned seed rows, empty sets; and the sign
    counts flm_check_signs reads back."""
    import torch
    g = rng(4242 + mode)
    eng.set_tuning("small", mode)
    try:
        for case in range(14):
            N, K = int(g.integers(0, 300)), int(g.integers(0, 600))
            L = int(g.integers(1, 20000)) if case % 3 else int(g.integers(1 << 16, 90000))
            pitch = (L + 3) // 4 * 4 + 4 * int(g.integers(0, 3))
            lo = int(g.integers(0, L // 16 + 1)) * 16 if g.random() < 0.5 else 0
            hi = L if g.random() < 0.5 else int(g.integers(lo // 16, L // 16 + 1)) * 16
            hi = max(hi, lo)
            slot0 = 16 * int(g.integers(0, 1 << 20)) if g.random() < 0.5 else 0
            rows, seeds, signs = rand_case(9000 + case, N, K, L)
            want = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8), L=L, threads=8) \
                if N else np.zeros(L, np.uint32)
            if K and hi > lo:
                want[lo:hi] += O.aggregate_unmask(np.zeros((0, 1), np.uint32), seeds, signs, L=hi - lo,
                                                  slot0=slot0 + lo, threads=8)
            d_rows = torch.zeros((max(N, 1), pitch), dtype=torch.int32, device="cuda")[:N]
            if N:
                d_rows[:, :L] = torch.from_numpy(rows.view(np.int32)).cuda()
            if K and case % 2:  # seed rows at an odd byte offset: the byte-load key path
                buf = torch.zeros(K * 32 + 1, dtype=torch.uint8, device="cuda")
                buf[1:] = torch.from_numpy(seeds.reshape(-1)).cuda()
                d_seeds = buf[1:].view(K, 32)
            else:
                d_seeds = torch.from_numpy(seeds).cuda() if K else torch.zeros((0, 32), dtype=torch.uint8,
                                                                               device="cuda")
            d_signs = torch.from_numpy(signs).cuda() if K else torch.zeros(0, dtype=torch.int8, device="cuda")
            out = torch.full((pitch,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
            eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L, mask_lo=lo, mask_hi=hi, prg_slot0=slot0)
            torch.cuda.synchronize()
            small = eng.last_plan()["variant"] == 100
            assert small == (mode == 2), (case, eng.last_plan())
            got = out[:L].cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (case, mode, N, K, L, pitch, lo, hi, slot0,
                                               np.flatnonzero(got != want)[:5])
            assert np.all(out[L:].cpu().numpy() == 0x5A5A5A5A), (case, "wrote past L")
            assert eng.check_signs() == 0
        # an invalid sign is counted by either path
        rows, seeds, signs = rand_case(1, 4, 40, 1000)
        signs[7] = 3
        out = torch.empty(1000, dtype=torch.int32, device="cuda")
        eng.aggregate_unmask_dev(torch.from_numpy(rows.view(np.int32)).cuda(), torch.from_numpy(seeds).cuda(),
                                 torch.from_numpy(signs).cuda(), out, L=1000)
        torch.cuda.synchronize()
        assert eng.check_signs() == 1
    finally:
        eng.set_tuning("small", 1)


def test_small_round_default_routing(eng):
    """Auto mode: c2 (N=128, L=16384) takes the one-launch kernel, c3-sized rounds do not; a
    flm_aggregate_dev after a small round must not silently reuse a seed table it never built."""
    import torch
    N, K, L = 128, 128, 16384
    rows, seeds, signs = rand_case(5, N, K, L)
    d_rows = torch.from_numpy(rows.view(np.int32)).cuda()
    d_seeds, d_signs = torch.from_numpy(seeds).cuda(), torch.from_numpy(signs).cuda()
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(d_rows, d_seeds, d_signs, out, L=L)
    torch.cuda.synchronize()
    assert eng.last_plan() == {"items": L // 32, "tile_slots": 32, "atomics": 0, "variant": 100}
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.aggregate_unmask(rows, seeds, signs, threads=8))
    with pytest.raises(RuntimeError, match="seed table"):
        eng.aggregate_dev(d_rows, K, out, L=L)
    big = torch.zeros((64, 1 << 17), dtype=torch.int32, device="cuda")
    eng.aggregate_unmask_dev(big, d_seeds, d_signs, torch.empty(1 << 17, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    assert eng.last_plan()["variant"] != 100


@pytest.mark.parametrize("mode", [0, 2])
def test_client_mask_small_vs_oracle(eng, mode):
    """Client masking (SA_ClientAgent.py:304-324) through the one-launch small kernel (SEG mode,
    "small" 2) and through the seed schedule + items path ("small" 0): rows with no seeds, rows
    with more than one 16-seed pass, odd L past several 256-slot tiles, with and without x."""
    import torch
    g = rng(31 + mode)
    eng.set_tuning("small", mode)
    try:
        for case in range(8):
            N, L = int(g.integers(1, 24)), int(g.integers(1, 3000))
            pitch = (L + 3) // 4 * 4 + 4 * int(g.integers(0, 3))
            deg = g.integers(0, 40, size=N) * (g.random(N) < 0.8)
            seg = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
            K = int(seg[-1])
            seeds = g.integers(0, 256, size=(max(K, 1), 32), dtype=np.uint8)[:K]
            signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
            x = g.integers(0, 2**32, size=(N, L), dtype=np.uint32) if case % 2 else None
            want = O.client_mask(seg, seeds, signs, L, x=x)
            d_seeds = torch.from_numpy(seeds.copy()).cuda() if K else torch.zeros((1, 32), dtype=torch.uint8,
                                                                                   device="cuda")
            out = torch.full((N, pitch), 0x3C3C3C3C, dtype=torch.int32, device="cuda")
            d_x = None
            if x is not None:
                d_x = torch.zeros((N, pitch), dtype=torch.int32, device="cuda")
                d_x[:, :L] = torch.from_numpy(x.view(np.int32)).cuda()
            eng.client_mask_dev(seg, d_seeds, signs, out, L, x=d_x)
            torch.cuda.synchronize()
            assert (eng.last_plan()["variant"] == 100) == (mode == 2), (case, eng.last_plan())
            got = out[:, :L].cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (case, mode, N, L, pitch, K)
            if pitch > L:
                assert np.all(out[:, L:].cpu().numpy() == 0x3C3C3C3C), (case, "wrote past L")
    finally:
        eng.set_tuning("small", 1)


def test_seed_table_not_reused_after_another_entry_point(eng):
    """flm_aggregate_dev unmasks against the table flm_seed_table_dev published; an entry point
    that rebuilds the device seed table in between (prg expansion, client masking, pair units)
    invalidates it, so a stale-table aggregate fails loudly instead of using other seeds
    (ADVICE r1)."""
    import torch
    K, L = 12, 4096
    g = np.random.Generator(np.random.PCG64(21))
    seeds = torch.from_numpy(g.integers(0, 256, (K, 32), dtype=np.uint8)).cuda()
    signs = torch.from_numpy(np.where(g.integers(0, 2, K) == 1, 1, -1).astype(np.int8)).cuda()
    other = torch.from_numpy(g.integers(0, 256, (K, 32), dtype=np.uint8)).cuda()
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    eng.seed_table_dev(seeds, signs)
    eng.aggregate_dev(None, K, out, L=L)         # the published table: fine
    torch.cuda.synchronize()
    want = O.aggregate_unmask(np.zeros((0, 1), np.uint32), seeds.cpu().numpy(), signs.cpu().numpy(), L=L)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    expanded = torch.empty((K, L), dtype=torch.int32, device="cuda")
    eng.prg_expand_dev(other, expanded, L)       # rebuilds the table with the same K
    with pytest.raises(RuntimeError, match="seed table"):
        eng.aggregate_dev(None, K, out, L=L)
    torch.cuda.synchronize()
