"""Property-based checks (hypothesis) of the host-side pieces the GPU path relies on, on CPU:
the multi-GPU geometry (the C ABI's flm_shard_bounds / flm_client_bounds against the Python
mirror), the oracle's PRG windows and linearity (the properties the full-size GPU tests lean on),
the protocol invariant out = |U| through the seed tables and dropout pairs
(SA_ClientAgent.py:304-324, SA_ServiceAgent.py:341-380, 529-605), and wire round trips
(util/util.py:179-252).  Sizes stay small so the whole file runs in seconds."""
import os
import sys

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (test infrastructure: the checker)

from flamingo_amd import params as P  # noqa: E402
from flamingo_amd.distributed import client_bounds, padded_length, shard_bounds  # noqa: E402

FAST = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
seed32 = st.binary(min_size=32, max_size=32)


@FAST
@given(L=st.integers(1, 1 << 22), world=st.integers(1, 16))
def test_shards_partition_the_slots(L, world):
    """Shards are contiguous, cover [0, L) exactly once, start on a 1024-slot boundary (or are empty
    at L), and the library computes the same bounds (host-only call, no GPU)."""
    from flamingo_amd.engine import shard_bounds as lib_shard_bounds
    Lp = padded_length(L, world)
    S = Lp // world
    assert Lp >= L and Lp % (1024 * world) == 0
    prev = 0
    for r in range(world):
        lo, hi = shard_bounds(L, world, r)
        assert lo == prev and lo <= hi and hi - lo <= S
        assert lo % 1024 == 0 or lo == hi == L  # an empty shard past the end sits at L
        assert lib_shard_bounds(L, world, r) == (lo, hi, S)
        prev = hi
    assert prev == L


@FAST
@given(N=st.integers(0, 5000), world=st.integers(1, 16))
def test_clients_partition_evenly(N, world):
    from flamingo_amd.engine import client_bounds as lib_client_bounds
    sizes, prev = [], 0
    for r in range(world):
        c0, c1 = client_bounds(N, world, r)
        assert c0 == prev and (c0, c1) == lib_client_bounds(N, world, r)
        sizes.append(c1 - c0)
        prev = c1
    assert prev == N and max(sizes) - min(sizes) <= 1


@FAST
@given(seed=seed32, L=st.integers(1, 300), slot0=st.integers(0, 5000))
def test_prg_windows_are_slices(seed, L, slot0):
    """PRG(seed)[slot0 : slot0 + L] from the counter offset equals the slice of the whole stream,
    and the numpy restatement agrees with the C one (partial ChaCha blocks at both ends)."""
    whole = O.prg(seed, slot0 + L)
    assert np.array_equal(O.prg(seed, L, slot0), whole[slot0:])
    assert np.array_equal(O.np_prg(seed, L, slot0), whole[slot0:])


@st.composite
def rounds(draw):
    N = draw(st.integers(0, 6))
    K = draw(st.integers(0, 6))
    L = draw(st.integers(1, 200))
    g = np.random.Generator(np.random.PCG64(draw(st.integers(0, 2**32 - 1))))
    rows = g.integers(0, 2**32, size=(N, L), dtype=np.uint32)
    seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
    signs = g.choice(np.array([-1, 1], np.int8), size=K)
    return rows, seeds, signs, L


@FAST
@given(rounds(), st.data())
def test_aggregate_is_linear_and_windowed(r, data):
    """out = S + sum sign * PRG: the rows and the masks add separately (mod 2^32); a +1 / -1 pair of
    the same seed cancels; a window [a, a + w) of the round equals the round of the row window with
    the PRG counter offset (slot0) -- the property the sharded and windowed GPU tests rely on."""
    rows, seeds, signs, L = r
    full = O.aggregate_unmask(rows, seeds, signs, L=L)
    S = rows.sum(axis=0, dtype=np.uint64).astype(np.uint32) if rows.shape[0] else np.zeros(L, np.uint32)
    M = O.aggregate_unmask(np.zeros((0, L), np.uint32), seeds, signs, L=L)
    assert np.array_equal(full, S + M)
    if seeds.shape[0]:  # the same seed once with +1 and once with -1 adds nothing
        s2 = np.concatenate([seeds, seeds[:1], seeds[:1]])
        g2 = np.concatenate([signs, np.array([1, -1], np.int8)])
        assert np.array_equal(O.aggregate_unmask(rows, s2, g2, L=L), full)
    a = data.draw(st.integers(0, L - 1))
    w = data.draw(st.integers(1, L - a))
    win = O.aggregate_unmask(rows[:, a:a + w] if rows.shape[0] else np.zeros((0, w), np.uint32),
                             seeds, signs, L=w, slot0=a)
    assert np.array_equal(win, full[a:a + w])


@FAST
@given(N=st.integers(2, 24), degree=st.integers(1, 8), gseed=st.integers(0, 1000),
       L=st.integers(1, 80), data=st.data())
def test_protocol_sum_is_number_online(N, degree, gseed, L, data):
    """The round's invariant with any dropout set: every client masks the all-ones vector with its
    self mask and its pair masks (client_seed_table), the server sums the online clients' vectors
    and unmasks with -PRG(m_i) for i in U and sigma * PRG(s_ij) for the (online, offline) pairs
    (server_seed_table / dropout_pairs): out == |U| in every slot."""
    nbrs = P.synthetic_neighbors(N, degree, seed=gseed)
    m = np.random.Generator(np.random.PCG64(gseed + 1)).integers(0, 256, size=(N, 32), dtype=np.uint8)
    offline = sorted(data.draw(st.sets(st.integers(0, N - 1), max_size=N - 1)))
    online = [i for i in range(N) if i not in set(offline)]
    seg, cs, csg = P.client_seed_table(m, nbrs, P.synthetic_pair_seed)
    y = O.client_mask(seg, cs, csg, L)
    ss, sg = P.server_seed_table(m, nbrs, online, offline, P.synthetic_pair_seed)
    out = O.aggregate_unmask(y[online], ss, sg, L=L)
    assert np.all(out == len(online))
    pairs, psg = P.dropout_pairs(nbrs, online, offline)
    for (i, j), s in zip(pairs, psg):
        assert i in online and j in offline and j in nbrs[i] and s == (1 if i > j else -1)


@FAST
@given(st.lists(st.tuples(st.binary(max_size=48), st.binary(max_size=16)), max_size=6),
       st.lists(st.integers(-2**70, 2**70), max_size=8))
def test_wire_round_trips(tuples, ints):
    from flamingo_amd.abides.flamingo import wire as W
    assert W.deserialize_tuples_bytes(W.serialize_tuples_bytes(tuples)) == tuples
    assert W.deserialize_dim1_list(W.serialize_dim1_list(ints)) == ints


@pytest.mark.parametrize("L,world", [(1, 8), (1023, 8), (1 << 20, 8), ((1 << 20) + 1, 3)])
def test_shard_edges(L, world):
    """Ranks past the end own empty shards (hi == lo == L); the last non-empty one ends at L."""
    b = [shard_bounds(L, world, r) for r in range(world)]
    assert b[-1][1] == L and all(lo <= hi for lo, hi in b)
