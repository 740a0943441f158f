"""Device-resident VECTOR ingestion (flamingo_amd.ingest.VectorStore) against the oracle.

The store is the drop-in server's path from arrival (SA_ServiceAgent.py:205-210) through the
partial sum (:346-350) to the final sum (:529-605): rows uploaded at arrival, S kept on the
device(s), masks added over each device's slot shard.  Checked bit-exactly on one engine and on
loopback groups (ranks sharing the one GPU), with a duplicate sender, an odd L, growth past the
initial capacity and a second iteration reusing the rows."""
from __future__ import annotations

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _case(N, K, L, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    rows = g.integers(0, 2**32, (N, L), dtype=np.uint32)
    seeds = g.integers(0, 256, (K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    return rows, seeds, signs


@pytest.mark.parametrize("G", [1, "1rccl", 3])
@pytest.mark.parametrize("N,K,L", [(20, 9, 16000), (7, 0, 4099), (33, 40, 1 << 17)])
def test_store_round_vs_oracle(G, N, K, L):
    """G = 1: one engine; 3: loopback ranks; "1rccl": a one-device group with an RCCL clique, whose
    partial sum takes the group's sharded round and grouped ncclReduceScatter."""
    from flamingo_amd import DeviceGroup, MaskEngine
    from flamingo_amd.ingest import VectorStore
    if G == "1rccl":
        eng, G = DeviceGroup([0], force_rccl=True), 1
        assert eng.rccl
    else:
        eng = MaskEngine(0) if G == 1 else DeviceGroup([0] * G)
    try:
        st = VectorStore(eng, L, capacity=max(1, N // 2))      # grows past its first capacity
        for it in range(2):                                      # second iteration reuses the rows
            rows, seeds, signs = _case(N, K, L, 100 * G + N + it)
            order = np.random.Generator(np.random.PCG64(it)).permutation(N)
            junk = np.full(L, 12345, np.uint32)
            st.add(int(order[0]), junk)                          # overwritten by the same sender below
            for i in order:
                st.add(int(i), rows[i])
            assert len(st) == N
            st.partial_sum()
            st.wait_partial()
            S = rows.sum(axis=0, dtype=np.uint64).astype(np.uint32)
            assert np.array_equal(st.host_partial(), S)
            got = st.unmask(seeds, signs)
            want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
            assert np.array_equal(got, want), (G, N, K, L, it)
            assert st.unmask_ms() > 0.0                          # the call's device time (flm_store_unmask_ms)
            st.reset()
        st.close()
    finally:
        eng.close()


def test_store_rejects_a_wrong_length():
    from flamingo_amd import MaskEngine
    from flamingo_amd.ingest import VectorStore
    with MaskEngine(0) as eng:
        st = VectorStore(eng, 1000, 4)
        st.add(1, np.zeros(1000, np.uint32))
        st.add(2, np.zeros(999, np.uint32))
        with pytest.raises(RuntimeError, match="incorrect length"):
            st.partial_sum()
        st.reset()
        st.add(3, np.zeros(1000, np.float32))      # not a uint32 body: never reinterpreted as one
        with pytest.raises(RuntimeError, match="incorrect length"):
            st.partial_sum()


def test_store_empty_round():
    from flamingo_amd import MaskEngine
    from flamingo_amd.ingest import VectorStore
    with MaskEngine(0) as eng:
        st = VectorStore(eng, 2048, 4)
        st.partial_sum()
        st.wait_partial()
        assert not st.host_partial().any()
        s = np.arange(32, dtype=np.uint8).reshape(1, 32)
        assert np.array_equal(st.unmask(s, [1]), O.prg(s.tobytes(), 2048))


def test_store_c_abi_checks_lengths_and_reset():
    """The library store itself (flm_store_*, not the Python guard): a body of the wrong length
    makes flm_store_partial fail with the reference's message; reset clears it; a sender sending
    twice keeps one row."""
    import ctypes
    from flamingo_amd import MaskEngine
    from flamingo_amd.ingest import VectorStore
    with MaskEngine(0) as eng:
        st = VectorStore(eng, 4096, 2)
        lib = st.lib
        row = np.arange(4096, dtype=np.uint32)
        assert lib.flm_store_add(st.h, 7, row.ctypes.data, 4095) == 0        # remembered, not an error yet
        assert lib.flm_store_partial(st.h) != 0
        assert b"incorrect length" in lib.flm_store_last_error(st.h)
        st.reset()
        for _ in range(2):
            assert lib.flm_store_add(st.h, 7, row.ctypes.data, 4096) == 0
        assert lib.flm_store_count(st.h) == 1
        st.partial_sum()
        assert st.wait_partial() >= 0.0
        assert np.array_equal(st.host_partial(), row)
        assert lib.flm_store_unmask(st.h, None, None, -1, ctypes.cast(row.ctypes.data, ctypes.POINTER(ctypes.c_uint32))) != 0
        st.close()


def test_store_add_after_partial_waits_for_the_sum():
    """A sender's row rewritten between flm_store_partial and flm_store_reset (a late VECTOR the
    reference-side binding forwards, integration/util_flm.py) must not corrupt S: the upload is
    ordered after the partial sum's reads."""
    from flamingo_amd import MaskEngine
    from flamingo_amd.ingest import VectorStore
    L, N = 1 << 20, 64
    rows, _, _ = _case(N, 0, L, 5)
    with MaskEngine(0) as eng:
        st = VectorStore(eng, L, N)
        for i in range(N):
            st.add(i, rows[i])
        st.partial_sum()
        for i in range(N):                              # immediately: the sum is still running
            st.add(i, np.zeros(L, np.uint32))
        st.wait_partial()
        assert st.has_partial
        assert np.array_equal(st.host_partial(), rows.sum(axis=0, dtype=np.uint64).astype(np.uint32))
        st.reset()
        assert not st.has_partial
        st.close()


def test_group_close_refused_while_a_store_is_open():
    from flamingo_amd import DeviceGroup
    from flamingo_amd.ingest import VectorStore
    grp = DeviceGroup([0, 0])
    st = VectorStore(grp, 4096, 2)
    with pytest.raises(RuntimeError, match="VectorStore"):
        grp.close()
    st.close()
    grp.close()


@pytest.mark.parametrize("G", [1, 2])
def test_store_unmask_seed_counts_grow_and_shrink(G):
    """K from call to call past the store's first seed buffer (made for 2 x capacity seeds) and back
    down: the device seed buffer and the pinned bounce buffers regrow (with slack) and stay exact; a
    call refused for its signs leaves the store usable."""
    from flamingo_amd import DeviceGroup, MaskEngine
    from flamingo_amd.ingest import VectorStore
    L, N = 5000, 4
    eng = MaskEngine(0) if G == 1 else DeviceGroup([0] * G)
    try:
        st = VectorStore(eng, L, capacity=N)
        rows, _, _ = _case(N, 0, L, 77)
        for i in range(N):
            st.add(i, rows[i])
        st.partial_sum()
        for j, K in enumerate([3, 200, 5000, 7, 6000]):
            _, seeds, signs = _case(1, K, 1, 1000 + j)
            if j == 3:
                bad = signs.copy()
                bad[0] = 0
                with pytest.raises(RuntimeError, match="signs"):
                    st.unmask(seeds, bad)
            got = st.unmask(seeds, signs)
            want = O.aggregate_unmask(rows, seeds, signs, L=L, threads=8)
            assert np.array_equal(got, want), (G, K)
            assert np.array_equal(st.host_partial(), rows.sum(axis=0, dtype=np.uint64).astype(np.uint32))
        st.close()
    finally:
        eng.close()
