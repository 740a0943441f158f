"""World-size-2 (and 3) gloo tests of the sharded server round on CPU.

The per-rank GPU kernel is replaced by the oracle (test infrastructure only):
each rank sums its own clients' rows over all slots and adds the masks over
its own slot shard; the reduce-scatter must then give every rank its shard of
the single-process round, bit-exactly, including mod-2^32 wrap.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def case(N, K, L):
    g = np.random.Generator(np.random.PCG64(N * 7 + K))
    rows = g.integers(0, 2**32, size=(N, L), dtype=np.uint32)
    rows[:, :5] = 0xFFFFFFFF                     # force wrap in the collective
    seeds = g.integers(0, 256, size=(K, 32), dtype=np.uint8)
    signs = np.where(g.random(K) < 0.5, 1, -1).astype(np.int8)
    return rows, seeds, signs


def worker(rank, world, port, N, K, L, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from flamingo_amd.distributed import ShardedRound, client_bounds

        class OracleRound(ShardedRound):
            """ShardedRound with the device kernel swapped for the CPU oracle."""

            def prepare_seeds(self, seeds, signs, stream=None):
                self.seeds, self.signs = seeds, signs

            def compute(self, rows, stream=None):
                part = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8), L=self.L)
                if self.hi > self.lo:
                    part[self.lo:self.hi] += O.aggregate_unmask(np.zeros((0, 1), np.uint32), self.seeds,
                                                                self.signs, L=self.hi - self.lo, slot0=self.lo)
                self.partial.zero_()
                self.partial[: self.L] = torch.from_numpy(part.view(np.int32))

        rows, seeds, signs = case(N, K, L)
        c0, c1 = client_bounds(N, world, rank)
        rnd = OracleRound(None, L, device=torch.device("cpu"))
        out = rnd.step(rows[c0:c1], seeds, signs)
        # pipelined: two rounds in flight on alternating buffers (async reduce-scatter),
        # the second with its rows negated-and-reused so the two results differ
        pipe = OracleRound(None, L, device=torch.device("cpu"), buffers=2)
        b0 = pipe.launch(rows[c0:c1], seeds, signs)
        b1 = pipe.launch((0 - rows[c0:c1]).astype(np.uint32), seeds, signs)
        b2 = pipe.launch(rows[c0:c1], seeds, signs)          # reuses buffer 0 after its collective
        r1, r2 = pipe.result(b1).numpy().view(np.uint32).copy(), pipe.result(b2).numpy().view(np.uint32).copy()
        assert b0 == b2 == 0 and b1 == 1
        q.put((rank, rnd.lo, rnd.hi, out.numpy().view(np.uint32).copy(), r1, r2))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,K,L", [(2, 6, 5, 5000), (2, 3, 0, 2048), (3, 7, 9, 4100), (4, 9, 11, 6000),
                                          (8, 13, 7, 9000)])  # G=8: ranks 5-7 own empty slot shards
def test_sharded_round_matches_single_process(world, N, K, L):
    rows, seeds, signs = case(N, K, L)
    want = O.aggregate_unmask(rows, seeds, signs, threads=4)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, N, K, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_neg = O.aggregate_unmask((0 - rows).astype(np.uint32), seeds, signs, threads=4)
    covered = np.zeros(L, bool)
    for rank, lo, hi, out, r1, r2 in got:
        assert np.array_equal(out, want[lo:hi]), rank
        assert np.array_equal(r1, want_neg[lo:hi]), rank      # pipelined round on buffer 1
        assert np.array_equal(r2, want[lo:hi]), rank          # buffer 0 reused
        covered[lo:hi] = True
    assert covered.all()


def test_shard_bounds_properties():
    from flamingo_amd.distributed import padded_length, shard_bounds, client_bounds
    for L in (1, 16, 1000, 16000, 2**20, 2**20 + 5):
        for G in (1, 2, 3, 8):
            b = [shard_bounds(L, G, r) for r in range(G)]
            assert b[0][0] == 0 and b[-1][1] == L
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 and (lo % 16 == 0 or lo == hi)
            assert padded_length(L, G) % (1024 * G) == 0
            assert sum(client_bounds(1000, G, r)[1] - client_bounds(1000, G, r)[0] for r in range(G)) == 1000


class _LoggingEngine:
    """Stands in for a MaskEngine in distributed.shutdown (isinstance is patched to accept it)."""

    def __init__(self):
        self.calls = []

    def comm_destroy(self):
        self.calls.append("comm_destroy")

    def close(self):
        self.calls.append("close")


def shutdown_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flamingo_amd import distributed as D
    from flamingo_amd import engine as E
    E.MaskEngine = _LoggingEngine                       # shutdown's isinstance check sees the stand-in
    eng = _LoggingEngine()
    D.shutdown(eng)
    q.put((rank, eng.calls, dist.is_initialized()))


@pytest.mark.parametrize("world", [2, 4])
def test_shutdown_tears_down_a_real_process_group(world):
    """distributed.shutdown on every rank of a real (gloo) world: library communicator first, the
    barrier, destroy_process_group, then the contexts -- no rank hangs, every rank ends uninitialised."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=shutdown_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [g[0] for g in got] == list(range(world))
    for _, calls, still_init in got:
        assert calls == ["comm_destroy", "close"] and not still_init
