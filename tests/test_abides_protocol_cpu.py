"""The full Flamingo protocol through the ABIDES agents on CPU.

The agents' engine (normally the GPU MaskEngine) is replaced by a test double
whose methods are the CPU oracle (oracle/oracle.py for masks and sums) and
the pure-Python / OpenSSL P-256 code (oracle/ec_oracle.py, flamingo_amd.crypto)
for the scalar multiplications and the threshold combine.  This checks the
protocol logic -- ECDH keys, h_ijt -> hash-to-curve seeds, ElGamal to the
system key, committee decryption shares, Lagrange combine, AES-GCM m_i
shares, JSON payloads -- end to end: the final sum must equal |U| in every
slot (all-ones inputs, SA_ClientAgent.py:304 + SA_ServiceAgent.py:605),
with and without dropouts.  The GPU versions of the same runs are in
tests/test_abides_gpu.py.
"""
import numpy as np
import pytest

import ec_oracle as E
import oracle as O
from flamingo_amd import crypto as C


class OracleStore:
    """The server's VECTOR store (flamingo_amd.ingest.VectorStore interface) on the host."""

    def __init__(self, L):
        self.L, self.G = L, 1
        self.reset()

    def reset(self):
        self.rows, self.bad, self.has_partial = {}, [], False

    def __len__(self):
        return len(self.rows)

    def add(self, sender, vec):
        v = np.asarray(vec)
        if v.shape != (self.L,):
            self.bad.append(sender)
        else:
            self.rows[sender] = v.astype(np.uint32)

    def partial_sum(self):
        rows = np.stack(list(self.rows.values())) if self.rows else np.zeros((0, self.L), np.uint32)
        self.S = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8), L=self.L)
        self.has_partial = True

    def wait_partial(self):
        return 0.0

    def host_partial(self):
        return self.S

    def unmask(self, seeds, signs):
        sd = np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32) if seeds else np.zeros((0, 32), np.uint8)
        return O.aggregate_unmask(self.S[None], sd, np.asarray(signs, np.int8), L=self.L)


class LazyH2C:
    """The (65536, 64) hash-to-curve table of hash_to_curve_decimal, computed row by row on demand
    by the pure-Python restatement (the whole table would take ~30 s of Python)."""

    def __init__(self, v0):
        self.v0, self.rows = v0, {}

    def _pt(self, i):
        if i not in self.rows:
            self.rows[i] = E.hash_str_to_curve(str(self.v0 + i))
        return self.rows[i]

    def table(self):
        outer = self

        class Rows:
            def __getitem__(self, i):
                return np.frombuffer(E.wire(outer._pt(int(i))), np.uint8)

        class Flags:
            def __getitem__(self, i):
                return 4 if outer._pt(int(i)) is None else 0
        return Rows(), Flags()


class OracleEngine:
    def hash_to_curve_decimal(self, v0=0, n=1 << 16):
        return LazyH2C(v0).table()

    def hash_to_curve_wire(self, msgs):
        pts = [E.hash_str_to_curve(m) for m in msgs]
        return (np.stack([np.frombuffer(E.wire(p), np.uint8) for p in pts]),
                np.array([4 if p is None else 0 for p in pts], np.uint32))

    def vector_store(self, L, capacity):
        return OracleStore(L)

    def client_mask(self, seg, seeds, signs, L, x=None):
        return O.client_mask(np.asarray(seg, np.int64), np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32),
                             np.asarray(signs, np.int8), L, x=x)

    def aggregate_unmask(self, vectors, seeds, signs, L=None):
        rows = np.stack(vectors) if len(vectors) else np.zeros((0, L), np.uint32)
        sd = np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32) if seeds else np.zeros((0, 32), np.uint8)
        return O.aggregate_unmask(rows, sd, np.asarray(signs, np.int8), L=L)

    def mask_accumulate(self, seeds, signs, acc, slot0=0):
        sd = np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32)
        return acc + O.aggregate_unmask(np.zeros((0, acc.shape[0]), np.uint32), sd, np.asarray(signs, np.int8),
                                        L=acc.shape[0])

    def chacha20_encrypt(self, key, data, nonce=bytes(8), counter=0):
        return O.chacha20_encrypt(key, data)

    def prg_expand(self, seeds, L, slot0=0):
        return np.stack([O.prg(bytes(s), L, slot0) for s in seeds])

    def ec_mul_wire(self, points_w, scalars_w):
        pts = C.points_from_wire(points_w)
        ks = [int.from_bytes(bytes(s), "big") for s in scalars_w]
        out = [C.mul(k, p) for k, p in zip(ks, pts)]
        return C.points_to_wire(out), np.array([4 if p is None else 0 for p in out], np.uint32)

    def shamir_combine(self, shares_by_term, lambdas):
        M = len(shares_by_term[0]) if lambdas else 0
        return [(sum(l * s[i] for l, s in zip(lambdas, shares_by_term)) % E.N).to_bytes(32, "big")
                for i in range(M)]

    def ec_combine_wire(self, c1_w, shares_w, lambdas_w, negate=True):
        c1 = C.points_from_wire(c1_w)
        shares = [C.points_from_wire(s) for s in shares_w]
        lam = [int.from_bytes(bytes(s), "big") for s in lambdas_w]
        pts, seeds = E.combine(c1, shares, lam, negate)
        return (C.points_to_wire(pts), np.frombuffer(b"".join(seeds), np.uint8).reshape(-1, 32),
                np.zeros(len(pts), np.uint32))


@pytest.fixture
def oracle_engine(monkeypatch):
    from flamingo_amd.abides.flamingo import protocol
    monkeypatch.setattr(protocol, "_engine", OracleEngine())
    yield
    protocol.configure(committee=60)


@pytest.mark.parametrize("offline", ["", "3,9,20"])
def test_protocol_end_to_end_on_oracle(oracle_engine, offline):
    from flamingo_amd.abides.config_flamingo import run
    argv = ["-c", "flamingo", "-n", "32", "-i", "2", "-s", "5", "-k", "--vector_len", "1000",
            "--committee_size", "9", "--root_seed_hex", "11" * 32, "--round_time", "30"]
    if offline:
        argv += ["--offline", offline]
    res = run(argv)
    srv = res["server"]
    assert sorted(srv.results) == [1, 2]
    for it, out in srv.results.items():
        assert np.all(out == srv.online_counts[it]), it
    if offline:
        assert len(srv.recon_symbol) > 0 and max(srv.online_counts.values()) <= 29


def test_wire_formats_roundtrip():
    from flamingo_amd.abides.flamingo import wire
    g2 = C.mul(2)
    el = {(1, 5): (E.G, g2), (7, 2): (g2, E.G)}
    s = wire.serialize_dim1_elgamal(el)
    assert wire.deserialize_dim1_elgamal(s) == el
    keys, c0, c1 = wire.elgamal_json_to_wire(s)
    assert keys == [(1, 5), (7, 2)] and C.points_from_wire(c0) == [E.G, g2] and C.points_from_wire(c1) == [g2, E.G]
    s = wire.serialize_dim1_ecp([E.G, g2])
    assert wire.deserialize_dim1_ecp(s) == [E.G, g2]
    assert wire.wire_to_ecp_json(wire.ecp_json_to_wire(s)) == s
    assert wire.deserialize_dim2_ecp(wire.serialize_dim2_ecp({"a": [E.G]})) == {"a": [E.G]}
    tb = [(b"\x01\x02", b"\xff" * 16)]
    assert wire.deserialize_tuples_bytes(wire.serialize_tuples_bytes(tb)) == tb


def test_vec_sum_partial_follows_the_store(oracle_engine):
    """SA_ServiceAgent.vec_sum_partial (:346-350): zeros before report, S after it (read from the
    store's has_partial flag, which the real VectorStore carries too), zeros again after the
    iteration's reset; a reference-style assignment works before report and is refused while S is
    device-resident."""
    from flamingo_amd.abides.flamingo.service_agent import SA_ServiceAgent
    from flamingo_amd.abides.flamingo import protocol
    protocol.configure(L=64)
    srv = SA_ServiceAgent(0, "srv", "SA_ServiceAgent", random_state=np.random.RandomState(1), num_clients=4,
                          users={1, 2, 3})
    srv.vector_len = 64
    assert not srv.vec_sum_partial.any()
    srv.vec_sum_partial = np.full(64, 5, np.uint32)
    assert np.all(srv.vec_sum_partial == 5)
    rows = {i: np.full(64, 10 * i, np.uint32) for i in (1, 2, 3)}
    for i, v in rows.items():
        srv.store().add(i, v)
    srv.store().partial_sum()
    assert np.all(srv.vec_sum_partial == 60)
    with pytest.raises(RuntimeError, match="device-resident"):
        srv.vec_sum_partial = np.zeros(64, np.uint32)
    srv.reconstruction_clear_pool()
    assert not srv.vec_sum_partial.any()


def test_offline_schedule_per_iteration():
    """--dropout F: a fresh PCG64(seed=t).choice(N, round(F N)) offline set per iteration."""
    from flamingo_amd.abides.config_flamingo import offline_schedule
    sch = offline_schedule(4096, 10, always={5}, dropout=0.01)
    for t in range(1, 11):
        off = sorted(i for i, its in sch.items() if t in its and i != 5)
        want = sorted(int(x) for x in np.random.Generator(np.random.PCG64(t)).choice(4096, 41, replace=False) if x != 5)
        assert off == want, t
        assert t in sch[5]
    assert offline_schedule(128, 3) == {}


def test_protocol_per_iteration_dropouts_on_oracle(oracle_engine, capsys):
    from flamingo_amd.abides.config_flamingo import offline_schedule, run
    argv = ["-c", "flamingo", "-n", "32", "-i", "3", "-s", "9", "-k", "--vector_len", "512",
            "--committee_size", "9", "--root_seed_hex", "22" * 32, "--round_time", "30", "--dropout", "0.1"]
    srv = run(argv)["server"]
    sch = offline_schedule(32, 3, dropout=0.1)
    assert sorted(srv.results) == [1, 2, 3]
    for it, out in srv.results.items():
        n_off = sum(1 for its in sch.values() if it in its)
        assert n_off == 3 and srv.online_counts[it] <= 32 - n_off
        assert np.all(out == srv.online_counts[it]) and srv.pairs_per_iteration[it] > 0
    assert "final_sum == |U| in every slot: True" in capsys.readouterr().out


def test_run_raises_the_gc_threshold_and_restores_it(monkeypatch):
    """config_flamingo.run raises the young-generation threshold for the event loop only
    (profiles/r05_sim_gc_threshold.log) and gives the caller's back, also when the run raises."""
    import gc
    from flamingo_amd.abides import config_flamingo as CF
    before = gc.get_threshold()
    seen = []

    def fake_run(args):
        seen.append(gc.get_threshold())
        raise RuntimeError("stop")

    monkeypatch.setattr(CF, "_run", fake_run)
    with pytest.raises(RuntimeError, match="stop"):
        CF.run(["-c", "flamingo", "-n", "8"])
    assert seen and seen[0][0] >= CF.GC_THRESHOLD0
    assert gc.get_threshold() == before
