"""End-to-end Flamingo simulation through the ABIDES surface with the GPU engine.

The reference's only correctness oracle is the printed final sum, which equals
|U| in every slot because client inputs are all ones (SA_ClientAgent.py:304,
SA_ServiceAgent.py:605).  Here it is asserted, with and without dropouts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_simulation_latency_dropouts():
    """Dropouts emerge from the cubic latency model alone (late VECTORs), as in the reference."""
    from flamingo_amd.abides.config_flamingo import run
    res = run(["-c", "flamingo", "-n", "128", "-i", "3", "-s", "7", "-k", "--root_seed_hex", "00" * 32])
    srv = res["server"]
    assert sorted(srv.results) == [1, 2, 3]
    for it, out in srv.results.items():
        assert out.dtype == np.uint32 and out.shape == (16000,)
        assert 0 < srv.online_counts[it] <= 128
        assert np.all(out == srv.online_counts[it]), it


def test_simulation_with_dropouts():
    from flamingo_amd.abides.config_flamingo import run
    res = run(["-c", "flamingo", "-n", "128", "-i", "2", "-s", "11", "-k", "--offline", "3,77,100",
               "--vector_len", "16384"])
    srv = res["server"]
    for it, out in srv.results.items():
        assert srv.online_counts[it] <= 125
        assert np.all(out == srv.online_counts[it]), it
    assert len(srv.recon_symbol) > 0          # dropout pairs were cancelled


@pytest.mark.parametrize("spec", ["loopback4", "rccl1"])
def test_simulation_on_a_device_group(monkeypatch, spec):
    """The server's vector steps over a DeviceGroup: 4 loopback ranks on the one GPU, or one device
    with an RCCL clique (FLM_GROUP_RCCL=1: the grouped ncclReduceScatter path the 8-GPU node runs).
    Same results; and right after every report the server's vec_sum_partial (read back from the
    device-resident S) equals the sum of the VECTOR bodies it received (SA_ServiceAgent.py:346-350)."""
    import oracle as O
    from flamingo_amd.abides.config_flamingo import run
    from flamingo_amd.abides.flamingo import protocol
    from flamingo_amd.abides.flamingo.service_agent import SA_ServiceAgent
    if spec == "loopback4":
        monkeypatch.setenv("FLM_GROUP_DEVICES", "0,0,0,0")
    else:
        monkeypatch.setenv("FLM_GROUP_RCCL", "1")
    checks = []
    orig = SA_ServiceAgent.report_process

    def report_and_check(self):
        orig(self)
        rows = np.stack([np.asarray(v, np.uint32) for v in self.user_vectors.values()])
        want = O.aggregate_unmask(rows, np.zeros((0, 32), np.uint8), np.zeros(0, np.int8), L=rows.shape[1])
        checks.append(bool(np.array_equal(self.vec_sum_partial, want)))

    monkeypatch.setattr(SA_ServiceAgent, "report_process", report_and_check)
    res = run(["-c", "flamingo", "-n", "128", "-i", "2", "-s", "11", "-k", "--offline", "3,77,100",
               "--vector_len", "16384"])
    grp = protocol._group
    assert grp is not None and grp.n == (4 if spec == "loopback4" else 1)
    assert grp.rccl == (spec == "rccl1")
    srv = res["server"]
    for it, out in srv.results.items():
        assert np.all(out == srv.online_counts[it]), it
    assert len(srv.recon_symbol) > 0
    assert checks == [True, True]
    srv._store.close()                      # the group refuses to close under a live store
    grp.close()
    protocol._group = None


@pytest.mark.parametrize("group", ["", "0,0,0,0"], ids=["one_gpu", "loopback4"])
def test_simulation_c5_shape_reduced(monkeypatch, group):
    """BASELINE c5's client count and per-iteration 1 % dropouts (--dropout 0.01: PCG64(seed=t)
    choice per iteration) through the agents, with L = 2^16 and 2 iterations; deterministic latency,
    so the offline sets are exactly the injected ones (41 per iteration).  loopback4: the server's
    store and sums over a 4-rank device group on the one GPU (client-sharded rows, slot-sharded S,
    the group's exchange) -- the drop-in server's multi-GPU form at c5's client count."""
    from flamingo_amd.abides.config_flamingo import offline_schedule, run
    from flamingo_amd.abides.flamingo import protocol
    if group:
        monkeypatch.setenv("FLM_GROUP_DEVICES", group)
    res = run(["-c", "flamingo", "-n", "4096", "--vector_len", "65536", "-i", "2", "--dropout", "0.01", "-k",
               "-s", "5", "--latency", "deterministic"])
    srv = res["server"]
    sch = offline_schedule(4096, 2, dropout=0.01)
    assert sorted(srv.results) == [1, 2]
    for it, out in srv.results.items():
        assert srv.online_counts[it] == 4096 - sum(1 for its in sch.values() if it in its) == 4055
        assert np.all(out == 4055), it
        assert srv.pairs_per_iteration[it] > 500
    if group:
        assert srv._store.G == 4
        srv._store.close()
        protocol._group.close()
        protocol._group = None


def test_assigned_vec_sum_partial_on_the_gpu():
    """ADVICE r4 (medium), with the GPU engine: an assigned vec_sum_partial is what the masks are
    added to when reconstruction_process runs without a report (SA_ServiceAgent.py:540/605)."""
    import oracle as O
    from flamingo_amd.abides.flamingo import protocol
    from flamingo_amd.abides.flamingo.service_agent import SA_ServiceAgent
    protocol.configure(L=4096)
    try:
        srv = SA_ServiceAgent(0, "srv", "SA_ServiceAgent", random_state=np.random.RandomState(1), num_clients=4,
                              users={1, 2, 3})
        base = np.random.default_rng(4).integers(0, 2**32, 4096, dtype=np.uint32)
        srv.vec_sum_partial = base
        m = 0xDEADBEEF12345
        srv.committee_threshold = 1
        srv.committee_shares_mi, srv.recon_index = {7: [m]}, {7: 1}
        srv.dec_target_pairwise, srv.recon_symbol = {}, {}
        srv.reconstruction_process()
        want = O.aggregate_unmask(base[None], np.frombuffer(m.to_bytes(32, "big"), np.uint8)[None],
                                  np.array([-1], np.int8), L=4096)
        assert np.array_equal(srv.final_sum, want)
    finally:
        protocol.configure(committee=60)
