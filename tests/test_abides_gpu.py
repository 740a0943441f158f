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
