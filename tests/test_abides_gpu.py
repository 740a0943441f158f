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


def test_simulation_on_a_device_group(monkeypatch):
    """The server's vector steps over a 4-rank DeviceGroup (loopback ranks on the one GPU; the
    driver's 8-GPU node gives it 8 distinct devices and an RCCL clique): same results."""
    from flamingo_amd.abides.config_flamingo import run
    from flamingo_amd.abides.flamingo import protocol
    monkeypatch.setenv("FLM_GROUP_DEVICES", "0,0,0,0")
    res = run(["-c", "flamingo", "-n", "128", "-i", "2", "-s", "11", "-k", "--offline", "3,77,100",
               "--vector_len", "16384"])
    assert protocol._group is not None and protocol._group.n == 4
    srv = res["server"]
    for it, out in srv.results.items():
        assert np.all(out == srv.online_counts[it]), it
    assert len(srv.recon_symbol) > 0
    protocol._group.close()
    protocol._group = None
