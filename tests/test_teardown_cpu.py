"""Host-side lifecycle logic, no GPU: the ordered RCCL teardown (distributed.shutdown), the
drop-in server's device-group reuse and retirement (protocol.server_engine, VectorStore.close),
the reference-style vec_sum_partial assignment feeding reconstruction_process
(SA_ServiceAgent.py:540/605), and ShardedReconstruction restoring the caller's ec_coop tuning."""
import numpy as np
import pytest
import torch

import oracle as O
from flamingo_amd import engine as E
from flamingo_amd.abides.flamingo import protocol


class FakeEngine(E.MaskEngine):
    def __init__(self, log, name):
        self.log, self.name, self.ctx = log, name, None

    def comm_destroy(self):
        self.log.append(("comm_destroy", self.name))

    def close(self):
        self.log.append(("close", self.name))

    def __del__(self):
        pass


class FakeOwner:
    def __init__(self, log, name):
        self.log, self.name = log, name

    def close(self):
        self.log.append(("close", self.name))


def test_shutdown_destroys_library_comms_before_the_process_group(monkeypatch):
    from flamingo_amd import distributed as D
    log = []
    monkeypatch.setattr(D.dist, "barrier", lambda *a, **k: log.append(("barrier",)))
    monkeypatch.setattr(D.dist, "destroy_process_group", lambda *a, **k: log.append(("destroy_pg",)))
    D.shutdown(FakeEngine(log, "eng"), FakeOwner(log, "store"), FakeOwner(log, "group"), None,
               group_initialized=True)
    assert log == [("comm_destroy", "eng"), ("close", "store"), ("close", "group"), ("barrier",),
                   ("destroy_pg",), ("close", "eng")]
    log.clear()
    D.shutdown(FakeEngine(log, "e"), group_initialized=False)        # world 1: no process group
    assert log == [("comm_destroy", "e"), ("close", "e")]


class FakeGroup:
    made = []

    def __init__(self, devices, force_rccl=False):
        self.devices, self.force_rccl = list(devices), bool(force_rccl)
        self.rccl = len(set(self.devices)) > 1 or self.force_rccl   # flm_group_init_flags' clique rule
        self._stores, self.retired, self.closed = 0, False, False
        FakeGroup.made.append(self)

    def close(self):
        if self._stores:
            raise RuntimeError("store open")
        self.closed = True


@pytest.fixture
def fake_groups(monkeypatch):
    FakeGroup.made = []
    monkeypatch.setattr(E, "DeviceGroup", FakeGroup)
    monkeypatch.setattr(protocol, "_group", None)
    monkeypatch.delenv("FLM_GROUP_RCCL", raising=False)
    monkeypatch.delenv("FLM_GPUS", raising=False)
    yield monkeypatch
    protocol._group = None


def test_server_engine_keeps_a_multi_gpu_group(fake_groups):
    """a group of distinct devices has a clique without FLM_GROUP_RCCL; it must be
    reused, not rebuilt (two ncclCommInitAll per iteration) on every server_engine() call."""
    fake_groups.setenv("FLM_GROUP_DEVICES", "0,1,2,3")
    a = protocol.server_engine()
    b = protocol.server_engine()
    assert a is b and len(FakeGroup.made) == 1 and a.rccl and not a.force_rccl
    fake_groups.setenv("FLM_GROUP_RCCL", "1")                   # the request changed: a new group
    c = protocol.server_engine()
    assert c is not a and c.force_rccl and a.closed


def test_replaced_group_is_closed_by_its_last_store(fake_groups):
    from flamingo_amd.ingest import VectorStore
    fake_groups.setenv("FLM_GROUP_DEVICES", "0,1")
    g = protocol.server_engine()
    freed = []

    class Lib:
        def flm_store_free(self, h):
            freed.append(h)

    st = VectorStore.__new__(VectorStore)                      # a store on g (no device needed)
    import ctypes
    st.lib, st.h, st._grp = Lib(), ctypes.c_void_p(1), g
    g._stores = 1
    fake_groups.setenv("FLM_GROUP_DEVICES", "0,1,2")
    g2 = protocol.server_engine()
    assert g2 is not g and g.retired and not g.closed          # still in use: not closed yet
    st.close()
    assert freed and g.closed and g._stores == 0


def test_assigned_vec_sum_partial_feeds_reconstruction(monkeypatch):
    """`server.vec_sum_partial = v` then reconstruction_process without a
    report adds the masks to v (the reference's attribute at :540/:605), instead of failing."""
    import sys
    sys.path.insert(0, __import__("os").path.dirname(__file__))
    from test_abides_protocol_cpu import OracleEngine
    from flamingo_amd.abides.flamingo.service_agent import SA_ServiceAgent
    monkeypatch.setattr(protocol, "_engine", OracleEngine())
    L = 64
    protocol.configure(L=L)
    try:
        srv = SA_ServiceAgent(0, "srv", "SA_ServiceAgent", random_state=np.random.RandomState(1), num_clients=4,
                              users={1, 2, 3})
        base = np.arange(L, dtype=np.uint32) * np.uint32(977)
        srv.vec_sum_partial = base
        with pytest.raises(RuntimeError, match="incorrect length"):
            srv.vec_sum_partial = np.zeros(L + 1, np.uint32)
        m = 0x1234567890ABCDEF
        srv.committee_threshold = 1
        srv.committee_shares_mi = {7: [m]}
        srv.recon_index = {7: 1}
        srv.dec_target_pairwise, srv.recon_symbol = {}, {}
        srv.reconstruction_process()
        want = O.aggregate_unmask(base[None], np.frombuffer(m.to_bytes(32, "big"), np.uint8)[None],
                                  np.array([-1], np.int8), L=L)
        assert np.array_equal(srv.final_sum, want)
    finally:
        protocol.configure(committee=60)


def test_ec_combine_restores_the_callers_ec_coop():
    """the confined-CU combine sets ec_coop for its launch and restores the value
    the caller had set on the shared engine, not -1."""
    from flamingo_amd.dist_recon import ShardedReconstruction

    class Eng:
        def __init__(self):
            self.t = {"ec_coop": 2}
            self.seen = None

        def get_tuning(self, k):
            return self.t[k]

        def set_tuning(self, k, v):
            self.t[k] = v

        def cu_count(self):
            return 256

        def cu_stream(self, cus):
            return None

        def has_comm(self):
            return False

        def ec_combine_dev(self, *a, **k):
            self.seen = self.t["ec_coop"]

    eng = Eng()
    rec = ShardedReconstruction(eng, 4096, device="cpu", ec_cus=72, ec_coop=1)
    rec._ec_combine(None, None, None, None, None)
    assert eng.seen == 1 and eng.t["ec_coop"] == 2
    assert torch.device("cpu") == rec.device


def test_protocol_shutdown_closes_group_and_engine(fake_groups):
    """The simulation's explicit teardown (python -m flamingo_amd.abides ends with it): the group, then
    the engine; nothing left to an exit-time finalizer."""
    fake_groups.setenv("FLM_GROUP_DEVICES", "0,1")
    g = protocol.server_engine()
    closed = []

    class Eng:
        def close(self):
            closed.append("engine")

    fake_groups.setattr(protocol, "_engine", Eng())
    protocol.shutdown()
    assert g.closed and closed == ["engine"] and protocol._group is None and protocol._engine is None
