"""CPU tests of the ABIDES surface (Kernel, Agent, Message, LatencyModel) and of
the agents' seed-sharing arithmetic.  No GPU."""
import numpy as np
import pandas as pd
import pytest

from flamingo_amd.abides import Agent, Kernel, LatencyModel, Message
from flamingo_amd.abides.flamingo.seeds import P256_N, lagrange_at_zero, shamir_recover, shamir_share


class Recorder(Agent):
    def __init__(self, id, peers, log):
        super().__init__(id, f"rec{id}", "Recorder", np.random.RandomState(id + 1))
        self.peers, self.events = peers, log

    def kernelStarting(self, startTime):
        self.setComputationDelay(1000)
        super().kernelStarting(startTime)

    def wakeup(self, t):
        super().wakeup(t)
        self.events.append(("wake", self.id, t))
        for p in self.peers:
            self.sendMessage(p, Message({"from": self.id}))

    def receiveMessage(self, t, msg):
        super().receiveMessage(t, msg)
        self.events.append(("msg", self.id, t, msg.body["from"]))


def run(agents, model=None, **kw):
    k = Kernel("test", random_state=np.random.RandomState(0))
    t0 = pd.Timestamp("2023-01-01")
    return k, k.runner(agents=agents, startTime=t0, stopTime=t0 + pd.Timedelta("1h"), agentLatencyModel=model,
                       defaultComputationDelay=5, skip_log=True, **kw)


def test_kernel_delivery_order_and_delays():
    log = []
    a0, a1 = Recorder(0, [1], log), Recorder(1, [], log)
    model = LatencyModel("deterministic", kwargs={"min_latency": np.array([[0, 777], [777, 0]])})
    k, state = run([a0, a1], model)
    t0 = pd.Timestamp("2023-01-01")
    # a0 wakes at t0, sends at t0 + its computation delay (1000 ns) + latency 777
    assert ("wake", 0, t0) in log
    msgs = [e for e in log if e[0] == "msg"]
    assert msgs == [("msg", 1, t0 + pd.Timedelta(1000 + 777), 0)]
    assert state["kernel_slowest_agent_finish_time"] == t0 + pd.Timedelta(1000 + 777 + 1000)


def test_agent_in_future_requeue():
    log = []

    class Busy(Recorder):
        def wakeup(self, t):
            super().wakeup(t)
            self.delay(10_000)        # busy for 10 us more after this wake

    a0, a1 = Busy(0, [], log), Recorder(1, [0], log)
    model = LatencyModel("deterministic", kwargs={"min_latency": 1})
    run([a0, a1], model)
    t0 = pd.Timestamp("2023-01-01")
    got = [e for e in log if e[0] == "msg"][0]
    # a1's message would arrive at t0+1001 but a0 is busy until t0 + 1000 + 10000
    assert got[2] == t0 + pd.Timedelta(11_000)


def test_latency_model_cubic_bounds():
    m = LatencyModel("cubic", random_state=np.random.RandomState(1),
                     kwargs={"min_latency": np.full((3, 3), 1000), "jitter": 0.3, "jitter_clip": 0.05,
                             "jitter_unit": 5})
    v = [m.get_latency(0, 1) for _ in range(1000)]
    assert min(v) >= 1000
    assert max(v) <= 1000 + (0.3 / 0.05 ** 3) * (1000 / 5)
    with pytest.raises(ValueError):
        LatencyModel("cubic", kwargs={})


def test_message_tiebreak_and_wakeup_validation():
    m1, m2 = Message({}), Message({})
    assert m1 < m2
    k = Kernel("t", random_state=np.random.RandomState(0))
    k.currentTime = pd.Timestamp("2023-01-02")
    with pytest.raises(ValueError):
        k.setWakeup(0, pd.Timestamp("2023-01-01"))
    with pytest.raises(ValueError):
        k.setAgentComputeDelay(0, 1.5)


def test_shamir_roundtrip_and_threshold():
    import random
    rng = random.Random(5)
    secret = int.from_bytes(bytes(range(32)), "big")
    pts = shamir_share(secret, 20, 60, rng=rng)
    assert shamir_recover(pts[:20]) == secret % P256_N
    assert shamir_recover(pts[17:37]) == secret % P256_N
    assert shamir_recover(pts[:19]) != secret % P256_N        # below threshold
    xs = [p[0] for p in pts[:20]]
    assert sum(lagrange_at_zero(xs)) % P256_N == 1            # interpolates constants exactly


def test_pair_seed_pipeline_symmetric():
    """s_ij derived by i (a_i A_j) equals the one derived by j (a_j A_i) (SA_ClientAgent.py:256-292).

    Reference quirk kept: h_ijt = ChaCha20(key).encrypt(t.to_bytes(16, 'big'))[0:4] & 0xFFFF
    (:276-279) only sees keystream bytes 0-3 XOR the zero high bytes of t, so s_ij is the
    same in every iteration t < 2^96, and differs only between pairs."""
    import hashlib
    import oracle as O                        # the checker's ChaCha20 (the product has only the GPU's)
    from flamingo_amd import crypto as C
    ai, aj = 1234567, 7654321
    Ai, Aj = C.mul(ai), C.mul(aj)

    def seed(a, B, it):
        key = hashlib.sha256(C.point_bytes(C.mul(a, B))).digest()
        h = O.chacha20_encrypt(key, it.to_bytes(16, "big"))
        H = C.hash_str_to_curve(str(int.from_bytes(h[:4], "big") & 0xFFFF))
        return hashlib.sha256(C.point_bytes(H)).digest()

    assert seed(ai, Aj, 1) == seed(aj, Ai, 1)
    assert seed(ai, Aj, 1) == seed(ai, Aj, 2)
    assert seed(ai, Aj, 1) != seed(ai, C.mul(99), 1)


def test_latency_model_matches_reference_golden():
    """Pinned to the reference itself: tests/golden/latency.json was produced by importing the
    reference's own model/LatencyModel.py (numpy-only, no shim; tests/golden/make_latency_golden.py).
    Same parameters and RandomState seed -> the same latency for every call, in order."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "latency.json")) as f:
        g = json.load(f)
    calls = [tuple(c) for c in g["calls"]]
    for name, c in g["cases"].items():
        kw = {k: (np.array(v) if isinstance(v, list) else v) for k, v in c["kwargs"].items()}
        m = LatencyModel(c["model"], random_state=np.random.RandomState(c["seed"]), kwargs=kw)
        got = [float(m.get_latency(s, r)) for s, r in calls]
        assert got == c["latencies"], name


def test_same_time_ties_follow_message_creation_order():
    """Kernel.py queues (time, (recipient, type, msg)): equal delivery times go to the message
    created first (Message.__lt__ on uniq), not the one sent first."""
    log = []

    class Sender(Agent):
        def __init__(self, id):
            super().__init__(id, "s", "Sender", np.random.RandomState(1))

        def kernelStarting(self, startTime):
            self.setComputationDelay(0)
            super().kernelStarting(startTime)

        def wakeup(self, t):
            super().wakeup(t)
            first, second = Message({"from": "first"}), Message({"from": "second"})
            self.sendMessage(1, second)          # sent first, created second
            self.sendMessage(1, first)

    class Sink(Recorder):
        def __init__(self):
            super().__init__(1, [], log)

    model = LatencyModel("deterministic", kwargs={"min_latency": 5})
    run([Sender(0), Sink()], model)
    got = [e[3] for e in log if e[0] == "msg"]
    assert got == ["first", "second"]
