"""Hash to curve on the GPU (flm_hash_to_curve*, flm_p256.hip hash_to_curve_kernel) against the
reference's table (tests/golden/h2c_golden.json, made by its own ecchash.py) and the oracle."""
import hashlib
import json
import os

import numpy as np
import pytest

import ec_oracle as E

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def eng():
    from flamingo_amd import MaskEngine
    e = MaskEngine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def table(eng):
    return eng.hash_to_curve_decimal(0, 1 << 16)


def test_gpu_h2c_table_matches_reference(table):
    """Every one of the 2^16 points the client can hash (SA_ClientAgent.py:280-286), one launch."""
    with open(os.path.join(HERE, "golden", "h2c_golden.json")) as f:
        g = json.load(f)
    out, fl = table
    assert not (fl & 12).any()
    for v, hx in g["points"].items():
        assert out[int(v)].tobytes().hex() == hx, v
    assert hashlib.sha256(out.tobytes()).hexdigest() == g["table_sha256"]


def test_gpu_h2c_random_rows_match_oracle(table):
    out, _ = table
    for v in np.random.default_rng(3).integers(0, 1 << 16, 64):
        assert out[v].tobytes() == E.wire(E.hash_str_to_curve(str(int(v)))), int(v)


def test_gpu_h2c_offsets_and_long_decimals(eng):
    """v0 > 0 and up to 10 digits (the table entry point takes any 32-bit range)."""
    for v0, n in ((65530, 12), (4294967290, 6), (999999995, 10)):
        out, fl = eng.hash_to_curve_decimal(v0, n)
        assert not fl.any()
        for i in range(n):
            assert out[i].tobytes() == E.wire(E.hash_str_to_curve(str(v0 + i))), v0 + i
    with pytest.raises(RuntimeError):
        eng.hash_to_curve_decimal(4294967290, 7)


def test_gpu_h2c_arbitrary_messages(eng):
    rng = np.random.default_rng(11)
    msgs = [b"", b"abcdeefekf", "h", "65535", bytes(64)] + \
        [bytes(rng.integers(0, 256, int(ln), dtype=np.uint8)) for ln in rng.integers(0, 65, 40)]
    out, fl = eng.hash_to_curve_wire(msgs)
    assert not fl.any()
    for m, row in zip(msgs, out):
        assert row.tobytes() == E.wire(E.hash_str_to_curve(m)), m
    with pytest.raises(RuntimeError):
        eng.hash_to_curve_wire([bytes(65)])


def test_gpu_h2c_dev_form_matches_host_form(eng, table):
    import torch
    out = torch.zeros((4096, 64), dtype=torch.uint8, device="cuda")
    fl = torch.full((4096,), -1, dtype=torch.int32, device="cuda")
    eng.hash_to_curve_decimal_dev(1000, 4096, out, fl)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), table[0][1000:5096]) and not fl.cpu().numpy().any()


def test_protocol_hash_to_curve_uses_the_gpu_table(eng):
    from flamingo_amd.abides.flamingo import protocol
    protocol.configure()
    try:
        for h in ("0", "7", "65535", "31337"):
            assert protocol.hash_to_curve(h) == E.hash_str_to_curve(h)
        assert protocol._h2c_table is not None
        assert protocol.hash_to_curve("007") == E.hash_str_to_curve("007")     # not a table key
    finally:
        protocol.configure()
