"""The row-sliced field layer of the cooperative EC kernel (flamingo_amd/csrc/flm_fe_row.h,
ec_mul_row_kernel) as its Python model tools/ec_row_model.py: the product columns, the NIST fold
with its 8x8 coefficient matrix and the signed carry passes give a value congruent mod p and below
2^256 on random and edge inputs, and the carry loops end after about one pass.  The GPU kernel is
checked end to end by tests/test_ec_gpu.py (the "row" parametrisation) and bit for bit against Python
integers by tools/probes/ec_row_probe.py."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import ec_row_model as M  # noqa: E402


def test_fold_matrix_is_the_nist_reduction():
    import random
    rng = random.Random(2)
    for _ in range(500):
        c = [rng.getrandbits(32) for _ in range(16)]
        v = sum(x << (32 * i) for i, x in enumerate(c))
        r = sum((c[j] + sum(M.A[j][k] * c[8 + k] for k in range(8))) << (32 * j) for j in range(8))
        assert (r - v) % M.P == 0
    # the top-carry fold: 2^256 = 2^224 - 2^192 - 2^96 + 1 (mod p)
    assert sum(f << (32 * r) for r, f in enumerate(M.FCO)) % M.P == 2**256 % M.P


def test_row_arithmetic_matches_python_ints():
    hist = M.check(n_random=600, seed=5)
    for k in ("mul_columns", "mul_fold", "add", "sub"):
        assert 0.5 < M.mean(hist[k]) < 1.5, (k, hist[k])


def test_model_predicts_the_threshold():
    """The decision rule of VERDICT r3 item 5: implement only if the model predicts >= 20 % off one
    G = 8 rank's combine."""
    p = M.predict(M.check(n_random=300, seed=7))
    assert p["dbl_chain_instr"][1] < 0.6 * p["dbl_chain_instr"][0]
    assert p["saving"] >= 0.20


def test_interleave_model_predicts_no_gain():
    """two products interleaved per row against the measured row kernel.  The
    SIMD already issues its waves into each other's DPP latency, so within-wave interleave cannot beat
    spreading the same products over waves; below the 20 % bar everywhere (not built)."""
    import ec_row_model as R
    for name, r in R.interleave_report():
        assert r["saving"] < 0.2, name
    assert R.interleave_model(2420, 256)["cycles_per_step_now"] > R.LONE_CPI      # D = 121 is issue-bound


def test_straus_row_model_prediction_and_measurement():
    """Round 5: g terms of a pair per row chain.  The model (g = 1 reproduces the measured one-rank-of-8
    shares -> final, 1.39-1.52 ms) predicted >= 20 % less at g = 4, so it was built
    (ec_mul_row_straus_kernel); measured, the chain ran 1.48x the latency the model assumed and the
    rank gained 3 %: the default stays g = 1 (flm_set_tuning ec_row_terms)."""
    import ec_row_model as R
    rep = {r["g"]: r for r in R.straus_report()}
    assert R.RANK8_NOW_MS[0] - 0.05 <= rep[1]["rank_ms"] <= R.RANK8_NOW_MS[1]
    assert rep[4]["saving"] >= 0.2 and rep[2]["chain_latency_ms"] < rep[2]["rank_ms"]
    assert 1 - R.MEASURED_RANK8_MS[4] / R.MEASURED_RANK8_MS[1] < 0.2             # measured: below the bar
    assert R.MEASURED_COMBINE_MS[4] / rep[4]["chain_latency_ms"] > 1.4
