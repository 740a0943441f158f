"""The binary-GCD inversion schedule ec_finish_kernel runs (flm_p256.hip fe_inv_bingcd: 18 outer
steps of 30 inner steps, int32 update factors, 64-bit approximations), as its Python model
tools/bingcd_model.py: it must converge within the 18 steps and agree with Fermat's a^(p-2).
The GPU kernel itself is checked end to end by tests/test_ec_gpu.py (every combine inverts Z)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import bingcd_model  # noqa: E402


def test_schedule_converges_and_matches_fermat():
    n, worst = bingcd_model.check(n_random=1500, seed=11)
    assert n > 1500 and worst <= 18


def test_single_step_bounds():
    # the inner loop's factors stay within int32 (|f|, |g| <= 2^30) on the extreme inputs
    for x in (1, 2, bingcd_model.P - 1, 2 ** 255, 2 ** 64 - 1):
        assert bingcd_model.inv(x) == pow(x, bingcd_model.P - 2, bingcd_model.P)
