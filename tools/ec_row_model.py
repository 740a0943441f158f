"""Model of the row-sliced P-256 field layer (flamingo_amd/csrc/flm_fe_row.h) and of what it buys
the cooperative scalar multiplication's latency chain.

1. The exact algorithm of flm_fe_row.h in Python integers -- one 32-bit limb per lane of a 16-lane
   row, the product columns, the carry passes, the NIST fold with the 8x8 coefficient matrix, the
   signed passes with the top carry folded back -- checked against Python's own mod-p arithmetic,
   and the number of carry passes each loop takes (the kernel loops while any lane of the wave
   carries, so the passes are part of the instruction count).
2. VALU instructions per field operation for both layouts: the per-lane Montgomery field of
   flm_p256.hip (gfx950 ISA counts, DESIGN.md section 5: fe_mul 258, fe_sqr 265, fe_add 28, fe_sub
   20) and the row field (ISA counts of tools/probes/ec_row_probe.hip's chains, plus the carry
   passes from 1.).
3. The critical path of the cooperative formulas (coop_dbl_w: 3 multiplication levels; coop_add_w: 5
   of them, six barrier levels) in each layout, and the predicted time of one G = 8 rank's combine
   (D = 120 pairs x T = 20) from the measured per-lane kernel: only the field arithmetic shrinks, the
   barriers, LDS exchanges and ec_finish stay.
Run: python tools/ec_row_model.py  (prints the model; tests/test_ec_row_model_cpu.py checks 1.)"""
import random
from collections import Counter

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
M32 = (1 << 32) - 1
# kFold of flm_fe_row.h: limb r of a*b mod p takes A[r][k] * c_(8+k) (NIST FIPS 186 fast reduction)
A = [[1, 1, 0, -1, -1, -1, -1, 0], [0, 1, 1, 0, -1, -1, -1, -1], [0, 0, 1, 1, 0, -1, -1, -1],
     [-1, -1, 0, 2, 2, 1, 0, -1], [0, -1, -1, 0, 2, 2, 1, 0], [0, 0, -1, -1, 0, 2, 2, 1],
     [-1, -1, 0, 0, 0, 1, 3, 2], [1, 0, -1, -1, -1, -1, 0, 3]]
FCO = [1, 0, 0, -1, 0, 0, -1, 1]      # where the carry out of limb 7 lands: t 2^256 = t (2^224 - 2^192 - 2^96 + 1)


def limbs(x, n=8):
    return [(x >> (32 * i)) & M32 for i in range(n)]


def val(w):
    return sum(v << (32 * i) for i, v in enumerate(w))


def snorm(v):
    """row::snorm: signed limb values -> limbs of a congruent value in [0, 2^256); returns (limbs, passes)."""
    passes = 0
    c = [x >> 32 for x in v]
    lo = [x & M32 for x in v]
    while any(c):
        t = c[7]
        v = [lo[r] + (c[r - 1] if r else 0) + t * FCO[r] for r in range(8)]
        c = [x >> 32 for x in v]
        lo = [x & M32 for x in v]
        passes += 1
    return lo, passes


def row_mul(a, b):
    """row::mul: returns (a*b mod p lazily in [0, 2^256), column passes, fold passes)."""
    la, lb = limbs(a), limbs(b)
    col = [sum(la[i] * lb[t - i] for i in range(8) if 0 <= t - i < 8) for t in range(16)]   # < 2^67
    acc = [x & ((1 << 64) - 1) for x in col]
    hi = [x >> 64 for x in col]
    s = [(acc[t] & M32) + ((acc[t - 1] >> 32) if t >= 1 else 0) + (hi[t - 2] if t >= 2 else 0) for t in range(16)]
    c = [x >> 32 for x in s]
    lo = [x & M32 for x in s]
    p1 = 0
    while any(c):
        s = [lo[t] + (c[t - 1] if t else 0) for t in range(16)]
        c = [x >> 32 for x in s]
        lo = [x & M32 for x in s]
        p1 += 1
    assert val(lo) == a * b
    v = [lo[r] + sum(A[r][k] * lo[8 + k] for k in range(8)) for r in range(8)]
    out, p2 = snorm(v)
    return val(out), p1, p2


def row_add(a, b):
    out, p = snorm([x + y for x, y in zip(limbs(a), limbs(b))])
    return val(out), p


def row_sub(a, b):
    out, p = snorm([x - y for x, y in zip(limbs(a), limbs(b))])
    return val(out), p


def check(n_random=2000, seed=3):
    """Every result congruent and in [0, 2^256) on random and edge inputs; returns pass histograms."""
    rng = random.Random(seed)
    edge = [0, 1, 2, P - 1, P, P + 1, 2**256 - 1, 2**255, 2**224, 2**96 - 1, 2**192, 2**256 - P]
    xs = edge + [rng.getrandbits(256) for _ in range(n_random)]
    hist = {"mul_columns": Counter(), "mul_fold": Counter(), "add": Counter(), "sub": Counter()}
    for k, a in enumerate(xs):
        for b in (edge if k < len(edge) else []) + [xs[(k * 7 + 1) % len(xs)], xs[(k * 13 + 5) % len(xs)]]:
            r, p1, p2 = row_mul(a, b)
            assert 0 <= r < 2**256 and r % P == a * b % P, (a, b)
            hist["mul_columns"][p1] += 1
            hist["mul_fold"][p2] += 1
            r, p = row_add(a, b)
            assert 0 <= r < 2**256 and r % P == (a + b) % P
            hist["add"][p] += 1
            r, p = row_sub(a, b)
            assert 0 <= r < 2**256 and r % P == (a - b) % P
            hist["sub"][p] += 1
    return hist


def mean(h):
    return sum(k * v for k, v in h.items()) / sum(h.values())


# VALU instructions per operation on one wave's critical path.
# Per-lane Montgomery field, gfx950 ISA of flm_p256.hip.
LANE = {"M": 258, "S": 265, "A": 28, "B": 20, "Z": 9}
# Row field, ISA of tools/probes/ec_row_probe.hip (hipcc -O3, gfx950): the carry loops are
# do-while (the first pass unconditional, then a wave-wide vote), so the multiply chain's loop is 93
# instructions with one pass of each loop, +7 per further column pass and +10 per further fold
# pass; an add or subtract is 14 with one pass, +10 per further pass.  A zero test is two ballots
# and compares (~10).  (Round 4's first version, with the votes before the passes and a
# cndmask/subtract per negative fold coefficient, was 103 + 5 + 8 = 116 and 9.5 + 8.)
ROW_BASE = {"M": 93, "M_col": 7, "M_fold": 10, "A": 14, "A_pass": 10, "Z": 10}

# The cooperative formulas' critical path (the longest wave of each barrier level), as op counts:
# coop_dbl_w: before barrier 1 every wave does 2 multiplications (w0: X^2, alpha^2) and 3 add/subs,
# after it w0 does alpha (4 beta - X3) and 3 subs -> 3 M + 6 A.
# coop_add_w: L1 1 M + 1 A, L2-L4 1 M + 2 A each, L5 1 M + 3 A, L6 1 A + 3 zero tests (+1 A for a
# negative digit's -Q.Y) -> 5 M + 12 A + 3 Z.
SCHED = {"dbl": {"M": 3, "A": 6, "Z": 0}, "add": {"M": 5, "A": 12, "Z": 3}}


def extra(h):
    """Mean passes beyond the first (the kernel's loops always run one)."""
    return sum(max(k - 1, 0) * v for k, v in h.items()) / sum(h.values())


def op_costs(hist):
    row = {"M": ROW_BASE["M"] + ROW_BASE["M_col"] * extra(hist["mul_columns"]) + ROW_BASE["M_fold"] * extra(hist["mul_fold"]),
           "A": ROW_BASE["A"] + ROW_BASE["A_pass"] * (extra(hist["add"]) + extra(hist["sub"])) / 2,
           "Z": ROW_BASE["Z"]}
    lane = {"M": (LANE["M"] + LANE["S"]) / 2, "A": (LANE["A"] + LANE["B"]) / 2, "Z": LANE["Z"]}
    return lane, row


def chain(cost, kind):
    return sum(SCHED[kind][k] * cost[k] for k in ("M", "A", "Z"))


def predict(hist, dbl_us=2.36, add_us=8.65, n_dbl=258, n_add=50, finish_ms=0.15, dbl_barrier_us=0.35,
            add_barrier_us=0.35):
    """One G = 8 rank's combine (D = 120, T = 20) with the row field: the measured per-lane
    cooperative kernel's doubling and addition times (2.36 / 8.65 us after round 3)
    minus their barrier/LDS overhead (2 and 6 barrier levels; ~0.35 us each, an assumption the
    measurement replaces) scale with the field-arithmetic instruction ratio."""
    lane, row = op_costs(hist)
    r_dbl = chain(row, "dbl") / chain(lane, "dbl")
    r_add = chain(row, "add") / chain(lane, "add")
    dbl_row = (dbl_us - 2 * dbl_barrier_us) * r_dbl + 2 * dbl_barrier_us
    add_row = (add_us - 6 * add_barrier_us) * r_add + 6 * add_barrier_us
    lane_ms = (n_dbl * dbl_us + n_add * add_us) / 1e3 + finish_ms
    row_ms = (n_dbl * dbl_row + n_add * add_row) / 1e3 + finish_ms
    return {"field_ops_lane": lane, "field_ops_row": row,
            "dbl_chain_instr": (chain(lane, "dbl"), chain(row, "dbl")),
            "add_chain_instr": (chain(lane, "add"), chain(row, "add")),
            "combine_ms_lane_model": lane_ms, "combine_ms_row_model": row_ms,
            "saving": 1 - row_ms / lane_ms}


# ---------------------------------------------------------------- interleave model
# Measured (DESIGN.md sections 5 and 10.2, profiles/r04_ec_kernel_sweep.log, r04_rank8_row.log):
LONE_MUL_NS = 279.0          # one row-field multiplication, one wave alone on its SIMD: 93 instructions
LONE_CPI = 6.5               # cycles per instruction of that lone chain (the DPP read waits on the last mad)
DBL_US_LONE = 1.78           # one doubling, lone wave
DBL_US_D120 = 2.38           # one doubling in the whole-GPU combine at D = 120, T = 20 (2,400 products)
ADD_US_LONE, ADD_US_D120 = 2.4, 3.2
SIMDS = 256 * 4


def interleave_model(products=2400, cus=256, k=2):
    """Cycles per formula step (one dependent instruction of every chain) on the busiest SIMD of the
    row kernel, now (one product per wave) and with k independent products interleaved per wave.

    A SIMD holding n waves, each a dependent chain, issues one instruction of each per step and takes
    max(L, n c) cycles for it: L = the lone chain's cycles per instruction (the DPP reads wait on the
    previous v_mad_u64_u32), c = the SIMD's issue cost of one wave instruction.  The busiest SIMD holds
    ceil(products / SIMDs) waves today, ceil(products / (k SIMDs)) waves of k instructions per step
    interleaved.  c is calibrated on the D = 120 measurement: 2,400 products on 1,024 SIMDs (3 waves
    on the busiest), 2.38 us per doubling against 1.78 us for a lone wave."""
    import math
    simds = cus * 4
    c = DBL_US_D120 / DBL_US_LONE * LONE_CPI / math.ceil(2400 / SIMDS)
    n_now = math.ceil(products / simds)
    n_int = math.ceil(products / (k * simds))
    now = max(LONE_CPI, n_now * c)
    inter = max(LONE_CPI, n_int * k * c)
    return {"busiest_simd_waves_now": n_now, "busiest_simd_waves_interleaved": n_int,
            "issue_cycles_per_instr": round(c, 3), "cycles_per_step_now": round(now, 3),
            "cycles_per_step_interleaved": round(inter, 3), "saving": round(1 - inter / now, 4)}


# ---------------------------------------------------------------- Straus in the row kernel (round 5)
# The issue-bound picture above, applied to one G = 8 rank's shares -> final: the combine's waves
# (priority 3) and the self-mask pass share the SIMDs, so the rank's time is about the SUM of the two
# issue workloads (bounded below by the combine's own chain latency).  Round 4 modelled Straus
# grouping against the combine ALONE (latency-bound: -7 %); beside the pass it is the issue work that
# counts.  Per-wave SIMD issue cost of one coop step, from the D = 120 calibration (3 waves on the
# busiest SIMD): a doubling 2.38 / 3 us, an addition 3.2 / 3 us; lone-wave latency 1.78 / 2.4 us.
DBL_ISSUE_US, ADD_ISSUE_US = DBL_US_D120 / 3, ADD_US_D120 / 3
PASS_MS_G8 = 0.82          # one G = 8 rank's self-mask pass alone (K = 4,055 + 121 over 2^17 slots)
RANK8_NOW_MS = (1.39, 1.52)  # measured: shares -> final, coop kernel on 72 CUs / row kernel unpartitioned


def straus_row_model(g, D=121, T=20, simds=SIMDS, pass_ms=PASS_MS_G8, adds_per_term=50):
    """g terms of one pair per row chain (a shared doubling chain, g tables of odd multiples):
    chains = D ceil(T / g), each (258 + g) doublings (258 of the chain + one per table) and
    g x 50 additions (43 wNAF + 7 table).  Returns the combine's issue work spread over the chip,
    its lone chain latency, and the predicted shares -> final = max(latency, pass + work)."""
    import math
    chains = D * math.ceil(T / g)
    dbl, add = 258 + g, adds_per_term * g
    work_ms = chains * (dbl * DBL_ISSUE_US + add * ADD_ISSUE_US) / simds / 1e3
    lat_ms = (dbl * DBL_US_LONE + add * ADD_US_LONE) / 1e3
    return {"g": g, "chains": chains, "combine_issue_ms": round(work_ms, 3), "chain_latency_ms": round(lat_ms, 3),
            "rank_ms": round(max(lat_ms, pass_ms + work_ms), 3)}


# Measured after building it (profiles/r05_ec_row_straus_combine_alone.log, r05_rank8_row_straus.log):
# the combine alone at D = 121 takes 0.825 / 0.994 / 1.405 ms at g = 1 / 2 / 4 -- the g = 4 chain runs
# 1.48x the lone-wave latency the model assumed (0.95 ms: 4 LDS tables, 4 digit strings, up to 26
# barriers per step against 8) -- and one rank's shares -> final 1.507 / 1.484 / 1.466 ms (-3 %).
MEASURED_RANK8_MS = {1: 1.507, 2: 1.484, 4: 1.466}
MEASURED_COMBINE_MS = {1: 0.825, 2: 0.994, 4: 1.405}


def straus_report():
    base = straus_row_model(1)["rank_ms"]
    return [dict(straus_row_model(g), saving=round(1 - straus_row_model(g)["rank_ms"] / base, 3)) for g in (1, 2, 4, 5)]


def interleave_report():
    rows = []
    for name, products, cus in (("whole-GPU combine, c5 one rank of G = 8 (D = 121 x T = 20)", 2420, 256),
                                ("the same on the rank's 72 EC CUs (beside the self-mask pass)", 2420, 72),
                                ("whole-GPU combine, c5 on one GPU (D = 962 x T = 20)", 19240, 256),
                                ("a small batch on 8 CUs, one product per SIMD (32 products)", 32, 8),
                                ("a small batch on 8 CUs, two products per SIMD (64 products)", 64, 8)):
        rows.append((name, interleave_model(products, cus)))
    return rows


if __name__ == "__main__":
    h = check()
    for k, v in h.items():
        print(f"{k} carry passes: mean {mean(v):.3f}, histogram {sorted(v.items())}")
    p = predict(h)
    print("instructions per op, per-lane field:", {k: round(v, 1) for k, v in p["field_ops_lane"].items()})
    print("instructions per op, row field:     ", {k: round(v, 1) for k, v in p["field_ops_row"].items()})
    print("doubling critical path (lane, row): %.0f, %.0f instructions" % p["dbl_chain_instr"])
    print("addition critical path (lane, row): %.0f, %.0f instructions" % p["add_chain_instr"])
    print("one G = 8 rank's combine (D = 120 x T = 20): per-lane model %.3f ms, row model %.3f ms: %.0f %% less"
          % (p["combine_ms_lane_model"], p["combine_ms_row_model"], 100 * p["saving"]))
    print()
    print("Straus in the row kernel, one G = 8 rank of c5 (D = 121, T = 20) beside its self-mask pass:")
    for r in straus_report():
        print("  ", r)
    print()
    print("two products interleaved per row (k = 2), cycles per formula step on one SIMD:")
    for name, r in interleave_report():
        print(f"  {name}: {r}")
