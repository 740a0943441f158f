"""Driver of tools/probes/ec_row_probe.hip: the row-sliced P-256 field layer (flm_fe_row.h) checked
against Python integers on random and edge inputs, then its lone-wave latency per dependent multiply
against the per-lane product-scanning multiply.  Writes the log to stdout."""
import os
import random
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "ec_row_probe")
P = 2**256 - 2**224 + 2**192 + 2**96 - 1


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def val(w):
    return sum(int(v) << (32 * i) for i, v in enumerate(w))


def main():
    rng = random.Random(7)
    edge = [0, 1, 2, P - 1, P, P + 1, 2**256 - 1, 2**255, 2**224, 2**96 - 1, 2**192, 2**256 - P, 2**32 - 1,
            2**256 - 2**32]
    pairs = [(a, b) for a in edge for b in edge] + [(rng.getrandbits(256), rng.getrandbits(256)) for _ in range(8000)]
    pairs += [(rng.getrandbits(256), b) for b in edge for _ in range(20)]
    n = len(pairs)
    inp = np.array([limbs(a) + limbs(b) for a, b in pairs], np.uint32)
    with tempfile.TemporaryDirectory() as td:
        fi, fo = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        inp.tofile(fi)
        r = subprocess.run([BIN, "check", fi, fo], capture_output=True, text=True, timeout=120)
        print(r.stdout.strip(), r.stderr.strip())
        if r.returncode:
            sys.exit(r.returncode)
        out = np.fromfile(fo, np.uint32)
    res, flags = out[: n * 48].reshape(n, 48), out[n * 48:]
    bad = 0
    for e, (a, b) in enumerate(pairs):
        w = res[e]
        m, s, d, mc, z, zc = (val(w[8 * k:8 * k + 8]) for k in range(6))
        chain = a % P
        for _ in range(64):
            chain = chain * b % P
        good = (m < 2**256 and m % P == a * b % P and s < 2**256 and s % P == (a + b) % P and d < 2**256
                and d % P == (a - b) % P and mc == a * b % P and z < 2**256 and z % P == chain and zc == chain
                and flags[e] == (1 | (2 if a % P == 0 else 0)))
        if not good:
            bad += 1
            if bad <= 5:
                print("MISMATCH", hex(a), hex(b), [hex(v) for v in (m, s, d, mc, z, zc)], flags[e])
    print(f"row field layer vs Python integers: {n - bad}/{n} elements exact (mul, add, sub, canon, 64-mul chain, "
          f"is_zero)")
    if bad:
        sys.exit(1)
    r = subprocess.run([BIN, "time"], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
