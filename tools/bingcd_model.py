"""Model of the GPU inversion: Pornin's optimized binary GCD (eprint 2020/972, Alg. 2) with
k-1 = 30 inner steps (int32 update factors), 64-bit approximations (low 30 bits + top 34 bits)."""
import random
P = 2**256 - 2**224 + 2**192 + 2**96 - 1
M64 = (1 << 64) - 1

def inv(x, outer=18, trace=None):
    a, b, u, v = x, P, 1, 0
    for it in range(outer):
        n = max(a.bit_length(), b.bit_length(), 64)
        sh = n - 64
        abar = ((a >> sh) & ~((1 << 30) - 1) & M64) | (a & ((1 << 30) - 1))
        bbar = ((b >> sh) & ~((1 << 30) - 1) & M64) | (b & ((1 << 30) - 1))
        f0, g0, f1, g1 = 1, 0, 0, 1
        for j in range(30):
            if abar & 1:
                if abar < bbar:
                    abar, bbar = bbar, abar
                    f0, g0, f1, g1 = f1, g1, f0, g0
                abar -= bbar
                f0, g0 = f0 - f1, g0 - g1
            abar >>= 1
            f1, g1 = 2 * f1, 2 * g1
        assert max(abs(f0), abs(g0), abs(f1), abs(g1)) <= 2**30
        na, nb = a * f0 + b * g0, a * f1 + b * g1
        assert na % (1 << 30) == 0 and nb % (1 << 30) == 0
        na >>= 30; nb >>= 30
        if na < 0: na, f0, g0 = -na, -f0, -g0
        if nb < 0: nb, f1, g1 = -nb, -f1, -g1
        a, b = na, nb
        w0, w1 = u * f0 + v * g0, u * f1 + v * g1
        q0, q1 = w0 % (1 << 30), w1 % (1 << 30)      # -p^-1 = 1 mod 2^30
        u, v = (w0 + q0 * P) >> 30, (w1 + q1 * P) >> 30
        assert -P <= u <= 2 * P and -P <= v <= 2 * P, (u, v)
        u %= P; v %= P
        if trace is not None and a == 0 and trace.get('done') is None: trace['done'] = it + 1
    assert a == 0 and b == 1, (x, a, b)
    return v

def check(n_random=20000, seed=5):
    """Every input converges within the 18 outer steps and matches Fermat; returns the worst
    number of outer steps any input needed."""
    rng = random.Random(seed)
    cases = [1, 2, 3, P - 1, P - 2, 2**255, 2**224, 2**96 - 1, (P - 1) // 2, 2**64 - 1, 2**30 + 1] + [rng.randrange(1, P) for _ in range(n_random)]
    worst = 0
    for x in cases:
        tr = {}
        r = inv(x, trace=tr)
        assert r == pow(x, P - 2, P), x
        worst = max(worst, tr['done'])
    return len(cases), worst


if __name__ == "__main__":
    n, worst = check()
    print("ok", n, "worst outer iterations to a == 0:", worst)
