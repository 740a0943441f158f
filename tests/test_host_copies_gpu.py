"""The host-pointer entry points never hand the caller's pageable memory to a HIP copy (DESIGN.md
section 6).  For a large pageable copy the HIP runtime pins the caller's pages (a KFD userptr
allocation); their later unmapping made the driver evict all of the process's GPU queues for
20-40 ms -- the agent run's unmask stall.  The library now copies every caller array through
pinned memory of its own: a bounce buffer for copies under 32 MiB, the two 32 MiB staging buffers
in pieces for larger ones (the CPU side split over the context's copy threads).

The check runs every host-pointer entry point with inputs and outputs of 1 KiB-300 MiB (40 MiB in
and out: a 32 MiB piece and a tail of one row; 300 MiB out: 10 pieces of 8 rows) in a child
process under AMD_LOG_LEVEL=4 (the runtime logs "HSA Copy Using Pinned resource" when it pins a
caller buffer for a copy) and asserts that no such line appears, while the results stay exact."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/oracle")
import oracle as O
from flamingo_amd import MaskEngine
eng = MaskEngine(0)
g = np.random.Generator(np.random.PCG64(7))
L = 1 << 20
seeds = g.integers(0, 256, (4, 32), dtype=np.uint8)
signs = np.array([1, -1, 1, -1], np.int8)
rows = g.integers(0, 2**32, (4, L), dtype=np.uint32)
print("== aggregate_unmask", flush=True)
out = eng.aggregate_unmask(rows, seeds, signs)
assert np.array_equal(out, O.aggregate_unmask(rows, seeds, signs, L=L))
print("== client_mask", flush=True)
y = eng.client_mask(np.array([0, 4], np.int64), seeds, signs, L, x=rows[:1])
assert np.array_equal(y, O.client_mask(np.array([0, 4], np.int64), seeds, signs, L, x=rows[:1]))
print("== client_mask 3 ragged rows", flush=True)
L2 = 100_003  # device rows padded to a wider pitch: 2-D copies whose thread slices cross rows
x3 = g.integers(0, 2**32, (3, L2), dtype=np.uint32)
seg3 = np.array([0, 2, 3, 4], np.int64)
assert np.array_equal(eng.client_mask(seg3, seeds, signs, L2, x=x3), O.client_mask(seg3, seeds, signs, L2, x=x3))
print("== prg_expand", flush=True)
e = eng.prg_expand(seeds, L)
assert all(np.array_equal(e[k], O.prg(seeds[k].tobytes(), L, 0)) for k in range(4))
print("== prg_expand 300 MiB", flush=True)
big = g.integers(0, 256, (75, 32), dtype=np.uint8)
e = eng.prg_expand(big, L)
for k in (0, 63, 64, 74):
    assert np.array_equal(e[k, -1024:], O.prg(big[k].tobytes(), 1024, L - 1024))
del e
print("== mask_accumulate", flush=True)
acc = rows[1].copy()
eng.mask_accumulate(seeds, signs, acc)
assert np.array_equal(acc, O.aggregate_unmask(rows[1:2], seeds, signs, L=L))
print("== chacha20", flush=True)
data = bytes(g.integers(0, 256, 4 << 20, dtype=np.uint8))
ct = eng.chacha20_encrypt(seeds[0].tobytes(), data)
assert eng.chacha20_encrypt(seeds[0].tobytes(), ct) == data
print("== chacha20 40 MiB", flush=True)
data = bytes(g.integers(0, 256, 40 << 20, dtype=np.uint8))  # one 32 MiB piece + a tail, each way
assert eng.chacha20_encrypt(seeds[1].tobytes(), data) == O.chacha20_encrypt(seeds[1].tobytes(), data)
del data
print("== hash_to_curve_decimal", flush=True)
pts, fl = eng.hash_to_curve_decimal(0, 1 << 16)
assert not fl.any() and pts.shape == (1 << 16, 64)
print("== ec_mul_wire", flush=True)
n = 20000
out, fl = eng.ec_mul_wire(np.repeat(pts[:1], n, axis=0), g.integers(0, 256, (n, 32), dtype=np.uint8))
assert not (fl & 2).any()
print("== ec_combine_wire", flush=True)
T, D = 20, 1000
eng.ec_combine_wire(pts[:D], np.repeat(pts[None, 1:D + 1], T, axis=0), g.integers(0, 128, (T, 32), dtype=np.uint8))
print("== shamir_combine", flush=True)
eng.shamir_combine([[int(v) for v in g.integers(1, 2**62, 5000)] for _ in range(20)],
                   [int(v) for v in g.integers(1, 2**62, 20)])
print("== done", flush=True)
"""


def test_host_pointer_calls_never_pin_caller_memory():
    env = dict(os.environ, AMD_LOG_LEVEL="4")
    r = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT))], capture_output=True, text=True,
                       timeout=110, env=env)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    assert "== done" in r.stdout
    pinned = [ln for ln in log.splitlines() if "Using Pinned resource" in ln]
    assert not pinned, "the HIP runtime pinned caller memory:\n" + "\n".join(pinned[:10])


def test_copy_threads_end_with_their_context():
    """A context's copy threads start on its first large host copy and are joined by flm_free: twelve
    contexts made, used and freed leave the process with as many threads as after the first."""
    import numpy as np
    from flamingo_amd import MaskEngine

    def nthreads():
        return len(os.listdir("/proc/self/task"))

    g = np.random.Generator(np.random.PCG64(11))
    seeds = g.integers(0, 256, (4, 32), dtype=np.uint8)
    after = []
    during = None
    for i in range(12):
        with MaskEngine(0) as eng:
            eng.prg_expand(seeds, 1 << 18)  # a 4 MiB output: the copy out runs on the copy threads
            if during is None:
                during = nthreads()
        after.append(nthreads())
    assert during >= after[0] + 3, (during, after)
    assert after[-1] == after[0], after


def test_host_calls_at_the_in_place_boundary():
    """One-client calls run in place below 32 MiB of bounce buffer and through DMA at or above it;
    both sides of that boundary, and tiny ragged lengths, are exact against the oracle."""
    import numpy as np
    sys.path.insert(0, ROOT + "/oracle")
    import oracle as O
    from flamingo_amd import MaskEngine

    g = np.random.Generator(np.random.PCG64(13))
    seeds = g.integers(0, 256, (3, 32), dtype=np.uint8)
    signs = np.array([1, -1, 1], np.int8)
    seg = np.array([0, 3], np.int64)
    big = 8 << 20  # words: 32 MiB
    with MaskEngine(0) as eng:
        for L in (1, 3, 5, 1021, big - 4, big - 3, big):
            x = g.integers(0, 2**32, (1, L), dtype=np.uint32)
            assert np.array_equal(eng.client_mask(seg, seeds, signs, L, x=x),
                                  O.client_mask(seg, seeds, signs, L, x=x)), L
            acc = x[0].copy()
            eng.mask_accumulate(seeds, signs, acc)
            assert np.array_equal(acc, O.aggregate_unmask(x, seeds, signs, L=L)), L
        for n in (1, 63, (32 << 20) - 1, 32 << 20):
            data = bytes(g.integers(0, 256, n, dtype=np.uint8))
            assert eng.chacha20_encrypt(seeds[0].tobytes(), data) == O.chacha20_encrypt(seeds[0].tobytes(), data), n
        for K, L in ((2, (4 << 20) - 4), (2, 4 << 20), (1, 7)):  # K x L words: just under, at 32 MiB; tiny
            e = eng.prg_expand(seeds[:K], L)
            for k in range(K):
                assert np.array_equal(e[k], O.prg(seeds[k].tobytes(), L, 0)), (K, L, k)
