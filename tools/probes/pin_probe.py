"""Which path does the HIP runtime take for the host-pointer calls' pageable copies?  Run under
AMD_LOG_LEVEL=4 (tools/gpu.sh pinprobe): one flm_client_mask of one client (x and out: 4 MiB
pageable numpy arrays, as client_agent.sendVectors makes them) and one flm_aggregate_unmask.  The
runtime logs "HSA Copy Using Pinned resource" when it registers (pins) the caller's pageable memory
with the driver -- a KFD userptr allocation, which an MMU-notifier invalidation of those pages
(e.g. a huge-page collapse of numpy's MADV_HUGEPAGE arrays) turns into an eviction of all of this
process's GPU queues -- and "Using Staging resource" when it copies through its own pinned buffers."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from flamingo_amd import MaskEngine  # noqa: E402

L = 1 << 20
eng = MaskEngine(0)
g = np.random.Generator(np.random.PCG64(1))
seeds = g.integers(0, 256, (3, 32), dtype=np.uint8)
x = g.integers(0, 2**32, (1, L), dtype=np.uint32)
print("=== client_mask 4 MiB pageable", flush=True)
eng.client_mask(np.array([0, 3], np.int64), seeds, np.array([1, -1, 1], np.int8), L, x=x)
print("=== aggregate_unmask 4 x 4 MiB pageable rows", flush=True)
eng.aggregate_unmask([x[0].copy() for _ in range(4)], seeds, np.array([1, -1, 1], np.int8))
print("=== done", flush=True)
