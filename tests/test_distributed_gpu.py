"""The pipelined multi-GPU round's RCCL path on a one-GPU box: tools/rccl_async_smoke.py runs
ShardedRound(buffers=2) with its async reduce-scatter forced on a one-rank nccl (RCCL) group and
checks every round against the synchronous round (the driver's 8-GPU run uses the same code)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_async_pipelined_round():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_async_smoke.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ok=True" in r.stdout
