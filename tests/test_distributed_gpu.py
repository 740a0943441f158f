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


@pytest.mark.parametrize("nproc,backend", [(1, "nccl"), (2, "gloo"), (3, "gloo")])
def test_sharded_reconstruction(nproc, backend):
    """flamingo_amd.dist_recon on 1 (library RCCL communicator) and 2/3 ranks (gloo, one GPU)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tools", "dist_recon_smoke.py"), backend]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sharded reconstruction ok=True" in r.stdout


def test_bench_spawns_its_own_ranks():
    """`python bench.py --gpus 2` (no torchrun around it) starts two ranks itself and reports
    n_gpus 2 from a correct round; gloo lets both ranks share the box's one GPU."""
    import json
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "3", "--warmup", "1", "--log2-L", "16", "--total-clients", "64", "--settle-ms", "0",
           "--no-cpu", "--no-copy", "--no-variants", "--no-configs", "--no-group"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["correct"] is True
    assert res["comm"]["world"] == 2 and res["comm"]["backend"] == "gloo"
    sc = res["scaling_check"]                     # the self-check fields of a G > 1 line (bench.scaling_check)
    assert sc["rccl_ranks_ok"] is False and sc["rccl_comm_ranks"] is None   # gloo: no library communicator
    assert len(res["roofline"]["kernel_ms_per_rank"]["ranks"]) == 2 and "predicted_vs_measured" in sc
