"""bench.py's launch decision (no GPU): `python bench.py --gpus G` starts G ranks itself, as
child processes of torch.distributed.run, before any GPU call; a rank started by a launcher
checks that the world it got is the one asked for, and fails otherwise."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_one_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, ["--gpus", "1"]) is None


def test_ranks_already_launched_run_in_process():
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, ["--gpus", "8"]) is None


def test_multi_gpu_spawns_torchrun_children():
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = bench.launch_plan(8, {}, argv, port=29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-len(argv) - 1] == os.path.abspath(os.path.join(ROOT, "bench.py"))
    assert cmd[-len(argv):] == argv            # the children see the same arguments


def test_bad_gpu_count_is_refused():
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {}, [])


def test_free_port_is_bindable():
    import socket
    p = bench.free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", p))


@pytest.mark.parametrize("gpus,world,backend,devices,ok", [
    (1, 1, "nccl", 1, True),
    (8, 8, "nccl", 8, True),
    (8, 1, "nccl", 8, False),     # asked for 8, got one rank: must not report n_gpus 1
    (2, 4, "nccl", 8, False),
    (4, 4, "nccl", 1, False),     # RCCL ranks need distinct GPUs
    (4, 4, "gloo", 1, True),      # gloo rehearsal: ranks share one GPU
])
def test_world_check(gpus, world, backend, devices, ok):
    assert (bench.world_check(gpus, world, backend, devices) == "") == ok


def test_world_mismatch_exits_nonzero_before_gpu():
    """A rank told --gpus 4 inside a 2-rank world refuses to run (exit 2, no JSON line)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "WORLD_SIZE=2" in r.stderr
    assert r.stdout.strip() == ""


def test_group_leg_failure_becomes_an_error_field():
    """The device-group leg runs in a child process; when it cannot run (here: no GPU) the bench
    line gets {"error": ...} instead of the bench failing or hanging."""
    import argparse
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible: the leg would run")
    args = argparse.Namespace(total_clients=64, log2_L=12, dropout=0.0, group_devices="", no_copy=True)
    res = bench.group_leg_subprocess(args, timeout=240)
    assert set(res) == {"error"} and "exited" in res["error"]


def test_pmc_csv_sums_instances_per_dispatch(tmp_path):
    """live_traffic's parser: rocprofv3 --pmc writes one CSV row per counter instance; the bytes of
    one dispatch are their sum; the round's kernel is the items_kernel with the most dispatches (the
    one-off items_kernel<16> that makes the rows is not mistaken for it); other counters are ignored."""
    d = tmp_path / "pass" / "host"
    d.mkdir(parents=True)
    hdr = "Dispatch_Id,Kernel_Name,Counter_Name,Counter_Value\n"
    rows = [(1, "void flm::items_kernel<1, true>(...)", "FETCH_SIZE", 100.0),
            (1, "void flm::items_kernel<1, true>(...)", "FETCH_SIZE", 50.5),
            (2, "void flm::items_kernel<1, true>(...)", "FETCH_SIZE", 120.0),
            (3, "void flm::items_kernel<16, true>(...)", "FETCH_SIZE", 999.0),
            (2, "void flm::items_kernel<1, true>(...)", "WRITE_SIZE", 7.0)]
    (d / "run_counter_collection.csv").write_text(
        hdr + "".join(f'{a},"{b}",{c},{v}\n' for a, b, c, v in rows))
    name, per = bench.pmc_per_dispatch(str(tmp_path / "pass"), "FETCH_SIZE")
    assert name.startswith("void flm::items_kernel<1, ") and per == {"1": 150.5, "2": 120.0}
    assert bench.pmc_per_dispatch(str(tmp_path / "pass"), "WRITE_SIZE")[1] == {"2": 7.0}
    assert bench.pmc_per_dispatch(str(tmp_path / "pass"), "FETCH_SIZE", kernel="items_kernel<16,")[1] == {"3": 999.0}
    assert bench.pmc_per_dispatch(str(tmp_path / "none"), "FETCH_SIZE") == (None, {})


def test_pmc_child_env_leaves_the_ranks_group():
    """A rank's profiling child runs as world 1: torchrun's per-rank variables are dropped."""
    env = bench.child_env({"RANK": "0", "WORLD_SIZE": "8", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                           "MASTER_PORT": "29500", "TORCHELASTIC_RUN_ID": "x", "PATH": "/usr/bin",
                           "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert env == {"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "TMPDIR": "/tmp"}


def test_scaling_check_fields():
    """A G > 1 line carries the self-check a first 8-GPU run is read with:
    the RCCL communicator's rank count, the one-GPU model's per-rank kernel time and value for
    that G, and measured / predicted."""
    b = 4.0 * 1024 * (1 << 20) + 4.0 * (1 << 20)
    r = bench.scaling_check(8, True, 1024, 1 << 20, [0.19, 0.2], 20000.0, b, 8, "rccl")
    assert r["rccl_ranks_ok"] is True and r["rccl_comm_ranks"] == 8
    assert r["predicted_rank_kernel_ms"] == 0.184 and r["measured_rank_kernel_ms_max"] == 0.2
    assert abs(r["predicted_value_gbs"] - b / 0.184e-3 / 1e9) < 0.1
    assert abs(r["predicted_vs_measured"]["rank_kernel_ms"] - 0.2 / 0.184) < 1e-3
    assert abs(r["predicted_vs_measured"]["value"] - 20000.0 / r["predicted_value_gbs"]) < 1e-3
    # gloo (no library communicator) or another shape: the fields are there, the model is not applied
    g = bench.scaling_check(2, True, 64, 1 << 16, [1.0, 1.1], 10.0, 1.0, None, "torch")
    assert g["rccl_ranks_ok"] is False and g["predicted_rank_kernel_ms"] is None
    assert g["predicted_vs_measured"] is None
    assert set(g) == set(r)
