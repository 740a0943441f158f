#!/usr/bin/env python3
"""Benchmark: device-resident aggregate+unmask GB/s for Flamingo's server round.

Contract (see README/DESIGN.md): ``python bench.py --gpus N --steps K --warmup W``
prints ONE JSON line on rank 0.  For N > 1 it is launched by torch.distributed.run
(one process per GPU, RCCL over xGMI).

Workload (BASELINE.json configs[3], "c4"): N = 1024 clients' masked vectors of
L = 2^20 uint32 slots in all, split over the G ranks (strong scaling, the config
literally: "n=1024 clients, L=2^20, vector slots sharded across 8 GPUs"); no
dropouts, so K = 1024 self-mask seeds are regenerated (SA_ServiceAgent.py:529-536)
and the output is sum(y_i) - sum PRG(m_i) = |U| in every slot (checked after
timing).  Rank r ingests clients [N r/G, N (r+1)/G) and regenerates the K masks over
its slot shard only.  --weak runs --clients-per-gpu clients on EVERY rank instead
(N = 1024 G; per-GPU work fixed), reported as "scaling": "weak".

A step = one round on device-resident inputs: seed-schedule launch +
row-sum/unmask launch (+ RCCL reduce-scatter of the L-slot partial for G > 1).
value = algorithmic bytes (4*|U|*L read + 4*L written) / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident aggregate+unmask GB/s, N clients × L int32 per round"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TOPS = 256 * 128 * 2.4e9 / 1e12   # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 Tops/s
# ChaCha20 ceiling of the chip from the issue probe (profiles/r01_issue_probe.log): quarter rounds
# with the four QRs of a half round in lockstep issue at 3.52 cycles per VALU instruction
# (v_add_u32 / v_xor_b32 ~2.1-2.4 cycles each, the v_alignbit_b32 rotate ~4.1); at 60.4
# instructions per word and 2.38 GHz that is 733 G words/s.  The bench reports it as a reference
# only: the ceiling it divides by is measured in the same run (mask_only_ceiling), and the
# committed PMC passes (profiles/r02_clock_cpi_summary.json) give cycles per instruction and
# clock for the c4 and the mask-only launch.
PROBE_CHACHA_CEILING_GWORDS = 733.0
CPI_SUMMARY = "profiles/r02_clock_cpi_summary.json"
CHACHA_MIX_CPI = 8.0 / 3.0       # cycles per VALU instruction of the add/xor/rotate mix at 2/2/4 cycles
# torchrun's per-rank environment: removed for the PMC child of a rank, so it runs as world 1
TORCHRUN_ENV = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")
CHACHA_OPS_PER_WORD = 61.5       # VALU instructions per mask word in items_kernel (PMC: 1.031e9 wave-instructions x 64 / 2^30 words, profiles/r02_profile_summary.json)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--total-clients", type=int, default=1024,
                    help="clients in all, split over the ranks (BASELINE c4: 1024 over 1-8 GPUs, strong scaling)")
    ap.add_argument("--weak", action="store_true",
                    help="weak scaling instead: --clients-per-gpu clients on every rank (N = clients-per-gpu * G)")
    ap.add_argument("--clients-per-gpu", type=int, default=1024)
    ap.add_argument("--log2-L", type=int, default=20)
    ap.add_argument("--dropout", type=float, default=0.0, help="fraction of clients offline (c5: 0.01)")
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed rounds before the warm-up until this much GPU time has passed: MI355X ramps its "
                         "clock over ~100 ms of load (tools/probes/tail_probe.py, DESIGN.md section 6)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-copy", action="store_true", help="skip the PCIe-inclusive measurement")
    ap.add_argument("--no-variants", action="store_true", help="skip the pairs-only variant")
    ap.add_argument("--no-prg-expand", action="store_true", help="skip the standalone mask-expansion leg")
    ap.add_argument("--profile", action="store_true", help="minimal run for rocprofv3 (no CPU/copy legs)")
    ap.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs (c2, c3, c5)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL; the real multi-GPU path) or gloo (test only: ranks sharing one GPU)")
    ap.add_argument("--no-group", action="store_true", help="skip the single-process device-group leg")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the live HBM-traffic passes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE over "
                         "bench.py --profile as child processes); the committed profile's figure is reported")
    ap.add_argument("--profile-rank", type=int, default=0,
                    help="internal, with --profile --profile-world G: run rank R's kernel of a G-rank round alone "
                         "on this GPU (its clients' rows, its slot shard's masks, no collective) for the PMC passes "
                         "of a G > 1 line")
    ap.add_argument("--profile-world", type=int, default=1, help="internal: see --profile-rank")
    ap.add_argument("--group-leg", action="store_true",
                    help="internal: run only the device-group leg and print its JSON (bench.py runs it as a child "
                         "process under a time limit, so a clique that cannot come up cannot hang the bench)")
    ap.add_argument("--group-devices", default="",
                    help="devices of the device-group leg, e.g. 0,0,0,0 (loopback ranks on one GPU); "
                         "default every visible GPU")
    return ap.parse_args()


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus: int, env, argv, port: int | None = None):
    """The command that runs `gpus` ranks of this bench as child processes (torch.distributed.run,
    one process per GPU, rendezvous on 127.0.0.1), or None when this process is to be the only
    rank (gpus == 1) or already is one (WORLD_SIZE set by a launcher).  No GPU call happens before
    this decision: the parent never touches HIP, it only waits for its children."""
    if gpus < 1:
        raise SystemExit(f"--gpus must be >= 1, got {gpus}")
    if gpus == 1 or "WORLD_SIZE" in env:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port or free_port()}",
            os.path.abspath(__file__), *argv]


def world_check(gpus: int, world: int, backend: str, devices: int) -> str:
    """'' when a run asked for `gpus` ranks may go on with `world`, else why not (the bench then
    exits non-zero instead of reporting a different n_gpus)."""
    if gpus != world:
        return f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
    if backend == "nccl" and world > devices:
        return f"{world} RCCL ranks need {world} GPUs, {devices} visible (gloo shares one GPU: --dist-backend gloo)"
    return ""


def client_table(torch, P, m, nbrs, c0, c1, dev):
    """The client seed table of clients [c0, c1) (ids are global: SA_ClientAgent.py:304-324):
    seg (host), seeds (device), signs (host), for flm_client_mask_dev."""
    seg_l, seeds_l, signs_l = [0], [], []
    for i in range(c0, c1):
        seeds_l.append(m[i].tobytes()); signs_l.append(1)
        for j in sorted(nbrs[i]):
            seeds_l.append(P.synthetic_pair_seed(i, j)); signs_l.append(1 if i < j else -1)
        seg_l.append(len(seeds_l))
    cseeds = np.frombuffer(b"".join(seeds_l), np.uint8).reshape(-1, 32)
    return np.array(seg_l, np.int64), torch.from_numpy(cseeds.copy()).to(dev), np.array(signs_l, np.int8)


def shard_windows(L, G, n=1024):
    """The parity windows of a G-way sharded round: the first and the last n slots of every
    non-empty shard (flm_shard_bounds), as (rank, start, length)."""
    from flamingo_amd.distributed import shard_bounds
    wins = []
    for r in range(G):
        lo, hi = shard_bounds(L, G, r)
        if hi <= lo:
            continue
        w = min(n, hi - lo)
        for a in sorted({lo, hi - w}):
            wins.append((r, a, w))
    return wins


def oracle_windows(torch, dist, rows, out_mine, lo, G, rank, seeds, signs, L, coll_dev, n=1024):
    """In-run parity of a (possibly sharded) round against the C oracle, outside the timed region:
    for the first and last n slots of every rank's shard, every rank sums ITS rows over the window
    on the host (uint64), an all-reduce adds the ranks' partial sums (G > 1), and each rank compares
    its own shard's windows of `out_mine` (slots lo.. of the round's output) with
    oracle.aggregate_unmask(S_window, seeds, signs, slot0=a) -- the reference's
    vec_sum_partial + cancel_vec + mi_vec (SA_ServiceAgent.py:346-350, 529-605) over that window.
    Results are all-reduced (MIN): True only if every rank's windows match bit for bit."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker only
    wins = shard_windows(L, G, n)
    host_rows = [rows[:, a:a + w].cpu().numpy().view(np.uint32) if rows is not None and rows.shape[0]
                 else np.zeros((0, w), np.uint32) for _, a, w in wins]
    part = np.concatenate([h.sum(axis=0, dtype=np.uint64) for h in host_rows]).astype(np.int64)
    coll_dev = torch.device("cpu") if coll_dev is None else coll_dev
    t = torch.from_numpy(part).to(coll_dev)
    if G > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    S_all = (t.cpu().numpy() % (1 << 32)).astype(np.uint32)
    seeds_h = seeds.cpu().numpy() if hasattr(seeds, "cpu") else np.asarray(seeds, np.uint8)
    signs_h = signs.cpu().numpy() if hasattr(signs, "cpu") else np.asarray(signs, np.int8)
    ok, o, mine = True, 0, []
    for r, a, w in wins:
        if r == rank:
            want = O.aggregate_unmask(S_all[o:o + w][None], seeds_h, signs_h, L=w, slot0=a, threads=8)
            got = out_mine[a - lo:a - lo + w].cpu().numpy().view(np.uint32)
            ok &= bool(np.array_equal(got, want))
            mine.append([a, w])
        o += w
    okt = torch.tensor([1 if ok else 0], device=coll_dev)
    if G > 1:
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    return {"match": bool(okt.item()), "windows": [[a, w] for _, a, w in wins], "seeds_K": int(seeds_h.shape[0]),
            "what": "oracle/flamingo_oracle.c aggregate_unmask over the first and last slots of every rank's shard "
                    "(row sums all-reduced over the ranks), bit-exact against the GPU output, outside the timed "
                    "region"}


def group_leg_main(args):
    """`bench.py --group-leg`: the c4 inputs of main() (same seeds, graph and offline set), then
    measure_group; prints one JSON object."""
    import torch
    from flamingo_amd import params as P
    N, L = args.total_clients, 1 << args.log2_L
    cfg = f"c4-n{N}-L{L}"
    m = np.frombuffer(b"".join(P.bench_seed(cfg, i) for i in range(N)), np.uint8).reshape(N, 32)
    nbrs = P.neighbor_graph(b"\x00" * 32, 1, N, 1, encrypt=None)
    g = np.random.Generator(np.random.PCG64(12345))
    n_off = int(round(args.dropout * N))
    offline = np.sort(g.choice(N, n_off, replace=False)) if n_off else np.zeros(0, np.int64)
    online = np.setdiff1d(np.arange(N), offline)
    sseeds, ssigns = P.server_seed_table(m, nbrs, online, offline, P.synthetic_pair_seed)
    print(json.dumps(measure_group(torch, P, m, nbrs, online, sseeds, ssigns, L, args.group_devices,
                                   copy=not args.no_copy)), flush=True)
    return 0


def group_leg_subprocess(args, timeout=240):
    """The device-group leg in a child process (never an exec: this process has touched the GPU),
    killed after `timeout` s; a failure or a hang becomes {"error": ...} in the line."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--group-leg", "--total-clients", str(args.total_clients),
           "--log2-L", str(args.log2_L), "--dropout", str(args.dropout)]
    if args.group_devices:
        cmd += ["--group-devices", args.group_devices]
    if args.no_copy:
        cmd.append("--no-copy")
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"device-group leg did not finish in {timeout} s (killed)"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"device-group leg exited {r.returncode}: {r.stderr.strip()[-400:]}"}
    return json.loads(lines[-1])


def main():
    args = parse()
    if args.group_leg:
        return group_leg_main(args)
    plan = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if plan is not None:
        import subprocess
        env = dict(os.environ)
        env.setdefault("OMP_NUM_THREADS", "1")
        # rank 0's JSON line reaches stdout straight through the inherited descriptor
        return subprocess.call(plan, env=env)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    why = world_check(args.gpus, world, args.dist_backend, torch.cuda.device_count())
    if why:
        print(f"bench.py: {why}", file=sys.stderr)
        return 2
    if world > 1:
        dev_id = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_id)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_id))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    G = world
    dev = torch.device("cuda", torch.cuda.current_device())

    from flamingo_amd import MaskEngine
    from flamingo_amd import params as P
    from flamingo_amd.distributed import ShardedRound, client_bounds, init_rccl

    eng = MaskEngine(torch.cuda.current_device())
    comm = "torch"
    if G > 1 and args.dist_backend == "nccl":
        # the library's own RCCL communicator: ncclUint32 reduce-scatter on our stream.  Should it fail
        # on any rank, every rank falls back to torch.distributed's collectives (RCCL too, int32 sums)
        err = ""
        try:
            init_rccl(eng)
        except Exception as e:
            err = f"{type(e).__name__}: {e}"
        ok_t = torch.tensor([0 if err else 1], device=dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        comm = "rccl" if int(ok_t.item()) else "torch"
        if comm == "torch" and err:
            print(f"warning: library RCCL communicator unavailable ({err}); using torch.distributed", file=sys.stderr)
    L = 1 << args.log2_L
    strong = not args.weak
    # --profile --profile-world G: rank R of a G-rank round, alone on this GPU (live_traffic's child)
    Gg, Rg = (args.profile_world, args.profile_rank) if (args.profile and args.profile_world > 1 and G == 1) \
        else (G, rank)
    N = args.total_clients if strong else args.clients_per_gpu * Gg
    Ng = N // Gg if strong else args.clients_per_gpu
    cfg = f"c4-n{N}-L{L}"

    # ---- inputs: valid masked rows, built on this GPU by the client-side kernel
    m = np.frombuffer(b"".join(P.bench_seed(cfg, i) for i in range(N)), np.uint8).reshape(N, 32)
    nbrs = P.neighbor_graph(b"\x00" * 32, 1, N, 1, encrypt=eng.chacha20_encrypt)
    c0, c1 = client_bounds(N, Gg, Rg)
    seg, d_cseeds, csigns = client_table(torch, P, m, nbrs, c0, c1, dev)

    g = np.random.Generator(np.random.PCG64(12345))
    n_off = int(round(args.dropout * N))
    offline = np.sort(g.choice(N, n_off, replace=False)) if n_off else np.zeros(0, np.int64)
    online = np.setdiff1d(np.arange(N), offline)
    sseeds, ssigns = P.server_seed_table(m, nbrs, online, offline, P.synthetic_pair_seed)
    K = sseeds.shape[0]
    D = K - len(online)
    my_online = online[(online >= c0) & (online < c1)] - c0
    d_seeds = torch.from_numpy(sseeds).to(dev)
    d_signs = torch.from_numpy(ssigns).to(dev)

    # all round work (both launches and the reduce-scatter) on one dedicated stream
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    # two partial buffers: round k's reduce-scatter (RCCL, async) runs under round k+1's kernel
    rnd = ShardedRound(eng, L, buffers=2 if G > 1 else 1, comm=comm)
    if Gg != G:  # the emulated rank's slot shard (its kernel's mask window; no exchange follows)
        from flamingo_amd.distributed import shard_bounds
        rnd.lo, rnd.hi = shard_bounds(L, Gg, Rg)

    # the rows are built last, right before the warm-up: the host-side preparation above leaves
    # the GPU idle, and MI355X ramps its clock back up over ~30 ms of load
    # (profiles/r01_c4_launch_series.log), so the warm-up starts on a busy GPU
    rows = torch.empty((c1 - c0, L), dtype=torch.int32, device=dev)
    eng.client_mask_dev(seg, d_cseeds, csigns, rows, L, stream=stream)
    rows_on = rows if len(my_online) == rows.shape[0] else rows[torch.from_numpy(my_online).to(dev)].contiguous()
    torch.cuda.synchronize()

    class _Timed:
        """ShardedRound.compute bracketed by HIP events on the round's stream."""
        def __init__(self, inner):
            self.inner = inner

        def __call__(self, rows, stream=None):
            ev_k[0].record(stream)
            self.inner(rows, stream)
            ev_k[1].record(stream)

    rnd.compute = _Timed(rnd.compute)

    def step():
        return rnd.launch(rows_on, d_seeds, d_signs, stream)

    ev_k = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    def agree_max(n):
        t = torch.tensor([n], dtype=torch.int64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    settle = settle_clock(torch, step, stream, args.settle_ms, agree=agree_max if G > 1 else None)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if G > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kern_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        # per-launch kernel time read back without stalling the next launch
        kern_ms.append((ev_k[0], ev_k[1]))
        ev_k = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    torch.cuda.synchronize()
    if G > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")
    if G > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_list = [a.elapsed_time(b) for a, b in kern_ms]
    kms = float(np.mean(kern_list))
    kq = np.percentile(kern_list, [10, 50, 90])

    # ---- correctness of the timed round: out == |U| in every slot of my shard
    out = rnd.result()
    torch.cuda.synchronize()
    # (an emulated rank's partial holds only its clients' rows: no |U| to check)
    ok = bool(torch.all(out == len(online)).item()) if Gg == G else True
    okt = torch.tensor([1 if ok else 0], device=coll_dev)
    if G > 1:
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    ok = bool(okt.item())
    xch = time_exchange(torch, dist, rnd, stream, coll_dev, L) if G > 1 else None
    # every rank's dominant-kernel time: the line shows the imbalance between ranks
    k_all = [kms]
    if G > 1:
        kt = torch.tensor([kms], dtype=torch.float64, device=coll_dev)
        k_all = [torch.zeros_like(kt) for _ in range(G)]
        dist.all_gather(k_all, kt)
        k_all = [float(x.item()) for x in k_all]
    # in-run parity of the timed round: windows of every rank's shard against the C oracle
    parity = None
    if not args.profile:
        parity = oracle_windows(torch, dist, rows_on, out, rnd.lo, G, rank, d_seeds, d_signs, L, coll_dev)

    ms_per_step = elapsed / args.steps * 1e3
    bytes_round = 4.0 * len(online) * L + 4.0 * L
    value = bytes_round / (elapsed / args.steps) / 1e9
    rows_rank = rows_on.shape[0]
    mask_slots = rnd.hi - rnd.lo
    ach_gbs = (4.0 * rows_rank * L + 4.0 * L) / (kms * 1e-3) / 1e9
    words = float(K) * mask_slots
    valu_tops = words * CHACHA_OPS_PER_WORD / (kms * 1e-3) / 1e12

    res = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": G, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None, "dtype": "u32", "correct": ok,
        "checked_against_oracle": parity,
        "comm": {"world": G, "backend": args.dist_backend if G > 1 else None,
                 "collective": (("library RCCL communicator (ncclReduceScatter, ncclUint32)" if rnd.comm == "rccl"
                                 else f"torch.distributed {args.dist_backend} reduce_scatter_tensor")
                                if G > 1 else None),
                 "rccl_comm_ranks": eng.comm_size()[0] if rnd.comm == "rccl" else None,
                 "reduce_scatter": xch},
        "clock_settle": settle,
        "data": "synthetic: valid masked rows y_i = 1 + PRG(m_i) +- PRG(s_ij) made on-GPU from SHA-256 bench "
                "seeds, neighbour graph of util/param.py findNeighbors (root 0^32, iter 1, o=1)",
        "config": {"workload": "c4: aggregate + self-mask and dropout-pair unmask, one server round",
                   "clients": N, "clients_per_gpu": Ng, "online": int(len(online)), "L": L, "seeds_K": int(K),
                   "dropout_pairs_D": int(D),
                   "parallelism": f"client-shard{G}+slot-shard{G}" + (
                       f"+{'rccl-uint32' if rnd.comm == 'rccl' else args.dist_backend}-reduce-scatter-overlapped"
                       if G > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": round(ach_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "items_kernel<1>", "kernel_ms": round(kms, 4),
                     "kernel_ms_p10_p50_p90": [round(float(x), 4) for x in kq],
                     "kernel_ms_per_rank": {"min": round(min(k_all), 4), "max": round(max(k_all), 4),
                                            "ranks": [round(x, 4) for x in k_all]},
                     "bytes_per_launch": 4 * rows_rank * L + 4 * L},
        "roofline_valu": {"bound": "valu", "mask_words_per_launch": int(words), "ops_per_word": CHACHA_OPS_PER_WORD,
                          "achieved_tops": round(valu_tops, 2), "peak_tops": round(VALU_PEAK_TOPS, 1),
                          "frac": round(valu_tops / VALU_PEAK_TOPS, 4),
                          # the mix's own peak: 4 adds + 4 xors at 2 cycles and 4 rotates at 4 cycles per
                          # quarter-round step = 2.67 cycles per instruction
                          "peak_tops_chacha_mix": round(VALU_PEAK_TOPS * 2.0 / CHACHA_MIX_CPI, 1),
                          "frac_of_chacha_mix_peak": round(valu_tops / (VALU_PEAK_TOPS * 2.0 / CHACHA_MIX_CPI), 4),
                          "mask_gwords_per_s": round(words / (kms * 1e-3) / 1e9, 1),
                          "probe_chacha_ceiling_gwords": PROBE_CHACHA_CEILING_GWORDS,
                          "probe_source": "profiles/r01_issue_probe.log (QR8 lockstep: 3.52 cycles per instruction at "
                                          "2.38 GHz)"},
    }

    if not args.profile:
        ceil = mask_only_ceiling(eng, torch, d_seeds, d_signs, L, rnd.lo, rnd.hi, stream)
        res["roofline_valu"]["same_run_ceiling"] = ceil
        res["roofline_valu"]["measured_chacha_ceiling_gwords"] = ceil["mask_gwords_per_s"]
        res["roofline_valu"]["frac_of_same_run_ceiling"] = round(
            words / (kms * 1e-3) / 1e9 / ceil["mask_gwords_per_s"], 4)
    cpi = committed_cpi()
    if cpi is not None:
        res["roofline_valu"]["pmc"] = cpi
    tr = committed_traffic(rows_rank, L, int(K))
    if tr is not None:
        res["roofline"]["traffic"] = tr["bytes"]
        res["roofline"]["traffic_source"] = tr["source"]
    if not args.profile:
        pk = practical_peak(eng, torch, rows_on, L, stream)
        res["roofline"]["practical_peak"] = pk
        res["roofline"]["frac_of_practical_peak"] = round(ach_gbs / pk["GB/s"], 4)
    if G > 1:
        res["scaling_check"] = scaling_check(G, strong, N, L, k_all, value, bytes_round,
                                             eng.comm_size()[0] if rnd.comm == "rccl" else None, rnd.comm)
    if rank == 0 and G == 1 and not args.profile and not args.no_prg_expand:
        res["prg_expand"] = measure_prg_expand(eng, torch, stream, res["roofline_valu"].get("measured_chacha_ceiling_gwords"))
    if not args.profile and not args.no_variants:
        # every rank at once (each over its own rows and its own slot shard), rank 0 reports
        po = variant_pairs_only(eng, torch, rows_on, nbrs, N, L, stream, P, rnd.lo, rnd.hi)["pairs_only"]
        po["frac_of_practical_peak"] = round(po["GB/s"] / res["roofline"]["practical_peak"]["GB/s"], 4)
        if G > 1:
            vt = torch.tensor([po["kernel_ms"]], dtype=torch.float64, device=coll_dev)
            v_all = [torch.zeros_like(vt) for _ in range(G)]
            dist.all_gather(v_all, vt)
            po["kernel_ms_per_rank"] = [round(float(x.item()), 4) for x in v_all]
        res["variants"] = {"pairs_only": po}
    if G > 1 and not args.profile and not args.no_cpu:
        # the reference's CPU path beside the G-GPU number: rank 0 rebuilds every client's row, runs
        # the reference loop on the whole c4 workload and compares it with the gathered shards
        full_out = gather_full_out(torch, dist, out, rnd.S, L, G, coll_dev)
        if rank == 0:
            seg_a, d_cs_a, cs_a = client_table(torch, P, m, nbrs, 0, N, dev)
            rows_all = torch.empty((N, L), dtype=torch.int32, device=dev)
            eng.client_mask_dev(seg_a, d_cs_a, cs_a, rows_all, L, stream=stream)
            if len(online) != N:
                rows_all = rows_all[torch.from_numpy(online).to(dev)].contiguous()
            res["cpu_baseline"] = cpu_baseline(rows_all, sseeds, ssigns, L, full_out)
            res["cpu_baseline"]["gpu_side"] = f"the {G} ranks' output shards, gathered"
            del rows_all, d_cs_a
            torch.cuda.empty_cache()
        dist.barrier()
    if rank == 0 and G == 1 and not args.profile:
        if not args.no_group:
            res["group"] = group_leg_subprocess(args)
        if not args.no_configs:
            res["other_configs"] = {
                "c2": measure_config(eng, torch, P, "c2", N=128, L=16384, o=1, dropout=0.0, check_oracle=True),
                "c3": measure_config(eng, torch, P, "c3", N=1024, L=1 << 18, o=2, dropout=0.0),
                "c5": measure_config(eng, torch, P, "c5", N=4096, L=1 << 20, o=1, dropout=0.01, rounds=10,
                                     recovery=True),
            }
            c5 = res["other_configs"]["c5"]
            rec = measure_recovery(eng, torch, D=int(round(c5["dropout_pairs_D_mean"])),
                                   M=int(round(c5["online_mean"])), T=20, cpu_pool=True)
            rec["server_reconstruction_ms"] = round(rec["gpu_ms"] + c5["ms_per_round"], 4)
            c5["seed_recovery"] = rec
            # one rank's share on 8 GPUs (dist_recon: every rank recovers all m_i and ceil(D/8) pairs):
            # the EC chain that sets the 8-GPU latency from the shares, measured on this one GPU
            d8 = -(-int(round(c5["dropout_pairs_D_mean"])) // 8)
            r8 = measure_recovery(eng, torch, D=d8, M=int(round(c5["online_mean"])), T=20)
            res["pair_seed_h2c"] = measure_h2c(eng, torch)
            c5["seed_recovery_one_rank_of_8"] = {
                "what": "the seed recovery one rank of an 8-GPU c5 runs (all m_i, ceil(D/8) dropout pairs), "
                        "timed alone on this GPU: the latency floor of shares -> final_sum at G = 8",
                "D_pairs": d8, "online_M": r8["online_M"], "gpu_ms": r8["gpu_ms"], "correct": r8["correct"]}
        if not args.no_copy:
            res["with_copy"] = with_copy(eng, torch, rows_on, sseeds, ssigns, L, len(online))
        if not args.no_cpu:
            res["cpu_baseline"] = cpu_baseline(rows_on, sseeds, ssigns, L, out)
        if not args.no_pmc:
            live = live_traffic(args, rows_rank, L, int(K))
            res["roofline"]["traffic_live"] = live
            if "bytes" in live:
                res["roofline"]["traffic_committed"] = res["roofline"].get("traffic")
                res["roofline"]["traffic"] = live["bytes"]
                res["roofline"]["traffic_source"] = live["source"]
    if G > 1 and not args.profile and not args.no_pmc:
        # the same-run HBM traffic of rank 0's kernel (its PMC child runs while the other ranks wait)
        if rank == 0:
            live = live_traffic(args, rows_rank, L, int(K), rank=0, world=G)
            res["roofline"]["traffic_live"] = live
            if "bytes" in live:
                res["roofline"]["traffic"] = live["bytes"]
                res["roofline"]["traffic_source"] = live["source"]
        dist.barrier()
    if G > 1 and not args.profile and not args.no_copy:
        res["with_copy"] = with_copy_sharded(torch, dist, rnd, rows_on, d_seeds, d_signs, stream, len(online), L,
                                             coll_dev)
    if G > 1 and not args.profile and not args.no_configs:
        res["other_configs"] = {"c5": measure_c5_sharded(eng, torch, dist, P, G, rank,
                                                         backend=args.dist_backend, comm=comm)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    # library communicator first, then torch's process group (distributed.shutdown)
    from flamingo_amd.distributed import shutdown
    del rnd
    shutdown(eng)
    return 0 if ok else 1


SETTLE_CONFIG_MS = 100.0  # clock settle before each config's first iteration (settle_clock)
RECON_EC_FRAC = 24 / 256  # share of the CUs given to the EC combine in the CU-split schedule (recon_probe sweep:
                          # 24 of MI355X's 256); a multiple of the 8 XCDs so every XCD loses the same count
RECON_MIN_ITEMS = 4096   # unmask items of the CU-split schedule's first pass
RECON_QUEUE_MIN_ITEMS = 4096  # its pass 1 plan: 4 same-tile row/seed parts per tile (merged kernel, atomics):
                             # 8.17 ms vs 8.28 at 1024 items (profiles/r02_recon_minitems.log)
RECON_QUEUE_EC_FRAC = 24 / 256  # EC CUs of the pair-queue schedule, with RECON_QUEUE_EC_TERMS combine terms per lane
RECON_QUEUE_EC_TERMS = 2        # (Straus): 16 / 24 / 32 CUs -> 9.78 / 8.05 / 8.28 ms; one term per lane on 32 CUs
RANK_EC_FRAC = 72 / 256  # EC CUs of one rank's CU-partitioned sharded reconstruction at G >= 8: one G = 8 rank's
                         # shares -> final 1.39-1.40 ms on 72 or 96 CUs against 1.63 unpartitioned (64 / 80 CUs
                         # bimodal; tools/probes/rank8_overlap_probe.py, profiles/r03_rank8_overlap_*.log)
RECON_STRIDE_EC_FRAC = 32 / 256  # the same queue schedule with the EC CUs strided over the logical ids: alone, the
                                 # combine runs 3.84 ms on 24 strided CUs against 5.36 on the first 24
                                 # (profiles/r02_ec_pick.log); beside the unmask 32 strided CUs measured best
                                # 8.46 (profiles/r02_straus_recon.log, r02_recon_sweep.log)


def settle_clock(torch, step, stream, ms, agree=None):
    """Untimed rounds, back to back, for about `ms` of GPU time (before the W warm-up steps).
    An MI355X coming off host-side preparation runs its first launches at a lower clock and takes
    ~100 ms of load to settle (profiles/r02_tail_probe.log: c4 launches flat at 1.42 ms after it;
    profiles/r01_c4_launch_series.log: 2.2 -> 1.68 ms over the first ~30 ms, pre-lockstep).
    The round count comes from the first 5 rounds' time; `agree` (multi-GPU: max over ranks)
    makes every rank run the same count, since each round ends in a collective."""
    if ms <= 0:
        return {"ms": 0.0, "rounds": 0}
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(5):
        step()
    e1.record(stream)
    e1.synchronize()
    per = max(e0.elapsed_time(e1) / 5, 1e-3)
    n = max(5, int(ms / per + 0.999))
    if agree is not None:
        n = agree(n)
    for _ in range(n - 5):
        step()
    e2 = torch.cuda.Event(enable_timing=True)
    e2.record(stream)
    e2.synchronize()
    return {"ms": round(e0.elapsed_time(e2), 1), "rounds": n,
            "what": "untimed rounds before the warm-up so the clock settles (outside the timed region)"}


def measure_config(eng, torch, P, name, N, L, o, dropout, rounds=1, steps=20, check_oracle=False, recovery=False):
    """One BASELINE config on this GPU: valid masked rows built on the GPU, `rounds` iterations
    (each its own neighbour graph and, with dropouts, its own offline set: PCG64(seed=iteration)),
    `steps` timed device-resident rounds per iteration; out == |U| checked every iteration.

    recovery=True: pair seeds are SHA-256 of group elements and the server gets m_i and s_ij only
    as decryption shares (flamingo_amd.synthetic); the whole reconstruction_process -- GPU seed
    recovery + unmask -- is also timed, sequential and with the recovery overlapped on a second
    stream (flamingo_amd.reconstruct), each checked out == |U|."""
    dev = torch.device("cuda", torch.cuda.current_device())
    m = np.frombuffer(b"".join(P.bench_seed(name, i) for i in range(N)), np.uint8).reshape(N, 32)
    stream = torch.cuda.current_stream()
    rows = torch.empty((N, L), dtype=torch.int32, device=dev)
    out = torch.empty(L, dtype=torch.int32, device=dev)
    per_round, ok_all, Ks, Ds, oks, cm_ms, cm_words = [], True, [], [], [], [], []
    parity = []
    cm_steady = None
    rec_seq, rec_ovl, rec_cu, rec_q, rec_s, rec_ok = [], [], [], [], [], True
    rep_ms, fp_ovl, fp_q, fp_s = [], [], [], []
    if recovery:
        from flamingo_amd.reconstruct import ServerReconstruction
        from flamingo_amd.synthetic import recovery_round
        recon, point_cache = ServerReconstruction(eng, dev), {}
        ec_cus = max(1, int(round(RECON_EC_FRAC * eng.cu_count() / 8)) * 8) if eng.cu_count() >= 64 else \
            max(1, int(round(RECON_EC_FRAC * eng.cu_count())))
        recon_cu = ServerReconstruction(eng, dev, pass1_min_items=RECON_MIN_ITEMS, ec_cus=ec_cus,
                                        cu_pick="first")
        q_cus = max(1, int(round(RECON_QUEUE_EC_FRAC * eng.cu_count() / 8)) * 8) if eng.cu_count() >= 64 else \
            max(1, int(round(RECON_QUEUE_EC_FRAC * eng.cu_count())))
        recon_q = ServerReconstruction(eng, dev, pass1_min_items=RECON_QUEUE_MIN_ITEMS, ec_cus=q_cus,
                                       cu_pick="first", pair_queue=True, ec_terms=RECON_QUEUE_EC_TERMS)
        s_cus = max(1, int(round(RECON_STRIDE_EC_FRAC * eng.cu_count() / 8)) * 8) if eng.cu_count() >= 64 else \
            max(1, int(round(RECON_STRIDE_EC_FRAC * eng.cu_count())))
        recon_s = ServerReconstruction(eng, dev, pass1_min_items=RECON_QUEUE_MIN_ITEMS, ec_cus=s_cus,
                                       cu_pick="stride", pair_queue=True, ec_terms=RECON_QUEUE_EC_TERMS)
    for it in range(1, rounds + 1):
        nbrs = P.neighbor_graph(b"\x00" * 32, it, N, o, encrypt=eng.chacha20_encrypt)
        n_off = int(round(dropout * N))
        off = np.sort(np.random.Generator(np.random.PCG64(it)).choice(N, n_off, replace=False)) if n_off else \
            np.zeros(0, np.int64)
        on = np.setdiff1d(np.arange(N), off)
        if recovery:
            R = recovery_round(eng, m, nbrs, on, off, T=20, committee=60, seed=it, point_cache=point_cache)
            seg, cs, csg = R["seg"], R["client_seeds"], R["client_signs"]
        else:
            seg, cs, csg = P.client_seed_table(m, nbrs, P.synthetic_pair_seed)
        d_cs = torch.from_numpy(cs).to(dev)
        # server seed table first (host work): the GPU then goes straight from the client masking
        # into the round's warm-up instead of idling (clock ramp)
        if recovery:
            ss, sg = R["server_seeds"], R["server_signs"]
        else:
            ss, sg = P.server_seed_table(m, nbrs, on, off, P.synthetic_pair_seed)
        d_s, d_g = torch.from_numpy(ss).to(dev), torch.from_numpy(sg).to(dev)
        eng.client_mask_dev(seg, d_cs, csg, rows, L, stream=stream)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        eng.client_mask_dev(seg, d_cs, csg, rows, L, stream=stream)   # timed: all N clients' masked vectors
        c1.record(stream)
        torch.cuda.synchronize()
        cm_ms.append(c0.elapsed_time(c1))
        cm_words.append(int(seg[-1]) * L)
        if it == 1 and cm_ms[-1] < 1.0:
            # a call this short ran on the clock an idle GPU starts from: also time it back to back
            # after ~50 ms of the same calls (median of 20), the kernel's own rate
            t_set, n_set = time.perf_counter(), 0
            while time.perf_counter() - t_set < 0.05 or n_set < 20:
                eng.client_mask_dev(seg, d_cs, csg, rows, L, stream=stream)
                n_set += 1
                if n_set % 50 == 0:
                    torch.cuda.synchronize()
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
            evs[0].record(stream)
            for i in range(20):
                eng.client_mask_dev(seg, d_cs, csg, rows, L, stream=stream)
                evs[i + 1].record(stream)
            torch.cuda.synchronize()
            cm_steady = float(np.median([evs[i].elapsed_time(evs[i + 1]) for i in range(20)]))
        r_on = rows if len(on) == N else rows[torch.from_numpy(on).to(dev)].contiguous()
        settle_clock(torch, lambda: eng.aggregate_unmask_dev(r_on, d_s, d_g, out, L=L, stream=stream), stream,
                     SETTLE_CONFIG_MS if it == 1 else 10.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            eng.aggregate_unmask_dev(r_on, d_s, d_g, out, L=L, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        per_round.append(e0.elapsed_time(e1) / steps)
        ok = bool(torch.all(out == len(on)).item())
        if check_oracle:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O  # checker only
            want = O.aggregate_unmask(r_on.cpu().numpy().view(np.uint32), ss, sg, threads=8)
            ok = ok and bool(np.array_equal(want, out.cpu().numpy().view(np.uint32)))
        elif it == 1 or it == rounds:
            # windows of the timed round's output against the C oracle (first and last iteration)
            w = oracle_windows(torch, None, r_on, out, 0, 1, 0, ss, sg, L, None, n=min(L, 2048))
            parity.append(w["match"])
            ok = ok and w["match"]
        ok_all &= ok
        if recovery:
            rt = {k: torch.from_numpy(R[k]).to(dev) for k in ("lambdas", "mi_shares", "c1", "pair_shares",
                                                              "pair_signs")}
            for rc, overlap, acc in ((recon, False, rec_seq), (recon, True, rec_ovl), (recon_cu, True, rec_cu),
                                     (recon_q, True, rec_q), (recon_s, True, rec_s)):
                args = (r_on, L, rt["lambdas"], rt["mi_shares"], rt["c1"], rt["pair_shares"], rt["pair_signs"], out)
                out.fill_(0)
                rc.run(*args, stream=stream, overlap=overlap)
                q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                q0.record(stream)
                for _ in range(max(2, steps // 4)):
                    rc.run(*args, stream=stream, overlap=overlap)
                q1.record(stream)
                torch.cuda.synchronize()
                acc.append(q0.elapsed_time(q1) / max(2, steps // 4))
                rec_ok &= bool(torch.all(out == len(on)).item())
                if it == 1 and rc is recon_q:
                    # the reconstruction from shares, windows against the oracle given the round's
                    # own server seeds (what the recovery must have produced)
                    w = oracle_windows(torch, None, r_on, out, 0, 1, 0, ss, sg, L, None)
                    parity.append(w["match"])
                    rec_ok &= w["match"]
            # the reference's own split: S = sum of the rows at report time (:346-350), before any
            # share exists; reconstruction_process then only adds the masks to S (:529-605).  The
            # latency from the shares to final_sum is the same schedules run over the one row S.
            S_row = torch.empty((1, L), dtype=torch.int32, device=dev)
            eng.aggregate_unmask_dev(r_on, None, None, S_row[0], L=L, stream=stream)
            reps = max(2, steps // 4)
            q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            q0.record(stream)
            for _ in range(reps):
                eng.aggregate_unmask_dev(r_on, None, None, S_row[0], L=L, stream=stream)
            q1.record(stream)
            torch.cuda.synchronize()
            rep_ms.append(q0.elapsed_time(q1) / reps)
            for rc, acc in ((recon, fp_ovl), (recon_q, fp_q), (recon_s, fp_s)):
                args = (S_row, L, rt["lambdas"], rt["mi_shares"], rt["c1"], rt["pair_shares"], rt["pair_signs"], out)
                out.fill_(0)
                rc.run(*args, stream=stream, overlap=True)
                q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                q0.record(stream)
                for _ in range(reps):
                    rc.run(*args, stream=stream, overlap=True)
                q1.record(stream)
                torch.cuda.synchronize()
                acc.append(q0.elapsed_time(q1) / reps)
                rec_ok &= bool(torch.all(out == len(on)).item())
            del S_row
        Ks.append(int(ss.shape[0]))
        Ds.append(int(ss.shape[0] - len(on)))
        oks.append(int(len(on)))
        del r_on
    ms = float(np.mean(per_round))
    nu = float(np.mean(oks))
    extra = {}
    if recovery:
        extra["server_reconstruction"] = {
            "what": "reconstruction_process from decryption shares: GPU m_i recovery (Shamir, mod n) + "
                    "threshold-ElGamal combine + SHA-256 seed derivation + unmask (SA_ServiceAgent.py:499-605)",
            "sequential_ms": round(float(np.mean(rec_seq)), 4),
            "overlapped_ms": round(float(np.mean(rec_ovl)), 4),
            "cu_split_ms": round(float(np.mean(rec_cu)), 4),
            "cu_split_queue_ms": round(float(np.mean(rec_q)), 4),
            "cu_split_queue_strided_ms": round(float(np.mean(rec_s)), 4),
            "unmask_only_ms": round(ms, 4), "correct": bool(rec_ok),
            "from_report_partial": {
                "what": "the reference's split (SA_ServiceAgent.py:346-350 at report, :499-605 at "
                        "reconstruction): S = sum of the rows computed at report time, before any share "
                        "exists; the reconstruction schedules then run over the one row S (mask work + "
                        "EC combine only): the latency from shares-in to final_sum",
                "report_rows_to_S_ms": round(float(np.mean(rep_ms)), 4),
                "overlapped_ms": round(float(np.mean(fp_ovl)), 4),
                "cu_split_queue_ms": round(float(np.mean(fp_q)), 4),
                "cu_split_queue_strided_ms": round(float(np.mean(fp_s)), 4)},
            "schedule": "overlapped: EC combine on a second stream under the self-mask unmask, pair masks in a "
                        "second pass; cu_split: the same with the two streams CU-partitioned (EC on "
                        f"{recon_cu.ec_cus} CUs, Shamir + self-mask unmask on the rest, min_items {RECON_MIN_ITEMS}); "
                        f"cu_split_queue: EC on {recon_q.ec_cus} CUs ({recon_q.ec_terms} combine terms per lane), which then claim pair-mask units from a "
                        "device work queue until the self-mask pass ends; the last pass takes the rest on all CUs; "
                        f"cu_split_queue_strided: the same with {recon_s.ec_cus} EC CUs strided over the logical CU ids"}
        recon_cu.close()
        recon_q.close()
        recon_s.close()
    return {"clients": N, "L": L, "neighborhood": o, "dropout": dropout, "iterations": rounds,
            "online_mean": nu, "seeds_K_mean": float(np.mean(Ks)), "dropout_pairs_D_mean": float(np.mean(Ds)),
            "ms_per_round": round(ms, 4), "GB/s": round((4.0 * nu * L + 4.0 * L) / (ms * 1e-3) / 1e9, 1),
            "correct": ok_all,
            "checked_against_oracle": bool(check_oracle or (parity and all(parity))),
            "oracle_check": ("the whole output of every iteration against oracle/flamingo_oracle.c" if check_oracle
                             else f"{len(parity)} checks: the first and last 2048 slots of the output (first and "
                                  "last iteration" + (", and the first iteration's reconstruction from shares"
                                                      if recovery else "") + ") against oracle/flamingo_oracle.c, "
                                  "bit-exact, outside the timed region"),
            "client_masks": {"what": "all N clients' masked vectors y_i = 1 + PRG(m_i) +- PRG(s_ij) "
                                     "(SA_ClientAgent.py:246-324), one flm_client_mask_dev launch",
                             "ms": round(float(np.mean(cm_ms)), 4), "mask_words": int(np.mean(cm_words)),
                             "G_words/s": round(float(np.mean(cm_words)) / float(np.mean(cm_ms)) / 1e6, 1),
                             **({"steady": {"what": "the same call back to back after ~50 ms of them, median of 20",
                                            "ms": round(cm_steady, 4),
                                            "G_words/s": round(cm_words[0] / cm_steady / 1e6, 1)}}
                                if cm_steady else {})},
            **extra}


def time_exchange(torch, dist, rnd, stream, coll_dev, L, reps=10):
    """The round's one collective on its own: `reps` reduce-scatters of the partial (Lp words, the
    same call ShardedRound makes) bracketed by HIP events on the round's stream after a barrier,
    max over ranks.  Outside the timed loop; there the collective overlaps the next round's kernel."""
    torch.cuda.synchronize()
    dist.barrier()
    rnd.exchange(stream)                                  # warm
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        rnd.exchange(stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    t = torch.tensor([ms], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = float(t.item())
    nbytes = 4 * rnd.Lp
    return {"what": "one reduce-scatter of the Lp-word partial, HIP events on the round's stream, max over ranks "
                    "(in the timed loop it overlaps the next round's kernel)",
            "ms": round(ms, 4), "bytes_per_rank": nbytes,
            "bus_GB_per_s": round(nbytes * (rnd.world - 1) / rnd.world / (ms * 1e-3) / 1e9, 1)}


def measure_recovery(eng, torch, D, M, T, steps=10, cpu_pool=False):
    """Seed recovery of one c5 round on the GPU (SA_ServiceAgent.py:506-526, 542-585):
    M self-mask seeds m_i = sum_j lambda_j y_{j,i} mod n and D dropout-pair seeds
    SHA-256(c1_i - sum_j lambda_j sk_j c0_i), T = 20 decryptors (committee 60, fraction 1/3).
    Inputs are real threshold-ElGamal ciphertexts and decryption shares built on the GPU
    (flm_ec_mul); checked: every recovered point equals the encrypted H_i, every seed equals
    hashlib's SHA-256 of it, every m_i equals Python's big-int sum.  CPU baseline: the
    reference's own arithmetic (Python ints for the Lagrange sum, OpenSSL P-256 for the
    scalar multiplications) timed on a bounded sample and scaled to the round."""
    import hashlib
    import random
    import time
    from flamingo_amd import crypto as C
    from flamingo_amd.abides.flamingo.seeds import lagrange_at_zero, shamir_share
    rng = random.Random(2024)
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    g = np.tile(np.frombuffer(C.point_bytes(C.G), np.uint8), (D, 1))
    rs = [rng.randrange(1, C.N) for _ in range(D)]
    hs = [rng.randrange(1, C.N) for _ in range(D)]
    sk = rng.randrange(1, C.N)
    members = sorted(rng.sample(range(1, 61), T))
    sk_sh = dict(shamir_share(sk, T, 60, rng=rng))
    lam = lagrange_at_zero(members)
    c0, _ = eng.ec_mul_wire(g, C.scalars_to_wire(rs))
    H, _ = eng.ec_mul_wire(g, C.scalars_to_wire(hs))
    skc0, _ = eng.ec_mul_wire(c0, C.scalars_to_wire([sk] * D))
    c1, _, _ = eng.ec_combine_wire(H, skc0[None], C.scalars_to_wire([1]), negate=False)
    dec, _ = eng.ec_mul_wire(np.tile(c0, (T, 1)), C.scalars_to_wire([sk_sh[x] for x in members for _ in range(D)]))
    ys = [[rng.randrange(0, C.N) for _ in range(M)] for _ in range(T)]
    d_c1 = torch.from_numpy(c1).to(dev)
    d_sh = torch.from_numpy(dec.reshape(T, D, 64)).to(dev)
    d_lam = torch.from_numpy(C.scalars_to_wire(lam)).to(dev)
    d_y = torch.from_numpy(np.stack([C.scalars_to_wire(y) for y in ys])).to(dev)
    seeds = torch.empty((M + D, 32), dtype=torch.uint8, device=dev)
    pts = torch.empty((D, 64), dtype=torch.uint8, device=dev)
    flags = torch.empty(D, dtype=torch.int32, device=dev)

    def recover():
        eng.shamir_combine_dev(d_y, d_lam, seeds[:M], stream=stream)
        eng.ec_combine_dev(d_c1, d_sh, d_lam, seeds[M:], flags, points_out=pts, stream=stream)

    recover()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        recover()
    e1.record(stream)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / steps
    got_pts = pts.cpu().numpy()
    got_seeds = seeds.cpu().numpy()
    ok = bool(np.array_equal(got_pts, H)) and int(flags.abs().sum()) == 0
    ok &= all(bytes(got_seeds[M + i]) == hashlib.sha256(bytes(H[i])).digest() for i in range(D))
    want_m = [(sum(l * y[i] for l, y in zip(lam, ys)) % C.N).to_bytes(32, "big") for i in range(M)]
    ok &= all(bytes(got_seeds[i]) == want_m[i] for i in range(M))
    base = {"1_core": cpu_seed_recovery(dec, c1, lam, ys, M, D, T, procs=1)}
    procs = min(host_threads()[0], T, CPU_POOL_MAX)
    # cpu_pool: only from a script whose top level is main-guarded (bench.py, tools/recovery_bench.py):
    # spawned workers re-import the caller's main module
    if cpu_pool and procs > 1:
        base["pool"] = cpu_seed_recovery(dec, c1, lam, ys, M, D, T, procs=procs)
    for b in base.values():
        ok &= b.pop("seeds") == [bytes(x) for x in got_seeds]
    best = min(base.values(), key=lambda b: b["ms"])
    return {"D_pairs": D, "online_M": M, "decryptors_T": T, "gpu_ms": round(gpu_ms, 4),
            "scalar_mults": D * T, "correct": bool(ok),
            "cpu_baseline": {"ms": best["ms"], "cores": best["cores"], "kind": "port",
                             "sample": f"the whole round, timed: Python big-int Lagrange of all {M} m_i, OpenSSL "
                                       f"EC_POINT_mul of all {D * T} lambda_j * share products (the reference's "
                                       f"parallel_mult; pool = its multiprocessing.Pool over the {T} terms, "
                                       f"{procs} spawned workers), "
                                       f"SA_ServiceAgent.py:552-572), EC_POINT_add sums, c1 - sum, SHA-256; its "
                                       f"seeds equal the GPU's",
                             "variants": base}}


def measure_h2c(eng, torch, reps=5, cpu_sample=4096):
    """The client's hash to curve (SA_ClientAgent.py:283-286 -> ecchash.hash_str_to_curve) for every
    h_ijt it can produce (str(v), v < 2^16, :280): one flm_hash_to_curve_decimal_dev launch, timed
    with HIP events on its stream.  Checked: the table's SHA-256 against the reference's own table
    (tests/golden/h2c_golden.json, made by make_h2c_golden.py) and the first `cpu_sample` rows
    against the CPU baseline's outputs.  CPU baseline: the restated reference algorithm
    (oracle/ec_oracle.py: hashlib SHA-256, Python big-int field) timed on those rows."""
    import hashlib
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream()
    n = 1 << 16
    out = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    fl = torch.empty(n, dtype=torch.int32, device=dev)
    eng.hash_to_curve_decimal_dev(0, n, out, fl, stream=stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        eng.hash_to_curve_decimal_dev(0, n, out, fl, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    table = out.cpu().numpy()
    res = {"points": n, "gpu_ms": round(ms, 4), "gpu_points_per_s": round(n / (ms * 1e-3)),
           "flags_clear": not bool(fl.cpu().numpy().any()),
           "table_sha256": hashlib.sha256(table.tobytes()).hexdigest()}
    try:
        with open(os.path.join(ROOT, "tests", "golden", "h2c_golden.json")) as f:
            gold = json.load(f)
        res["matches_reference_table"] = gold["table_sha256"] == res["table_sha256"]
        res["parity"] = gold.get("parity")
    except OSError:
        res["matches_reference_table"] = None
    # cpu_baseline leg: the oracle restatement (checker only, outside the GPU timing)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ec_oracle as E
    t = time.perf_counter()
    rows = [E.wire(E.hash_str_to_curve(str(v))) for v in range(cpu_sample)]
    cpu_s = time.perf_counter() - t
    res["matches_cpu_sample"] = all(table[v].tobytes() == rows[v] for v in range(cpu_sample))
    res["cpu_baseline"] = {"points_per_s": round(cpu_sample / cpu_s, 1), "cores": 1, "kind": "port",
                           "sample": f"oracle/ec_oracle.hash_str_to_curve (the reference's algorithm: SHA-256 "
                                     f"XMD, big-int map_to_curve, Q0 + Q1) on v = 0..{cpu_sample - 1}, timed",
                           "table_s_at_this_rate": round(n * cpu_s / cpu_sample, 1)}
    return res


_TLS = None


CPU_POOL_MAX = 8   # spawned CPU-baseline workers (each may open the GPU under rocprofv3; the box allows 16)


def _cpu_mul_column(args):
    """One decryptor's column lambda_j * share_{j,i} (parallel_mult, SA_ServiceAgent.py:27-34), OpenSSL,
    on a curve context of this worker's own."""
    import threading
    global _TLS
    col, lam = args
    from flamingo_amd import crypto as C
    if _TLS is None:
        _TLS = threading.local()
    cv = getattr(_TLS, "curve", None)
    if cv is None:
        cv = _TLS.curve = C._Curve()
    pts = C.points_from_wire(np.frombuffer(col, np.uint8).reshape(-1, 64))
    return [cv.mul(lam, p) for p in pts]


def cpu_seed_recovery(dec, c1, lam, ys, M, D, T, procs=1):
    """The reference's reconstruction seed recovery on the host, the whole round (not a sample):
    m_i = sum_j lambda_j y_{j,i} mod n (:518-526); for every dropout pair the T products
    lambda_j share_{j,i} (:552-567; procs > 1: one task per term j on a pool of `procs` spawned
    worker processes, as the reference's multiprocessing.Pool), their sum, c1 - sum, SHA-256
    (:572-585).  At most CPU_POOL_MAX workers: under rocprofv3 every spawned worker inherits the
    profiler's preload and opens the GPU, and the box allows 16 processes on it (16 workers + this
    one tripped that guard once); threads were tried instead and lose to the GIL (1,061 ms on 16
    against 777 on one core)."""
    import hashlib
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor
    from flamingo_amd import crypto as C
    cols = [(dec[j * D:(j + 1) * D].tobytes(), lam[j]) for j in range(T)]
    pool = ProcessPoolExecutor(procs, mp_context=mp.get_context("spawn")) if procs > 1 else None
    try:
        if pool:
            list(pool.map(_cpu_mul_column, [(dec[:64].tobytes(), 1)] * procs))        # workers up
        t0 = time.perf_counter()
        seeds = [(sum(l * y[i] for l, y in zip(lam, ys)) % C.N).to_bytes(32, "big") for i in range(M)]
        t1 = time.perf_counter()
        prods = list(pool.map(_cpu_mul_column, cols)) if pool else [_cpu_mul_column(c) for c in cols]
        t2 = time.perf_counter()
        c1p = C.points_from_wire(c1)
        for i in range(D):
            acc = None
            for j in range(T):
                acc = C.add(acc, prods[j][i])
            pt = C.add(c1p[i], C.neg(acc))
            seeds.append(hashlib.sha256(C.point_bytes(pt)).digest())
        t3 = time.perf_counter()
    finally:
        if pool:
            pool.shutdown()
    return {"ms": round((t3 - t0) * 1e3, 1), "cores": procs, "lagrange_ms": round((t1 - t0) * 1e3, 1),
            "scalar_mults_ms": round((t2 - t1) * 1e3, 1), "sums_sha_ms": round((t3 - t2) * 1e3, 1), "seeds": seeds}


def mask_only_ceiling(eng, torch, d_seeds, d_signs, L, lo, hi, stream, reps=10):
    """The ChaCha ceiling measured in the same run: the timed round's own K seeds over its own
    slot window, no rows (a mask-only items_kernel launch), right after the timed loop so the
    clock is the one the round ran at.  Median of `reps` launches."""
    K = d_seeds.shape[0]
    out = torch.empty(L, dtype=torch.int32, device=d_seeds.device)
    eng.seed_table_dev(d_seeds, d_signs, stream=stream)
    for _ in range(3):
        eng.aggregate_dev(None, K, out, L=L, mask_lo=lo, mask_hi=hi, stream=stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        eng.aggregate_dev(None, K, out, L=L, mask_lo=lo, mask_hi=hi, stream=stream)
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    ms = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))
    words = float(K) * (hi - lo)
    return {"what": "mask-only launch of the same K seeds over the same slot window (no rows), same run",
            "kernel_ms": round(ms, 4), "mask_gwords_per_s": round(words / (ms * 1e-3) / 1e9, 1)}


PRG_EXPAND_K = 962  # the c5 round's dropout pairs D (bench other_configs.c5.dropout_pairs_D_mean, round 5)


def measure_prg_expand(eng, torch, stream, ceil_gwords=None, K=PRG_EXPAND_K, L=1 << 20, reps=5):
    """north_star (i) on its own: expand K recovered pair seeds into K masks of L slots in device
    memory, one seed per row (flm_prg_expand_dev; the cancel_vec idiom of SA_ServiceAgent.py:596-603
    for the whole batch of dropout pairs), outside the headline's timed loop.  Median of `reps`
    launches on the bench stream.  Reports the bytes written against HBM peak and the mask words
    per second against the same run's ChaCha ceiling (mask_only_ceiling: the summing kernel's
    words/s with no rows), and checks the first and last 4096 slots of three rows against
    oracle.prg (checker only)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker only
    dev = torch.device("cuda", torch.cuda.current_device())
    seeds = np.random.Generator(np.random.PCG64(962)).integers(0, 256, (K, 32), dtype=np.uint8)
    d_seeds = torch.from_numpy(seeds).to(dev)
    out = torch.empty((K, L), dtype=torch.int32, device=dev)
    for _ in range(2):
        eng.prg_expand_dev(d_seeds, out, L, stream=stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(stream)
    for i in range(reps):
        eng.prg_expand_dev(d_seeds, out, L, stream=stream)
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    times = [ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]
    ms = float(np.median(times))
    plan = eng.last_plan()
    n = 4096
    ok = True
    for k in (0, K // 2, K - 1):
        for a in (0, L - n):
            got = out[k, a:a + n].cpu().numpy().view(np.uint32)
            ok &= bool(np.array_equal(got, O.prg(seeds[k].tobytes(), n, a)))
    words = float(K) * L
    gbs = 4.0 * words / (ms * 1e-3) / 1e9
    gw = words / (ms * 1e-3) / 1e9
    res = {"what": f"flm_prg_expand_dev: {K} pair seeds (c5's D) x L = {L} slots into device memory, one mask "
                   f"row per seed, median of {reps} launches (SA_ServiceAgent.py:596-603)",
           "K": K, "L": L, "kernel": "prg_expand_kernel (one-wave workgroups, runs of (seed, 1024-slot) units, "
                                     "LDS-staged 1 KiB-contiguous stores)",
           "workgroups": plan["items"], "note": "kernel_ms = seed schedule + expansion launch (HIP events around the call)", "kernel_ms": round(ms, 4), "kernel_ms_all": [round(t, 4) for t in times],
           "bytes_written_per_launch": int(4 * words), "GB/s_written": round(gbs, 1),
           "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 4), "mask_gwords_per_s": round(gw, 1),
           "checked_against_oracle": {"match": ok, "rows": [0, K // 2, K - 1], "windows": [[0, n], [L - n, n]]}}
    if ceil_gwords:
        res["chacha_ceiling_gwords"] = ceil_gwords
        res["frac_of_same_run_chacha_ceiling"] = round(gw / ceil_gwords, 4)
    del out
    torch.cuda.empty_cache()
    return res


# strong-scaled c4 (N = 1024, L = 2^20): one rank's shard kernel timed alone on one GPU with that rank's
# exact shapes (G = 1 is the round-5 driver bench), the prediction a SCALE line is read against
SCALING_MODEL_RANK_MS = {1: 1.31, 2: 0.69, 4: 0.35, 8: 0.184}


def scaling_check(G, strong, N, L, kernel_ms_per_rank, value_gbs, bytes_round, rccl_ranks, comm):
    """What a multi-GPU line must show for its scaling to be read: the exchange
    through the library's RCCL communicator with G ranks, and each rank's kernel against the
    one-GPU model.  Pure host arithmetic (tested on the CPU, tests/test_bench_cpu.py)."""
    pred = SCALING_MODEL_RANK_MS.get(G) if strong and N == 1024 and L == 1 << 20 else None
    kmax = max(kernel_ms_per_rank)
    res = {"model_source": "DESIGN.md section 7 (one rank's shard kernel timed alone on one GPU)",
           "rccl_comm_ranks": rccl_ranks, "rccl_ranks_ok": bool(comm == "rccl" and rccl_ranks == G),
           "predicted_rank_kernel_ms": pred, "measured_rank_kernel_ms_max": round(kmax, 4),
           "predicted_value_gbs": None, "predicted_vs_measured": None}
    if pred is not None:
        pv = bytes_round / (pred * 1e-3) / 1e9
        res["predicted_value_gbs"] = round(pv, 1)
        res["predicted_vs_measured"] = {"rank_kernel_ms": round(kmax / pred, 4), "value": round(value_gbs / pv, 4)}
    return res


# the fastest rows-only stream configuration measured (merged accumulator, 4 rows in
# flight, 4096-slot tiles, 512 items; profiles/r01_ab_rows_minitems.log)
STREAM_TUNING = (("variant", 4, -1), ("subtiles", 4, 0), ("min_items", 512, 1024))


def practical_peak(eng, torch, rows, L, stream, reps=10):
    """The chip's practical HBM read rate measured in the same run: rows-only launches of the
    same items_kernel (K = 0: every row summed, no seeds) over the same rows buffer, median of
    `reps` launches each, in the default plan and in the fastest stream configuration measured
    (STREAM_TUNING); the faster of the two is the SURVEY 8(d) "read-only stream kernel on the box"
    denominator."""
    out = torch.empty(L, dtype=torch.int32, device=rows.device)
    nbytes = 4.0 * rows.shape[0] * L + 4.0 * L

    def timed():
        for _ in range(3):
            eng.aggregate_unmask_dev(rows, None, None, out, L=L, stream=stream)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record(stream)
        for i in range(reps):
            eng.aggregate_unmask_dev(rows, None, None, out, L=L, stream=stream)
            ev[i + 1].record(stream)
        torch.cuda.synchronize()
        return float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))

    ms_default = timed()
    try:
        for key, val, _ in STREAM_TUNING:
            eng.set_tuning(key, val)
        ms_tuned = timed()
    finally:
        for key, _, dflt in STREAM_TUNING:
            eng.set_tuning(key, dflt)
    ms = min(ms_default, ms_tuned)
    return {"what": f"rows-only launches of items_kernel (K = 0) over the same rows, same run, median of {reps}: "
                    "the faster of the default plan and the fastest stream configuration measured "
                    "(merged accumulator, 4 rows in flight, 4096-slot tiles, 512 items)",
            "kernel_ms": round(ms, 4), "GB/s": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "frac_of_spec": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "default_plan_ms": round(ms_default, 4), "stream_config_ms": round(ms_tuned, 4)}


def measure_group(torch, P, m, nbrs, online, sseeds, ssigns, L, spec="", copy=True, steps=20):
    """The drop-in server's multi-GPU form (Kernel.py:190-271 is ONE process): flm_group over
    `spec`'s devices (default every visible GPU), the c4 round through
    flm_group_aggregate_unmask_dev (rows resident on each device: client-sharded rows,
    slot-sharded masks, one RCCL reduce-scatter over the clique -- no RCCL for one device) and,
    with copy, flm_group_aggregate_unmask (pinned host rows, one upload thread per device, shards
    back to the host).  Host-timed per round including the group's launch and sync; checked
    out == |U| in every slot."""
    from flamingo_amd import DeviceGroup, PinnedArena, _lib
    from flamingo_amd.engine import client_bounds, shard_bounds
    devs = [int(d) for d in spec.split(",")] if spec else list(range(max(1, _lib.load().flm_device_count())))
    grp = DeviceGroup(devs)
    G, n_on = grp.n, len(online)
    try:
        rows, seeds, signs, shards = [], [], [], []
        S = shard_bounds(L, G, 0)[2]
        for r, d in enumerate(devs):
            dev = torch.device("cuda", d)
            c0, c1 = client_bounds(n_on, G, r)
            ids = online[c0:c1]
            seg_l, cs, cg = [0], [], []
            for i in ids:
                cs.append(m[i].tobytes()); cg.append(1)
                for j in sorted(nbrs[i]):
                    cs.append(P.synthetic_pair_seed(int(i), j)); cg.append(1 if i < j else -1)
                seg_l.append(len(cs))
            rr = torch.empty((len(ids), L), dtype=torch.int32, device=dev)
            if len(ids):
                d_cs = torch.from_numpy(np.frombuffer(b"".join(cs), np.uint8).reshape(-1, 32).copy()).to(dev)
                grp.engines[r].client_mask_dev(np.array(seg_l, np.int64), d_cs, np.array(cg, np.int8), rr, L,
                                               stream=torch.cuda.current_stream(dev))
            rows.append(rr)
            seeds.append(torch.from_numpy(sseeds).to(dev))
            signs.append(torch.from_numpy(ssigns).to(dev))
            shards.append(torch.empty(S, dtype=torch.int32, device=dev))
        for d in set(devs):
            torch.cuda.synchronize(torch.device("cuda", d))

        def run():
            grp.aggregate_unmask_dev(rows, seeds, signs, shards, L, after_current=False)
        t_set = time.perf_counter()
        n_settle = 0
        while time.perf_counter() - t_set < 0.2 or n_settle < 3:   # clock settle, then warm-up
            run()
            grp.sync()
            n_settle += 1
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        grp.sync()
        dt = (time.perf_counter() - t0) / steps
        ok = True
        for r in range(G):
            lo, hi, _ = shard_bounds(L, G, r)
            ok &= bool(torch.all(shards[r][: hi - lo] == n_on).item())
        nbytes = 4.0 * n_on * L + 4.0 * L
        res = {"devices": devs, "ranks": G, "loopback": grp.loopback,
               "exchange": ("none (one device)" if G == 1 else
                            "shard_sum kernel (loopback ranks on one GPU)" if grp.loopback else
                            "ncclReduceScatter over the ncclCommInitAll clique"),
               "dev": {"what": "flm_group_aggregate_unmask_dev: rows resident, rounds on the ranks' streams, "
                               "host-timed with flm_group_sync after the last of the rounds",
                       "ms_per_round": round(dt * 1e3, 4), "GB/s": round(nbytes / dt / 1e9, 1), "correct": ok,
                       "rounds": steps}}
        if copy:
            arena = PinnedArena(int(n_on) * L * 4 + 4096)
            host = arena.array((n_on, L), np.uint32)
            o = 0
            for rr in rows:
                host.view(np.int32)[o:o + rr.shape[0]] = rr.cpu().numpy()
                o += rr.shape[0]
            vecs = [host[i] for i in range(n_on)]
            best, okc = None, True
            for _ in range(3):
                t0 = time.perf_counter()
                out = grp.aggregate_unmask(vecs, sseeds, ssigns, L=L)
                t = time.perf_counter() - t0
                best = t if best is None else min(best, t)
                okc &= bool(np.all(out == n_on))
            arena.free()
            res["host"] = {"what": "flm_group_aggregate_unmask: pinned host rows, each device uploads its "
                                   "clients over its own link, shards back to host; best of 3",
                           "ms_per_round": round(best * 1e3, 2), "GB/s": round(nbytes / best / 1e9, 2),
                           "correct": okc}
        return res
    finally:
        grp.close()


def measure_c5_sharded(eng, torch, dist, P, G, rank, backend="nccl", rounds=10, steps=5, comm=None):
    """BASELINE c5 on G GPUs (n=4096, L=2^20, 1 % dropouts, 10 iterations): every rank runs
    flamingo_amd.dist_recon.ShardedReconstruction on its share -- its online clients' rows, all
    m_i (Shamir), its chunk of the dropout pairs (EC combine on a side stream), one all-gather of
    the pair keys, the pair masks over its slot shard, one reduce-scatter.  Wall time per round,
    barrier-bracketed, max over ranks; every rank checks its shard == |U|."""
    from flamingo_amd.dist_recon import ShardedReconstruction, pair_chunk
    from flamingo_amd.distributed import client_bounds
    from flamingo_amd.synthetic import recovery_round
    dev = torch.device("cuda", torch.cuda.current_device())
    N, L, T = 4096, 1 << 20, 20
    m = np.frombuffer(b"".join(P.bench_seed("c5", i) for i in range(N)), np.uint8).reshape(N, 32)
    stream = torch.cuda.current_stream()
    rec = ShardedReconstruction(eng, L, comm=comm or ("rccl" if backend == "nccl" else "torch"))
    # at G = 8 one rank's self-mask pass is shorter than its combine's chain: also time the schedule
    # with the combine on its own CUs (dist_recon ec_cus; RANK_EC_FRAC of the CUs).  At G = 2 / 4 the
    # pass on the remaining CUs is the longer leg and it loses (profiles/r03_rank_overlap_G{2,4}.log)
    rec_cu = None
    if G >= 8 and eng.cu_count() >= 64:
        rec_cu = ShardedReconstruction(eng, L, comm=rec.comm, ec_cus=int(round(RANK_EC_FRAC * eng.cu_count() / 8)) * 8)
    out = torch.empty(rec.S, dtype=torch.int32, device=dev)
    per_round, oks, Ds, parity = [], True, [], []
    rep_ms, fp_ms, fp_cu_ms = [], [], []
    S_shard = torch.empty(rec.S, dtype=torch.int32, device=dev)
    cache = {}
    coll = dev if backend == "nccl" else torch.device("cpu")

    def timed(fn):
        """fn() `steps` times between barriers; max-over-ranks ms per call."""
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()) / steps * 1e3
    for it in range(1, rounds + 1):
        nbrs = P.neighbor_graph(b"\x00" * 32, it, N, 1, encrypt=eng.chacha20_encrypt)
        off = np.sort(np.random.Generator(np.random.PCG64(it)).choice(N, int(round(0.01 * N)), replace=False))
        on = np.setdiff1d(np.arange(N), off)
        R = recovery_round(eng, m, nbrs, on, off, T=T, committee=60, seed=it, point_cache=cache)
        c0, c1 = client_bounds(len(on), G, rank)
        ids = on[c0:c1]
        seg = R["seg"]
        st, en = seg[ids], seg[ids + 1]
        sub_seeds = np.concatenate([R["client_seeds"][a:b] for a, b in zip(st, en)])
        sub_signs = np.concatenate([R["client_signs"][a:b] for a, b in zip(st, en)])
        sub_seg = np.concatenate([[0], np.cumsum(en - st)]).astype(np.int64)
        rows = torch.empty((len(ids), L), dtype=torch.int32, device=dev)
        eng.client_mask_dev(sub_seg, torch.from_numpy(sub_seeds).to(dev), sub_signs, rows, L, stream=stream)
        D = R["D"]
        a, b, _ = pair_chunk(D, G, rank)
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
        args = (rows, t(R["lambdas"]), t(R["mi_shares"]), t(R["c1"][a:b]), t(R["pair_shares"][:, a:b]),
                t(R["pair_signs"]), D, out)
        for _ in range(2):
            rec.run(*args, stream=stream)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            rec.run(*args, stream=stream)
        torch.cuda.synchronize()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=coll)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        per_round.append(float(el.item()) / steps * 1e3)
        oks &= bool(torch.all(out[: rec.hi - rec.lo] == len(on)).item())
        if it == 1:
            # windows of every rank's shard against the oracle (row sums all-reduced over the ranks)
            w = oracle_windows(torch, dist, rows, out, rec.lo, G, rank, R["server_seeds"], R["server_signs"], L,
                               coll)
            parity.append(w["match"])
        # the reference's split: S shards at report time, then shares -> final over them
        rep_ms.append(timed(lambda: rec.report(rows, S_shard, stream=stream)))
        out.fill_(0)
        fp_ms.append(timed(lambda: rec.run_from_partial(S_shard, *args[1:], stream=stream)))
        oks &= bool(torch.all(out[: rec.hi - rec.lo] == len(on)).item())
        if it == rounds:
            w = oracle_windows(torch, dist, rows, out, rec.lo, G, rank, R["server_seeds"], R["server_signs"], L,
                               coll)
            parity.append(w["match"])
        if rec_cu is not None:
            out.fill_(0)
            fp_cu_ms.append(timed(lambda: rec_cu.run_from_partial(S_shard, *args[1:], stream=stream)))
            oks &= bool(torch.all(out[: rec.hi - rec.lo] == len(on)).item())
        Ds.append(D)
        del rows
    okt = torch.tensor([1 if oks else 0], device=coll)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    ms = float(np.mean(per_round))
    return {"clients": N, "L": L, "dropout": 0.01, "iterations": rounds, "decryptors_T": T,
            "dropout_pairs_D_mean": float(np.mean(Ds)),
            "server_reconstruction_ms": round(ms, 4),
            "GB/s": round((4.0 * (N - round(0.01 * N)) * L + 4.0 * L) / (ms * 1e-3) / 1e9, 1),
            "from_report_partial": {"report_rows_to_S_shards_ms": round(float(np.mean(rep_ms)), 4),
                                    "shares_to_final_ms": round(float(np.mean(fp_ms)), 4),
                                    "what": "ShardedReconstruction.report (rows -> reduce-scattered S shards, at "
                                            "report time) and run_from_partial (shares -> final over each rank's "
                                            "S shard: the all-gather of pair keys is the one exchange)",
                                    **({"shares_to_final_ec_cus_ms": round(float(np.mean(fp_cu_ms)), 4),
                                        "ec_cus": rec_cu.ec_cus,
                                        "what_ec_cus": "the same with the combine on its own first ec_cus CUs and "
                                                       "Shamir + self masks on the rest (dist_recon ec_cus)"}
                                       if rec_cu is not None else {})},
            "correct": bool(okt.item()) and all(parity),
            "checked_against_oracle": bool(parity) and all(parity),
            "oracle_check": "the first and last 1024 slots of every rank's shard (run of iteration 1, "
                            f"run_from_partial of iteration {rounds}) against oracle/flamingo_oracle.c given the "
                            "round's server seeds, row sums all-reduced over the ranks; bit-exact",
            "schedule": "per rank: Shamir of all m_i; EC combine of its ceil(D/G) pair chunk on a side stream under "
                        "rows + self masks over its slot shard; all-gather of the pair keys; pair masks over its "
                        "shard; reduce-scatter ("
                        + ("library RCCL communicator, ncclUint32" if rec.comm == "rccl" else f"torch.distributed {backend}")
                        + ")"}


def pmc_per_dispatch(d, ctr, kernel=None):
    """rocprofv3 --pmc CSV output under directory d: counter `ctr` per dispatch, summed over the CSV's
    per-instance rows (one row per XCD / block instance), for one kernel: the one whose name contains
    `kernel`, or (None) the `items_kernel` instance with the most dispatches -- the timed round's
    kernel, whatever its template arguments (a G > 1 rank's shard kernel may differ from c4's); the
    bench's one-off launches, such as the `items_kernel<16, ...>` that makes the rows, are single
    dispatches.  (A name prefix is not enough: `items_kernel<1` also matches `items_kernel<16`.)
    Returns (kernel name, {dispatch id: value}); (None, {}) when nothing matches."""
    import csv
    import glob
    by_kernel = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if row["Counter_Name"] != ctr or (kernel not in name if kernel else "items_kernel<" not in name):
                    continue
                per = by_kernel.setdefault(name, {})
                per[row["Dispatch_Id"]] = per.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    if not by_kernel:
        return None, {}
    name = max(by_kernel, key=lambda k: len(by_kernel[k]))
    return name, by_kernel[name]


def child_env(environ):
    """The environment of a profiling child: this process's without torchrun's per-rank variables
    (the child must run as world 1, not join the ranks' group), TMPDIR=/tmp for rocprofv3."""
    env = {k: v for k, v in environ.items() if k not in TORCHRUN_ENV and not k.startswith("TORCHELASTIC_")}
    env["TMPDIR"] = "/tmp"
    return env


def live_traffic(args, rows, L, K, timeout=180, rank=0, world=1):
    """HBM bytes per launch of the dominant kernel, measured in this run on this box: two rocprofv3
    PMC passes over `bench.py --profile` (the same workload), run as child processes of this one
    (never an exec), one counter group each -- FETCH_SIZE takes 3 of the 4 TCC counters and
    WRITE_SIZE 2 (MI355X_MICROARCH.md) -- with gfx950's correction: FETCH_SIZE reports half the bytes
    of a wide coalesced stream, so read bytes = 2 x FETCH_SIZE KiB; WRITE_SIZE is exact for 16-B
    stores.  Averaged over the child's dispatches of the round's kernel (pmc_per_dispatch).
    world > 1: the child runs rank `rank`'s kernel of a `world`-rank round alone on this GPU
    (--profile-rank / --profile-world: its clients' rows over all L slots, its shard's masks, no
    collective), with torchrun's environment removed so it does not join the running ranks' group.
    A pass that fails or exceeds `timeout` s (killed) gives {"error": ...}."""
    import shutil
    import subprocess
    import tempfile
    rp = shutil.which("rocprofv3")
    if not rp:
        return {"error": "rocprofv3 not found"}
    child = [sys.executable, os.path.abspath(__file__), "--profile", "--steps", "10", "--warmup", "2",
             "--settle-ms", "50", "--total-clients", str(args.total_clients), "--log2-L", str(args.log2_L),
             "--dropout", str(args.dropout)]
    if args.weak:
        child += ["--weak", "--clients-per-gpu", str(args.clients_per_gpu)]
    if world > 1:
        child += ["--profile-rank", str(rank), "--profile-world", str(world)]
    env = child_env(os.environ)
    kib = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, ctr)
            try:
                r = subprocess.run([rp, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--", *child],
                                   capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
            except subprocess.TimeoutExpired:
                return {"error": f"rocprofv3 --pmc {ctr} did not finish in {timeout} s (killed)"}
            if r.returncode != 0:
                return {"error": f"rocprofv3 --pmc {ctr} exited {r.returncode}: {r.stderr.strip()[-300:]}"}
            name, per = pmc_per_dispatch(d, ctr)
            if not per:
                return {"error": f"no items_kernel dispatch in the {ctr} pass"}
            kib[ctr] = (sum(per.values()) / len(per), len(per), name)
    read = 2.0 * kib["FETCH_SIZE"][0] * 1024
    write = kib["WRITE_SIZE"][0] * 1024
    alg = 4.0 * rows * L + 4.0 * L
    return {"bytes": int(read + write), "read_bytes_corrected": int(read), "write_bytes": int(write),
            "algorithmic_bytes": int(alg), "traffic_over_algorithmic": round((read + write) / alg, 4),
            "dispatches": {"FETCH_SIZE": kib["FETCH_SIZE"][1], "WRITE_SIZE": kib["WRITE_SIZE"][1]},
            "kernel": kib["FETCH_SIZE"][2],
            "source": "this run: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, over bench.py --profile (same workload, "
                      "this box), FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, per launch of the round's kernel"
                      + (f"; rank {rank} of {world} alone on its GPU" if world > 1 else "")}


def committed_cpi():
    """Shader clock and cycles per VALU instruction per SIMD of the c4 launch and of the mask-only
    launch (same seeds, no rows) from the committed rocprofv3 PMC passes (tools/gpu_clock.sh)."""
    try:
        d = json.load(open(os.path.join(ROOT, CPI_SUMMARY)))
    except (OSError, ValueError):
        return None
    out = {"source": CPI_SUMMARY}
    for m in ("full", "mask"):
        if m in d and "cycles_per_valu_inst_per_simd" in d[m]:
            out[m] = {"kernel_ms": round(d[m]["duration_ns"] / 1e6, 4), "clock_ghz": round(d[m]["clock_ghz"], 3),
                      "cycles_per_valu_inst": round(d[m]["cycles_per_valu_inst_per_simd"], 3)}
    return out


def committed_traffic(rows, L, K):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes
    (profiles/*_profile_summary.json: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), when the
    profiled command was this same workload; None otherwise."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_profile_summary.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        wl = d.get("workload", {"rows": 1024, "L": 1 << 20, "K": 1024})
        if (wl.get("rows"), wl.get("L"), wl.get("K")) != (rows, L, K):
            continue
        for k, v in d.get("counters", {}).items():
            if k.startswith("flm::items_kernel<1,") and "hbm_traffic_bytes" in v:
                best = {"bytes": int(v["hbm_traffic_bytes"]), "source": os.path.relpath(f, ROOT)}
    return best


def gather_full_out(torch, dist, out_mine, S, L, G, coll_dev):
    """Every rank's output shard (out_mine: slots [lo, hi) of this rank) assembled into the whole
    uint32[L] vector on every rank (one all-gather of S words per rank; outside the timed region)."""
    buf = torch.zeros(S, dtype=torch.int32, device=coll_dev)
    buf[: out_mine.shape[0]] = out_mine.to(coll_dev)
    parts = [torch.empty_like(buf) for _ in range(G)]
    dist.all_gather(parts, buf)
    return torch.cat(parts)[:L].cpu().numpy().view(np.uint32)


def variant_pairs_only(eng, torch, rows, nbrs, N, L, stream, P, lo=0, hi=None):
    """Aggregate + dropout-pair unmask only (K = D), the HBM-bound half of the round: this rank's
    rows over all L slots plus the pair masks of a 1 % offline set of the N clients over its slot
    shard [lo, hi) (the whole vector on one GPU)."""
    hi = L if hi is None else hi
    g = np.random.Generator(np.random.PCG64(99))
    off = np.sort(g.choice(N, max(1, N // 100), replace=False))
    on = np.setdiff1d(np.arange(N), off)
    pairs, pairs_signs = P.dropout_pairs(nbrs, on, off)
    seeds = np.frombuffer(b"".join(P.synthetic_pair_seed(i, j) for i, j in pairs), np.uint8).reshape(-1, 32)
    d_seeds = torch.from_numpy(seeds.copy()).cuda()
    d_signs = torch.from_numpy(np.array(pairs_signs, np.int8)).cuda()
    out = torch.empty(L, dtype=torch.int32, device="cuda")
    K = seeds.shape[0]
    res = {}
    for name, rr in (("pairs_only", rows),):
        eng.seed_table_dev(d_seeds, d_signs, stream=stream)
        for _ in range(10):
            eng.aggregate_dev(rr, K, out, L=L, mask_lo=lo, mask_hi=hi, stream=stream)
        reps = 20
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        ev[0].record(stream)
        for i in range(reps):
            eng.aggregate_dev(rr, K, out, L=L, mask_lo=lo, mask_hi=hi, stream=stream)
            ev[i + 1].record(stream)
        torch.cuda.synchronize()
        ms = float(np.median([ev[i].elapsed_time(ev[i + 1]) for i in range(reps)]))   # per launch, median
        gbs = (4.0 * rr.shape[0] * L + 4.0 * L) / (ms * 1e-3) / 1e9
        res[name] = {"rows": int(rr.shape[0]), "seeds_K": int(K), "mask_slots": [int(lo), int(hi)],
                     "kernel_ms": round(ms, 4), "GB/s": round(gbs, 1),
                     "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                     "note": "rows summed + dropout-pair masks only (self masks excluded): HBM-bound half"}
    return res


def with_copy(eng, torch, rows, seeds, signs, L, n_online):
    """PCIe-inclusive round: pinned host rows -> device -> round -> host out."""
    from flamingo_amd import PinnedArena
    N = rows.shape[0]
    arena = PinnedArena(N * L * 4 + L * 4 + 4096)
    host = arena.array((N, L), np.uint32)
    host_out = arena.array((L,), np.uint32)
    host.view(np.int32)[:] = rows.cpu().numpy()
    vecs = [host[i] for i in range(N)]
    t = []
    for _ in range(3):
        t0 = time.perf_counter()
        out = eng.aggregate_unmask(vecs, seeds, signs, L=L)
        t.append(time.perf_counter() - t0)
    ok = bool(np.all(out == n_online))
    arena.free()
    best = min(t)
    return {"ms_per_round": round(best * 1e3, 2), "GB/s": round((4.0 * N * L + 4.0 * L) / best / 1e9, 2),
            "correct": ok, "path": "flm_aggregate_unmask: pinned host rows, host-contiguous runs of <=16 rows per "
                    "hipMemcpyAsync over 4 copy streams, + D2H of out"}


def with_copy_sharded(torch, dist, rnd, rows_on, d_seeds, d_signs, stream, n_online, L, coll_dev, tries=3):
    """PCIe-inclusive round on G ranks: every rank's clients' rows from pinned host memory over its
    own link (one H2D into the same device rows), its shard kernel, the reduce-scatter, and its
    shard of `out` back to pinned host memory; max over ranks, best of `tries`."""
    n_out = rnd.hi - rnd.lo
    try:  # every rank agrees the buffers exist before any rank enters the timed collectives
        host = rows_on.cpu().pin_memory()
        host_out = torch.empty(max(1, n_out), dtype=torch.int32).pin_memory()
        err = ""
    except Exception as e:
        err = f"{type(e).__name__}: {e}"
    okp = torch.tensor([0 if err else 1], device=coll_dev)
    dist.all_reduce(okp, op=dist.ReduceOp.MIN)
    if not int(okp.item()):
        return {"error": err or "another rank could not allocate its pinned buffers"}
    best, ok = None, True
    for _ in range(tries):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            rows_on.copy_(host, non_blocking=True)
        b = rnd.launch(rows_on, d_seeds, d_signs, stream)
        res = rnd.result(b)                      # the current stream waits for the reduce-scatter
        if n_out:
            host_out[:n_out].copy_(res, non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ok &= bool(torch.all(host_out[:n_out] == n_online).item()) if n_out else True
        t = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        best = float(t.item()) if best is None else min(best, float(t.item()))
    okt = torch.tensor([1 if ok else 0], device=coll_dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    G = dist.get_world_size()
    return {"ms_per_round": round(best * 1e3, 2), "GB/s": round((4.0 * n_online * L + 4.0 * L) / best / 1e9, 2),
            "correct": bool(okt.item()),
            "path": f"{G} ranks: pinned host rows of each rank's clients over its own link (one H2D each), shard "
                    "kernel, reduce-scatter, D2H of each rank's out shard; max over ranks"}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def host_threads():
    """(threads, quota): every core this job may use -- nproc, capped by the cgroup CPU quota
    (cpu.max) when one is set -- and that quota in cores (None when unlimited)."""
    n = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    if hasattr(os, "sched_getaffinity"):
        n = min(n, len(os.sched_getaffinity(0)))
    return (max(1, min(n, int(quota))) if quota else n), quota


def cpu_baseline(rows, seeds, signs, L, gpu_out):
    """CPU baseline on this host, same inputs, also cross-checking the GPU bit for bit (gpu_out: the
    GPU's whole output, a device tensor or, at G > 1, the uint32 vector gathered from the ranks).

    value: oracle/ref_numpy.py -- the reference's server loop as written there (numpy uint32
    accumulate, one ChaCha20 keystream + frombuffer + temporary per seed), over OpenSSL's C
    ChaCha20 in place of the un-installable pycryptodomex; single thread like the reference.
    Also reported: the scalar C restatement (1 thread) and its OpenMP all-core run."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker / CPU baseline only
    import ref_numpy as R
    N = rows.shape[0]
    host = rows.cpu().numpy().view(np.uint32)
    gpu = gpu_out.cpu().numpy().view(np.uint32) if hasattr(gpu_out, "cpu") else np.asarray(gpu_out, np.uint32)
    bytes_round = 4.0 * N * L + 4.0 * L
    neg = signs < 0
    assert neg.all(), "c4 baseline round has self masks only"
    t0 = time.perf_counter()
    out = R.server_round(list(host), [s.tobytes() for s in seeds], [], [], L)
    dt = time.perf_counter() - t0
    res = {"value": round(bytes_round / dt / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"the full workload: {N} rows x {L} slots, {seeds.shape[0]} self-mask seeds; the reference's "
                     "numpy loop (SA_ServiceAgent.py:346-350,530-536,605) over OpenSSL ChaCha20, 1 thread",
           "seconds": round(dt, 3), "matches_gpu": bool(np.array_equal(out, gpu))}
    t0 = time.perf_counter()
    out_c = O.aggregate_unmask(host, seeds, signs, L=L, threads=1)
    dt_c = time.perf_counter() - t0
    res["c_port_1_thread"] = {"value": round(bytes_round / dt_c / 1e9, 3), "seconds": round(dt_c, 3),
                              "matches_gpu": bool(np.array_equal(out_c, gpu))}
    threads, quota = host_threads()
    t0 = time.perf_counter()
    out2 = O.aggregate_unmask(host, seeds, signs, L=L, threads=threads)
    dt2 = time.perf_counter() - t0
    res["c_port_all_cores"] = {"value": round(bytes_round / dt2 / 1e9, 3), "cores": threads,
                               "seconds": round(dt2, 3), "matches_gpu": bool(np.array_equal(out2, gpu)),
                               "note": "OpenMP over every core this job may use: min(nproc, cgroup CPU quota)"}
    res["cpu"] = cpu_model()
    res["nproc"] = os.cpu_count()
    res["cgroup_cpu_quota_cores"] = quota
    return res


if __name__ == "__main__":
    sys.exit(main())
