"""Flamingo experiment driver (config/flamingo.py surface).

    python -m flamingo_amd.abides -c flamingo -n 128 -i 1 [-o 1] [-s SEED] [-v]

Same flags as the reference (config/flamingo.py:24-52), same agent
construction (:179-215), cubic latency model (:225-238) and result print
(:253-266).  Extra flags: --vector_len (reference constant 16000,
util/param.py:8), --root_seed_hex (the reference draws it at random,
util/param.py:31), --offline id,id,... (clients that crash before sending in
every iteration: explicit dropout injection), --dropout F (in each iteration t a
fresh offline set PCG64(seed=t).choice(N, round(F N), replace=False), SURVEY 8d's
c5 recipe: BASELINE c5 is -n 4096 --vector_len 1048576 -i 10 --dropout 0.01),
--latency deterministic (model/LatencyModel.py:142-143: min latency only, so no
VECTOR arrives late and the offline sets are exactly the injected ones; the
reference config's cubic model, the default, adds emergent late-message dropouts).
At the end the run prints, per iteration, |U| and whether final_sum == |U| in
every slot (the all-ones known answer, SA_ClientAgent.py:304 + SA_ServiceAgent.py:605).
"""
from __future__ import annotations

import argparse
import gc
from datetime import timedelta
from time import time

import numpy as np
import pandas as pd

from . import log
from .kernel import Kernel
from .latency import LatencyModel
from .flamingo import SA_ClientAgent as ClientAgent
from .flamingo import SA_ServiceAgent as ServiceAgent
from .flamingo import protocol as param
from .. import params as P


def parse(argv):
    ap = argparse.ArgumentParser(description="Detailed options for the Flamingo config.")
    ap.add_argument("-a", "--clear_learning", action="store_true")
    ap.add_argument("-c", "--config", required=True)
    ap.add_argument("-i", "--num_iterations", type=int, default=5)
    ap.add_argument("-k", "--skip_log", action="store_true")
    ap.add_argument("-l", "--log_dir", default=None)
    ap.add_argument("-n", "--num_clients", type=int, default=5)
    ap.add_argument("-o", "--neighborhood_size", type=int, default=1)
    ap.add_argument("--round_time", type=int, default=10)
    ap.add_argument("-s", "--seed", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-p", "--parallel_mode", type=bool, default=True)   # type=bool quirk kept
    ap.add_argument("-d", "--debug_mode", type=bool, default=False)
    ap.add_argument("--config_help", action="store_true")
    ap.add_argument("--vector_len", type=int, default=P.vector_len)
    ap.add_argument("--root_seed_hex", default=None)
    ap.add_argument("--offline", default="")
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--latency", choices=("cubic", "deterministic"), default="cubic")
    ap.add_argument("--committee_size", type=int, default=P.committee_size)
    args, _ = ap.parse_known_args(argv)
    return ap, args


def offline_schedule(n: int, iterations: int, always=(), dropout: float = 0.0) -> dict:
    """client id -> iterations in which it crashes before sending: `always` in every iteration, plus
    a fresh PCG64(seed=t).choice(n, round(dropout n), replace=False) set in each iteration t."""
    out = {i: set(range(1, iterations + 1)) for i in always}
    k = int(round(dropout * n))
    for t in range(1, iterations + 1):
        if k:
            for i in np.random.Generator(np.random.PCG64(t)).choice(n, k, replace=False):
                out.setdefault(int(i), set()).add(t)
    return out


# Young-generation threshold for the run: the simulation allocates ~1.7 M container objects per
# iteration at n = 4096 (messages, payload dicts), and at CPython's default of 700 the resulting
# full collections over the agents' state took 5.7 s of a 67 s c5 event loop; at 50,000 they take
# 0.5 s and the loop 61.5 s (tools/probes/sim_gc_probe.py, profiles/r05_sim_gc_threshold.log).
GC_THRESHOLD0 = 50_000


def run(argv=None):
    ap, args = parse(argv)
    if args.config_help:
        ap.print_help()
        return None
    old_gc = gc.get_threshold()
    gc.set_threshold(max(old_gc[0], GC_THRESHOLD0), *old_gc[1:])
    try:
        return _run(args)
    finally:
        gc.set_threshold(*old_gc)


def _run(args):
    seed = args.seed or int(pd.Timestamp.now().timestamp() * 1000000) % (2**32 - 1)
    np.random.seed(seed)
    log.silent_mode = not args.verbose
    n = args.num_clients
    if not P.assert_power_of_two(n):
        raise ValueError("Number of clients must be power of 2")
    root = bytes.fromhex(args.root_seed_hex) if args.root_seed_hex else None
    if args.committee_size > args.num_clients:
        raise ValueError("committee_size cannot exceed num_clients")
    param.configure(root=root, L=args.vector_len, committee=args.committee_size)
    offline = {int(x) for x in args.offline.split(",") if x.strip()}
    offline_its = offline_schedule(n, args.num_iterations, offline, args.dropout)
    print(f"Silent mode: {log.silent_mode}")
    print(f"Configuration seed: {seed}\n")

    start = pd.to_datetime("2023-01-01")
    stop = start + pd.to_timedelta("2000:00:00")
    default_delay = 1000000000 * 0.1
    kernel = Kernel("Base Kernel",
                    random_state=np.random.RandomState(seed=np.random.randint(low=0, high=2**32, dtype="uint64")))
    latency_rstate = np.random.RandomState(seed=np.random.randint(low=0, high=2**32, dtype="uint64"))
    agents = []
    t0 = time()
    for i in range(n):
        agents.append(ClientAgent(
            id=i, name=f"PPFL Client Agent {i}", type="ClientAgent", iterations=args.num_iterations, num_clients=n,
            neighborhood_size=args.neighborhood_size, debug_mode=args.debug_mode,
            random_state=np.random.RandomState(seed=np.random.randint(low=0, high=2**32, dtype="uint64")),
            offline_iterations=offline_its.get(i, ())))
    print(f"Client init took {timedelta(seconds=time() - t0)}")
    server = ServiceAgent(
        id=n, name="PPFL Service Agent", type="ServiceAgent",
        random_state=np.random.RandomState(seed=np.random.randint(low=0, high=2**32, dtype="uint64")),
        msg_fwd_delay=0, users=[*range(n)], iterations=args.num_iterations,
        round_time=pd.Timedelta(f"{args.round_time}s"), num_clients=n, neighborhood_size=args.neighborhood_size,
        parallel_mode=args.parallel_mode, debug_mode=args.debug_mode)
    agents.append(server)
    pairwise = (len(agents), len(agents))
    model_args = {"connected": True,
                  "min_latency": np.random.uniform(low=10000000, high=100000000, size=pairwise),
                  "jitter": 0.3, "jitter_clip": 0.05, "jitter_unit": 5}
    latency = LatencyModel(latency_model=args.latency, random_state=latency_rstate, kwargs=model_args)
    results = kernel.runner(agents=agents, startTime=start, stopTime=stop, agentLatencyModel=latency,
                            defaultComputationDelay=default_delay, skip_log=args.skip_log, log_dir=args.log_dir)
    print()
    print("######## Microbenchmarks ########")
    print(f"Protocol Iterations: {args.num_iterations}, Clients: {n}, ")
    print()
    print("Service Agent mean time per iteration (except setup)...")
    print(f"    Report step:         {results['srv_report']}")
    print(f"    Crosscheck step:     {results['srv_crosscheck']}")
    print(f"    Reconstruction step: {results['srv_reconstruction']}")
    print()
    print("Client Agent mean time per iteration (except setup)...")
    print(f"    Report step:         {results['clt_report'] / n}")
    print(f"    Crosscheck step:     {results['clt_crosscheck'] / param.committee_size}")
    print(f"    Reconstruction step: {results['clt_reconstruction'] / param.committee_size}")
    print()
    print("######## Known answer (all-ones inputs: final_sum == |U| in every slot) ########")
    for it in sorted(server.results):
        out, u = server.results[it], server.online_counts[it]
        gpu = server.gpu_ms.get(it, {})
        print(f"    iteration {it}: |U| = {u}, dropout pairs = {server.pairs_per_iteration.get(it, 0)}, "
              f"final_sum == |U| in every slot: {bool(np.all(out == u))}; report GPU {gpu.get('report', 0):.3f} ms, "
              f"unmask + D2H {gpu.get('reconstruction_unmask_gpu', 0):.3f} ms GPU "
              f"({gpu.get('reconstruction_unmask_wall', 0):.3f} ms wall)")
    print()
    results["server"] = server
    return results
