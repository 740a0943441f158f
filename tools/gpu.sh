#!/bin/bash
# The one launcher for GPU sessions (replaces round 1-2's per-session gpu_*.sh scripts).
#   usage: tools/gpu.sh TAG STEP [STEP ...]      (run through gpurun from the repo root)
# Steps, each under its own time limit, chained so the first failure ends the session:
#   tests        pytest -m gpu (whole GPU suite)          -> gpurun_out/TAG_pytest_gpu.log
#   tests:EXPR   pytest -m gpu -k EXPR                     -> gpurun_out/TAG_pytest_gpu_k.log
#   smoke        __graft_entry__.smoke()                   -> gpurun_out/TAG_smoke.log
#   bench        python bench.py (N=1 default line)        -> gpurun_out/TAG_bench.json/.err
#   bench2       bench.py --gpus 2 --dist-backend gloo (self-launched ranks sharing the GPU)
#   benchG:N     bench.py --gpus N --dist-backend gloo --steps 3 (N self-launched ranks on the one GPU:
#                the sharded c4 and c5 paths end to end, correctness only)
#   sim          ABIDES simulations c1 (n=128) and n=1024 x 2 iterations -> TAG_sim_*.log
#   simc3 / simc5 / simc5r   the agents at BASELINE c3, c5 (n=4096, L=2^20, 10 iterations, 1 % dropouts), reduced c5
#   simprof      cProfile of the reduced c5 run;  simtrace  rocprofv3 kernel trace of a 4-iteration c5 run
#   h2c          the hash-to-curve table launch under a kernel trace
#   rccl         tools/rccl_clique_smoke.py (forced one-device RCCL clique + world-1 forced collectives),
#                then the same with AMD_LOG_LEVEL=4: the kernels it dispatched (RCCL's included)
#   rccltrace    the same script under rocprofv3 --kernel-trace --stats (put it last in a call)
#   ecpmc:K      rocprofv3 PMC pass (VALU/SALU instructions, wave cycles, waits) of the combine at D = 4
#                with ec_coop K (1: per-lane field, 2: row field)
#   pmc:SCRIPT   one rocprofv3 PMC pass (SQ/GRBM issue counters) over python tools/SCRIPT -> TAG_pmc_<name>/
#   prof         rocprofv3 kernel trace + stats and PMC passes of bench.py --profile (gpu_prof.sh)
#   clock        PMC clock/CPI passes (gpu_clock.sh)
#   py:SCRIPT[:ARG]  python tools/SCRIPT [ARG] (e.g. probes/recon_partial_sweep.py) -> gpurun_out/TAG_<name>.log
#   expand       tools/expand_bench.py (the prg_expand leg alone)
#   stallab / stallscr / stallnuma / stallthp / stallpin / pinprobe / stallevict
#                round 6's unmask-stall diagnosis: c5 agent runs with the HIP API
#                trace, scratch / NUMA / THP / pinning settings, the runtime's copy log, and KFD's
#                per-process evicted_ms around every unmask (stallevict: 5 runs x 3 iterations)
#   hostab       tools/probes/host_path_ab.py: host-pointer calls' wall time, this build against lib_v/
TAG=${1:?usage: tools/gpu.sh TAG STEP...}
shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
for step in "$@"; do
  echo "[gpu.sh] $(date +%T) step $step"
  case $step in
    tests)
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$O/${TAG}_pytest_gpu.log" 2>&1 || { tail -30 "$O/${TAG}_pytest_gpu.log"; exit 1; }
      tail -3 "$O/${TAG}_pytest_gpu.log" ;;
    tests:*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${step#tests:}" \
        > "$O/${TAG}_pytest_gpu_k.log" 2>&1 || { tail -30 "$O/${TAG}_pytest_gpu_k.log"; exit 1; }
      tail -3 "$O/${TAG}_pytest_gpu_k.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1 || exit 1 ;;
    bench)
      timeout -k 10 900 python bench.py > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || { tail -20 "$O/${TAG}_bench.err"; exit 1; }
      cat "$O/${TAG}_bench.json" ;;
    bench2)
      timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --no-cpu --no-configs --no-group \
        > "$O/${TAG}_bench2_gloo.json" 2> "$O/${TAG}_bench2_gloo.err" || { tail -20 "$O/${TAG}_bench2_gloo.err"; exit 1; }
      cat "$O/${TAG}_bench2_gloo.json" ;;
    benchG:*)
      n=${step#benchG:}
      timeout -k 10 900 python bench.py --gpus "$n" --dist-backend gloo --steps 3 --warmup 1 \
        > "$O/${TAG}_bench_g${n}_gloo.json" 2> "$O/${TAG}_bench_g${n}_gloo.err" || { tail -20 "$O/${TAG}_bench_g${n}_gloo.err"; exit 1; }
      cut -c1-400 "$O/${TAG}_bench_g${n}_gloo.json" ;;
    sim)
      timeout -k 10 300 python -m flamingo_amd.abides -c flamingo -n 128 -i 1 -p 1 > "$O/${TAG}_sim_c1_n128.log" 2>&1 || exit 1
      timeout -k 10 600 python -m flamingo_amd.abides -c flamingo -n 1024 -i 2 -p 1 > "$O/${TAG}_sim_n1024_i2.log" 2>&1 || exit 1 ;;
    simc5r)
      # BASELINE c5's shape with L = 2^16 and 2 iterations (1 % per-iteration dropouts) through the agents
      timeout -k 10 900 python -u -m flamingo_amd.abides -c flamingo -n 4096 --vector_len 65536 -i 2 --dropout 0.01 --latency deterministic \
        -k -s 5 > "$O/${TAG}_sim_c5r.log" 2>&1 || { tail -30 "$O/${TAG}_sim_c5r.log"; exit 1; }
      tail -12 "$O/${TAG}_sim_c5r.log" ;;
    simprof)
      # where the host time of the agent simulation goes: cProfile of the reduced c5 run
      timeout -k 10 900 python -u -m cProfile -o "$O/${TAG}_sim_c5r.prof" -m flamingo_amd.abides -c flamingo -n 4096 \
        --vector_len 65536 -i 2 --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_sim_c5r_prof.log" 2>&1 \
        || { tail -30 "$O/${TAG}_sim_c5r_prof.log"; exit 1; }
      python -c "import pstats,sys; p=pstats.Stats(sys.argv[1]); p.sort_stats('tottime').print_stats(40); p.sort_stats('cumulative').print_stats(60)" \
        "$O/${TAG}_sim_c5r.prof" > "$O/${TAG}_sim_c5r_pstats.txt" 2>&1
      head -70 "$O/${TAG}_sim_c5r_pstats.txt" | tail -50 ;;
    simtrace)
      # rocprofv3 kernel trace of the c5 agent simulation, 4 iterations (are slow wall times GPU time?)
      (cd /tmp && PYTHONPATH="$R" timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$O/${TAG}_simtrace" \
        -o run -- python3 -u -m flamingo_amd.abides -c flamingo -n 4096 --vector_len 1048576 -i 4 --dropout 0.01 \
        --latency deterministic -k -s 5 > "$O/${TAG}_simtrace.log" 2>&1) || { tail -30 "$O/${TAG}_simtrace.log"; exit 1; }
      grep "iteration [0-9]*:" "$O/${TAG}_simtrace.log" ;;
    stallab)
      # the agent run's first-iteration unmask stall: c5 with 4 iterations, alternating
      # the default allocator with glibc's mmap threshold pinned at 32 MiB and trimming off (freed numpy
      # bodies then stay in the heap instead of being unmapped)
      for v in base mmap base mmap; do
        if [ $v = mmap ]; then envs="MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=68719476736"; else envs=""; fi
        env $envs timeout -k 10 300 python -u -m flamingo_amd.abides -c flamingo -n 4096 --vector_len 1048576 -i 4 \
          --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_stall_$v.log" 2>&1 || { tail -30 "$O/${TAG}_stall_$v.log"; exit 1; }
        echo "== $v"; grep "iteration [0-9]*:" "$O/${TAG}_stall_$v.log" | sed 's/.*iteration/iteration/' | cut -c1-40,150-230
        cat "$O/${TAG}_stall_$v.log" >> "$O/${TAG}_stall_all.txt"
      done ;;
    stallscr)
      # the same c5 run (3 iterations) with ROCr's scratch reclaim off, two ways, then the default under a
      # kernel + copy + scratch-memory trace (the EC kernels use scratch: is the stall a scratch reclaim?)
      for v in noreclaim noasync noreclaim noasync; do
        if [ $v = noreclaim ]; then envs="HSA_NO_SCRATCH_RECLAIM=1"; else envs="HSA_ENABLE_SCRATCH_ASYNC_RECLAIM=0"; fi
        env $envs timeout -k 10 300 python -u -m flamingo_amd.abides -c flamingo -n 4096 --vector_len 1048576 -i 3 \
          --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_stall_$v.log" 2>&1 || { tail -30 "$O/${TAG}_stall_$v.log"; exit 1; }
        echo "== $v"; grep -h "iteration [0-9]*:" "$O/${TAG}_stall_$v.log" | sed 's/.*iteration \([0-9]*\):.*unmask + D2H \(.*\)/it \1: \2/'
        cat "$O/${TAG}_stall_$v.log" >> "$O/${TAG}_stall_all.txt"
      done
      (cd /tmp && PYTHONPATH="$R" timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --scratch-memory-trace \
        --output-format csv -d "$O/${TAG}_scrtrace" -o run -- python3 -u -m flamingo_amd.abides -c flamingo -n 4096 \
        --vector_len 1048576 -i 3 --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_scrtrace.log" 2>&1) \
        || { tail -30 "$O/${TAG}_scrtrace.log"; exit 1; }
      echo "== traced"; grep -h "iteration [0-9]*:" "$O/${TAG}_scrtrace.log" | sed 's/.*iteration \([0-9]*\):.*unmask + D2H \(.*\)/it \1: \2/'
      find "$O/${TAG}_scrtrace" -name '*.csv' -exec gzip -f {} + ; true ;;
    stallnuma)
      # is the stall a KFD queue eviction from an MMU-notifier invalidation of a pinned (userptr) buffer,
      # e.g. by automatic NUMA balancing?  The kernel's settings, then c5 (3 iterations) alternating the
      # default with MPOL_LOCAL (no NUMA-balancing scans of this process: tools/probes/mempolicy_run.py)
      for f in /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/enabled \
               /sys/kernel/mm/transparent_hugepage/defrag /proc/sys/kernel/numa_balancing_scan_delay_ms \
               /proc/sys/kernel/numa_balancing_scan_period_min_ms; do echo "$f: $(cat $f 2>&1)"; done
      grep -h "numa_\|thp_\|pgmigrate" /proc/vmstat 2>/dev/null | head -20 > "$O/${TAG}_vmstat_before.txt"
      for v in local base local base local local; do
        if [ $v = local ]; then pre="tools/probes/mempolicy_run.py"; else pre="-m"; fi
        timeout -k 10 300 python -u $pre flamingo_amd.abides -c flamingo -n 4096 --vector_len 1048576 -i 3 \
          --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_stall_$v.log" 2>&1 || { tail -30 "$O/${TAG}_stall_$v.log"; exit 1; }
        echo "== $v"; grep -h "iteration [0-9]*:" "$O/${TAG}_stall_$v.log" | sed 's/.*iteration \([0-9]*\):.*unmask + D2H \(.*\)/it \1: \2/'
        cat "$O/${TAG}_stall_$v.log" >> "$O/${TAG}_stall_all.txt"
      done
      grep -h "numa_\|thp_\|pgmigrate" /proc/vmstat 2>/dev/null | head -20 > "$O/${TAG}_vmstat_after.txt"; true ;;
    expand)
      timeout -k 10 300 python -u tools/probes/expand_probe.py > "$O/${TAG}_expand_probe.log" 2>&1 \
        || { tail -30 "$O/${TAG}_expand_probe.log"; exit 1; }
      cat "$O/${TAG}_expand_probe.log" | grep -v amdgpu.ids ;;
    stallevict)
      # KFD's per-process queue-eviction counter (sysfs evicted_ms) around every server unmask of the
      # c5 agent run (tools/probes/evict_probe_run.py), 3 runs x 3 iterations
      ls /sys/class/kfd/kfd 2>&1 | head; ls /sys/class/kfd/kfd/proc 2>&1 | head
      for v in 1 2 3 4 5; do
        timeout -k 10 300 python -u tools/probes/evict_probe_run.py -c flamingo -n 4096 --vector_len 1048576 -i 3 \
          --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_evict_$v.log" 2>&1 || { tail -30 "$O/${TAG}_evict_$v.log"; exit 1; }
        echo "== run $v"; grep -h "evict_probe" "$O/${TAG}_evict_$v.log" | cut -c1-400
      done ;;
    stallthp)
      # the eviction counter with transparent huge pages off for the process (PR_SET_THP_DISABLE) vs on,
      # alternating, 3 iterations each; then /proc/vmstat's THP / compaction / migration counters
      grep -h "thp_\|compact_\|pgmigrate" /proc/vmstat > "$O/${TAG}_vmstat_before.txt" 2>/dev/null
      for v in off on off on off off; do
        if [ $v = off ]; then fl="--thp-off"; else fl=""; fi
        timeout -k 10 300 python -u tools/probes/evict_probe_run.py $fl -c flamingo -n 4096 --vector_len 1048576 -i 3 \
          --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_thp_$v.log" 2>&1 || { tail -30 "$O/${TAG}_thp_$v.log"; exit 1; }
        echo "== thp $v"; grep -h "evict_probe\] unmask" "$O/${TAG}_thp_$v.log" | cut -c1-60
        cat "$O/${TAG}_thp_$v.log" >> "$O/${TAG}_thp_all.txt"
      done
      grep -h "thp_\|compact_\|pgmigrate" /proc/vmstat > "$O/${TAG}_vmstat_after.txt" 2>/dev/null; true ;;
    pinprobe)
      # the HIP runtime's own log of the host-pointer calls' copies: pinned (the caller's pages registered
      # with the driver) or staged (tools/probes/pin_probe.py)
      env $PINENV AMD_LOG_LEVEL=4 timeout -k 10 120 python -u tools/probes/pin_probe.py > "$O/${TAG}_pin_probe.out" 2> "$O/${TAG}_pin_probe.err" \
        || { tail -20 "$O/${TAG}_pin_probe.err"; exit 1; }
      grep -h "===\|Pinned resource\|Staging resource\|Unpinned\|staging\|hsa_amd_memory_lock\|Pin" "$O/${TAG}_pin_probe.out" "$O/${TAG}_pin_probe.err" \
        | cut -c1-220 | head -60 > "$O/${TAG}_pin_probe_summary.txt"; cat "$O/${TAG}_pin_probe_summary.txt"; rm -f "$O/${TAG}_pin_probe.err" ;;
    stallpin)
      # the eviction counter with the HIP runtime never pinning the caller's pageable memory for a copy
      # (GPU_PINNED_MIN_XFER_SIZE, MB: every pageable copy staged through the runtime's own buffers) vs default
      for v in nopin base nopin base nopin nopin; do
        if [ $v = nopin ]; then envs="GPU_PINNED_MIN_XFER_SIZE=1048576"; else envs=""; fi
        env $envs timeout -k 10 300 python -u tools/probes/evict_probe_run.py -c flamingo -n 4096 --vector_len 1048576 -i 3 \
          --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_pin_$v.log" 2>&1 || { tail -30 "$O/${TAG}_pin_$v.log"; exit 1; }
        echo "== $v"; grep -h "evict_probe\] unmask" "$O/${TAG}_pin_$v.log" | cut -c1-60
        cat "$O/${TAG}_pin_$v.log" >> "$O/${TAG}_pin_all.txt"
      done ;;
    hostab)
      # host-pointer entry points' wall time per call: this build against the pre-bounce build (lib_v)
      for v in new simple old new simple old; do
        envs=""
        if [ $v = old ]; then envs="FLM_LIB_PATH=$R/flamingo_amd/lib_v/libflamingo_hip_pre_bounce.so"; fi
        if [ $v = simple ]; then envs="FLM_LIB_PATH=$R/flamingo_amd/lib_v/libflamingo_hip_bounce_simple.so"; fi
        env $envs timeout -k 10 200 python -u tools/probes/host_path_ab.py > "$O/${TAG}_hostab_$v.log" 2>&1 || { tail -20 "$O/${TAG}_hostab_$v.log"; exit 1; }
        cat "$O/${TAG}_hostab_$v.log" | grep -v amdgpu.ids
      done ;;
    simc3)
      # BASELINE c3 through the agents: n = 1024, -o 2, L = 2^18
      timeout -k 10 900 python -u -m flamingo_amd.abides -c flamingo -n 1024 -o 2 --vector_len 262144 -i 2 -k -s 3 \
        > "$O/${TAG}_sim_c3.log" 2>&1 || { tail -30 "$O/${TAG}_sim_c3.log"; exit 1; }
      tail -12 "$O/${TAG}_sim_c3.log" ;;
    simc5)
      # BASELINE c5 through the agents: n = 4096, L = 2^20, 10 iterations, 1 % per-iteration dropouts;
      # FLM_GPUS=all: the server's steps over every visible GPU (one here, all 8 on the 8-GPU node)
      FLM_GPUS=all timeout -k 10 1100 python -u -m flamingo_amd.abides -c flamingo -n 4096 --vector_len 1048576 -i 10 \
        --dropout 0.01 --latency deterministic -k -s 5 > "$O/${TAG}_sim_c5.log" 2>&1 || { tail -30 "$O/${TAG}_sim_c5.log"; exit 1; }
      tail -24 "$O/${TAG}_sim_c5.log" ;;
    rccl)
      # every RCCL branch of the multi-GPU path on the one GPU (tools/rccl_clique_smoke.py), then the
      # same script under a kernel + memory-copy trace: the RCCL kernels / copies it launched
      timeout -k 10 300 python -u tools/rccl_clique_smoke.py > "$O/${TAG}_rccl_clique.log" 2>&1 \
        || { tail -30 "$O/${TAG}_rccl_clique.log"; exit 1; }
      tail -2 "$O/${TAG}_rccl_clique.log"
      # the HIP runtime's own launch log names every kernel dispatched (RCCL's included)
      AMD_LOG_LEVEL=4 timeout -k 10 300 python -u tools/rccl_clique_smoke.py gloo > "$O/${TAG}_rccl_amdlog.out" \
        2> "$O/${TAG}_rccl_amdlog.err" || { tail -20 "$O/${TAG}_rccl_amdlog.out"; exit 1; }
      python tools/kernel_log_summary.py "$O/${TAG}_rccl_amdlog.err" "$O/${TAG}_rccl_kernels.json" && rm -f "$O/${TAG}_rccl_amdlog.err" ;;
    rccltrace|rccltrace:*)
      # rocprofv3 kernel trace of the same script with torch's process group on backend ${step#rccltrace:}
      # (default nccl: torch's ProcessGroupNCCL beside the library communicator, torn down in the order
      # of distributed.shutdown); /proc/self/maps at interpreter exit goes next to the log
      be=nccl; [ "$step" != rccltrace ] && be=${step#rccltrace:}
      (cd /tmp && FLM_EXIT_MAPS="$O/${TAG}_rccl_trace_${be}.maps" timeout -k 10 300 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$O/${TAG}_rccl_trace_${be}" -o run -- python3 "$R/tools/rccl_clique_smoke.py" "$be" \
        > "$O/${TAG}_rccl_trace_${be}.log" 2>&1) || { tail -40 "$O/${TAG}_rccl_trace_${be}.log"; exit 1; }
      tail -3 "$O/${TAG}_rccl_trace_${be}.log" ;;
    h2c)
      # the hash-to-curve table launch under a kernel trace (tools/h2c_bench.py)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${TAG}_h2c" -o run \
        -- python3 "$R/tools/h2c_bench.py" > "$O/${TAG}_h2c.log" 2>&1) || { tail -20 "$O/${TAG}_h2c.log"; exit 1; }
      grep '^{' "$O/${TAG}_h2c.log" | cut -c1-600 ;;
    ecpmc:*)
      # one PMC pass over tools/ec_bench.py (the combine, T = 20, Lagrange scalars) with ec_coop ${step#ecpmc:}
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
        SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv \
        -d "$O/${TAG}_ecpmc${step#ecpmc:}" -o run -- python3 "$R/tools/ec_bench.py" --D 4 --T 20 --reps 3 \
        --scalars lagrange --coop "${step#ecpmc:}" > "$O/${TAG}_ecpmc${step#ecpmc:}.log" 2>&1) \
        || { tail -20 "$O/${TAG}_ecpmc${step#ecpmc:}.log"; exit 1; } ;;
    pmc:*)
      # one PMC pass (VALU/SALU instructions, waves, wave cycles, busy, waits) over python tools/SCRIPT
      s=${step#pmc:}
      n=$(basename "${s%.py}")
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
        SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv \
        -d "$O/${TAG}_pmc_$n" -o run -- python3 "$R/tools/$s" > "$O/${TAG}_pmc_$n.log" 2>&1) \
        || { tail -20 "$O/${TAG}_pmc_$n.log"; exit 1; }
      tail -2 "$O/${TAG}_pmc_$n.log" ;;
    prof)
      bash tools/gpu_prof.sh "$TAG" || exit 1 ;;
    clock)
      bash tools/gpu_clock.sh "$TAG" > "$O/${TAG}_clock_run.log" 2>&1 || exit 1 ;;
    py:*)
      s=${step#py:}
      a=""
      case $s in *:*) a=${s#*:}; s=${s%%:*} ;; esac   # py:SCRIPT:ARG passes one argument
      n=$(basename "${s%.py}")
      timeout -k 10 600 python -u "tools/$s" $a > "$O/${TAG}_$n.log" 2>&1 || { tail -20 "$O/${TAG}_$n.log"; exit 1; }
      tail -5 "$O/${TAG}_$n.log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] $(date +%T) done"
