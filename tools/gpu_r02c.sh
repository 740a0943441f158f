#!/bin/bash
# Evidence refresh after the claimed-units kernel: non-temporal row loads A/B, the default bench
# line, the profile set (tools/gpu_prof.sh r02c), clock/CPI passes, 2-rank rehearsal.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/ab_items.py --workloads full --variants merged,merged_nt --subtiles 1 --rounds 3 --reps 10 > gpurun_out/ab_nt.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r02c.json 2> gpurun_out/bench_r02c.err || exit $?
bash tools/gpu_prof.sh r02c || exit $?
cd $R
bash tools/gpu_clock.sh r02c > gpurun_out/clock_run.log 2>&1 || exit $?
bash tools/dist2.sh
