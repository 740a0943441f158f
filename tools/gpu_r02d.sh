#!/bin/bash
# Final round-2 evidence with the claimed-units kernel: the default bench line, the profile set
# (tools/gpu_prof.sh r02d), clock/CPI passes, 2-rank rehearsal.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r02d.json 2> gpurun_out/bench_r02d.err || exit $?
bash tools/gpu_prof.sh r02d || exit $?
cd $R
bash tools/gpu_clock.sh r02d > gpurun_out/clock_run.log 2>&1 || exit $?
bash tools/dist2.sh
