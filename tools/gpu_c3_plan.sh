#!/bin/bash
# c3 (N=1024, L=2^18) plans with the claimed units: sub-tiles 1/4 x item targets, alternated over 8
# rounds, two processes; then the bench line (roofline.traffic from the committed PMC summary).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/ab_c3_plan.log
for i in 1 2; do
timeout -k 10 300 python3 -u tools/ab_items.py --workloads c3 --variants auto \
  --subtiles 1,4 --min-items 512,1024,2048,4096 --rounds 8 --reps 10 >> gpurun_out/ab_c3_plan.log 2>&1 || exit $?
done
timeout -k 10 400 python3 bench.py > gpurun_out/bench_r02e.json 2> gpurun_out/bench_r02e.err
