#!/bin/bash
# c4 whole round (and mask-only) with the claimed units: 1024 one-tile items (default) vs 4096-slot
# tiles at 512 (P=2, atomics) and 2048 items, alternated over 8 rounds, two processes.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/ab_c4_plan.log
for i in 1 2; do
timeout -k 10 300 python3 -u tools/ab_items.py --workloads full,mask --variants auto \
  --subtiles 1,4 --min-items 512,1024 --rounds 8 --reps 10 >> gpurun_out/ab_c4_plan.log 2>&1 || exit $?
done
