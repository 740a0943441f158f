#!/bin/bash
# One rank of the strong-scaled c4 round: the default plan (1 sub-tile, 1024 items) against
# 4 sub-tiles with 512 items, alternated over 8 rounds, two processes.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/ab_strong_plan2.log
for i in 1 2; do
timeout -k 10 300 python3 -u tools/ab_items.py --workloads strong8,strong4,strong2 --variants auto \
  --subtiles 1,4 --min-items 512,1024 --pairing 1 --rounds 8 --reps 10 >> gpurun_out/ab_strong_plan2.log 2>&1 || exit $?
done
