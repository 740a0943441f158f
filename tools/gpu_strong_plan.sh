#!/bin/bash
# One rank of the strong-scaled c4 round (G = 2/4/8, production dual-tile pairing): sub-tiles x
# planner item count, after the claimed units.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab_items.py --workloads strong8,strong4,strong2 --variants auto,block,block_spread \
  --subtiles 1,4 --min-items 512,1024,2048,4096 --pairing 1 --rounds 2 --reps 10 > gpurun_out/ab_strong_plan.log 2>&1
