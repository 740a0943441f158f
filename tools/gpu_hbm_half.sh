#!/bin/bash
# The HBM-bound half (rows only; rows + 204 dropout-pair masks): every items_kernel variant x
# sub-tiles x planner item count, one process (tools/ab_items.py), after the claimed units.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python3 -u tools/ab_items.py --workloads pairs,rows \
  --variants auto,coalesced,block,merged,merged_nt,merged_ru4,merged_ru4_nt,merged_spread,block_spread \
  --subtiles 1,4 --min-items 512,1024,2048 --rounds 2 --reps 5 > gpurun_out/ab_hbm_half.log 2>&1
