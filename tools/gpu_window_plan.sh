#!/bin/bash
# Windowed plans (4096-slot tiles, 512 items): GPU tests, then the new default (subtiles 0) against
# the previous plan (subtiles 1) on the strong-scaled ranks and the weak-scaled shard, alternated;
# 2-rank rehearsal.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_window.log 2>&1 || exit $?
: > gpurun_out/ab_window_plan.log
for i in 1 2; do
timeout -k 10 300 python3 -u tools/ab_items.py --workloads strong8,strong4,strong2,shard8 --variants auto \
  --subtiles 0,1 --min-items 1024 --pairing 1 --rounds 8 --reps 10 >> gpurun_out/ab_window_plan.log 2>&1 || exit $?
done
bash tools/dist2.sh
