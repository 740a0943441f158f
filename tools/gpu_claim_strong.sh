#!/bin/bash
# Claimed units vs the static split (lib_v/static) on one rank of the strong-scaled c4 round
# (tools/ab_items.py strong2/4/8) and on c3; alternating processes.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/ab_claim_strong.log
for i in 1 2; do
  for V in base static; do
    if [ $V = base ]; then unset FLM_LIB_PATH; else export FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so; fi
    echo "# $V" >> gpurun_out/ab_claim_strong.log
    timeout -k 10 200 python3 -u tools/ab_items.py --workloads strong2,strong4,strong8,c3 --variants auto --subtiles 0 --rounds 3 --reps 10 --settle-ms 100 2>/dev/null >> gpurun_out/ab_claim_strong.log || exit $?
  done
done
