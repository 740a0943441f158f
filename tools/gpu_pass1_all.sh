#!/bin/bash
# c5 reconstruction: pass 1 on every CU (EC still on its CU-masked stream, priority 3) vs the
# CU-partitioned pass 1, at 16/24/32 EC CUs.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/recon_pass1_all.log
for A in 0 1 0 1; do
  echo "# PASS1_ALL=$A" >> gpurun_out/recon_pass1_all.log
  PASS1_ALL=$A EC_CUS=16,24,32 SPLIT=q MIN_ITEMS=4096 EC_TERMS=2 timeout -k 10 300 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_pass1_all.log || exit $?
done
