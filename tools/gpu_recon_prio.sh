#!/bin/bash
# EC wave priority x schedule: queue with 32 EC CUs; overlap without a CU split (pairs in a last pass)
R=$(pwd)
: > gpurun_out/recon_prio.log
for V in base prio0 prio1; do
  for CFG in "32 q" "0 0"; do
    set -- $CFG
    echo -n "$V " >> gpurun_out/recon_prio.log
    FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so EC_CUS=$1 SPLIT=$2 MIN_ITEMS=4096 timeout -k 10 200 \
      python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_prio.log || exit $?
  done
done
