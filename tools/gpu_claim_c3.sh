#!/bin/bash
# c3 and the strong-scaled ranks (production dual-tile pairing) with claimed units vs the static
# split, and workgroup timelines of c3 for both.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/ab_claim_strong.log
for i in 1 2; do
  for V in base static; do
    if [ $V = base ]; then unset FLM_LIB_PATH; else export FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so; fi
    echo "# $V" >> gpurun_out/ab_claim_strong.log
    timeout -k 10 200 python3 -u tools/ab_items.py --workloads strong2,strong4,strong8,c3 --variants auto --subtiles 0 --pairing 1 --rounds 3 --reps 10 --settle-ms 100 2>/dev/null >> gpurun_out/ab_claim_strong.log || exit $?
  done
done
unset FLM_LIB_PATH
for V in wgt wgts; do
  WG_TRACE_DUMP=gpurun_out/wgt_c3_$V FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 120 python3 tools/wg_trace.py c3 > gpurun_out/wg_trace_c3_$V.log 2>&1 || exit $?
done
