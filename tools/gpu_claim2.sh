#!/bin/bash
# Claimed units, two-loop body with the counter add in asm: GPU tests, A/B against the static split
# on the c4 / client shapes and on the strong-scaled ranks + c3.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_claim2.log 2>&1 || exit $?
bash tools/ab_variants.sh gpurun_out/ab_claim2.log 3 "mask full client" static || exit $?
: > gpurun_out/ab_claim2_strong.log
for i in 1 2; do
  for V in base static; do
    if [ $V = base ]; then unset FLM_LIB_PATH; else export FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so; fi
    echo "# $V" >> gpurun_out/ab_claim2_strong.log
    timeout -k 10 200 python3 -u tools/ab_items.py --workloads strong2,strong4,strong8,c3 --variants auto --subtiles 0 --pairing 1 --rounds 3 --reps 10 --settle-ms 100 2>/dev/null >> gpurun_out/ab_claim2_strong.log || exit $?
  done
done
