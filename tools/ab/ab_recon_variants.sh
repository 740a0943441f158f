#!/bin/bash
# c5 reconstruction (pair queue, 32 EC CUs, 4096 pass-1 items) with library variants, alternating;
# the pair-unit parity tests first.  usage: tools/ab/ab_recon_variants.sh OUT ROUNDS name...
OUT=$1; N=$2; shift 2
R=$(pwd)
: > $OUT
for V in "$@"; do
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 200 python -m pytest tests/test_reconstruct_gpu.py -x -q -k "not pair_units_queue" \
    --timeout 120 --timeout-method thread > ${OUT%.log}_parity_$V.log 2>&1 || { echo "parity FAILED for $V"; exit 1; }
done
for i in $(seq $N); do
  for V in "$@"; do
    echo -n "$V " >> $OUT
    FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so EC_CUS=32 SPLIT=q MIN_ITEMS=4096 timeout -k 10 200 \
      python -u tools/probes/recon_split_sweep.py 2>/dev/null >> $OUT || exit $?
  done
done
