#!/bin/bash
# Parity subset of every variant build (flamingo_amd/lib_v/<name>), then the A/B of tools/ab/ab_variants.sh.
# usage: tools/ab/ab_variants_check.sh OUT ROUNDS "MODES" name...
OUT=$1; N=$2; MODES=$3; shift 3
R=$(pwd)
for V in "$@"; do
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -x -q \
    --timeout 120 --timeout-method thread -k "aggregate or client_mask or prg" > ${OUT%.log}_parity_$V.log 2>&1 || { echo "parity FAILED for $V"; exit 1; }
done
bash tools/ab/ab_variants.sh $OUT $N "$MODES" "$@"
