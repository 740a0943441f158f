#!/bin/bash
# A/B P-256 builds (flamingo_amd/lib_v/<name>) with the cooperative EC kernel: parity, then the
# c5-size combine on the whole chip and one rank's share at G = 8.  usage: tools/ab/ab_ec_coop.sh OUT ROUNDS name...
OUT=$1; N=$2; shift 2
R=$(pwd)
: > $OUT
for V in "$@"; do
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 200 python -m pytest tests/test_ec_gpu.py -x -q \
    --timeout 120 --timeout-method thread > ${OUT%.log}_parity_$V.log 2>&1 || { echo "parity FAILED for $V"; exit 1; }
done
for i in $(seq $N); do
  for D in 962 120; do
    for V in "$@"; do
      echo -n "$V " >> $OUT
      FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 120 python3 tools/ec_bench.py --D $D --T 20 \
        --reps 10 --cpu-sample 1 --scalars lagrange --coop 1 2>/dev/null >> $OUT || exit $?
    done
  done
done
