#!/bin/bash
# A/B P-256 library builds (flamingo_amd/lib_v/<name>) on every EC kernel form: the EC GPU tests
# against each build first, then tools/ec_bench.py on the c5 combine (D = 962) and one G = 8 rank's
# share (D = 120), cooperative (coop 1) and one lane per product (coop 0), alternating builds.
# usage: tools/ab/ab_ec_kernels.sh OUT ROUNDS name...
OUT=$1; N=$2; shift 2
R=$(pwd)
: > $OUT
for V in "$@"; do
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 200 python -m pytest tests/test_ec_gpu.py -x -q \
    --timeout 120 --timeout-method thread > ${OUT%.log}_parity_$V.log 2>&1 || { echo "parity FAILED for $V"; exit 1; }
done
for i in $(seq $N); do
  for CO in 1 0; do
    for D in 962 120; do
      for V in "$@"; do
        echo -n "$V " >> $OUT
        FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 120 python3 tools/ec_bench.py --D $D --T 20 \
          --reps 10 --cpu-sample 1 --scalars lagrange --coop $CO 2>/dev/null >> $OUT || exit $?
      done
    done
  done
done
