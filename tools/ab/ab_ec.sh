#!/bin/bash
# A/B P-256 builds (flamingo_amd/lib_v/<name>) on the c5 EC combine shape (D=962, T=20), on the whole
# chip and on 32 CUs.  usage: tools/ab/ab_ec.sh OUT ROUNDS name...
OUT=$1; N=$2; shift 2
R=$(pwd)
: > $OUT
for i in $(seq $N); do
  for CU in ${EC_AB_CUS:-0 32}; do
    for V in "$@"; do
      export FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so
      echo -n "$V " >> $OUT
      timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --cus $CU 2>/dev/null >> $OUT || exit $?
    done
  done
done
