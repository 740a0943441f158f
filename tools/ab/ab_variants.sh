#!/bin/bash
# A/B library variants (flamingo_amd/lib_v/<name>) against the default build on the c4 mask-only
# and full launch shapes, alternating processes.  usage: tools/ab/ab_variants.sh OUT ROUNDS MODES name...
OUT=$1; N=$2; MODES=$3; shift 3
R=$(pwd)
: > $OUT
for i in $(seq $N); do
  for M in $MODES; do
    for V in base "$@"; do
      if [ $V = base ]; then unset FLM_LIB_PATH; else export FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so; fi
      echo -n "$V " >> $OUT
      timeout -k 10 120 python3 tools/clock_probe.py $M --reps 30 2>/dev/null >> $OUT || exit $?
    done
  done
done
