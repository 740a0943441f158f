#!/bin/bash
# A/B two builds of the library (A = flamingo_amd/lib, B = flamingo_amd/lib_ab) on the c4 launch
# shapes, alternating processes so both see the same box state: tools/clock_probe.py full / mask.
# usage: tools/ab/ab_lib.sh OUT ROUNDS
OUT=${1:-gpurun_out/ab_lib.log}; N=${2:-3}
R=$(pwd)
: > $OUT
for i in $(seq $N); do
  for M in full mask; do
    for V in A B; do
      if [ $V = B ]; then export FLM_LIB_PATH=$R/flamingo_amd/lib_ab/libflamingo_hip.so; else unset FLM_LIB_PATH; fi
      echo -n "$V " >> $OUT
      timeout -k 10 120 python3 tools/clock_probe.py $M --reps 40 2>/dev/null >> $OUT || exit $?
    done
  done
done
