#!/bin/bash
# Where the masked-CU slowdown of the per-lane combine starts: D = 962, T = 20, 2 terms, 64 / 80 / 96 / 112 CUs.
mkdir -p gpurun_out
: > gpurun_out/ec_alone3.log
for C in 64 80 96 112; do
  echo -n "terms 2 cus $C " >> gpurun_out/ec_alone3.log
  timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 2 --cus $C 2>/dev/null >> gpurun_out/ec_alone3.log || exit $?
done
