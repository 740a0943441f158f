#!/bin/bash
# The combine alone on part of ONE XCD / one whole XCD / one and a half ('xcd' pick: XCD 0's CUs first).
mkdir -p gpurun_out
: > gpurun_out/ec_onexcd.log
for C in 8 16 24 32 48; do
  echo -n "pick xcd cus $C " >> gpurun_out/ec_onexcd.log
  timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 2 --cus $C --pick xcd 2>/dev/null >> gpurun_out/ec_onexcd.log || exit $?
done
