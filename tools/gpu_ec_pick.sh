#!/bin/bash
# Masked-CU combine (D = 962, T = 20, 2 terms per lane): 'first' vs 'stride' CU picks at 24 / 32 / 48 CUs.
mkdir -p gpurun_out
: > gpurun_out/ec_pick.log
for P in first stride; do
  for C in 24 32 48; do
    echo -n "pick $P cus $C " >> gpurun_out/ec_pick.log
    timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 2 --cus $C --pick $P 2>/dev/null >> gpurun_out/ec_pick.log || exit $?
  done
done
