#!/bin/bash
# Is the CU-masked combine slow because waves share a CU (the EC kernels are ~174 KB of straight-line code:
# instruction-cache pressure) rather than because of the mask?  Per-lane Straus kernel, D = 962, T = 20.
mkdir -p gpurun_out
: > gpurun_out/ec_alone2.log
for cfg in "128 0" "128 64" "256 0" "256 64" "0 64" "64 64"; do
  set -- $cfg
  echo -n "terms 2 cus $1 spread $2 " >> gpurun_out/ec_alone2.log
  timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 2 --cus $1 --spread $2 2>/dev/null >> gpurun_out/ec_alone2.log || exit $?
done
