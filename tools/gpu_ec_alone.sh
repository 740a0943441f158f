#!/bin/bash
# The c5 combine (D = 962, T = 20, per-lane Straus kernel) ALONE on CU-masked streams ('first' pick) and on the
# whole chip, with and without an LDS reservation that caps EC workgroups per CU (ec_spread KiB): is a CU-masked
# dispatch packing two EC waves per SIMD?
mkdir -p gpurun_out
: > gpurun_out/ec_alone.log
for SP in 0 40; do
  for C in 24 32 48 0; do
    echo -n "terms 2 spread $SP cus $C " >> gpurun_out/ec_alone.log
    timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 2 --cus $C --spread $SP 2>/dev/null >> gpurun_out/ec_alone.log || exit $?
  done
  echo -n "terms 4 spread $SP cus 24 " >> gpurun_out/ec_alone.log
  timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 4 --cus 24 --spread $SP 2>/dev/null >> gpurun_out/ec_alone.log || exit $?
done
