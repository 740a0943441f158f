#!/bin/bash
# EC CUs picked xcd_stride (k/8 per XCD, spread over each XCD's CUs): the combine alone, then the c5
# reconstruction timeline, against the strided pick (which lands on three XCDs only).
mkdir -p gpurun_out
: > gpurun_out/ec_xcd.log
for C in 24 32; do
  echo -n "pick xcd_stride cus $C " >> gpurun_out/ec_xcd.log
  timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 0 --terms 2 --cus $C --pick xcd_stride 2>/dev/null >> gpurun_out/ec_xcd.log || exit $?
done
PICKS="xcd_stride stride" CUSET="24 32" bash tools/gpu_recon_pick.sh
