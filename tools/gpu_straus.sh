#!/bin/bash
timeout -k 10 400 python -u -m pytest tests/test_ec_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/straus_tests.log 2>&1 || exit $?
: > gpurun_out/straus_bench.log
for TM in 1 2 4; do
  timeout -k 10 120 python3 tools/ec_bench.py --D 962 --T 20 --reps 5 --cpu-sample 1 --scalars lagrange --coop 0 --terms $TM --cus 32 2>/dev/null >> gpurun_out/straus_bench.log || exit $?
done
: > gpurun_out/straus_recon.log
for TM in 1 2 4; do
  EC_TERMS=$TM EC_CUS=16,24,32 SPLIT=q MIN_ITEMS=4096 timeout -k 10 300 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/straus_recon.log || exit $?
done
