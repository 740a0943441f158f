#!/bin/bash
# pair-queue reconstruction with and without the CU split, several pass-1 item counts
timeout -k 10 300 python -u -m pytest tests/test_reconstruct_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/recon_tests.log 2>&1 || exit $?
: > gpurun_out/recon_nosplit.log
for MI in 4096 8192 16384; do
  echo "min_items=$MI" >> gpurun_out/recon_nosplit.log
  EC_CUS=0,32 SPLIT=q MIN_ITEMS=$MI timeout -k 10 200 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_nosplit.log || exit $?
done
