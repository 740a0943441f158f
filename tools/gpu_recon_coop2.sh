#!/bin/bash
: > gpurun_out/recon_coop2.log
for r in 1 2; do
  EC_COOP=0 EC_CUS=32 SPLIT=q MIN_ITEMS=4096 timeout -k 10 200 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_coop2.log || exit $?
  EC_COOP=1 EC_CUS=56,64,72,80 SPLIT=q MIN_ITEMS=4096 timeout -k 10 300 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_coop2.log || exit $?
done
