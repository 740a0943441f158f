#!/bin/bash
# c5 reconstruction (pair queue, 32 EC CUs) at several pass-1 item counts (same-tile parts since round 2)
: > gpurun_out/recon_minitems_r02.log
for MI in 1024 2048 4096 8192; do
  echo "min_items=$MI" >> gpurun_out/recon_minitems_r02.log
  EC_CUS=32 SPLIT=q MIN_ITEMS=$MI timeout -k 10 200 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_minitems_r02.log || exit $?
done
