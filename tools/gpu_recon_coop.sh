#!/bin/bash
# c5 reconstruction with the per-lane and the cooperative EC kernel: CU-split + queue at 24-64 EC CUs,
# and the sequential / overlapped (no split) schedules
: > gpurun_out/recon_coop.log
for C in 0 1; do
  EC_COOP=$C EC_CUS=24,32,48,64 SPLIT=q MIN_ITEMS=4096 timeout -k 10 300 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_coop.log || exit $?
done
