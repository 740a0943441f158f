#!/bin/bash
# c5 reconstruction (pair queue, 2 combine terms per lane) after the claimed-units kernel: pass-1
# item count x EC CU count.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/recon_claim.log
for MI in 1024 2048 4096; do
  echo "min_items=$MI" >> gpurun_out/recon_claim.log
  EC_CUS=16,24,32 SPLIT=q MIN_ITEMS=$MI EC_TERMS=2 timeout -k 10 300 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_claim.log || exit $?
done
