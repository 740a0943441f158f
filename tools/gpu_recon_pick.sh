#!/bin/bash
# c5 reconstruction (pair queue, 2 terms per lane) with the EC CUs picked 'first' (k/8 per XCD, in-XCD CUs 0..k/8-1)
# or 'stride' (evenly over the logical ids), 24 and 32 EC CUs: HIP-event timeline per run (tools/recon_events.py).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
: > gpurun_out/recon_pick.log
for P in ${PICKS:-first stride}; do
  for C in ${CUSET:-24 32}; do
    echo "# pick $P ec_cus $C" >> gpurun_out/recon_pick.log
    EC_PICK=$P EC_CUS=$C timeout -k 10 300 python3 -u tools/recon_events.py 2>/dev/null | grep -v amdgpu >> gpurun_out/recon_pick.log || exit $?
  done
done
