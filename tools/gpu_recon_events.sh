#!/bin/bash
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/recon_events.py > gpurun_out/recon_events.log 2>&1 || exit $?
EC_CUS=32 timeout -k 10 300 python3 -u tools/recon_events.py >> gpurun_out/recon_events.log 2>&1
