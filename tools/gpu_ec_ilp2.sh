#!/bin/bash
# P-256 field multiply with two accumulator chains per column (lib_v/ilp2) vs the same tree without
# (lib_v/ecbase): EC combine alone (whole chip, 24 CUs) and the c5 reconstruction sweep; EC GPU tests.
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
EC_AB_CUS="0 24" bash tools/ab_ec.sh gpurun_out/ab_ec_ilp2.log 2 ecbase ilp2 || exit $?
FLM_LIB_PATH=$R/flamingo_amd/lib_v/ilp2/libflamingo_hip.so timeout -k 10 300 python3 -u -m pytest tests/test_ec_gpu.py tests/test_reconstruct_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ec_ilp2.log 2>&1 || exit $?
: > gpurun_out/recon_ilp2.log
for V in ecbase ilp2; do
  echo "# $V" >> gpurun_out/recon_ilp2.log
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so EC_CUS=16,24,32 SPLIT=q MIN_ITEMS=4096 EC_TERMS=2 timeout -k 10 300 python -u tools/recon_split_sweep.py 2>/dev/null >> gpurun_out/recon_ilp2.log || exit $?
done
