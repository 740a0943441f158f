#!/bin/bash
# Claimed work units in items_kernel: GPU tests, A/B against the static split (lib_v/static), and
# workgroup timelines of both (lib_v/wgt, lib_v/wgts).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_claim.log 2>&1 || exit $?
bash tools/ab_variants.sh gpurun_out/ab_claim.log 3 "mask full client" static || exit $?
for V in wgt wgts; do
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 120 python3 tools/wg_trace.py mask > gpurun_out/wg_trace_$V.log 2>&1 || exit $?
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 120 python3 tools/wg_trace.py full >> gpurun_out/wg_trace_$V.log 2>&1 || exit $?
done
