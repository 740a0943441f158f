#!/bin/bash
# Issue priority by progress on top of the claimed units (lib_v/prio) vs the default build, plus
# the workgroup timeline of the priority build (lib_v/wgtp).
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
bash tools/ab_variants.sh gpurun_out/ab_prio.log 3 "mask full" prio || exit $?
FLM_LIB_PATH=$R/flamingo_amd/lib_v/wgtp/libflamingo_hip.so timeout -k 10 120 python3 tools/wg_trace.py mask > gpurun_out/wg_trace_wgtp.log 2>&1 || exit $?
FLM_LIB_PATH=$R/flamingo_amd/lib_v/wgtp/libflamingo_hip.so timeout -k 10 120 python3 tools/wg_trace.py full >> gpurun_out/wg_trace_wgtp.log 2>&1
