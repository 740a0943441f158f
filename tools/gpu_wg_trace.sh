#!/bin/bash
# Workgroup timelines of the c4 launches (tools/wg_trace.py on the -DFLM_WG_TRACE probe build).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export FLM_LIB_PATH=$R/flamingo_amd/lib_v/wgt/libflamingo_hip.so
cd $R
WG_TRACE_DUMP=gpurun_out/wgt_mask.npy timeout -k 10 120 python3 tools/wg_trace.py mask > gpurun_out/wg_trace.log 2>&1 && \
WG_TRACE_DUMP=gpurun_out/wgt_full.npy timeout -k 10 120 python3 tools/wg_trace.py full >> gpurun_out/wg_trace.log 2>&1 && \
timeout -k 10 120 python3 tools/wg_trace.py mask --min-items 16384 >> gpurun_out/wg_trace.log 2>&1
