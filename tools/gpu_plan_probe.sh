#!/bin/bash
# plan_probe timing, then per-case PMC passes (one counter set per run; no trace domains with --pmc)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/plan_probe.py > $R/gpurun_out/plan_probe.log 2>&1 || exit $?
for c in agg client fused; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pp_$c -o run -- python3 $R/tools/plan_probe.py --case $c --reps 10 > $R/gpurun_out/pp_$c.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_INSTS_LDS GRBM_COUNT --output-format csv -d $R/gpurun_out/pp2_$c -o run -- python3 $R/tools/plan_probe.py --case $c --reps 10 > $R/gpurun_out/pp2_$c.log 2>&1 || exit $?
done
