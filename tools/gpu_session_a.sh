#!/bin/bash
# clock/CPI PMC passes, then the split-plan A/B (merged same-tile items with atomics)
timeout -k 10 120 python3 tools/clock_probe.py rows > gpurun_out/clock_r02_rows.json 2>/dev/null || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d $R/gpurun_out/clock_r02_pmc_rows -o run -- python3 $R/tools/clock_probe.py rows > $R/gpurun_out/clock_r02_pmc_rows.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python -u tools/ab_items.py --workloads full,c3 --variants auto --subtiles 1 --pairing 1 --min-items 512,1024,2048,4096 --rounds 3 --reps 5 > gpurun_out/ab_split2.log 2>&1
