#!/bin/bash
# Sub-tile A/B of the mask-heavy launches (tools/ab_items.py: c4 full / mask-only at 1, 4, 16
# sub-tiles per workgroup, plus the client-masking launch) and PMC passes (clock, cycles per VALU
# instruction) of the mask-only launch at 1 and 16 sub-tiles and of client masking.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 240 python3 -u $R/tools/ab_items.py --workloads mask,full,client --variants auto --subtiles 1,4,16 \
  --rounds 3 --reps 5 > $R/gpurun_out/ab_subtiles.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
for M in "mask 1" "mask 16" "client 0"; do
  set -- $M
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d $R/gpurun_out/sub_pmc_$1_$2 -o run -- python3 $R/tools/clock_probe.py $1 --subtiles $2 > $R/gpurun_out/sub_pmc_$1_$2.log 2>&1 || exit $?
done
