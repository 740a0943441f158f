#!/bin/bash
# PMC passes of tools/clock_probe.py, one process per mode (full / mask / rows): shader clock and
# cycles per VALU instruction of the c4 launch vs the mask-only launch.  usage: tools/gpu_clock.sh TAG
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for M in full mask rows; do
  timeout -k 10 120 python3 $R/tools/clock_probe.py $M > $R/gpurun_out/clock_${TAG}_$M.json 2>/dev/null || exit $?
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES --output-format csv -d $R/gpurun_out/clock_${TAG}_pmc_$M -o run -- python3 $R/tools/clock_probe.py $M > $R/gpurun_out/clock_${TAG}_pmc_$M.log 2>&1 || exit $?
done
cd $R && python3 tools/clock_summary.py gpurun_out/clock_${TAG}_summary.json gpurun_out/clock_${TAG}_pmc_full gpurun_out/clock_${TAG}_pmc_mask gpurun_out/clock_${TAG}_pmc_rows
