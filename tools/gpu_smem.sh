#!/bin/bash
# Scalar-load latency and scalar-cache hit rate of the seed-record loads: PMC passes of the c4
# mask-only launch (1 and 16 sub-tiles per workgroup) and of client masking (tools/clock_probe.py).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for M in "mask 1" "mask 16" "client 0" "full 1"; do
  set -- $M
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/smem_$1_$2 -o run -- python3 $R/tools/clock_probe.py $1 --subtiles $2 > $R/gpurun_out/smem_$1_$2.log 2>&1 || exit $?
done
