#!/bin/bash
# PMC passes on the cooperative EC combine (one G = 8 rank's D = 120 share): instruction-cache
# traffic and the wave's instruction / wait mix, one counter group per run.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/tools/ec_bench.py --D 120 --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop 1"
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_REQ --output-format csv -d $R/gpurun_out/ecic_a -o run -- $B > $R/gpurun_out/ecic_a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_IFETCH SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/ecic_b -o run -- $B > $R/gpurun_out/ecic_b.log 2>&1 || exit $?
