#!/bin/bash
# Profile session: kernel trace + stats, then separate PMC passes (no trace domains with --pmc).
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trace -o run -- python3 $R/bench.py --profile --steps 10 --warmup 2 > $R/gpurun_out/prof_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_pmc1 -o run -- python3 $R/bench.py --profile --steps 4 --warmup 1 > $R/gpurun_out/prof_pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_pmc2 -o run -- python3 $R/bench.py --profile --steps 4 --warmup 1 > $R/gpurun_out/prof_pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/prof_pmc3 -o run -- python3 $R/bench.py --profile --steps 4 --warmup 1 > $R/gpurun_out/prof_pmc3.log 2>&1 || exit $?
