#!/bin/bash
# Profile session for the committed profiles/: bench (live numbers), kernel trace + stats of
# the same command, then separate PMC passes (no trace domains combined with --pmc).
# usage: tools/gpu_prof.sh TAG   (outputs under gpurun_out/prof_TAG*)
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --profile --steps 20 --warmup 3"
timeout -k 10 300 $B > $R/gpurun_out/prof_${TAG}_bench.json 2> $R/gpurun_out/prof_${TAG}_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_trace -o run -- $B > $R/gpurun_out/prof_${TAG}_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_${TAG}_pmc1 -o run -- $B > $R/gpurun_out/prof_${TAG}_pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_${TAG}_pmc2 -o run -- $B > $R/gpurun_out/prof_${TAG}_pmc2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/prof_${TAG}_pmc3 -o run -- $B > $R/gpurun_out/prof_${TAG}_pmc3.log 2>&1 || exit $?
cd $R && python3 tools/summarize_profile.py gpurun_out/prof_${TAG}_summary.json gpurun_out/prof_${TAG}_trace gpurun_out/prof_${TAG}_pmc1 gpurun_out/prof_${TAG}_pmc2 gpurun_out/prof_${TAG}_pmc3 > /dev/null
# seed recovery (c5 shape): kernel trace + stats of tools/recovery_bench.py
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_recovery -o run -- python3 $R/tools/recovery_bench.py > $R/gpurun_out/prof_${TAG}_recovery.log 2>&1 || exit $?
# standalone mask expansion (flm_prg_expand_dev, c5's D seeds x 2^20): kernel trace + stats, then its write traffic
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_expand -o run -- python3 $R/tools/expand_bench.py > $R/gpurun_out/prof_${TAG}_expand.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_${TAG}_expand_pmc -o run -- python3 $R/tools/expand_bench.py > $R/gpurun_out/prof_${TAG}_expand_pmc.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/prof_${TAG}_expand_pmc3 -o run -- python3 $R/tools/expand_bench.py > $R/gpurun_out/prof_${TAG}_expand_pmc3.log 2>&1 || exit $?
cd $R && python3 tools/summarize_profile.py gpurun_out/prof_${TAG}_expand_summary.json gpurun_out/prof_${TAG}_expand gpurun_out/prof_${TAG}_expand_pmc gpurun_out/prof_${TAG}_expand_pmc3 > /dev/null
