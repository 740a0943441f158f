#!/bin/bash
# Final round-2 evidence after the cooperative EC changes: full GPU suite, smoke(), default bench, and the
# seed-recovery kernel trace (rocprofv3 --kernel-trace --stats of tools/recovery_bench.py).
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final2.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_final2.json 2> gpurun_out/bench_final2.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final2_recovery -o run -- python3 $R/tools/recovery_bench.py > $R/gpurun_out/prof_final2_recovery.log 2>&1 || exit $?
