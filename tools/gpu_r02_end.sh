#!/bin/bash
# End-of-round-2 evidence: the full GPU suite, smoke(), the default bench line.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_end.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_end.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_end.json 2> gpurun_out/bench_end.err || exit $?
