#!/bin/bash
# Round-2 re-entry check: full GPU test suite, then the default bench line.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_check.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_check.json 2> gpurun_out/bench_check.err || exit $?
