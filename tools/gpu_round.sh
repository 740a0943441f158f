#!/bin/bash
# One GPU session: parity tests, smoke, bench.  Stops at the first fault/timeout.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python __graft_entry__.py > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py "$@" > gpurun_out/bench.log 2>&1 || exit $?
