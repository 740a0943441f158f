#!/bin/bash
# Round-2 session: new GPU tests, full bench, then the 2-rank rehearsal on the one GPU.
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_integration_binding.py tests/test_abides_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_r02.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || exit $?
bash tools/dist2.sh
