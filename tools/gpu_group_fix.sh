#!/bin/bash
# Device-group loopback ordering fix + stream fixes in dist_recon: the group, distributed and reconstruction GPU tests.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_group_gpu.py tests/test_distributed_gpu.py tests/test_reconstruct_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_group_fix.log 2>&1
