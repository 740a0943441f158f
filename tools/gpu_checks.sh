#!/bin/bash
# Wrapper input checks + strided-row pitch: the GPU parity, group and reconstruction tests.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_group_gpu.py tests/test_reconstruct_gpu.py tests/test_ec_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_checks.log 2>&1
