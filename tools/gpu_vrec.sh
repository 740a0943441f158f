#!/bin/bash
# Vector-loaded seed records (FLM_VREC=1, the default build) against the scalar-load path
# (flamingo_amd/lib_v/old, FLM_VREC=0): parity tests first, then the c4 full / mask-only A/B.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_ref_golden_gpu.py tests/test_reconstruct_gpu.py tests/test_group_gpu.py tests/test_distributed_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_vrec.log 2>&1 || exit $?
bash tools/ab_variants.sh gpurun_out/ab_vrec.log 4 "full mask" old
