#!/bin/bash
# Cooperative doubling with its additions moved off wave 0's last level (lib_v/new = the default build)
# against the previous kernel (lib_v/ecold): EC parity for both, then the combine at D = 962 / 120.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ec_gpu.py tests/test_reconstruct_gpu.py tests/test_ref_golden_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_coop_dbl.log 2>&1 || exit $?
bash tools/ab_ec_coop.sh gpurun_out/ab_coop_dbl.log 3 new ecold
