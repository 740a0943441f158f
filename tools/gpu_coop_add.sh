#!/bin/bash
# Cooperative addition with one multiplication per level and 2v / 2 s1 j precomputed (lib_v/add2 = the default build)
# against the previous kernel (lib_v/dbl1): EC parity for both, then the combine at D = 962 / 120.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ec_gpu.py tests/test_reconstruct_gpu.py tests/test_ref_golden_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_coop_add.log 2>&1 || exit $?
bash tools/ab_ec_coop.sh gpurun_out/ab_coop_add.log 3 add2 dbl1
