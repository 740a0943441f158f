#!/bin/bash
# rotl16 as v_pack_b32_f16: exhaustive bit check + issue cost (tools/pack_probe), parity tests with the
# pack build (lib_v/pk_a), then the c4 full / mask-only A/B of the pack builds (gap variants).
mkdir -p gpurun_out
timeout -k 5 90 ./tools/pack_probe > gpurun_out/pack_probe.log 2>&1 || exit $?
grep -q "mismatches 0 of" gpurun_out/pack_probe.log || exit 3
FLM_LIB_PATH=$PWD/flamingo_amd/lib_v/pk_a/libflamingo_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_ref_golden_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1 || exit $?
bash tools/ab_variants.sh gpurun_out/ab_pack.log 3 "full mask" pk_a pk_b pk_c pk_d
