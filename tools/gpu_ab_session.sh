FLM_LIB_PATH=$PWD/flamingo_amd/lib_ab/libflamingo_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_configs_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || exit $?
bash tools/ab_lib.sh gpurun_out/ab_lib.log 3
