timeout -k 10 300 python -u -m pytest tests/test_reconstruct_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pu_tests.log 2>&1 || exit $?
EC_CUS=32 SPLIT=q MIN_ITEMS=4096 timeout -k 10 200 python -u tools/recon_split_sweep.py > gpurun_out/pu_recon.log 2>&1 || exit $?
MIN_ITEMS=4096 bash tools/gpu_queue_trace.sh
