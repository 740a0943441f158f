# pair-queue reconstruction: parity tests, then the c5 schedule sweep (tools/recon_split_sweep.py)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_reconstruct_gpu.py > gpurun_out/q_tests.log 2>&1 || exit $?
EC_CUS=${EC_CUS:-24,32,40} SPLIT=${SPLIT:-0,q,0,q} CU_PICK=${CU_PICK:-first} timeout -k 10 400 python -u tools/recon_split_sweep.py > gpurun_out/q_sweep.log 2>&1
