R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do for V in prio noprio; do
  echo "== $V" >> gpurun_out/r03_rank8_prio_ab.log
  FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 200 python -u tools/probes/rank8_overlap_probe.py >> gpurun_out/r03_rank8_prio_ab.log 2>&1 || exit 1
done; done
FLM_LIB_PATH=$R/flamingo_amd/lib_v/prio/libflamingo_hip.so timeout -k 10 200 python -m pytest tests/test_ec_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_rank8_prio_parity.log 2>&1 || exit 1
