timeout -k 10 400 python -u -m pytest tests/test_ec_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ec_coop_tests.log 2>&1 || exit $?
: > gpurun_out/ec_coop_bench.log
for C in 0 1; do
  for D in 962 120; do
    FLM_EC_COOP=$C timeout -k 10 120 python3 tools/ec_bench.py --D $D --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop $C 2>/dev/null >> gpurun_out/ec_coop_bench.log || exit $?
  done
done
