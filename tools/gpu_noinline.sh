#!/bin/bash
# Field multiply / square as shared routines (lib_v/noinl, FLM_FE_LINKAGE=noinline: kernels 174 KB -> 47-54 KB)
# against inlined copies (lib_v/base): EC parity, then the combine alone on 24 masked CUs / the whole chip
# (per-lane Straus kernel) and the cooperative kernel at D = 962 / 120.
mkdir -p gpurun_out
R=$(pwd)
FLM_LIB_PATH=$R/flamingo_amd/lib_v/noinl/libflamingo_hip.so timeout -k 10 200 python -m pytest tests/test_ec_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_noinl.log 2>&1 || exit $?
: > gpurun_out/ab_noinl.log
for rep in 1 2; do
  for V in base noinl; do
    for cfg in "0 2 24" "0 2 0" "1 1 0"; do
      set -- $cfg
      for D in 962 120; do
        [ "$1" = 0 ] && [ "$D" = 120 ] && continue
        echo -n "$V coop $1 terms $2 cus $3 D $D " >> gpurun_out/ab_noinl.log
        FLM_LIB_PATH=$R/flamingo_amd/lib_v/$V/libflamingo_hip.so timeout -k 10 120 python3 tools/ec_bench.py --D $D --T 20 --reps 10 --cpu-sample 1 --scalars lagrange --coop $1 --terms $2 --cus $3 2>/dev/null >> gpurun_out/ab_noinl.log || exit $?
      done
    done
  done
done
