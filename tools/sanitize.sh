#!/bin/bash
# ASan + UBSan on the CPU-side code (no GPU sanitizer on this pool):
#   * the C oracle (oracle/_asan/liboracle.so);
#   * the host side of libflamingo_hip.so -- planner (flm_plan_aggregate / build_aggregate_items),
#     shard geometry, argument checks, context lifecycle -- built with -Xarch_host sanitizers
#     (device code is not instrumented) into build/asan/;
# then the CPU tests that exercise them run with the sanitizer runtimes preloaded.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT"
make -s -B -C oracle asan
mkdir -p build/asan
hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
  -o build/asan/libflamingo_hip.so flamingo_amd/csrc/flm_kernels.hip flamingo_amd/csrc/flm_runtime.hip \
  flamingo_amd/csrc/flm_p256.hip flamingo_amd/csrc/flm_comm.hip flamingo_amd/csrc/flm_store.hip


CLANG_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so 2>/dev/null | head -1)
echo "runtimes: $CLANG_RT"
LD_PRELOAD="$CLANG_RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  FLM_LIB_PATH="$ROOT/build/asan/libflamingo_hip.so" FLM_ORACLE_LIB="$ROOT/oracle/_asan/liboracle.so" \
  python -m pytest tests/test_oracle.py tests/test_planner_cpu.py tests/test_lib_abi.py tests/test_ref_golden_cpu.py \
  -q -m "not gpu" -p no:cacheprovider "$@"
