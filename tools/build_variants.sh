#!/bin/bash
# Build libflamingo_hip.so variants of flm_kernels.hip (compile-time -D flags) for A/B runs:
# flamingo_amd/lib_v/<name>/libflamingo_hip.so.  usage: tools/build_variants.sh name1 'flags1' name2 'flags2' ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/flamingo_amd/csrc
O=/tmp/flm_var_objs
mkdir -p $O
for f in flm_runtime flm_p256 flm_comm; do
  [ $O/$f.o -nt $C/$f.hip ] || hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -o $O/$f.o $C/$f.hip &
done
wait
pids=()
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p $R/flamingo_amd/lib_v/$name
  ( eval hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c -o $O/k_$name.o $C/flm_kernels.hip 2>/dev/null && \
    hipcc --offload-arch=gfx950 -fPIC -shared -o $R/flamingo_amd/lib_v/$name/libflamingo_hip.so $O/k_$name.o $O/flm_runtime.o $O/flm_p256.o $O/flm_comm.o && echo built $name ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
