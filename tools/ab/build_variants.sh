#!/bin/bash
# Build libflamingo_hip.so variants with compile-time -D flags on ONE source file (VAR_SRC, default
# flm_kernels; the others are built once, plain) for A/B runs: flamingo_amd/lib_v/<name>/libflamingo_hip.so.
# usage: [VAR_SRC=flm_p256] tools/ab/build_variants.sh name1 'flags1' name2 'flags2' ...
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/flamingo_amd/csrc
O=/tmp/flm_var_objs
V=${VAR_SRC:-flm_kernels}
mkdir -p $O
others=()
for f in flm_kernels flm_runtime flm_p256 flm_comm flm_store; do
  [ $f = $V ] && continue
  others+=($O/$f.o)
  if [ ! $O/$f.o -nt $C/$f.hip ] || [ ! $O/$f.o -nt $C/flm_internal.h ]; then
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -o $O/$f.o $C/$f.hip &
  fi
done
wait
pids=()
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p $R/flamingo_amd/lib_v/$name
  ( eval hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c -o $O/v_$name.o $C/$V.hip 2>/dev/null && \
    hipcc --offload-arch=gfx950 -fPIC -shared -o $R/flamingo_amd/lib_v/$name/libflamingo_hip.so $O/v_$name.o ${others[@]} && echo built $name ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
