// bank_probe.hip -- does VGPR bank placement of VALU source operands cost issue cycles on gfx950?
// Fixed physical registers via inline asm (clobbers), 8 independent chains, 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define BODY_SAME \
  "v_add_u32 v40, v40, v44\n v_add_u32 v41, v41, v45\n v_add_u32 v42, v42, v46\n v_add_u32 v43, v43, v47\n" \
  "v_add_u32 v48, v48, v52\n v_add_u32 v49, v49, v53\n v_add_u32 v50, v50, v54\n v_add_u32 v51, v51, v55\n"
#define BODY_DIFF \
  "v_add_u32 v40, v40, v45\n v_add_u32 v41, v41, v46\n v_add_u32 v42, v42, v47\n v_add_u32 v43, v43, v44\n" \
  "v_add_u32 v48, v48, v53\n v_add_u32 v49, v49, v54\n v_add_u32 v50, v50, v55\n v_add_u32 v51, v51, v52\n"
#define ALIGN_SAME \
  "v_alignbit_b32 v40, v40, v44, 7\n v_alignbit_b32 v41, v41, v45, 7\n v_alignbit_b32 v42, v42, v46, 7\n v_alignbit_b32 v43, v43, v47, 7\n" \
  "v_alignbit_b32 v48, v48, v52, 7\n v_alignbit_b32 v49, v49, v53, 7\n v_alignbit_b32 v50, v50, v54, 7\n v_alignbit_b32 v51, v51, v55, 7\n"
#define ALIGN_DIFF \
  "v_alignbit_b32 v40, v40, v45, 7\n v_alignbit_b32 v41, v41, v46, 7\n v_alignbit_b32 v42, v42, v47, 7\n v_alignbit_b32 v43, v43, v44, 7\n" \
  "v_alignbit_b32 v48, v48, v53, 7\n v_alignbit_b32 v49, v49, v54, 7\n v_alignbit_b32 v50, v50, v55, 7\n v_alignbit_b32 v51, v51, v52, 7\n"
#define ROT_SELF \
  "v_alignbit_b32 v40, v40, v40, 7\n v_alignbit_b32 v41, v41, v41, 7\n v_alignbit_b32 v42, v42, v42, 7\n v_alignbit_b32 v43, v43, v43, 7\n" \
  "v_alignbit_b32 v48, v48, v48, 7\n v_alignbit_b32 v49, v49, v49, 7\n v_alignbit_b32 v50, v50, v50, 7\n v_alignbit_b32 v51, v51, v51, 7\n"
#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"

#define K(NAME, BODY) \
__global__ __launch_bounds__(256) void k_##NAME(int iters, uint32_t *out, uint64_t *clk) { \
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    for (int i = 0; i < iters; ++i) asm volatile(BODY BODY BODY BODY ::: CLOB); \
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    uint32_t v; asm volatile("v_mov_b32 %0, v40" : "=v"(v) :: CLOB); out[blockIdx.x * 256 + threadIdx.x] = v; \
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; } \
}
K(add_same, BODY_SAME)
K(add_diff, BODY_DIFF)
K(align_same, ALIGN_SAME)
K(align_diff, ALIGN_DIFF)
K(rot_self, ROT_SELF)

int main() {
    uint32_t *out; uint64_t *clk, h[2];
    const int grid = 8192, iters = 2000;
    hipMalloc(&out, grid * 256 * 4); hipMalloc(&clk, 16);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
#define RUN(NAME) { \
    hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk); hipDeviceSynchronize(); \
    hipEventRecord(a); hipLaunchKernelGGL(k_##NAME, dim3(grid), dim3(256), 0, 0, iters, out, clk); hipEventRecord(b); \
    hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost); \
    double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9; double wi = (double)grid * 4 * iters * 32; \
    printf("%-12s %7.3f ms clk %.2f GHz cycles/wave-instr/SIMD %.2f\n", #NAME, ms, ghz, (ms * 1e-3 * ghz * 1e9) / (wi / 1024)); }
    RUN(add_same) RUN(add_diff) RUN(align_same) RUN(align_diff) RUN(rot_self)
    return 0;
}
