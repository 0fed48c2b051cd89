#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){fprintf(stderr,"%s: %s\n",#x,hipGetErrorString(e)); exit(2);} } while(0)
__global__ __launch_bounds__(256) void k_xor(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_alignbit(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_add3(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %0, %16, %0\nv_add3_u32 %1, %1, %16, %1\nv_add3_u32 %2, %2, %16, %2\nv_add3_u32 %3, %3, %16, %3\nv_add3_u32 %4, %4, %16, %4\nv_add3_u32 %5, %5, %16, %5\nv_add3_u32 %6, %6, %16, %6\nv_add3_u32 %7, %7, %16, %7\nv_add3_u32 %0, %0, %16, %0\nv_add3_u32 %1, %1, %16, %1\nv_add3_u32 %2, %2, %16, %2\nv_add3_u32 %3, %3, %16, %3\nv_add3_u32 %4, %4, %16, %4\nv_add3_u32 %5, %5, %16, %5\nv_add3_u32 %6, %6, %16, %6\nv_add3_u32 %7, %7, %16, %7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_sdwa_xor_hi(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_xor_b32_sdwa %8, %0, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %9, %1, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %10, %2, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %11, %3, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %12, %4, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %13, %5, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %14, %6, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %15, %7, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %8, %0, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %9, %1, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %10, %2, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %11, %3, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %12, %4, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %13, %5, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %14, %6, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %15, %7, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_sdwa_xor_lo_pres(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_xor_b32_sdwa %0, %8, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %1, %9, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %2, %10, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %3, %11, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %4, %12, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %5, %13, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %6, %14, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %7, %15, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %0, %8, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %1, %9, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %2, %10, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %3, %11, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %4, %12, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %5, %13, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %6, %14, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %7, %15, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_xor_alignbit(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_add_add3(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_add3_u32 %0, %0, %16, %0\nv_add3_u32 %1, %1, %16, %1\nv_add3_u32 %2, %2, %16, %2\nv_add3_u32 %3, %3, %16, %3\nv_add3_u32 %4, %4, %16, %4\nv_add3_u32 %5, %5, %16, %5\nv_add3_u32 %6, %6, %16, %6\nv_add3_u32 %7, %7, %16, %7\nv_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_add3_u32 %0, %0, %16, %0\nv_add3_u32 %1, %1, %16, %1\nv_add3_u32 %2, %2, %16, %2\nv_add3_u32 %3, %3, %16, %3\nv_add3_u32 %4, %4, %16, %4\nv_add3_u32 %5, %5, %16, %5\nv_add3_u32 %6, %6, %16, %6\nv_add3_u32 %7, %7, %16, %7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_xor_xor_alignbit(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_add_xor(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_add_u32 %0, %0, %16\nv_add_u32 %1, %1, %16\nv_add_u32 %2, %2, %16\nv_add_u32 %3, %3, %16\nv_add_u32 %4, %4, %16\nv_add_u32 %5, %5, %16\nv_add_u32 %6, %6, %16\nv_add_u32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_alignbit_alignbit_xor_xor(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %0, %0, %0, 9\nv_alignbit_b32 %1, %1, %1, 9\nv_alignbit_b32 %2, %2, %2, 9\nv_alignbit_b32 %3, %3, %3, 9\nv_alignbit_b32 %4, %4, %4, 9\nv_alignbit_b32 %5, %5, %5, 9\nv_alignbit_b32 %6, %6, %6, 9\nv_alignbit_b32 %7, %7, %7, 9\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %0, %0, %0, 9\nv_alignbit_b32 %1, %1, %1, 9\nv_alignbit_b32 %2, %2, %2, 9\nv_alignbit_b32 %3, %3, %3, 9\nv_alignbit_b32 %4, %4, %4, 9\nv_alignbit_b32 %5, %5, %5, 9\nv_alignbit_b32 %6, %6, %6, 9\nv_alignbit_b32 %7, %7, %7, 9\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_mov_sdwa_byte3(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_mov_b32_sdwa %0, %8 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %1, %9 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %2, %10 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %3, %11 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %4, %12 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %5, %13 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %6, %14 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %7, %15 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %0, %8 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %1, %9 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %2, %10 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %3, %11 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %4, %12 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %5, %13 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %6, %14 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %7, %15 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_lshr(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_lshrrev_b32 %0, 8, %0\nv_lshrrev_b32 %1, 8, %1\nv_lshrrev_b32 %2, 8, %2\nv_lshrrev_b32 %3, 8, %3\nv_lshrrev_b32 %4, 8, %4\nv_lshrrev_b32 %5, 8, %5\nv_lshrrev_b32 %6, 8, %6\nv_lshrrev_b32 %7, 8, %7\nv_lshrrev_b32 %0, 8, %0\nv_lshrrev_b32 %1, 8, %1\nv_lshrrev_b32 %2, 8, %2\nv_lshrrev_b32 %3, 8, %3\nv_lshrrev_b32 %4, 8, %4\nv_lshrrev_b32 %5, 8, %5\nv_lshrrev_b32 %6, 8, %6\nv_lshrrev_b32 %7, 8, %7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_perm(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_perm_b32 %0, %0, %0, %16\nv_perm_b32 %1, %1, %1, %16\nv_perm_b32 %2, %2, %2, %16\nv_perm_b32 %3, %3, %3, %16\nv_perm_b32 %4, %4, %4, %16\nv_perm_b32 %5, %5, %5, %16\nv_perm_b32 %6, %6, %6, %16\nv_perm_b32 %7, %7, %7, %16\nv_perm_b32 %0, %0, %0, %16\nv_perm_b32 %1, %1, %1, %16\nv_perm_b32 %2, %2, %2, %16\nv_perm_b32 %3, %3, %3, %16\nv_perm_b32 %4, %4, %4, %16\nv_perm_b32 %5, %5, %5, %16\nv_perm_b32 %6, %6, %6, %16\nv_perm_b32 %7, %7, %7, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_xor_3reg(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_xor_b32 %0, %8, %16\nv_xor_b32 %1, %9, %16\nv_xor_b32 %2, %10, %16\nv_xor_b32 %3, %11, %16\nv_xor_b32 %4, %12, %16\nv_xor_b32 %5, %13, %16\nv_xor_b32 %6, %14, %16\nv_xor_b32 %7, %15, %16\nv_xor_b32 %0, %8, %16\nv_xor_b32 %1, %9, %16\nv_xor_b32 %2, %10, %16\nv_xor_b32 %3, %11, %16\nv_xor_b32 %4, %12, %16\nv_xor_b32 %5, %13, %16\nv_xor_b32 %6, %14, %16\nv_xor_b32 %7, %15, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_add3_3reg(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %8, %16, %0\nv_add3_u32 %1, %9, %16, %1\nv_add3_u32 %2, %10, %16, %2\nv_add3_u32 %3, %11, %16, %3\nv_add3_u32 %4, %12, %16, %4\nv_add3_u32 %5, %13, %16, %5\nv_add3_u32 %6, %14, %16, %6\nv_add3_u32 %7, %15, %16, %7\nv_add3_u32 %0, %8, %16, %0\nv_add3_u32 %1, %9, %16, %1\nv_add3_u32 %2, %10, %16, %2\nv_add3_u32 %3, %11, %16, %3\nv_add3_u32 %4, %12, %16, %4\nv_add3_u32 %5, %13, %16, %5\nv_add3_u32 %6, %14, %16, %6\nv_add3_u32 %7, %15, %16, %7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_alignbit_2reg(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[8]; for (int i = 0; i < 8; ++i) { r[i] = threadIdx.x * 16 + i; t[i] = i * 77; }
  uint32_t k = blockIdx.x | 1;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_alignbit_b32 %0, %8, %8, 7\nv_alignbit_b32 %1, %9, %9, 7\nv_alignbit_b32 %2, %10, %10, 7\nv_alignbit_b32 %3, %11, %11, 7\nv_alignbit_b32 %4, %12, %12, 7\nv_alignbit_b32 %5, %13, %13, 7\nv_alignbit_b32 %6, %14, %14, 7\nv_alignbit_b32 %7, %15, %15, 7\nv_alignbit_b32 %0, %8, %8, 7\nv_alignbit_b32 %1, %9, %9, 7\nv_alignbit_b32 %2, %10, %10, 7\nv_alignbit_b32 %3, %11, %11, 7\nv_alignbit_b32 %4, %12, %12, 7\nv_alignbit_b32 %5, %13, %13, 7\nv_alignbit_b32 %6, %14, %14, 7\nv_alignbit_b32 %7, %15, %15, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(k));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i] ^ t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
int main() { uint32_t *out; uint64_t *clk; CK(hipMalloc(&out, 8192*256*4)); CK(hipMalloc(&clk, 16));
hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); const uint32_t iters = 512, grid = 8192;
{ hipLaunchKernelGGL(k_xor, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_xor, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "xor", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_alignbit, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_alignbit, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "alignbit", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_add3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_add3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "add3", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_sdwa_xor_hi, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_sdwa_xor_hi, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "sdwa_xor_hi", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_sdwa_xor_lo_pres, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_sdwa_xor_lo_pres, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "sdwa_xor_lo_pres", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_xor_alignbit, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_xor_alignbit, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 32; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "xor+alignbit", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_add_add3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_add_add3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 32; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "add+add3", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_xor_xor_alignbit, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_xor_xor_alignbit, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 48; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "xor+xor+alignbit", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_add_xor, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_add_xor, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 32; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "add+xor", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_alignbit_alignbit_xor_xor, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_alignbit_alignbit_xor_xor, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 64; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "alignbit+alignbit+xor+xor", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_mov_sdwa_byte3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_mov_sdwa_byte3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "mov_sdwa_byte3", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_lshr, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_lshr, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "lshr", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_perm, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_perm, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "perm", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_xor_3reg, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_xor_3reg, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "xor_3reg", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_add3_3reg, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_add3_3reg, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "add3_3reg", ghz, cyc_per_instr); }
{ hipLaunchKernelGGL(k_alignbit_2reg, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_alignbit_2reg, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double wave_instr = double(grid) * 4 * iters * 4 * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  double cyc_per_instr = (ms * 1e-3 * ghz * 1e9) * 1024.0 / wave_instr;
  printf("%-28s clk %.2f GHz  cycles/wave-instr %.2f\n", "alignbit_2reg", ghz, cyc_per_instr); }
return 0; }