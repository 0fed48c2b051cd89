#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){fprintf(stderr,"%s: %s\n",#x,hipGetErrorString(e)); exit(2);} } while(0)
__global__ __launch_bounds__(256) void k_A_cur(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t m = blockIdx.x, t0_ = 1, t1_ = 2, t2_ = 3, t3_ = 4;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_alignbit_b32 %3, %3, %3, 16\nv_alignbit_b32 %7, %7, %7, 16\nv_alignbit_b32 %11, %11, %11, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_alignbit_b32 %3, %3, %3, 8\nv_alignbit_b32 %7, %7, %7, 8\nv_alignbit_b32 %11, %11, %11, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) ,"+v"(t0_),"+v"(t1_),"+v"(t2_),"+v"(t3_) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = t0_ ^ t1_ ^ t2_ ^ t3_; for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_B_sdwa16(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t m = blockIdx.x, t0_ = 1, t1_ = 2, t2_ = 3, t3_ = 4;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_add_u32 %2, %2, %16\nv_add_u32 %6, %6, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %14, %14, %19\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %16, %16, %0\nv_xor_b32 %17, %17, %4\nv_xor_b32 %18, %18, %8\nv_xor_b32 %19, %19, %12\nv_alignbit_b32 %3, %16, %16, 8\nv_alignbit_b32 %7, %17, %17, 8\nv_alignbit_b32 %11, %18, %18, 8\nv_alignbit_b32 %15, %19, %19, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) ,"+v"(t0_),"+v"(t1_),"+v"(t2_),"+v"(t3_) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = t0_ ^ t1_ ^ t2_ ^ t3_; for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_C_split_add3(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t m = blockIdx.x, t0_ = 1, t1_ = 2, t2_ = 3, t3_ = 4;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add_u32 %0, %0, %1\nv_add_u32 %4, %4, %5\nv_add_u32 %8, %8, %9\nv_add_u32 %12, %12, %13\nv_add_u32 %0, %0, %20\nv_add_u32 %4, %4, %20\nv_add_u32 %8, %8, %20\nv_add_u32 %12, %12, %20\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_alignbit_b32 %3, %3, %3, 16\nv_alignbit_b32 %7, %7, %7, 16\nv_alignbit_b32 %11, %11, %11, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add_u32 %0, %0, %1\nv_add_u32 %4, %4, %5\nv_add_u32 %8, %8, %9\nv_add_u32 %12, %12, %13\nv_add_u32 %0, %0, %20\nv_add_u32 %4, %4, %20\nv_add_u32 %8, %8, %20\nv_add_u32 %12, %12, %20\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_alignbit_b32 %3, %3, %3, 8\nv_alignbit_b32 %7, %7, %7, 8\nv_alignbit_b32 %11, %11, %11, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) ,"+v"(t0_),"+v"(t1_),"+v"(t2_),"+v"(t3_) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = t0_ ^ t1_ ^ t2_ ^ t3_; for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_D_sdwa16_split(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t m = blockIdx.x, t0_ = 1, t1_ = 2, t2_ = 3, t3_ = 4;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add_u32 %0, %0, %1\nv_add_u32 %4, %4, %5\nv_add_u32 %8, %8, %9\nv_add_u32 %12, %12, %13\nv_add_u32 %0, %0, %20\nv_add_u32 %4, %4, %20\nv_add_u32 %8, %8, %20\nv_add_u32 %12, %12, %20\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_add_u32 %2, %2, %16\nv_add_u32 %6, %6, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %14, %14, %19\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add_u32 %0, %0, %1\nv_add_u32 %4, %4, %5\nv_add_u32 %8, %8, %9\nv_add_u32 %12, %12, %13\nv_add_u32 %0, %0, %20\nv_add_u32 %4, %4, %20\nv_add_u32 %8, %8, %20\nv_add_u32 %12, %12, %20\nv_xor_b32 %16, %16, %0\nv_xor_b32 %17, %17, %4\nv_xor_b32 %18, %18, %8\nv_xor_b32 %19, %19, %12\nv_alignbit_b32 %3, %16, %16, 8\nv_alignbit_b32 %7, %17, %17, 8\nv_alignbit_b32 %11, %18, %18, 8\nv_alignbit_b32 %15, %19, %19, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) ,"+v"(t0_),"+v"(t1_),"+v"(t2_),"+v"(t3_) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = t0_ ^ t1_ ^ t2_ ^ t3_; for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_E_sdwa16_sdwa8(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t m = blockIdx.x, t0_ = 1, t1_ = 2, t2_ = 3, t3_ = 4;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_add_u32 %2, %2, %16\nv_add_u32 %6, %6, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %14, %14, %19\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %16, %16, %0\nv_xor_b32 %17, %17, %4\nv_xor_b32 %18, %18, %8\nv_xor_b32 %19, %19, %12\nv_lshrrev_b32 %3, 8, %16\nv_lshrrev_b32 %7, 8, %17\nv_lshrrev_b32 %11, 8, %18\nv_lshrrev_b32 %15, 8, %19\nv_mov_b32_sdwa %3, %16 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %7, %17 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %11, %18 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %15, %19 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) ,"+v"(t0_),"+v"(t1_),"+v"(t2_),"+v"(t3_) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = t0_ ^ t1_ ^ t2_ ^ t3_; for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
int main() { uint32_t *out; uint64_t *clk; CK(hipMalloc(&out, 8192*256*4)); CK(hipMalloc(&clk, 16));
hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); const uint32_t iters = 1024, grid = 8192;
{ hipLaunchKernelGGL(k_A_cur, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_cur, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 4 * 4; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-18s %8.3f ms  %8.2f G-func/ns  clk %.2f GHz  cyc/G/wave(per SIMD) %.2f\n", "A_cur", ms, gs / (ms * 1e-3) / 1e12, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ hipLaunchKernelGGL(k_B_sdwa16, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_B_sdwa16, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 4 * 4; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-18s %8.3f ms  %8.2f G-func/ns  clk %.2f GHz  cyc/G/wave(per SIMD) %.2f\n", "B_sdwa16", ms, gs / (ms * 1e-3) / 1e12, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ hipLaunchKernelGGL(k_C_split_add3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_C_split_add3, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 4 * 4; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-18s %8.3f ms  %8.2f G-func/ns  clk %.2f GHz  cyc/G/wave(per SIMD) %.2f\n", "C_split_add3", ms, gs / (ms * 1e-3) / 1e12, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ hipLaunchKernelGGL(k_D_sdwa16_split, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_D_sdwa16_split, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 4 * 4; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-18s %8.3f ms  %8.2f G-func/ns  clk %.2f GHz  cyc/G/wave(per SIMD) %.2f\n", "D_sdwa16_split", ms, gs / (ms * 1e-3) / 1e12, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ hipLaunchKernelGGL(k_E_sdwa16_sdwa8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_sdwa16_sdwa8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 4 * 4; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-18s %8.3f ms  %8.2f G-func/ns  clk %.2f GHz  cyc/G/wave(per SIMD) %.2f\n", "E_sdwa16_sdwa8", ms, gs / (ms * 1e-3) / 1e12, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
return 0; }