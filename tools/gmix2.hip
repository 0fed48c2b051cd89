#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){fprintf(stderr,"%s: %s\n",#x,hipGetErrorString(e)); exit(2);} } while(0)
__global__ __launch_bounds__(256) void k_A_ilp2(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[2]; for (int i = 0; i < 8; ++i) r[i] = threadIdx.x * 16 + i; for (int i = 0; i < 2; ++i) t[i] = i;
  uint32_t m = blockIdx.x;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 8; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %10\nv_add3_u32 %4, %4, %5, %10\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_alignbit_b32 %3, %3, %3, 16\nv_alignbit_b32 %7, %7, %7, 16\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_add3_u32 %0, %0, %1, %10\nv_add3_u32 %4, %4, %5, %10\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_alignbit_b32 %3, %3, %3, 8\nv_alignbit_b32 %7, %7, %7, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i]; for (int i = 0; i < 2; ++i) x ^= t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_A_ilp4(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16], t[4]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i; for (int i = 0; i < 4; ++i) t[i] = i;
  uint32_t m = blockIdx.x;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_alignbit_b32 %3, %3, %3, 16\nv_alignbit_b32 %7, %7, %7, 16\nv_alignbit_b32 %11, %11, %11, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_alignbit_b32 %3, %3, %3, 8\nv_alignbit_b32 %7, %7, %7, 8\nv_alignbit_b32 %11, %11, %11, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 16; ++i) x ^= r[i]; for (int i = 0; i < 4; ++i) x ^= t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_A_ilp8(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[32], t[8]; for (int i = 0; i < 32; ++i) r[i] = threadIdx.x * 16 + i; for (int i = 0; i < 8; ++i) t[i] = i;
  uint32_t m = blockIdx.x;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 2; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %40\nv_add3_u32 %4, %4, %5, %40\nv_add3_u32 %8, %8, %9, %40\nv_add3_u32 %12, %12, %13, %40\nv_add3_u32 %16, %16, %17, %40\nv_add3_u32 %20, %20, %21, %40\nv_add3_u32 %24, %24, %25, %40\nv_add3_u32 %28, %28, %29, %40\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_xor_b32 %19, %19, %16\nv_xor_b32 %23, %23, %20\nv_xor_b32 %27, %27, %24\nv_xor_b32 %31, %31, %28\nv_alignbit_b32 %3, %3, %3, 16\nv_alignbit_b32 %7, %7, %7, 16\nv_alignbit_b32 %11, %11, %11, 16\nv_alignbit_b32 %15, %15, %15, 16\nv_alignbit_b32 %19, %19, %19, 16\nv_alignbit_b32 %23, %23, %23, 16\nv_alignbit_b32 %27, %27, %27, 16\nv_alignbit_b32 %31, %31, %31, 16\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_add_u32 %18, %18, %19\nv_add_u32 %22, %22, %23\nv_add_u32 %26, %26, %27\nv_add_u32 %30, %30, %31\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_xor_b32 %17, %17, %18\nv_xor_b32 %21, %21, %22\nv_xor_b32 %25, %25, %26\nv_xor_b32 %29, %29, %30\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_alignbit_b32 %17, %17, %17, 12\nv_alignbit_b32 %21, %21, %21, 12\nv_alignbit_b32 %25, %25, %25, 12\nv_alignbit_b32 %29, %29, %29, 12\nv_add3_u32 %0, %0, %1, %40\nv_add3_u32 %4, %4, %5, %40\nv_add3_u32 %8, %8, %9, %40\nv_add3_u32 %12, %12, %13, %40\nv_add3_u32 %16, %16, %17, %40\nv_add3_u32 %20, %20, %21, %40\nv_add3_u32 %24, %24, %25, %40\nv_add3_u32 %28, %28, %29, %40\nv_xor_b32 %3, %3, %0\nv_xor_b32 %7, %7, %4\nv_xor_b32 %11, %11, %8\nv_xor_b32 %15, %15, %12\nv_xor_b32 %19, %19, %16\nv_xor_b32 %23, %23, %20\nv_xor_b32 %27, %27, %24\nv_xor_b32 %31, %31, %28\nv_alignbit_b32 %3, %3, %3, 8\nv_alignbit_b32 %7, %7, %7, 8\nv_alignbit_b32 %11, %11, %11, 8\nv_alignbit_b32 %15, %15, %15, 8\nv_alignbit_b32 %19, %19, %19, 8\nv_alignbit_b32 %23, %23, %23, 8\nv_alignbit_b32 %27, %27, %27, 8\nv_alignbit_b32 %31, %31, %31, 8\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_add_u32 %18, %18, %19\nv_add_u32 %22, %22, %23\nv_add_u32 %26, %26, %27\nv_add_u32 %30, %30, %31\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_xor_b32 %17, %17, %18\nv_xor_b32 %21, %21, %22\nv_xor_b32 %25, %25, %26\nv_xor_b32 %29, %29, %30\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %17, %17, %17, 7\nv_alignbit_b32 %21, %21, %21, 7\nv_alignbit_b32 %25, %25, %25, 7\nv_alignbit_b32 %29, %29, %29, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]),"+v"(r[16]),"+v"(r[17]),"+v"(r[18]),"+v"(r[19]),"+v"(r[20]),"+v"(r[21]),"+v"(r[22]),"+v"(r[23]),"+v"(r[24]),"+v"(r[25]),"+v"(r[26]),"+v"(r[27]),"+v"(r[28]),"+v"(r[29]),"+v"(r[30]),"+v"(r[31]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 32; ++i) x ^= r[i]; for (int i = 0; i < 8; ++i) x ^= t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_E_ilp2(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[8], t[2]; for (int i = 0; i < 8; ++i) r[i] = threadIdx.x * 16 + i; for (int i = 0; i < 2; ++i) t[i] = i;
  uint32_t m = blockIdx.x;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 8; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %10\nv_add3_u32 %4, %4, %5, %10\nv_xor_b32_sdwa %8, %3, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %9, %7, %4 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %8, %3, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %9, %7, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_add_u32 %2, %2, %8\nv_add_u32 %6, %6, %9\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_add3_u32 %0, %0, %1, %10\nv_add3_u32 %4, %4, %5, %10\nv_xor_b32 %8, %8, %0\nv_xor_b32 %9, %9, %4\nv_lshrrev_b32 %3, 8, %8\nv_lshrrev_b32 %7, 8, %9\nv_mov_b32_sdwa %3, %8 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %7, %9 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(t[0]),"+v"(t[1]) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 8; ++i) x ^= r[i]; for (int i = 0; i < 2; ++i) x ^= t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_E_ilp4(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16], t[4]; for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i; for (int i = 0; i < 4; ++i) t[i] = i;
  uint32_t m = blockIdx.x;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 4; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %16, %3, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %17, %7, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %18, %11, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %19, %15, %12 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_add_u32 %2, %2, %16\nv_add_u32 %6, %6, %17\nv_add_u32 %10, %10, %18\nv_add_u32 %14, %14, %19\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_add3_u32 %0, %0, %1, %20\nv_add3_u32 %4, %4, %5, %20\nv_add3_u32 %8, %8, %9, %20\nv_add3_u32 %12, %12, %13, %20\nv_xor_b32 %16, %16, %0\nv_xor_b32 %17, %17, %4\nv_xor_b32 %18, %18, %8\nv_xor_b32 %19, %19, %12\nv_lshrrev_b32 %3, 8, %16\nv_lshrrev_b32 %7, 8, %17\nv_lshrrev_b32 %11, 8, %18\nv_lshrrev_b32 %15, 8, %19\nv_mov_b32_sdwa %3, %16 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %7, %17 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %11, %18 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %15, %19 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 16; ++i) x ^= r[i]; for (int i = 0; i < 4; ++i) x ^= t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(256) void k_E_ilp8(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[32], t[8]; for (int i = 0; i < 32; ++i) r[i] = threadIdx.x * 16 + i; for (int i = 0; i < 8; ++i) t[i] = i;
  uint32_t m = blockIdx.x;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t it = 0; it < iters; ++it) {
    #pragma unroll
    for (int u = 0; u < 2; ++u)
    asm volatile("v_add3_u32 %0, %0, %1, %40\nv_add3_u32 %4, %4, %5, %40\nv_add3_u32 %8, %8, %9, %40\nv_add3_u32 %12, %12, %13, %40\nv_add3_u32 %16, %16, %17, %40\nv_add3_u32 %20, %20, %21, %40\nv_add3_u32 %24, %24, %25, %40\nv_add3_u32 %28, %28, %29, %40\nv_xor_b32_sdwa %32, %3, %0 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %33, %7, %4 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %34, %11, %8 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %35, %15, %12 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %36, %19, %16 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %37, %23, %20 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %38, %27, %24 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %39, %31, %28 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\nv_xor_b32_sdwa %32, %3, %0 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %33, %7, %4 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %34, %11, %8 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %35, %15, %12 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %36, %19, %16 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %37, %23, %20 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %38, %27, %24 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_xor_b32_sdwa %39, %31, %28 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\nv_add_u32 %2, %2, %32\nv_add_u32 %6, %6, %33\nv_add_u32 %10, %10, %34\nv_add_u32 %14, %14, %35\nv_add_u32 %18, %18, %36\nv_add_u32 %22, %22, %37\nv_add_u32 %26, %26, %38\nv_add_u32 %30, %30, %39\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_xor_b32 %17, %17, %18\nv_xor_b32 %21, %21, %22\nv_xor_b32 %25, %25, %26\nv_xor_b32 %29, %29, %30\nv_alignbit_b32 %1, %1, %1, 12\nv_alignbit_b32 %5, %5, %5, 12\nv_alignbit_b32 %9, %9, %9, 12\nv_alignbit_b32 %13, %13, %13, 12\nv_alignbit_b32 %17, %17, %17, 12\nv_alignbit_b32 %21, %21, %21, 12\nv_alignbit_b32 %25, %25, %25, 12\nv_alignbit_b32 %29, %29, %29, 12\nv_add3_u32 %0, %0, %1, %40\nv_add3_u32 %4, %4, %5, %40\nv_add3_u32 %8, %8, %9, %40\nv_add3_u32 %12, %12, %13, %40\nv_add3_u32 %16, %16, %17, %40\nv_add3_u32 %20, %20, %21, %40\nv_add3_u32 %24, %24, %25, %40\nv_add3_u32 %28, %28, %29, %40\nv_xor_b32 %32, %32, %0\nv_xor_b32 %33, %33, %4\nv_xor_b32 %34, %34, %8\nv_xor_b32 %35, %35, %12\nv_xor_b32 %36, %36, %16\nv_xor_b32 %37, %37, %20\nv_xor_b32 %38, %38, %24\nv_xor_b32 %39, %39, %28\nv_lshrrev_b32 %3, 8, %32\nv_lshrrev_b32 %7, 8, %33\nv_lshrrev_b32 %11, 8, %34\nv_lshrrev_b32 %15, 8, %35\nv_lshrrev_b32 %19, 8, %36\nv_lshrrev_b32 %23, 8, %37\nv_lshrrev_b32 %27, 8, %38\nv_lshrrev_b32 %31, 8, %39\nv_mov_b32_sdwa %3, %32 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %7, %33 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %11, %34 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %15, %35 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %19, %36 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %23, %37 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %27, %38 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_mov_b32_sdwa %31, %39 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0\nv_add_u32 %2, %2, %3\nv_add_u32 %6, %6, %7\nv_add_u32 %10, %10, %11\nv_add_u32 %14, %14, %15\nv_add_u32 %18, %18, %19\nv_add_u32 %22, %22, %23\nv_add_u32 %26, %26, %27\nv_add_u32 %30, %30, %31\nv_xor_b32 %1, %1, %2\nv_xor_b32 %5, %5, %6\nv_xor_b32 %9, %9, %10\nv_xor_b32 %13, %13, %14\nv_xor_b32 %17, %17, %18\nv_xor_b32 %21, %21, %22\nv_xor_b32 %25, %25, %26\nv_xor_b32 %29, %29, %30\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %17, %17, %17, 7\nv_alignbit_b32 %21, %21, %21, 7\nv_alignbit_b32 %25, %25, %25, 7\nv_alignbit_b32 %29, %29, %29, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]),"+v"(r[16]),"+v"(r[17]),"+v"(r[18]),"+v"(r[19]),"+v"(r[20]),"+v"(r[21]),"+v"(r[22]),"+v"(r[23]),"+v"(r[24]),"+v"(r[25]),"+v"(r[26]),"+v"(r[27]),"+v"(r[28]),"+v"(r[29]),"+v"(r[30]),"+v"(r[31]),"+v"(t[0]),"+v"(t[1]),"+v"(t[2]),"+v"(t[3]),"+v"(t[4]),"+v"(t[5]),"+v"(t[6]),"+v"(t[7]) : "v"(m));
  }
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0; for (int i = 0; i < 32; ++i) x ^= r[i]; for (int i = 0; i < 8; ++i) x ^= t[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
int main() { uint32_t *out; uint64_t *clk; CK(hipMalloc(&out, 8192*256*4)); CK(hipMalloc(&clk, 16));
hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); const uint32_t iters = 1024;
{ const uint32_t grid = 4096; hipLaunchKernelGGL(k_A_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp2", 16, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 8192; hipLaunchKernelGGL(k_A_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp2", 32, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 2048; hipLaunchKernelGGL(k_A_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp2", 8, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 4096; hipLaunchKernelGGL(k_A_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp4", 16, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 8192; hipLaunchKernelGGL(k_A_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp4", 32, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 2048; hipLaunchKernelGGL(k_A_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp4", 8, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 4096; hipLaunchKernelGGL(k_A_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp8", 16, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 8192; hipLaunchKernelGGL(k_A_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp8", 32, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 2048; hipLaunchKernelGGL(k_A_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_A_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "A_ilp8", 8, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 4096; hipLaunchKernelGGL(k_E_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp2", 16, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 8192; hipLaunchKernelGGL(k_E_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp2", 32, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 2048; hipLaunchKernelGGL(k_E_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp2, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp2", 8, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 4096; hipLaunchKernelGGL(k_E_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp4", 16, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 8192; hipLaunchKernelGGL(k_E_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp4", 32, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 2048; hipLaunchKernelGGL(k_E_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp4, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp4", 8, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 4096; hipLaunchKernelGGL(k_E_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp8", 16, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 8192; hipLaunchKernelGGL(k_E_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp8", 32, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
{ const uint32_t grid = 2048; hipLaunchKernelGGL(k_E_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(k_E_ilp8, dim3(grid), dim3(256), 0, 0, out, iters, clk); CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1)); uint64_t c[2]; CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
  double gs = double(grid) * 256 * iters * 16; double ghz = double(c[0]) / (double(c[1]) * 10.0);
  printf("%-10s waves/SIMD %d  %8.3f ms  clk %.2f GHz  cyc/G/wave %.2f\n", "E_ilp8", 8, ms, ghz, (ms*1e-3*ghz*1e9) * 1024.0 / (gs/64)); }
return 0; }