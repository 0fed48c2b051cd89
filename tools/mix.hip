#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__device__ __forceinline__ void body_xor(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %8, %8, %16\nv_xor_b32 %9, %9, %16\nv_xor_b32 %10, %10, %16\nv_xor_b32 %11, %11, %16\nv_xor_b32 %12, %12, %16\nv_xor_b32 %13, %13, %16\nv_xor_b32 %14, %14, %16\nv_xor_b32 %15, %15, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %8, %8, %16\nv_xor_b32 %9, %9, %16\nv_xor_b32 %10, %10, %16\nv_xor_b32 %11, %11, %16\nv_xor_b32 %12, %12, %16\nv_xor_b32 %13, %13, %16\nv_xor_b32 %14, %14, %16\nv_xor_b32 %15, %15, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %8, %8, %16\nv_xor_b32 %9, %9, %16\nv_xor_b32 %10, %10, %16\nv_xor_b32 %11, %11, %16\nv_xor_b32 %12, %12, %16\nv_xor_b32 %13, %13, %16\nv_xor_b32 %14, %14, %16\nv_xor_b32 %15, %15, %16\nv_xor_b32 %0, %0, %16\nv_xor_b32 %1, %1, %16\nv_xor_b32 %2, %2, %16\nv_xor_b32 %3, %3, %16\nv_xor_b32 %4, %4, %16\nv_xor_b32 %5, %5, %16\nv_xor_b32 %6, %6, %16\nv_xor_b32 %7, %7, %16\nv_xor_b32 %8, %8, %16\nv_xor_b32 %9, %9, %16\nv_xor_b32 %10, %10, %16\nv_xor_b32 %11, %11, %16\nv_xor_b32 %12, %12, %16\nv_xor_b32 %13, %13, %16\nv_xor_b32 %14, %14, %16\nv_xor_b32 %15, %15, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_xor(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_xor(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_alignbit(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %8, %8, %8, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %10, %10, %10, 7\nv_alignbit_b32 %11, %11, %11, 7\nv_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %8, %8, %8, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %10, %10, %10, 7\nv_alignbit_b32 %11, %11, %11, 7\nv_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %8, %8, %8, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %10, %10, %10, 7\nv_alignbit_b32 %11, %11, %11, 7\nv_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7\nv_alignbit_b32 %0, %0, %0, 7\nv_alignbit_b32 %1, %1, %1, 7\nv_alignbit_b32 %2, %2, %2, 7\nv_alignbit_b32 %3, %3, %3, 7\nv_alignbit_b32 %4, %4, %4, 7\nv_alignbit_b32 %5, %5, %5, 7\nv_alignbit_b32 %6, %6, %6, 7\nv_alignbit_b32 %7, %7, %7, 7\nv_alignbit_b32 %8, %8, %8, 7\nv_alignbit_b32 %9, %9, %9, 7\nv_alignbit_b32 %10, %10, %10, 7\nv_alignbit_b32 %11, %11, %11, 7\nv_alignbit_b32 %12, %12, %12, 7\nv_alignbit_b32 %13, %13, %13, 7\nv_alignbit_b32 %14, %14, %14, 7\nv_alignbit_b32 %15, %15, %15, 7" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_alignbit(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_alignbit(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshr1(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshrrev_b32 %0, 1, %0\nv_lshrrev_b32 %1, 1, %1\nv_lshrrev_b32 %2, 1, %2\nv_lshrrev_b32 %3, 1, %3\nv_lshrrev_b32 %4, 1, %4\nv_lshrrev_b32 %5, 1, %5\nv_lshrrev_b32 %6, 1, %6\nv_lshrrev_b32 %7, 1, %7\nv_lshrrev_b32 %8, 1, %8\nv_lshrrev_b32 %9, 1, %9\nv_lshrrev_b32 %10, 1, %10\nv_lshrrev_b32 %11, 1, %11\nv_lshrrev_b32 %12, 1, %12\nv_lshrrev_b32 %13, 1, %13\nv_lshrrev_b32 %14, 1, %14\nv_lshrrev_b32 %15, 1, %15\nv_lshrrev_b32 %0, 1, %0\nv_lshrrev_b32 %1, 1, %1\nv_lshrrev_b32 %2, 1, %2\nv_lshrrev_b32 %3, 1, %3\nv_lshrrev_b32 %4, 1, %4\nv_lshrrev_b32 %5, 1, %5\nv_lshrrev_b32 %6, 1, %6\nv_lshrrev_b32 %7, 1, %7\nv_lshrrev_b32 %8, 1, %8\nv_lshrrev_b32 %9, 1, %9\nv_lshrrev_b32 %10, 1, %10\nv_lshrrev_b32 %11, 1, %11\nv_lshrrev_b32 %12, 1, %12\nv_lshrrev_b32 %13, 1, %13\nv_lshrrev_b32 %14, 1, %14\nv_lshrrev_b32 %15, 1, %15\nv_lshrrev_b32 %0, 1, %0\nv_lshrrev_b32 %1, 1, %1\nv_lshrrev_b32 %2, 1, %2\nv_lshrrev_b32 %3, 1, %3\nv_lshrrev_b32 %4, 1, %4\nv_lshrrev_b32 %5, 1, %5\nv_lshrrev_b32 %6, 1, %6\nv_lshrrev_b32 %7, 1, %7\nv_lshrrev_b32 %8, 1, %8\nv_lshrrev_b32 %9, 1, %9\nv_lshrrev_b32 %10, 1, %10\nv_lshrrev_b32 %11, 1, %11\nv_lshrrev_b32 %12, 1, %12\nv_lshrrev_b32 %13, 1, %13\nv_lshrrev_b32 %14, 1, %14\nv_lshrrev_b32 %15, 1, %15\nv_lshrrev_b32 %0, 1, %0\nv_lshrrev_b32 %1, 1, %1\nv_lshrrev_b32 %2, 1, %2\nv_lshrrev_b32 %3, 1, %3\nv_lshrrev_b32 %4, 1, %4\nv_lshrrev_b32 %5, 1, %5\nv_lshrrev_b32 %6, 1, %6\nv_lshrrev_b32 %7, 1, %7\nv_lshrrev_b32 %8, 1, %8\nv_lshrrev_b32 %9, 1, %9\nv_lshrrev_b32 %10, 1, %10\nv_lshrrev_b32 %11, 1, %11\nv_lshrrev_b32 %12, 1, %12\nv_lshrrev_b32 %13, 1, %13\nv_lshrrev_b32 %14, 1, %14\nv_lshrrev_b32 %15, 1, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshr1(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshr1(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshr7(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshrrev_b32 %0, 7, %0\nv_lshrrev_b32 %1, 7, %1\nv_lshrrev_b32 %2, 7, %2\nv_lshrrev_b32 %3, 7, %3\nv_lshrrev_b32 %4, 7, %4\nv_lshrrev_b32 %5, 7, %5\nv_lshrrev_b32 %6, 7, %6\nv_lshrrev_b32 %7, 7, %7\nv_lshrrev_b32 %8, 7, %8\nv_lshrrev_b32 %9, 7, %9\nv_lshrrev_b32 %10, 7, %10\nv_lshrrev_b32 %11, 7, %11\nv_lshrrev_b32 %12, 7, %12\nv_lshrrev_b32 %13, 7, %13\nv_lshrrev_b32 %14, 7, %14\nv_lshrrev_b32 %15, 7, %15\nv_lshrrev_b32 %0, 7, %0\nv_lshrrev_b32 %1, 7, %1\nv_lshrrev_b32 %2, 7, %2\nv_lshrrev_b32 %3, 7, %3\nv_lshrrev_b32 %4, 7, %4\nv_lshrrev_b32 %5, 7, %5\nv_lshrrev_b32 %6, 7, %6\nv_lshrrev_b32 %7, 7, %7\nv_lshrrev_b32 %8, 7, %8\nv_lshrrev_b32 %9, 7, %9\nv_lshrrev_b32 %10, 7, %10\nv_lshrrev_b32 %11, 7, %11\nv_lshrrev_b32 %12, 7, %12\nv_lshrrev_b32 %13, 7, %13\nv_lshrrev_b32 %14, 7, %14\nv_lshrrev_b32 %15, 7, %15\nv_lshrrev_b32 %0, 7, %0\nv_lshrrev_b32 %1, 7, %1\nv_lshrrev_b32 %2, 7, %2\nv_lshrrev_b32 %3, 7, %3\nv_lshrrev_b32 %4, 7, %4\nv_lshrrev_b32 %5, 7, %5\nv_lshrrev_b32 %6, 7, %6\nv_lshrrev_b32 %7, 7, %7\nv_lshrrev_b32 %8, 7, %8\nv_lshrrev_b32 %9, 7, %9\nv_lshrrev_b32 %10, 7, %10\nv_lshrrev_b32 %11, 7, %11\nv_lshrrev_b32 %12, 7, %12\nv_lshrrev_b32 %13, 7, %13\nv_lshrrev_b32 %14, 7, %14\nv_lshrrev_b32 %15, 7, %15\nv_lshrrev_b32 %0, 7, %0\nv_lshrrev_b32 %1, 7, %1\nv_lshrrev_b32 %2, 7, %2\nv_lshrrev_b32 %3, 7, %3\nv_lshrrev_b32 %4, 7, %4\nv_lshrrev_b32 %5, 7, %5\nv_lshrrev_b32 %6, 7, %6\nv_lshrrev_b32 %7, 7, %7\nv_lshrrev_b32 %8, 7, %8\nv_lshrrev_b32 %9, 7, %9\nv_lshrrev_b32 %10, 7, %10\nv_lshrrev_b32 %11, 7, %11\nv_lshrrev_b32 %12, 7, %12\nv_lshrrev_b32 %13, 7, %13\nv_lshrrev_b32 %14, 7, %14\nv_lshrrev_b32 %15, 7, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshr7(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshr7(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshr16(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshrrev_b32 %0, 16, %0\nv_lshrrev_b32 %1, 16, %1\nv_lshrrev_b32 %2, 16, %2\nv_lshrrev_b32 %3, 16, %3\nv_lshrrev_b32 %4, 16, %4\nv_lshrrev_b32 %5, 16, %5\nv_lshrrev_b32 %6, 16, %6\nv_lshrrev_b32 %7, 16, %7\nv_lshrrev_b32 %8, 16, %8\nv_lshrrev_b32 %9, 16, %9\nv_lshrrev_b32 %10, 16, %10\nv_lshrrev_b32 %11, 16, %11\nv_lshrrev_b32 %12, 16, %12\nv_lshrrev_b32 %13, 16, %13\nv_lshrrev_b32 %14, 16, %14\nv_lshrrev_b32 %15, 16, %15\nv_lshrrev_b32 %0, 16, %0\nv_lshrrev_b32 %1, 16, %1\nv_lshrrev_b32 %2, 16, %2\nv_lshrrev_b32 %3, 16, %3\nv_lshrrev_b32 %4, 16, %4\nv_lshrrev_b32 %5, 16, %5\nv_lshrrev_b32 %6, 16, %6\nv_lshrrev_b32 %7, 16, %7\nv_lshrrev_b32 %8, 16, %8\nv_lshrrev_b32 %9, 16, %9\nv_lshrrev_b32 %10, 16, %10\nv_lshrrev_b32 %11, 16, %11\nv_lshrrev_b32 %12, 16, %12\nv_lshrrev_b32 %13, 16, %13\nv_lshrrev_b32 %14, 16, %14\nv_lshrrev_b32 %15, 16, %15\nv_lshrrev_b32 %0, 16, %0\nv_lshrrev_b32 %1, 16, %1\nv_lshrrev_b32 %2, 16, %2\nv_lshrrev_b32 %3, 16, %3\nv_lshrrev_b32 %4, 16, %4\nv_lshrrev_b32 %5, 16, %5\nv_lshrrev_b32 %6, 16, %6\nv_lshrrev_b32 %7, 16, %7\nv_lshrrev_b32 %8, 16, %8\nv_lshrrev_b32 %9, 16, %9\nv_lshrrev_b32 %10, 16, %10\nv_lshrrev_b32 %11, 16, %11\nv_lshrrev_b32 %12, 16, %12\nv_lshrrev_b32 %13, 16, %13\nv_lshrrev_b32 %14, 16, %14\nv_lshrrev_b32 %15, 16, %15\nv_lshrrev_b32 %0, 16, %0\nv_lshrrev_b32 %1, 16, %1\nv_lshrrev_b32 %2, 16, %2\nv_lshrrev_b32 %3, 16, %3\nv_lshrrev_b32 %4, 16, %4\nv_lshrrev_b32 %5, 16, %5\nv_lshrrev_b32 %6, 16, %6\nv_lshrrev_b32 %7, 16, %7\nv_lshrrev_b32 %8, 16, %8\nv_lshrrev_b32 %9, 16, %9\nv_lshrrev_b32 %10, 16, %10\nv_lshrrev_b32 %11, 16, %11\nv_lshrrev_b32 %12, 16, %12\nv_lshrrev_b32 %13, 16, %13\nv_lshrrev_b32 %14, 16, %14\nv_lshrrev_b32 %15, 16, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshr16(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshr16(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshl1(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshlrev_b32 %0, 1, %0\nv_lshlrev_b32 %1, 1, %1\nv_lshlrev_b32 %2, 1, %2\nv_lshlrev_b32 %3, 1, %3\nv_lshlrev_b32 %4, 1, %4\nv_lshlrev_b32 %5, 1, %5\nv_lshlrev_b32 %6, 1, %6\nv_lshlrev_b32 %7, 1, %7\nv_lshlrev_b32 %8, 1, %8\nv_lshlrev_b32 %9, 1, %9\nv_lshlrev_b32 %10, 1, %10\nv_lshlrev_b32 %11, 1, %11\nv_lshlrev_b32 %12, 1, %12\nv_lshlrev_b32 %13, 1, %13\nv_lshlrev_b32 %14, 1, %14\nv_lshlrev_b32 %15, 1, %15\nv_lshlrev_b32 %0, 1, %0\nv_lshlrev_b32 %1, 1, %1\nv_lshlrev_b32 %2, 1, %2\nv_lshlrev_b32 %3, 1, %3\nv_lshlrev_b32 %4, 1, %4\nv_lshlrev_b32 %5, 1, %5\nv_lshlrev_b32 %6, 1, %6\nv_lshlrev_b32 %7, 1, %7\nv_lshlrev_b32 %8, 1, %8\nv_lshlrev_b32 %9, 1, %9\nv_lshlrev_b32 %10, 1, %10\nv_lshlrev_b32 %11, 1, %11\nv_lshlrev_b32 %12, 1, %12\nv_lshlrev_b32 %13, 1, %13\nv_lshlrev_b32 %14, 1, %14\nv_lshlrev_b32 %15, 1, %15\nv_lshlrev_b32 %0, 1, %0\nv_lshlrev_b32 %1, 1, %1\nv_lshlrev_b32 %2, 1, %2\nv_lshlrev_b32 %3, 1, %3\nv_lshlrev_b32 %4, 1, %4\nv_lshlrev_b32 %5, 1, %5\nv_lshlrev_b32 %6, 1, %6\nv_lshlrev_b32 %7, 1, %7\nv_lshlrev_b32 %8, 1, %8\nv_lshlrev_b32 %9, 1, %9\nv_lshlrev_b32 %10, 1, %10\nv_lshlrev_b32 %11, 1, %11\nv_lshlrev_b32 %12, 1, %12\nv_lshlrev_b32 %13, 1, %13\nv_lshlrev_b32 %14, 1, %14\nv_lshlrev_b32 %15, 1, %15\nv_lshlrev_b32 %0, 1, %0\nv_lshlrev_b32 %1, 1, %1\nv_lshlrev_b32 %2, 1, %2\nv_lshlrev_b32 %3, 1, %3\nv_lshlrev_b32 %4, 1, %4\nv_lshlrev_b32 %5, 1, %5\nv_lshlrev_b32 %6, 1, %6\nv_lshlrev_b32 %7, 1, %7\nv_lshlrev_b32 %8, 1, %8\nv_lshlrev_b32 %9, 1, %9\nv_lshlrev_b32 %10, 1, %10\nv_lshlrev_b32 %11, 1, %11\nv_lshlrev_b32 %12, 1, %12\nv_lshlrev_b32 %13, 1, %13\nv_lshlrev_b32 %14, 1, %14\nv_lshlrev_b32 %15, 1, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshl1(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshl1(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshl7(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %8, 7, %8\nv_lshlrev_b32 %9, 7, %9\nv_lshlrev_b32 %10, 7, %10\nv_lshlrev_b32 %11, 7, %11\nv_lshlrev_b32 %12, 7, %12\nv_lshlrev_b32 %13, 7, %13\nv_lshlrev_b32 %14, 7, %14\nv_lshlrev_b32 %15, 7, %15\nv_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %8, 7, %8\nv_lshlrev_b32 %9, 7, %9\nv_lshlrev_b32 %10, 7, %10\nv_lshlrev_b32 %11, 7, %11\nv_lshlrev_b32 %12, 7, %12\nv_lshlrev_b32 %13, 7, %13\nv_lshlrev_b32 %14, 7, %14\nv_lshlrev_b32 %15, 7, %15\nv_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %8, 7, %8\nv_lshlrev_b32 %9, 7, %9\nv_lshlrev_b32 %10, 7, %10\nv_lshlrev_b32 %11, 7, %11\nv_lshlrev_b32 %12, 7, %12\nv_lshlrev_b32 %13, 7, %13\nv_lshlrev_b32 %14, 7, %14\nv_lshlrev_b32 %15, 7, %15\nv_lshlrev_b32 %0, 7, %0\nv_lshlrev_b32 %1, 7, %1\nv_lshlrev_b32 %2, 7, %2\nv_lshlrev_b32 %3, 7, %3\nv_lshlrev_b32 %4, 7, %4\nv_lshlrev_b32 %5, 7, %5\nv_lshlrev_b32 %6, 7, %6\nv_lshlrev_b32 %7, 7, %7\nv_lshlrev_b32 %8, 7, %8\nv_lshlrev_b32 %9, 7, %9\nv_lshlrev_b32 %10, 7, %10\nv_lshlrev_b32 %11, 7, %11\nv_lshlrev_b32 %12, 7, %12\nv_lshlrev_b32 %13, 7, %13\nv_lshlrev_b32 %14, 7, %14\nv_lshlrev_b32 %15, 7, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshl7(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshl7(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshl16(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshlrev_b32 %0, 16, %0\nv_lshlrev_b32 %1, 16, %1\nv_lshlrev_b32 %2, 16, %2\nv_lshlrev_b32 %3, 16, %3\nv_lshlrev_b32 %4, 16, %4\nv_lshlrev_b32 %5, 16, %5\nv_lshlrev_b32 %6, 16, %6\nv_lshlrev_b32 %7, 16, %7\nv_lshlrev_b32 %8, 16, %8\nv_lshlrev_b32 %9, 16, %9\nv_lshlrev_b32 %10, 16, %10\nv_lshlrev_b32 %11, 16, %11\nv_lshlrev_b32 %12, 16, %12\nv_lshlrev_b32 %13, 16, %13\nv_lshlrev_b32 %14, 16, %14\nv_lshlrev_b32 %15, 16, %15\nv_lshlrev_b32 %0, 16, %0\nv_lshlrev_b32 %1, 16, %1\nv_lshlrev_b32 %2, 16, %2\nv_lshlrev_b32 %3, 16, %3\nv_lshlrev_b32 %4, 16, %4\nv_lshlrev_b32 %5, 16, %5\nv_lshlrev_b32 %6, 16, %6\nv_lshlrev_b32 %7, 16, %7\nv_lshlrev_b32 %8, 16, %8\nv_lshlrev_b32 %9, 16, %9\nv_lshlrev_b32 %10, 16, %10\nv_lshlrev_b32 %11, 16, %11\nv_lshlrev_b32 %12, 16, %12\nv_lshlrev_b32 %13, 16, %13\nv_lshlrev_b32 %14, 16, %14\nv_lshlrev_b32 %15, 16, %15\nv_lshlrev_b32 %0, 16, %0\nv_lshlrev_b32 %1, 16, %1\nv_lshlrev_b32 %2, 16, %2\nv_lshlrev_b32 %3, 16, %3\nv_lshlrev_b32 %4, 16, %4\nv_lshlrev_b32 %5, 16, %5\nv_lshlrev_b32 %6, 16, %6\nv_lshlrev_b32 %7, 16, %7\nv_lshlrev_b32 %8, 16, %8\nv_lshlrev_b32 %9, 16, %9\nv_lshlrev_b32 %10, 16, %10\nv_lshlrev_b32 %11, 16, %11\nv_lshlrev_b32 %12, 16, %12\nv_lshlrev_b32 %13, 16, %13\nv_lshlrev_b32 %14, 16, %14\nv_lshlrev_b32 %15, 16, %15\nv_lshlrev_b32 %0, 16, %0\nv_lshlrev_b32 %1, 16, %1\nv_lshlrev_b32 %2, 16, %2\nv_lshlrev_b32 %3, 16, %3\nv_lshlrev_b32 %4, 16, %4\nv_lshlrev_b32 %5, 16, %5\nv_lshlrev_b32 %6, 16, %6\nv_lshlrev_b32 %7, 16, %7\nv_lshlrev_b32 %8, 16, %8\nv_lshlrev_b32 %9, 16, %9\nv_lshlrev_b32 %10, 16, %10\nv_lshlrev_b32 %11, 16, %11\nv_lshlrev_b32 %12, 16, %12\nv_lshlrev_b32 %13, 16, %13\nv_lshlrev_b32 %14, 16, %14\nv_lshlrev_b32 %15, 16, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshl16(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshl16(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshl_v(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshlrev_b32 %0, %16, %0\nv_lshlrev_b32 %1, %16, %1\nv_lshlrev_b32 %2, %16, %2\nv_lshlrev_b32 %3, %16, %3\nv_lshlrev_b32 %4, %16, %4\nv_lshlrev_b32 %5, %16, %5\nv_lshlrev_b32 %6, %16, %6\nv_lshlrev_b32 %7, %16, %7\nv_lshlrev_b32 %8, %16, %8\nv_lshlrev_b32 %9, %16, %9\nv_lshlrev_b32 %10, %16, %10\nv_lshlrev_b32 %11, %16, %11\nv_lshlrev_b32 %12, %16, %12\nv_lshlrev_b32 %13, %16, %13\nv_lshlrev_b32 %14, %16, %14\nv_lshlrev_b32 %15, %16, %15\nv_lshlrev_b32 %0, %16, %0\nv_lshlrev_b32 %1, %16, %1\nv_lshlrev_b32 %2, %16, %2\nv_lshlrev_b32 %3, %16, %3\nv_lshlrev_b32 %4, %16, %4\nv_lshlrev_b32 %5, %16, %5\nv_lshlrev_b32 %6, %16, %6\nv_lshlrev_b32 %7, %16, %7\nv_lshlrev_b32 %8, %16, %8\nv_lshlrev_b32 %9, %16, %9\nv_lshlrev_b32 %10, %16, %10\nv_lshlrev_b32 %11, %16, %11\nv_lshlrev_b32 %12, %16, %12\nv_lshlrev_b32 %13, %16, %13\nv_lshlrev_b32 %14, %16, %14\nv_lshlrev_b32 %15, %16, %15\nv_lshlrev_b32 %0, %16, %0\nv_lshlrev_b32 %1, %16, %1\nv_lshlrev_b32 %2, %16, %2\nv_lshlrev_b32 %3, %16, %3\nv_lshlrev_b32 %4, %16, %4\nv_lshlrev_b32 %5, %16, %5\nv_lshlrev_b32 %6, %16, %6\nv_lshlrev_b32 %7, %16, %7\nv_lshlrev_b32 %8, %16, %8\nv_lshlrev_b32 %9, %16, %9\nv_lshlrev_b32 %10, %16, %10\nv_lshlrev_b32 %11, %16, %11\nv_lshlrev_b32 %12, %16, %12\nv_lshlrev_b32 %13, %16, %13\nv_lshlrev_b32 %14, %16, %14\nv_lshlrev_b32 %15, %16, %15\nv_lshlrev_b32 %0, %16, %0\nv_lshlrev_b32 %1, %16, %1\nv_lshlrev_b32 %2, %16, %2\nv_lshlrev_b32 %3, %16, %3\nv_lshlrev_b32 %4, %16, %4\nv_lshlrev_b32 %5, %16, %5\nv_lshlrev_b32 %6, %16, %6\nv_lshlrev_b32 %7, %16, %7\nv_lshlrev_b32 %8, %16, %8\nv_lshlrev_b32 %9, %16, %9\nv_lshlrev_b32 %10, %16, %10\nv_lshlrev_b32 %11, %16, %11\nv_lshlrev_b32 %12, %16, %12\nv_lshlrev_b32 %13, %16, %13\nv_lshlrev_b32 %14, %16, %14\nv_lshlrev_b32 %15, %16, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshl_v(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshl_v(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshr_v(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshrrev_b32 %0, %16, %0\nv_lshrrev_b32 %1, %16, %1\nv_lshrrev_b32 %2, %16, %2\nv_lshrrev_b32 %3, %16, %3\nv_lshrrev_b32 %4, %16, %4\nv_lshrrev_b32 %5, %16, %5\nv_lshrrev_b32 %6, %16, %6\nv_lshrrev_b32 %7, %16, %7\nv_lshrrev_b32 %8, %16, %8\nv_lshrrev_b32 %9, %16, %9\nv_lshrrev_b32 %10, %16, %10\nv_lshrrev_b32 %11, %16, %11\nv_lshrrev_b32 %12, %16, %12\nv_lshrrev_b32 %13, %16, %13\nv_lshrrev_b32 %14, %16, %14\nv_lshrrev_b32 %15, %16, %15\nv_lshrrev_b32 %0, %16, %0\nv_lshrrev_b32 %1, %16, %1\nv_lshrrev_b32 %2, %16, %2\nv_lshrrev_b32 %3, %16, %3\nv_lshrrev_b32 %4, %16, %4\nv_lshrrev_b32 %5, %16, %5\nv_lshrrev_b32 %6, %16, %6\nv_lshrrev_b32 %7, %16, %7\nv_lshrrev_b32 %8, %16, %8\nv_lshrrev_b32 %9, %16, %9\nv_lshrrev_b32 %10, %16, %10\nv_lshrrev_b32 %11, %16, %11\nv_lshrrev_b32 %12, %16, %12\nv_lshrrev_b32 %13, %16, %13\nv_lshrrev_b32 %14, %16, %14\nv_lshrrev_b32 %15, %16, %15\nv_lshrrev_b32 %0, %16, %0\nv_lshrrev_b32 %1, %16, %1\nv_lshrrev_b32 %2, %16, %2\nv_lshrrev_b32 %3, %16, %3\nv_lshrrev_b32 %4, %16, %4\nv_lshrrev_b32 %5, %16, %5\nv_lshrrev_b32 %6, %16, %6\nv_lshrrev_b32 %7, %16, %7\nv_lshrrev_b32 %8, %16, %8\nv_lshrrev_b32 %9, %16, %9\nv_lshrrev_b32 %10, %16, %10\nv_lshrrev_b32 %11, %16, %11\nv_lshrrev_b32 %12, %16, %12\nv_lshrrev_b32 %13, %16, %13\nv_lshrrev_b32 %14, %16, %14\nv_lshrrev_b32 %15, %16, %15\nv_lshrrev_b32 %0, %16, %0\nv_lshrrev_b32 %1, %16, %1\nv_lshrrev_b32 %2, %16, %2\nv_lshrrev_b32 %3, %16, %3\nv_lshrrev_b32 %4, %16, %4\nv_lshrrev_b32 %5, %16, %5\nv_lshrrev_b32 %6, %16, %6\nv_lshrrev_b32 %7, %16, %7\nv_lshrrev_b32 %8, %16, %8\nv_lshrrev_b32 %9, %16, %9\nv_lshrrev_b32 %10, %16, %10\nv_lshrrev_b32 %11, %16, %11\nv_lshrrev_b32 %12, %16, %12\nv_lshrrev_b32 %13, %16, %13\nv_lshrrev_b32 %14, %16, %14\nv_lshrrev_b32 %15, %16, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshr_v(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshr_v(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_add_self(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_add_u32 %0, %0, %0\nv_add_u32 %1, %1, %1\nv_add_u32 %2, %2, %2\nv_add_u32 %3, %3, %3\nv_add_u32 %4, %4, %4\nv_add_u32 %5, %5, %5\nv_add_u32 %6, %6, %6\nv_add_u32 %7, %7, %7\nv_add_u32 %8, %8, %8\nv_add_u32 %9, %9, %9\nv_add_u32 %10, %10, %10\nv_add_u32 %11, %11, %11\nv_add_u32 %12, %12, %12\nv_add_u32 %13, %13, %13\nv_add_u32 %14, %14, %14\nv_add_u32 %15, %15, %15\nv_add_u32 %0, %0, %0\nv_add_u32 %1, %1, %1\nv_add_u32 %2, %2, %2\nv_add_u32 %3, %3, %3\nv_add_u32 %4, %4, %4\nv_add_u32 %5, %5, %5\nv_add_u32 %6, %6, %6\nv_add_u32 %7, %7, %7\nv_add_u32 %8, %8, %8\nv_add_u32 %9, %9, %9\nv_add_u32 %10, %10, %10\nv_add_u32 %11, %11, %11\nv_add_u32 %12, %12, %12\nv_add_u32 %13, %13, %13\nv_add_u32 %14, %14, %14\nv_add_u32 %15, %15, %15\nv_add_u32 %0, %0, %0\nv_add_u32 %1, %1, %1\nv_add_u32 %2, %2, %2\nv_add_u32 %3, %3, %3\nv_add_u32 %4, %4, %4\nv_add_u32 %5, %5, %5\nv_add_u32 %6, %6, %6\nv_add_u32 %7, %7, %7\nv_add_u32 %8, %8, %8\nv_add_u32 %9, %9, %9\nv_add_u32 %10, %10, %10\nv_add_u32 %11, %11, %11\nv_add_u32 %12, %12, %12\nv_add_u32 %13, %13, %13\nv_add_u32 %14, %14, %14\nv_add_u32 %15, %15, %15\nv_add_u32 %0, %0, %0\nv_add_u32 %1, %1, %1\nv_add_u32 %2, %2, %2\nv_add_u32 %3, %3, %3\nv_add_u32 %4, %4, %4\nv_add_u32 %5, %5, %5\nv_add_u32 %6, %6, %6\nv_add_u32 %7, %7, %7\nv_add_u32 %8, %8, %8\nv_add_u32 %9, %9, %9\nv_add_u32 %10, %10, %10\nv_add_u32 %11, %11, %11\nv_add_u32 %12, %12, %12\nv_add_u32 %13, %13, %13\nv_add_u32 %14, %14, %14\nv_add_u32 %15, %15, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_add_self(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_add_self(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshr_b64(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]\nv_lshrrev_b64 v[40:41], 7, v[42:43]" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshr_b64(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshr_b64(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_lshl_b64(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]\nv_lshlrev_b64 v[40:41], 7, v[42:43]" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_lshl_b64(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_lshl_b64(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_pk_mov(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]\nv_pk_mov_b32 v[40:41], v[42:43], v[44:45] op_sel:[1,0]" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_pk_mov(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_pk_mov(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_bfe(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_bfe_u32 %0, %0, 3, 9\nv_bfe_u32 %1, %1, 3, 9\nv_bfe_u32 %2, %2, 3, 9\nv_bfe_u32 %3, %3, 3, 9\nv_bfe_u32 %4, %4, 3, 9\nv_bfe_u32 %5, %5, 3, 9\nv_bfe_u32 %6, %6, 3, 9\nv_bfe_u32 %7, %7, 3, 9\nv_bfe_u32 %8, %8, 3, 9\nv_bfe_u32 %9, %9, 3, 9\nv_bfe_u32 %10, %10, 3, 9\nv_bfe_u32 %11, %11, 3, 9\nv_bfe_u32 %12, %12, 3, 9\nv_bfe_u32 %13, %13, 3, 9\nv_bfe_u32 %14, %14, 3, 9\nv_bfe_u32 %15, %15, 3, 9\nv_bfe_u32 %0, %0, 3, 9\nv_bfe_u32 %1, %1, 3, 9\nv_bfe_u32 %2, %2, 3, 9\nv_bfe_u32 %3, %3, 3, 9\nv_bfe_u32 %4, %4, 3, 9\nv_bfe_u32 %5, %5, 3, 9\nv_bfe_u32 %6, %6, 3, 9\nv_bfe_u32 %7, %7, 3, 9\nv_bfe_u32 %8, %8, 3, 9\nv_bfe_u32 %9, %9, 3, 9\nv_bfe_u32 %10, %10, 3, 9\nv_bfe_u32 %11, %11, 3, 9\nv_bfe_u32 %12, %12, 3, 9\nv_bfe_u32 %13, %13, 3, 9\nv_bfe_u32 %14, %14, 3, 9\nv_bfe_u32 %15, %15, 3, 9\nv_bfe_u32 %0, %0, 3, 9\nv_bfe_u32 %1, %1, 3, 9\nv_bfe_u32 %2, %2, 3, 9\nv_bfe_u32 %3, %3, 3, 9\nv_bfe_u32 %4, %4, 3, 9\nv_bfe_u32 %5, %5, 3, 9\nv_bfe_u32 %6, %6, 3, 9\nv_bfe_u32 %7, %7, 3, 9\nv_bfe_u32 %8, %8, 3, 9\nv_bfe_u32 %9, %9, 3, 9\nv_bfe_u32 %10, %10, 3, 9\nv_bfe_u32 %11, %11, 3, 9\nv_bfe_u32 %12, %12, 3, 9\nv_bfe_u32 %13, %13, 3, 9\nv_bfe_u32 %14, %14, 3, 9\nv_bfe_u32 %15, %15, 3, 9\nv_bfe_u32 %0, %0, 3, 9\nv_bfe_u32 %1, %1, 3, 9\nv_bfe_u32 %2, %2, 3, 9\nv_bfe_u32 %3, %3, 3, 9\nv_bfe_u32 %4, %4, 3, 9\nv_bfe_u32 %5, %5, 3, 9\nv_bfe_u32 %6, %6, 3, 9\nv_bfe_u32 %7, %7, 3, 9\nv_bfe_u32 %8, %8, 3, 9\nv_bfe_u32 %9, %9, 3, 9\nv_bfe_u32 %10, %10, 3, 9\nv_bfe_u32 %11, %11, 3, 9\nv_bfe_u32 %12, %12, 3, 9\nv_bfe_u32 %13, %13, 3, 9\nv_bfe_u32 %14, %14, 3, 9\nv_bfe_u32 %15, %15, 3, 9" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_bfe(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_bfe(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_mul24(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_mul_u32_u24 %0, 128, %0\nv_mul_u32_u24 %1, 128, %1\nv_mul_u32_u24 %2, 128, %2\nv_mul_u32_u24 %3, 128, %3\nv_mul_u32_u24 %4, 128, %4\nv_mul_u32_u24 %5, 128, %5\nv_mul_u32_u24 %6, 128, %6\nv_mul_u32_u24 %7, 128, %7\nv_mul_u32_u24 %8, 128, %8\nv_mul_u32_u24 %9, 128, %9\nv_mul_u32_u24 %10, 128, %10\nv_mul_u32_u24 %11, 128, %11\nv_mul_u32_u24 %12, 128, %12\nv_mul_u32_u24 %13, 128, %13\nv_mul_u32_u24 %14, 128, %14\nv_mul_u32_u24 %15, 128, %15\nv_mul_u32_u24 %0, 128, %0\nv_mul_u32_u24 %1, 128, %1\nv_mul_u32_u24 %2, 128, %2\nv_mul_u32_u24 %3, 128, %3\nv_mul_u32_u24 %4, 128, %4\nv_mul_u32_u24 %5, 128, %5\nv_mul_u32_u24 %6, 128, %6\nv_mul_u32_u24 %7, 128, %7\nv_mul_u32_u24 %8, 128, %8\nv_mul_u32_u24 %9, 128, %9\nv_mul_u32_u24 %10, 128, %10\nv_mul_u32_u24 %11, 128, %11\nv_mul_u32_u24 %12, 128, %12\nv_mul_u32_u24 %13, 128, %13\nv_mul_u32_u24 %14, 128, %14\nv_mul_u32_u24 %15, 128, %15\nv_mul_u32_u24 %0, 128, %0\nv_mul_u32_u24 %1, 128, %1\nv_mul_u32_u24 %2, 128, %2\nv_mul_u32_u24 %3, 128, %3\nv_mul_u32_u24 %4, 128, %4\nv_mul_u32_u24 %5, 128, %5\nv_mul_u32_u24 %6, 128, %6\nv_mul_u32_u24 %7, 128, %7\nv_mul_u32_u24 %8, 128, %8\nv_mul_u32_u24 %9, 128, %9\nv_mul_u32_u24 %10, 128, %10\nv_mul_u32_u24 %11, 128, %11\nv_mul_u32_u24 %12, 128, %12\nv_mul_u32_u24 %13, 128, %13\nv_mul_u32_u24 %14, 128, %14\nv_mul_u32_u24 %15, 128, %15\nv_mul_u32_u24 %0, 128, %0\nv_mul_u32_u24 %1, 128, %1\nv_mul_u32_u24 %2, 128, %2\nv_mul_u32_u24 %3, 128, %3\nv_mul_u32_u24 %4, 128, %4\nv_mul_u32_u24 %5, 128, %5\nv_mul_u32_u24 %6, 128, %6\nv_mul_u32_u24 %7, 128, %7\nv_mul_u32_u24 %8, 128, %8\nv_mul_u32_u24 %9, 128, %9\nv_mul_u32_u24 %10, 128, %10\nv_mul_u32_u24 %11, 128, %11\nv_mul_u32_u24 %12, 128, %12\nv_mul_u32_u24 %13, 128, %13\nv_mul_u32_u24 %14, 128, %14\nv_mul_u32_u24 %15, 128, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_mul24(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_mul24(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_mad24(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_mad_u32_u24 %0, %16, %0, %0\nv_mad_u32_u24 %1, %16, %1, %1\nv_mad_u32_u24 %2, %16, %2, %2\nv_mad_u32_u24 %3, %16, %3, %3\nv_mad_u32_u24 %4, %16, %4, %4\nv_mad_u32_u24 %5, %16, %5, %5\nv_mad_u32_u24 %6, %16, %6, %6\nv_mad_u32_u24 %7, %16, %7, %7\nv_mad_u32_u24 %8, %16, %8, %8\nv_mad_u32_u24 %9, %16, %9, %9\nv_mad_u32_u24 %10, %16, %10, %10\nv_mad_u32_u24 %11, %16, %11, %11\nv_mad_u32_u24 %12, %16, %12, %12\nv_mad_u32_u24 %13, %16, %13, %13\nv_mad_u32_u24 %14, %16, %14, %14\nv_mad_u32_u24 %15, %16, %15, %15\nv_mad_u32_u24 %0, %16, %0, %0\nv_mad_u32_u24 %1, %16, %1, %1\nv_mad_u32_u24 %2, %16, %2, %2\nv_mad_u32_u24 %3, %16, %3, %3\nv_mad_u32_u24 %4, %16, %4, %4\nv_mad_u32_u24 %5, %16, %5, %5\nv_mad_u32_u24 %6, %16, %6, %6\nv_mad_u32_u24 %7, %16, %7, %7\nv_mad_u32_u24 %8, %16, %8, %8\nv_mad_u32_u24 %9, %16, %9, %9\nv_mad_u32_u24 %10, %16, %10, %10\nv_mad_u32_u24 %11, %16, %11, %11\nv_mad_u32_u24 %12, %16, %12, %12\nv_mad_u32_u24 %13, %16, %13, %13\nv_mad_u32_u24 %14, %16, %14, %14\nv_mad_u32_u24 %15, %16, %15, %15\nv_mad_u32_u24 %0, %16, %0, %0\nv_mad_u32_u24 %1, %16, %1, %1\nv_mad_u32_u24 %2, %16, %2, %2\nv_mad_u32_u24 %3, %16, %3, %3\nv_mad_u32_u24 %4, %16, %4, %4\nv_mad_u32_u24 %5, %16, %5, %5\nv_mad_u32_u24 %6, %16, %6, %6\nv_mad_u32_u24 %7, %16, %7, %7\nv_mad_u32_u24 %8, %16, %8, %8\nv_mad_u32_u24 %9, %16, %9, %9\nv_mad_u32_u24 %10, %16, %10, %10\nv_mad_u32_u24 %11, %16, %11, %11\nv_mad_u32_u24 %12, %16, %12, %12\nv_mad_u32_u24 %13, %16, %13, %13\nv_mad_u32_u24 %14, %16, %14, %14\nv_mad_u32_u24 %15, %16, %15, %15\nv_mad_u32_u24 %0, %16, %0, %0\nv_mad_u32_u24 %1, %16, %1, %1\nv_mad_u32_u24 %2, %16, %2, %2\nv_mad_u32_u24 %3, %16, %3, %3\nv_mad_u32_u24 %4, %16, %4, %4\nv_mad_u32_u24 %5, %16, %5, %5\nv_mad_u32_u24 %6, %16, %6, %6\nv_mad_u32_u24 %7, %16, %7, %7\nv_mad_u32_u24 %8, %16, %8, %8\nv_mad_u32_u24 %9, %16, %9, %9\nv_mad_u32_u24 %10, %16, %10, %10\nv_mad_u32_u24 %11, %16, %11, %11\nv_mad_u32_u24 %12, %16, %12, %12\nv_mad_u32_u24 %13, %16, %13, %13\nv_mad_u32_u24 %14, %16, %14, %14\nv_mad_u32_u24 %15, %16, %15, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_mad24(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_mad24(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_mul_lo(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_mul_lo_u32 %0, %0, %16\nv_mul_lo_u32 %1, %1, %16\nv_mul_lo_u32 %2, %2, %16\nv_mul_lo_u32 %3, %3, %16\nv_mul_lo_u32 %4, %4, %16\nv_mul_lo_u32 %5, %5, %16\nv_mul_lo_u32 %6, %6, %16\nv_mul_lo_u32 %7, %7, %16\nv_mul_lo_u32 %8, %8, %16\nv_mul_lo_u32 %9, %9, %16\nv_mul_lo_u32 %10, %10, %16\nv_mul_lo_u32 %11, %11, %16\nv_mul_lo_u32 %12, %12, %16\nv_mul_lo_u32 %13, %13, %16\nv_mul_lo_u32 %14, %14, %16\nv_mul_lo_u32 %15, %15, %16\nv_mul_lo_u32 %0, %0, %16\nv_mul_lo_u32 %1, %1, %16\nv_mul_lo_u32 %2, %2, %16\nv_mul_lo_u32 %3, %3, %16\nv_mul_lo_u32 %4, %4, %16\nv_mul_lo_u32 %5, %5, %16\nv_mul_lo_u32 %6, %6, %16\nv_mul_lo_u32 %7, %7, %16\nv_mul_lo_u32 %8, %8, %16\nv_mul_lo_u32 %9, %9, %16\nv_mul_lo_u32 %10, %10, %16\nv_mul_lo_u32 %11, %11, %16\nv_mul_lo_u32 %12, %12, %16\nv_mul_lo_u32 %13, %13, %16\nv_mul_lo_u32 %14, %14, %16\nv_mul_lo_u32 %15, %15, %16\nv_mul_lo_u32 %0, %0, %16\nv_mul_lo_u32 %1, %1, %16\nv_mul_lo_u32 %2, %2, %16\nv_mul_lo_u32 %3, %3, %16\nv_mul_lo_u32 %4, %4, %16\nv_mul_lo_u32 %5, %5, %16\nv_mul_lo_u32 %6, %6, %16\nv_mul_lo_u32 %7, %7, %16\nv_mul_lo_u32 %8, %8, %16\nv_mul_lo_u32 %9, %9, %16\nv_mul_lo_u32 %10, %10, %16\nv_mul_lo_u32 %11, %11, %16\nv_mul_lo_u32 %12, %12, %16\nv_mul_lo_u32 %13, %13, %16\nv_mul_lo_u32 %14, %14, %16\nv_mul_lo_u32 %15, %15, %16\nv_mul_lo_u32 %0, %0, %16\nv_mul_lo_u32 %1, %1, %16\nv_mul_lo_u32 %2, %2, %16\nv_mul_lo_u32 %3, %3, %16\nv_mul_lo_u32 %4, %4, %16\nv_mul_lo_u32 %5, %5, %16\nv_mul_lo_u32 %6, %6, %16\nv_mul_lo_u32 %7, %7, %16\nv_mul_lo_u32 %8, %8, %16\nv_mul_lo_u32 %9, %9, %16\nv_mul_lo_u32 %10, %10, %16\nv_mul_lo_u32 %11, %11, %16\nv_mul_lo_u32 %12, %12, %16\nv_mul_lo_u32 %13, %13, %16\nv_mul_lo_u32 %14, %14, %16\nv_mul_lo_u32 %15, %15, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_mul_lo(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_mul_lo(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_add_sgpr(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_add_u32 %0, %17, %0\nv_add_u32 %1, %17, %1\nv_add_u32 %2, %17, %2\nv_add_u32 %3, %17, %3\nv_add_u32 %4, %17, %4\nv_add_u32 %5, %17, %5\nv_add_u32 %6, %17, %6\nv_add_u32 %7, %17, %7\nv_add_u32 %8, %17, %8\nv_add_u32 %9, %17, %9\nv_add_u32 %10, %17, %10\nv_add_u32 %11, %17, %11\nv_add_u32 %12, %17, %12\nv_add_u32 %13, %17, %13\nv_add_u32 %14, %17, %14\nv_add_u32 %15, %17, %15\nv_add_u32 %0, %17, %0\nv_add_u32 %1, %17, %1\nv_add_u32 %2, %17, %2\nv_add_u32 %3, %17, %3\nv_add_u32 %4, %17, %4\nv_add_u32 %5, %17, %5\nv_add_u32 %6, %17, %6\nv_add_u32 %7, %17, %7\nv_add_u32 %8, %17, %8\nv_add_u32 %9, %17, %9\nv_add_u32 %10, %17, %10\nv_add_u32 %11, %17, %11\nv_add_u32 %12, %17, %12\nv_add_u32 %13, %17, %13\nv_add_u32 %14, %17, %14\nv_add_u32 %15, %17, %15\nv_add_u32 %0, %17, %0\nv_add_u32 %1, %17, %1\nv_add_u32 %2, %17, %2\nv_add_u32 %3, %17, %3\nv_add_u32 %4, %17, %4\nv_add_u32 %5, %17, %5\nv_add_u32 %6, %17, %6\nv_add_u32 %7, %17, %7\nv_add_u32 %8, %17, %8\nv_add_u32 %9, %17, %9\nv_add_u32 %10, %17, %10\nv_add_u32 %11, %17, %11\nv_add_u32 %12, %17, %12\nv_add_u32 %13, %17, %13\nv_add_u32 %14, %17, %14\nv_add_u32 %15, %17, %15\nv_add_u32 %0, %17, %0\nv_add_u32 %1, %17, %1\nv_add_u32 %2, %17, %2\nv_add_u32 %3, %17, %3\nv_add_u32 %4, %17, %4\nv_add_u32 %5, %17, %5\nv_add_u32 %6, %17, %6\nv_add_u32 %7, %17, %7\nv_add_u32 %8, %17, %8\nv_add_u32 %9, %17, %9\nv_add_u32 %10, %17, %10\nv_add_u32 %11, %17, %11\nv_add_u32 %12, %17, %12\nv_add_u32 %13, %17, %13\nv_add_u32 %14, %17, %14\nv_add_u32 %15, %17, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_add_sgpr(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_add_sgpr(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_add_sgpr_e64(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_add_u32_e64 %0, %0, %17\nv_add_u32_e64 %1, %1, %17\nv_add_u32_e64 %2, %2, %17\nv_add_u32_e64 %3, %3, %17\nv_add_u32_e64 %4, %4, %17\nv_add_u32_e64 %5, %5, %17\nv_add_u32_e64 %6, %6, %17\nv_add_u32_e64 %7, %7, %17\nv_add_u32_e64 %8, %8, %17\nv_add_u32_e64 %9, %9, %17\nv_add_u32_e64 %10, %10, %17\nv_add_u32_e64 %11, %11, %17\nv_add_u32_e64 %12, %12, %17\nv_add_u32_e64 %13, %13, %17\nv_add_u32_e64 %14, %14, %17\nv_add_u32_e64 %15, %15, %17\nv_add_u32_e64 %0, %0, %17\nv_add_u32_e64 %1, %1, %17\nv_add_u32_e64 %2, %2, %17\nv_add_u32_e64 %3, %3, %17\nv_add_u32_e64 %4, %4, %17\nv_add_u32_e64 %5, %5, %17\nv_add_u32_e64 %6, %6, %17\nv_add_u32_e64 %7, %7, %17\nv_add_u32_e64 %8, %8, %17\nv_add_u32_e64 %9, %9, %17\nv_add_u32_e64 %10, %10, %17\nv_add_u32_e64 %11, %11, %17\nv_add_u32_e64 %12, %12, %17\nv_add_u32_e64 %13, %13, %17\nv_add_u32_e64 %14, %14, %17\nv_add_u32_e64 %15, %15, %17\nv_add_u32_e64 %0, %0, %17\nv_add_u32_e64 %1, %1, %17\nv_add_u32_e64 %2, %2, %17\nv_add_u32_e64 %3, %3, %17\nv_add_u32_e64 %4, %4, %17\nv_add_u32_e64 %5, %5, %17\nv_add_u32_e64 %6, %6, %17\nv_add_u32_e64 %7, %7, %17\nv_add_u32_e64 %8, %8, %17\nv_add_u32_e64 %9, %9, %17\nv_add_u32_e64 %10, %10, %17\nv_add_u32_e64 %11, %11, %17\nv_add_u32_e64 %12, %12, %17\nv_add_u32_e64 %13, %13, %17\nv_add_u32_e64 %14, %14, %17\nv_add_u32_e64 %15, %15, %17\nv_add_u32_e64 %0, %0, %17\nv_add_u32_e64 %1, %1, %17\nv_add_u32_e64 %2, %2, %17\nv_add_u32_e64 %3, %3, %17\nv_add_u32_e64 %4, %4, %17\nv_add_u32_e64 %5, %5, %17\nv_add_u32_e64 %6, %6, %17\nv_add_u32_e64 %7, %7, %17\nv_add_u32_e64 %8, %8, %17\nv_add_u32_e64 %9, %9, %17\nv_add_u32_e64 %10, %10, %17\nv_add_u32_e64 %11, %11, %17\nv_add_u32_e64 %12, %12, %17\nv_add_u32_e64 %13, %13, %17\nv_add_u32_e64 %14, %14, %17\nv_add_u32_e64 %15, %15, %17" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_add_sgpr_e64(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_add_sgpr_e64(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_pk_lshl16(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_pk_lshlrev_b16 %0, 3, %0\nv_pk_lshlrev_b16 %1, 3, %1\nv_pk_lshlrev_b16 %2, 3, %2\nv_pk_lshlrev_b16 %3, 3, %3\nv_pk_lshlrev_b16 %4, 3, %4\nv_pk_lshlrev_b16 %5, 3, %5\nv_pk_lshlrev_b16 %6, 3, %6\nv_pk_lshlrev_b16 %7, 3, %7\nv_pk_lshlrev_b16 %8, 3, %8\nv_pk_lshlrev_b16 %9, 3, %9\nv_pk_lshlrev_b16 %10, 3, %10\nv_pk_lshlrev_b16 %11, 3, %11\nv_pk_lshlrev_b16 %12, 3, %12\nv_pk_lshlrev_b16 %13, 3, %13\nv_pk_lshlrev_b16 %14, 3, %14\nv_pk_lshlrev_b16 %15, 3, %15\nv_pk_lshlrev_b16 %0, 3, %0\nv_pk_lshlrev_b16 %1, 3, %1\nv_pk_lshlrev_b16 %2, 3, %2\nv_pk_lshlrev_b16 %3, 3, %3\nv_pk_lshlrev_b16 %4, 3, %4\nv_pk_lshlrev_b16 %5, 3, %5\nv_pk_lshlrev_b16 %6, 3, %6\nv_pk_lshlrev_b16 %7, 3, %7\nv_pk_lshlrev_b16 %8, 3, %8\nv_pk_lshlrev_b16 %9, 3, %9\nv_pk_lshlrev_b16 %10, 3, %10\nv_pk_lshlrev_b16 %11, 3, %11\nv_pk_lshlrev_b16 %12, 3, %12\nv_pk_lshlrev_b16 %13, 3, %13\nv_pk_lshlrev_b16 %14, 3, %14\nv_pk_lshlrev_b16 %15, 3, %15\nv_pk_lshlrev_b16 %0, 3, %0\nv_pk_lshlrev_b16 %1, 3, %1\nv_pk_lshlrev_b16 %2, 3, %2\nv_pk_lshlrev_b16 %3, 3, %3\nv_pk_lshlrev_b16 %4, 3, %4\nv_pk_lshlrev_b16 %5, 3, %5\nv_pk_lshlrev_b16 %6, 3, %6\nv_pk_lshlrev_b16 %7, 3, %7\nv_pk_lshlrev_b16 %8, 3, %8\nv_pk_lshlrev_b16 %9, 3, %9\nv_pk_lshlrev_b16 %10, 3, %10\nv_pk_lshlrev_b16 %11, 3, %11\nv_pk_lshlrev_b16 %12, 3, %12\nv_pk_lshlrev_b16 %13, 3, %13\nv_pk_lshlrev_b16 %14, 3, %14\nv_pk_lshlrev_b16 %15, 3, %15\nv_pk_lshlrev_b16 %0, 3, %0\nv_pk_lshlrev_b16 %1, 3, %1\nv_pk_lshlrev_b16 %2, 3, %2\nv_pk_lshlrev_b16 %3, 3, %3\nv_pk_lshlrev_b16 %4, 3, %4\nv_pk_lshlrev_b16 %5, 3, %5\nv_pk_lshlrev_b16 %6, 3, %6\nv_pk_lshlrev_b16 %7, 3, %7\nv_pk_lshlrev_b16 %8, 3, %8\nv_pk_lshlrev_b16 %9, 3, %9\nv_pk_lshlrev_b16 %10, 3, %10\nv_pk_lshlrev_b16 %11, 3, %11\nv_pk_lshlrev_b16 %12, 3, %12\nv_pk_lshlrev_b16 %13, 3, %13\nv_pk_lshlrev_b16 %14, 3, %14\nv_pk_lshlrev_b16 %15, 3, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_pk_lshl16(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_pk_lshl16(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_sub(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_sub_u32 %0, %0, %16\nv_sub_u32 %1, %1, %16\nv_sub_u32 %2, %2, %16\nv_sub_u32 %3, %3, %16\nv_sub_u32 %4, %4, %16\nv_sub_u32 %5, %5, %16\nv_sub_u32 %6, %6, %16\nv_sub_u32 %7, %7, %16\nv_sub_u32 %8, %8, %16\nv_sub_u32 %9, %9, %16\nv_sub_u32 %10, %10, %16\nv_sub_u32 %11, %11, %16\nv_sub_u32 %12, %12, %16\nv_sub_u32 %13, %13, %16\nv_sub_u32 %14, %14, %16\nv_sub_u32 %15, %15, %16\nv_sub_u32 %0, %0, %16\nv_sub_u32 %1, %1, %16\nv_sub_u32 %2, %2, %16\nv_sub_u32 %3, %3, %16\nv_sub_u32 %4, %4, %16\nv_sub_u32 %5, %5, %16\nv_sub_u32 %6, %6, %16\nv_sub_u32 %7, %7, %16\nv_sub_u32 %8, %8, %16\nv_sub_u32 %9, %9, %16\nv_sub_u32 %10, %10, %16\nv_sub_u32 %11, %11, %16\nv_sub_u32 %12, %12, %16\nv_sub_u32 %13, %13, %16\nv_sub_u32 %14, %14, %16\nv_sub_u32 %15, %15, %16\nv_sub_u32 %0, %0, %16\nv_sub_u32 %1, %1, %16\nv_sub_u32 %2, %2, %16\nv_sub_u32 %3, %3, %16\nv_sub_u32 %4, %4, %16\nv_sub_u32 %5, %5, %16\nv_sub_u32 %6, %6, %16\nv_sub_u32 %7, %7, %16\nv_sub_u32 %8, %8, %16\nv_sub_u32 %9, %9, %16\nv_sub_u32 %10, %10, %16\nv_sub_u32 %11, %11, %16\nv_sub_u32 %12, %12, %16\nv_sub_u32 %13, %13, %16\nv_sub_u32 %14, %14, %16\nv_sub_u32 %15, %15, %16\nv_sub_u32 %0, %0, %16\nv_sub_u32 %1, %1, %16\nv_sub_u32 %2, %2, %16\nv_sub_u32 %3, %3, %16\nv_sub_u32 %4, %4, %16\nv_sub_u32 %5, %5, %16\nv_sub_u32 %6, %6, %16\nv_sub_u32 %7, %7, %16\nv_sub_u32 %8, %8, %16\nv_sub_u32 %9, %9, %16\nv_sub_u32 %10, %10, %16\nv_sub_u32 %11, %11, %16\nv_sub_u32 %12, %12, %16\nv_sub_u32 %13, %13, %16\nv_sub_u32 %14, %14, %16\nv_sub_u32 %15, %15, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_sub(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_sub(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_not(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_not_b32 %0, %0\nv_not_b32 %1, %1\nv_not_b32 %2, %2\nv_not_b32 %3, %3\nv_not_b32 %4, %4\nv_not_b32 %5, %5\nv_not_b32 %6, %6\nv_not_b32 %7, %7\nv_not_b32 %8, %8\nv_not_b32 %9, %9\nv_not_b32 %10, %10\nv_not_b32 %11, %11\nv_not_b32 %12, %12\nv_not_b32 %13, %13\nv_not_b32 %14, %14\nv_not_b32 %15, %15\nv_not_b32 %0, %0\nv_not_b32 %1, %1\nv_not_b32 %2, %2\nv_not_b32 %3, %3\nv_not_b32 %4, %4\nv_not_b32 %5, %5\nv_not_b32 %6, %6\nv_not_b32 %7, %7\nv_not_b32 %8, %8\nv_not_b32 %9, %9\nv_not_b32 %10, %10\nv_not_b32 %11, %11\nv_not_b32 %12, %12\nv_not_b32 %13, %13\nv_not_b32 %14, %14\nv_not_b32 %15, %15\nv_not_b32 %0, %0\nv_not_b32 %1, %1\nv_not_b32 %2, %2\nv_not_b32 %3, %3\nv_not_b32 %4, %4\nv_not_b32 %5, %5\nv_not_b32 %6, %6\nv_not_b32 %7, %7\nv_not_b32 %8, %8\nv_not_b32 %9, %9\nv_not_b32 %10, %10\nv_not_b32 %11, %11\nv_not_b32 %12, %12\nv_not_b32 %13, %13\nv_not_b32 %14, %14\nv_not_b32 %15, %15\nv_not_b32 %0, %0\nv_not_b32 %1, %1\nv_not_b32 %2, %2\nv_not_b32 %3, %3\nv_not_b32 %4, %4\nv_not_b32 %5, %5\nv_not_b32 %6, %6\nv_not_b32 %7, %7\nv_not_b32 %8, %8\nv_not_b32 %9, %9\nv_not_b32 %10, %10\nv_not_b32 %11, %11\nv_not_b32 %12, %12\nv_not_b32 %13, %13\nv_not_b32 %14, %14\nv_not_b32 %15, %15" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_not(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_not(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_cndmask(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_cndmask_b32 %0, %0, %16, vcc\nv_cndmask_b32 %1, %1, %16, vcc\nv_cndmask_b32 %2, %2, %16, vcc\nv_cndmask_b32 %3, %3, %16, vcc\nv_cndmask_b32 %4, %4, %16, vcc\nv_cndmask_b32 %5, %5, %16, vcc\nv_cndmask_b32 %6, %6, %16, vcc\nv_cndmask_b32 %7, %7, %16, vcc\nv_cndmask_b32 %8, %8, %16, vcc\nv_cndmask_b32 %9, %9, %16, vcc\nv_cndmask_b32 %10, %10, %16, vcc\nv_cndmask_b32 %11, %11, %16, vcc\nv_cndmask_b32 %12, %12, %16, vcc\nv_cndmask_b32 %13, %13, %16, vcc\nv_cndmask_b32 %14, %14, %16, vcc\nv_cndmask_b32 %15, %15, %16, vcc\nv_cndmask_b32 %0, %0, %16, vcc\nv_cndmask_b32 %1, %1, %16, vcc\nv_cndmask_b32 %2, %2, %16, vcc\nv_cndmask_b32 %3, %3, %16, vcc\nv_cndmask_b32 %4, %4, %16, vcc\nv_cndmask_b32 %5, %5, %16, vcc\nv_cndmask_b32 %6, %6, %16, vcc\nv_cndmask_b32 %7, %7, %16, vcc\nv_cndmask_b32 %8, %8, %16, vcc\nv_cndmask_b32 %9, %9, %16, vcc\nv_cndmask_b32 %10, %10, %16, vcc\nv_cndmask_b32 %11, %11, %16, vcc\nv_cndmask_b32 %12, %12, %16, vcc\nv_cndmask_b32 %13, %13, %16, vcc\nv_cndmask_b32 %14, %14, %16, vcc\nv_cndmask_b32 %15, %15, %16, vcc\nv_cndmask_b32 %0, %0, %16, vcc\nv_cndmask_b32 %1, %1, %16, vcc\nv_cndmask_b32 %2, %2, %16, vcc\nv_cndmask_b32 %3, %3, %16, vcc\nv_cndmask_b32 %4, %4, %16, vcc\nv_cndmask_b32 %5, %5, %16, vcc\nv_cndmask_b32 %6, %6, %16, vcc\nv_cndmask_b32 %7, %7, %16, vcc\nv_cndmask_b32 %8, %8, %16, vcc\nv_cndmask_b32 %9, %9, %16, vcc\nv_cndmask_b32 %10, %10, %16, vcc\nv_cndmask_b32 %11, %11, %16, vcc\nv_cndmask_b32 %12, %12, %16, vcc\nv_cndmask_b32 %13, %13, %16, vcc\nv_cndmask_b32 %14, %14, %16, vcc\nv_cndmask_b32 %15, %15, %16, vcc\nv_cndmask_b32 %0, %0, %16, vcc\nv_cndmask_b32 %1, %1, %16, vcc\nv_cndmask_b32 %2, %2, %16, vcc\nv_cndmask_b32 %3, %3, %16, vcc\nv_cndmask_b32 %4, %4, %16, vcc\nv_cndmask_b32 %5, %5, %16, vcc\nv_cndmask_b32 %6, %6, %16, vcc\nv_cndmask_b32 %7, %7, %16, vcc\nv_cndmask_b32 %8, %8, %16, vcc\nv_cndmask_b32 %9, %9, %16, vcc\nv_cndmask_b32 %10, %10, %16, vcc\nv_cndmask_b32 %11, %11, %16, vcc\nv_cndmask_b32 %12, %12, %16, vcc\nv_cndmask_b32 %13, %13, %16, vcc\nv_cndmask_b32 %14, %14, %16, vcc\nv_cndmask_b32 %15, %15, %16, vcc" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_cndmask(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_cndmask(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_mov(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_mov_b32 %0, %16\nv_mov_b32 %1, %16\nv_mov_b32 %2, %16\nv_mov_b32 %3, %16\nv_mov_b32 %4, %16\nv_mov_b32 %5, %16\nv_mov_b32 %6, %16\nv_mov_b32 %7, %16\nv_mov_b32 %8, %16\nv_mov_b32 %9, %16\nv_mov_b32 %10, %16\nv_mov_b32 %11, %16\nv_mov_b32 %12, %16\nv_mov_b32 %13, %16\nv_mov_b32 %14, %16\nv_mov_b32 %15, %16\nv_mov_b32 %0, %16\nv_mov_b32 %1, %16\nv_mov_b32 %2, %16\nv_mov_b32 %3, %16\nv_mov_b32 %4, %16\nv_mov_b32 %5, %16\nv_mov_b32 %6, %16\nv_mov_b32 %7, %16\nv_mov_b32 %8, %16\nv_mov_b32 %9, %16\nv_mov_b32 %10, %16\nv_mov_b32 %11, %16\nv_mov_b32 %12, %16\nv_mov_b32 %13, %16\nv_mov_b32 %14, %16\nv_mov_b32 %15, %16\nv_mov_b32 %0, %16\nv_mov_b32 %1, %16\nv_mov_b32 %2, %16\nv_mov_b32 %3, %16\nv_mov_b32 %4, %16\nv_mov_b32 %5, %16\nv_mov_b32 %6, %16\nv_mov_b32 %7, %16\nv_mov_b32 %8, %16\nv_mov_b32 %9, %16\nv_mov_b32 %10, %16\nv_mov_b32 %11, %16\nv_mov_b32 %12, %16\nv_mov_b32 %13, %16\nv_mov_b32 %14, %16\nv_mov_b32 %15, %16\nv_mov_b32 %0, %16\nv_mov_b32 %1, %16\nv_mov_b32 %2, %16\nv_mov_b32 %3, %16\nv_mov_b32 %4, %16\nv_mov_b32 %5, %16\nv_mov_b32 %6, %16\nv_mov_b32 %7, %16\nv_mov_b32 %8, %16\nv_mov_b32 %9, %16\nv_mov_b32 %10, %16\nv_mov_b32 %11, %16\nv_mov_b32 %12, %16\nv_mov_b32 %13, %16\nv_mov_b32 %14, %16\nv_mov_b32 %15, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_mov(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_mov(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__device__ __forceinline__ void body_split_fast_slow_dep(uint32_t *r, uint32_t k, uint32_t ks) {
  asm volatile("v_lshrrev_b32 %0, 7, %0\nv_xor_b32 %1, %1, %16\nv_lshrrev_b32 %2, 7, %2\nv_xor_b32 %3, %3, %16\nv_lshrrev_b32 %4, 7, %4\nv_xor_b32 %5, %5, %16\nv_lshrrev_b32 %6, 7, %6\nv_xor_b32 %7, %7, %16\nv_lshrrev_b32 %8, 7, %8\nv_xor_b32 %9, %9, %16\nv_lshrrev_b32 %10, 7, %10\nv_xor_b32 %11, %11, %16\nv_lshrrev_b32 %12, 7, %12\nv_xor_b32 %13, %13, %16\nv_lshrrev_b32 %14, 7, %14\nv_xor_b32 %15, %15, %16\nv_lshrrev_b32 %0, 7, %0\nv_xor_b32 %1, %1, %16\nv_lshrrev_b32 %2, 7, %2\nv_xor_b32 %3, %3, %16\nv_lshrrev_b32 %4, 7, %4\nv_xor_b32 %5, %5, %16\nv_lshrrev_b32 %6, 7, %6\nv_xor_b32 %7, %7, %16\nv_lshrrev_b32 %8, 7, %8\nv_xor_b32 %9, %9, %16\nv_lshrrev_b32 %10, 7, %10\nv_xor_b32 %11, %11, %16\nv_lshrrev_b32 %12, 7, %12\nv_xor_b32 %13, %13, %16\nv_lshrrev_b32 %14, 7, %14\nv_xor_b32 %15, %15, %16\nv_lshrrev_b32 %0, 7, %0\nv_xor_b32 %1, %1, %16\nv_lshrrev_b32 %2, 7, %2\nv_xor_b32 %3, %3, %16\nv_lshrrev_b32 %4, 7, %4\nv_xor_b32 %5, %5, %16\nv_lshrrev_b32 %6, 7, %6\nv_xor_b32 %7, %7, %16\nv_lshrrev_b32 %8, 7, %8\nv_xor_b32 %9, %9, %16\nv_lshrrev_b32 %10, 7, %10\nv_xor_b32 %11, %11, %16\nv_lshrrev_b32 %12, 7, %12\nv_xor_b32 %13, %13, %16\nv_lshrrev_b32 %14, 7, %14\nv_xor_b32 %15, %15, %16\nv_lshrrev_b32 %0, 7, %0\nv_xor_b32 %1, %1, %16\nv_lshrrev_b32 %2, 7, %2\nv_xor_b32 %3, %3, %16\nv_lshrrev_b32 %4, 7, %4\nv_xor_b32 %5, %5, %16\nv_lshrrev_b32 %6, 7, %6\nv_xor_b32 %7, %7, %16\nv_lshrrev_b32 %8, 7, %8\nv_xor_b32 %9, %9, %16\nv_lshrrev_b32 %10, 7, %10\nv_xor_b32 %11, %11, %16\nv_lshrrev_b32 %12, 7, %12\nv_xor_b32 %13, %13, %16\nv_lshrrev_b32 %14, 7, %14\nv_xor_b32 %15, %15, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k), "s"(ks) : "v40", "v41", "v42", "v43", "v44", "v45", "vcc");
}
__global__ __launch_bounds__(256) void k_split_fast_slow_dep(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  for (uint32_t it = 0; it < iters; ++it) body_split_fast_slow_dep(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ __launch_bounds__(512) void k_split_xor_alignbit(uint32_t *out, uint32_t iters) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1, ks = __builtin_amdgcn_readfirstlane(blockIdx.x) | 3;
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 1)
    for (uint32_t it = 0; it < iters; ++it) body_alignbit(r, k, ks);
  else
    for (uint32_t it = 0; it < iters; ++it) body_xor(r, k, ks);
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

struct K { const char *name; void *fn; int threads; };
static K ks_[] = {
  {"xor", (void*)k_xor, 256},
  {"alignbit", (void*)k_alignbit, 256},
  {"lshr1", (void*)k_lshr1, 256},
  {"lshr7", (void*)k_lshr7, 256},
  {"lshr16", (void*)k_lshr16, 256},
  {"lshl1", (void*)k_lshl1, 256},
  {"lshl7", (void*)k_lshl7, 256},
  {"lshl16", (void*)k_lshl16, 256},
  {"lshl_v", (void*)k_lshl_v, 256},
  {"lshr_v", (void*)k_lshr_v, 256},
  {"add_self", (void*)k_add_self, 256},
  {"lshr_b64", (void*)k_lshr_b64, 256},
  {"lshl_b64", (void*)k_lshl_b64, 256},
  {"pk_mov", (void*)k_pk_mov, 256},
  {"bfe", (void*)k_bfe, 256},
  {"mul24", (void*)k_mul24, 256},
  {"mad24", (void*)k_mad24, 256},
  {"mul_lo", (void*)k_mul_lo, 256},
  {"add_sgpr", (void*)k_add_sgpr, 256},
  {"add_sgpr_e64", (void*)k_add_sgpr_e64, 256},
  {"pk_lshl16", (void*)k_pk_lshl16, 256},
  {"sub", (void*)k_sub, 256},
  {"not", (void*)k_not, 256},
  {"cndmask", (void*)k_cndmask, 256},
  {"mov", (void*)k_mov, 256},
  {"split_fast_slow_dep", (void*)k_split_fast_slow_dep, 256},
  {"split_xor_alignbit", (void*)k_split_xor_alignbit, 512}
};
int main(int argc, char **argv) {
  const uint32_t iters = 4096;
  int cus = 256;
  uint32_t *out;
  hipMalloc(&out, size_t(1) << 28);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int occ : {2, 4, 8}) {
    for (auto &k : ks_) {
      if (argc > 1 && !strstr(k.name, argv[1])) continue;
      const int waves_per_block = k.threads / 64;
      const int blocks = cus * 4 * occ / waves_per_block;
      void *args[] = {&out, (void *)&iters};
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernel(k.fn, dim3(blocks), dim3(k.threads), args, 0, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      // wave-instructions per SIMD = occ waves x iters x 64
      const double per_simd = double(occ) * iters * 64;
      printf("%-20s occ %d  %8.3f ms  %6.3f ns/instr/SIMD  (= %.2f cyc at 2.1 GHz)\n", k.name, occ,
             best, best * 1e6 / per_simd, best * 1e6 / per_simd * 2.1);
    }
  }
  return 0;
}
