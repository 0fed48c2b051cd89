#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__device__ __forceinline__ void body_F(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_H(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_alt1(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_alignbit_b32 %1, %1, %1, 7\nv_add_u32 %2, %2, %7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_alignbit_b32 %5, %5, %5, 7\nv_add_u32 %6, %6, %11\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_alignbit_b32 %9, %9, %9, 7\nv_add_u32 %10, %10, %15\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_alignbit_b32 %13, %13, %13, 7\nv_add_u32 %14, %14, %3\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_alignbit_b32 %1, %1, %1, 7\nv_add_u32 %2, %2, %7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_alignbit_b32 %5, %5, %5, 7\nv_add_u32 %6, %6, %11\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_alignbit_b32 %9, %9, %9, 7\nv_add_u32 %10, %10, %15\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_alignbit_b32 %13, %13, %13, 7\nv_add_u32 %14, %14, %3\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_alignbit_b32 %1, %1, %1, 7\nv_add_u32 %2, %2, %7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_alignbit_b32 %5, %5, %5, 7\nv_add_u32 %6, %6, %11\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_alignbit_b32 %9, %9, %9, 7\nv_add_u32 %10, %10, %15\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_alignbit_b32 %13, %13, %13, 7\nv_add_u32 %14, %14, %3\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_alignbit_b32 %1, %1, %1, 7\nv_add_u32 %2, %2, %7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_alignbit_b32 %5, %5, %5, 7\nv_add_u32 %6, %6, %11\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_alignbit_b32 %9, %9, %9, 7\nv_add_u32 %10, %10, %15\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_alignbit_b32 %13, %13, %13, 7\nv_add_u32 %14, %14, %3\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b2(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b4(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b8(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b16(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b32(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_qr4(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_qr_b16(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b4_rot(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b8_rot(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b16_rot(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_b32_rot(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_qr_b16_rot(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %1, %1, %6, %16\nv_alignbit_b32 %2, %2, %2, 7\nv_add3_u32 %3, %3, %8, %16\nv_alignbit_b32 %4, %4, %4, 7\nv_add3_u32 %5, %5, %10, %16\nv_alignbit_b32 %6, %6, %6, 7\nv_add3_u32 %7, %7, %12, %16\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_alignbit_b32 %8, %8, %8, 7\nv_add3_u32 %9, %9, %14, %16\nv_alignbit_b32 %10, %10, %10, 7\nv_add3_u32 %11, %11, %0, %16\nv_alignbit_b32 %12, %12, %12, 7\nv_add3_u32 %13, %13, %2, %16\nv_alignbit_b32 %14, %14, %14, 7\nv_add3_u32 %15, %15, %4, %16\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4\nv_xor_b32 %0, %0, %5\nv_add_u32 %1, %1, %6\nv_xor_b32 %2, %2, %7\nv_add_u32 %3, %3, %8\nv_xor_b32 %4, %4, %9\nv_add_u32 %5, %5, %10\nv_xor_b32 %6, %6, %11\nv_add_u32 %7, %7, %12\nv_xor_b32 %8, %8, %13\nv_add_u32 %9, %9, %14\nv_xor_b32 %10, %10, %15\nv_add_u32 %11, %11, %0\nv_xor_b32 %12, %12, %1\nv_add_u32 %13, %13, %2\nv_xor_b32 %14, %14, %3\nv_add_u32 %15, %15, %4" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_qr_c1(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_qr_c1_nop(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_qr_c2(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_qr_c2_nop(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_qr_c4(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %2, %2, %2, 7\nv_xor_b32 %3, %3, %11\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %2, %2, %10\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %2, %2, %2, 7\nv_xor_b32 %3, %3, %11\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %2, %2, %10\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %2, %2, %2, 7\nv_xor_b32 %3, %3, %11\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %2, %2, %10\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %2, %2, %2, 7\nv_xor_b32 %3, %3, %11\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %2, %2, %10\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %2, %2, %2, 7\nv_xor_b32 %3, %3, %11\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %2, %2, %10\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %2, %2, %2, 7\nv_xor_b32 %3, %3, %11" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_qr_c4_nop(uint32_t *r, uint32_t k) {
  asm volatile("v_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %2, %2, %2, 7\ns_nop 0\nv_xor_b32 %3, %3, %11\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %2, %2, %10\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %2, %2, %2, 7\ns_nop 0\nv_xor_b32 %3, %3, %11\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %2, %2, %10\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %2, %2, %2, 7\ns_nop 0\nv_xor_b32 %3, %3, %11\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %2, %2, %10\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %2, %2, %2, 7\ns_nop 0\nv_xor_b32 %3, %3, %11\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %2, %2, %10\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %2, %2, %2, 7\ns_nop 0\nv_xor_b32 %3, %3, %11\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %2, %2, %10\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %2, %2, %2, 7\ns_nop 0\nv_xor_b32 %3, %3, %11" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_g_c1(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %0, %0, %8\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_add3_u32 %0, %0, %8, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8\nv_xor_b32 %0, %0, %8\nv_add_u32 %0, %0, %8" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_g_c1_nop(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %0, %0, %8" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_g_c2(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %0, %0, %8, %16\nv_add_u32 %1, %1, %9\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %0, %0, %8\nv_add3_u32 %1, %1, %9, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_g_c2_nop(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %0, %0, %8, %16\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %0, %0, %8\ns_nop 0\nv_add3_u32 %1, %1, %9, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_g_c4(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_xor_b32 %0, %0, %8\nv_alignbit_b32 %1, %1, %1, 7\nv_add3_u32 %2, %2, %10, %16\nv_add_u32 %3, %3, %11\nv_alignbit_b32 %0, %0, %0, 7\nv_xor_b32 %1, %1, %9\nv_add_u32 %2, %2, %10\nv_add3_u32 %3, %3, %11, %16\nv_xor_b32 %0, %0, %8\nv_add_u32 %1, %1, %9\nv_xor_b32 %2, %2, %10\nv_add_u32 %3, %3, %11" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__device__ __forceinline__ void body_dep_g_c4_nop(uint32_t *r, uint32_t k) {
  asm volatile("v_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_alignbit_b32 %1, %1, %1, 7\ns_nop 0\nv_add3_u32 %2, %2, %10, %16\ns_nop 0\nv_add_u32 %3, %3, %11\ns_nop 0\nv_alignbit_b32 %0, %0, %0, 7\ns_nop 0\nv_xor_b32 %1, %1, %9\ns_nop 0\nv_add_u32 %2, %2, %10\ns_nop 0\nv_add3_u32 %3, %3, %11, %16\ns_nop 0\nv_xor_b32 %0, %0, %8\ns_nop 0\nv_add_u32 %1, %1, %9\ns_nop 0\nv_xor_b32 %2, %2, %10\ns_nop 0\nv_add_u32 %3, %3, %11" : "+v"(r[0]),"+v"(r[1]),"+v"(r[2]),"+v"(r[3]),"+v"(r[4]),"+v"(r[5]),"+v"(r[6]),"+v"(r[7]),"+v"(r[8]),"+v"(r[9]),"+v"(r[10]),"+v"(r[11]),"+v"(r[12]),"+v"(r[13]),"+v"(r[14]),"+v"(r[15]) : "v"(k));
}
__global__ __launch_bounds__(64) void k_F(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_F(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_F(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_H(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_H(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_H(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_alt1(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_alt1(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_alt1(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b2(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b2(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b2(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b4(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b4(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b4(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b8(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b8(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b8(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b16(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b16(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b16(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b32(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b32(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b32(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_qr4(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_qr4(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_qr4(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_qr_b16(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_qr_b16(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_qr_b16(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_split_F_H(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_H(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_F(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b4_phase(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b4_rot(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b4(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b8_phase(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b8_rot(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b8(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b16_phase(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b16_rot(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b16(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_b32_phase(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_b32_rot(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_b32(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_qr_b16_phase(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_qr_b16_rot(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_qr_b16(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_qr_c1(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c1(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c1(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_qr_c1_nop(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c1_nop(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c1_nop(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_qr_c2(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c2(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c2(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_qr_c2_nop(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c2_nop(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c2_nop(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_qr_c4(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c4(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c4(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_qr_c4_nop(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c4_nop(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_qr_c4_nop(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_g_c1(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c1(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c1(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_g_c1_nop(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c1_nop(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c1_nop(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_g_c2(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c2(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c2(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_g_c2_nop(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c2_nop(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c2_nop(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_g_c4(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c4(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c4(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
__global__ __launch_bounds__(64) void k_dep_g_c4_nop(uint32_t *out, uint32_t iters, uint64_t *clk) {
  uint32_t r[16];
  for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
  uint32_t k = blockIdx.x | 1;
  const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID
  const bool odd = (hw & 1) != 0;
  uint64_t s0 = __builtin_amdgcn_s_memtime(), w0 = __builtin_amdgcn_s_memrealtime();
  if (odd)
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c4_nop(r, k);
  else
    for (uint32_t it = 0; it < iters; ++it) body_dep_g_c4_nop(r, k);
  uint64_t s1 = __builtin_amdgcn_s_memtime(), w1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= r[i];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = s1 - s0; clk[1] = w1 - w0; }
}
struct K { const char *name; void *fn; };
static K ks_[] = {
  {"F", (void*)k_F},
  {"H", (void*)k_H},
  {"alt1", (void*)k_alt1},
  {"b2", (void*)k_b2},
  {"b4", (void*)k_b4},
  {"b8", (void*)k_b8},
  {"b16", (void*)k_b16},
  {"b32", (void*)k_b32},
  {"qr4", (void*)k_qr4},
  {"qr_b16", (void*)k_qr_b16},
  {"split_F_H", (void*)k_split_F_H},
  {"b4_phase", (void*)k_b4_phase},
  {"b8_phase", (void*)k_b8_phase},
  {"b16_phase", (void*)k_b16_phase},
  {"b32_phase", (void*)k_b32_phase},
  {"qr_b16_phase", (void*)k_qr_b16_phase},
  {"dep_qr_c1", (void*)k_dep_qr_c1},
  {"dep_qr_c1_nop", (void*)k_dep_qr_c1_nop},
  {"dep_qr_c2", (void*)k_dep_qr_c2},
  {"dep_qr_c2_nop", (void*)k_dep_qr_c2_nop},
  {"dep_qr_c4", (void*)k_dep_qr_c4},
  {"dep_qr_c4_nop", (void*)k_dep_qr_c4_nop},
  {"dep_g_c1", (void*)k_dep_g_c1},
  {"dep_g_c1_nop", (void*)k_dep_g_c1_nop},
  {"dep_g_c2", (void*)k_dep_g_c2},
  {"dep_g_c2_nop", (void*)k_dep_g_c2_nop},
  {"dep_g_c4", (void*)k_dep_g_c4},
  {"dep_g_c4_nop", (void*)k_dep_g_c4_nop}
};
int main(int argc, char **argv) {
  const uint32_t iters = 2048;
  const int simds = 1024;
  uint32_t *out; uint64_t *clk;
  hipMalloc(&out, size_t(1) << 26);
  hipMalloc(&clk, 64);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int occ : {2, 4, 6, 8}) {
    for (auto &k : ks_) {
      if (argc > 1 && !strstr(k.name, argv[1])) continue;
      const int blocks = simds * occ;
      void *args[] = {&out, (void *)&iters, &clk};
      float best = 1e30f; double ghz = 0;
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernel(k.fn, dim3(blocks), dim3(64), args, 0, nullptr);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        if (ms < best) { best = ms; ghz = double(c[0]) / (double(c[1]) * 10.0); }
      }
      const double per_simd = double(occ) * iters * 64;
      printf("%-14s occ %d  %8.3f ms  clk %.2f GHz  cyc/instr/SIMD %.2f\n", k.name, occ, best,
             ghz, best * 1e6 * ghz / per_simd);
    }
  }
  return 0;
}
