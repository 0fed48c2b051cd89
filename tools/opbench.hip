// opbench.hip -- per-instruction VALU throughput on gfx950 (not product code).
// Each kernel runs 8 independent dependency chains per lane of one opcode in
// inline asm; grid = 8192 x 256 threads (8 waves/SIMD on 256 CUs).  Also reads
// the in-kernel clock (s_memtime / s_memrealtime @ 100 MHz).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));        \
      exit(2);                                                      \
    }                                                               \
  } while (0)

#define REP8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

#define KERNEL(NAME, ASMSTR)                                                   \
  __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t iters,   \
                                              uint64_t *clk) {                 \
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3,          \
             r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;               \
    uint32_t k = blockIdx.x | 1;                                               \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                \
    uint64_t w0 = __builtin_amdgcn_s_memrealtime();                            \
    for (uint32_t i = 0; i < iters; ++i) {                                     \
      _Pragma("unroll") for (int u = 0; u < 8; ++u) {                          \
        asm volatile(ASMSTR                                                    \
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4),       \
                       "+v"(r5), "+v"(r6), "+v"(r7)                            \
                     : "v"(k));                                                \
      }                                                                        \
    }                                                                          \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                \
    uint64_t w1 = __builtin_amdgcn_s_memrealtime();                            \
    out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7; \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                 \
      clk[0] = t1 - t0;                                                        \
      clk[1] = w1 - w0;                                                        \
    }                                                                          \
  }

#define X8(I) "I %0, %0, %8\n I %1, %1, %8\n I %2, %2, %8\n I %3, %3, %8\n I %4, %4, %8\n I %5, %5, %8\n I %6, %6, %8\n I %7, %7, %8\n"
#define X8_3(I, EXTRA) \
  I " %0, %0, %8, " EXTRA "\n" I " %1, %1, %8, " EXTRA "\n" I " %2, %2, %8, " EXTRA "\n" I " %3, %3, %8, " EXTRA "\n" \
  I " %4, %4, %8, " EXTRA "\n" I " %5, %5, %8, " EXTRA "\n" I " %6, %6, %8, " EXTRA "\n" I " %7, %7, %8, " EXTRA "\n"
#define X8_2(I) \
  I " %0, %0, %8\n" I " %1, %1, %8\n" I " %2, %2, %8\n" I " %3, %3, %8\n" \
  I " %4, %4, %8\n" I " %5, %5, %8\n" I " %6, %6, %8\n" I " %7, %7, %8\n"
#define X8_ROT(I) \
  I " %0, %0, %0, 7\n" I " %1, %1, %1, 7\n" I " %2, %2, %2, 7\n" I " %3, %3, %3, 7\n" \
  I " %4, %4, %4, 7\n" I " %5, %5, %5, 7\n" I " %6, %6, %6, 7\n" I " %7, %7, %7, 7\n"

KERNEL(k_xor, X8_2("v_xor_b32"))
KERNEL(k_add, X8_2("v_add_u32"))
KERNEL(k_add3, X8_3("v_add3_u32", "%0"))
KERNEL(k_alignbit, X8_ROT("v_alignbit_b32"))
KERNEL(k_perm, X8_3("v_perm_b32", "%8"))
KERNEL(k_bitop3, X8_3("v_bitop3_b32", "%8 bitop3:0x96"))
KERNEL(k_xad, X8_3("v_xad_u32", "%8"))
KERNEL(k_addf, X8_2("v_add_f32"))
KERNEL(k_fmaf, X8_3("v_fma_f32", "%0"))
KERNEL(k_lshlor, X8_3("v_lshl_or_b32", "%8"))

int main() {
  uint32_t *out;
  uint64_t *clk;
  CK(hipMalloc(&out, 8192 * 256 * 4));
  CK(hipMalloc(&clk, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const uint32_t iters = 2048, grid = 8192;
  struct K {
    const char *name;
    void (*fn)(uint32_t *, uint32_t, uint64_t *);
  } ks[] = {{"v_xor_b32", k_xor},       {"v_add_u32", k_add},
            {"v_add3_u32", k_add3},     {"v_alignbit_b32", k_alignbit},
            {"v_perm_b32", k_perm},     {"v_bitop3_b32", k_bitop3},
            {"v_xad_u32", k_xad},       {"v_add_f32", k_addf},
            {"v_fma_f32", k_fmaf},      {"v_lshl_or_b32", k_lshlor}};
  for (auto &k : ks) {
    hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, iters, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, out, iters, clk);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    uint64_t c[2];
    CK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
    const double ops = double(grid) * 256 * iters * 8 * 8;
    const double ghz = double(c[0]) / (double(c[1]) * 10.0);
    printf("%-16s %8.3f ms  %7.2f Tops/s  clk %.2f GHz  lanes/clk/SIMD %.1f\n",
           k.name, ms, ops / (ms * 1e-3) / 1e12, ghz,
           ops / (ms * 1e-3) / (256.0 * 4 * ghz * 1e9));
  }
  return 0;
}
