// chainlat.hip -- dependent-issue latency of the instructions on the
// quad-layout BLAKE3 chain (quad_compress, post_kernels.hip), on gfx950 (not
// product code).  Each kernel runs ONE dependent chain
// per lane of REPS instructions x iters in inline asm, at one wave per SIMD
// (256 workgroups of 256 lanes = 4 waves per CU); thread 0 of workgroup 0
// reads s_memtime (shader clock) and s_memrealtime (100 MHz) around the loop.
// cycles per instruction = clk / (iters x REPS).  DPP reads of a VGPR written
// by the previous VALU instruction need two wait states on gfx9 (the
// compiler's hazard recognizer inserts `s_nop 1`), so the DPP chains carry
// them explicitly, as compiled code does.
//   hipcc -O3 --offload-arch=gfx950 tools/chainlat.hip -o tools/chainlat
//   ./tools/chainlat  -> one JSON line
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e = (x);                                       \
    if (e != hipSuccess) {                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));  \
      exit(2);                                                \
    }                                                         \
  } while (0)

constexpr int REPS = 32;

#define R4(S) S S S S
#define R32(S) R4(R4(S)) R4(R4(S))

// one operand chain: x depends on itself; k is loop-invariant
#define CHAIN1(NAME, INSN)                                                       \
  __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t iters,     \
                                              unsigned long long *clk) {         \
    uint32_t x = threadIdx.x * 2654435761u, k = blockIdx.x | 1u;                 \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                  \
    const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();              \
    for (uint32_t i = 0; i < iters; ++i) asm volatile(R32(INSN "\n") : "+v"(x) : "v"(k)); \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                  \
    const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();              \
    out[blockIdx.x * 256 + threadIdx.x] = x;                                     \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                   \
      clk[0] = t1 - t0;                                                          \
      clk[1] = w1 - w0;                                                          \
    }                                                                            \
  }

CHAIN1(k_add, "v_add_u32 %0, %0, %1")
CHAIN1(k_add3, "v_add3_u32 %0, %0, %1, %0")
CHAIN1(k_xor, "v_xor_b32 %0, %0, %1")
CHAIN1(k_alignbit, "v_alignbit_b32 %0, %0, %0, 7")
CHAIN1(k_alignbit16, "v_alignbit_b32 %0, %0, %0, 16")
CHAIN1(k_perm, "v_perm_b32 %0, %0, %0, %1")
CHAIN1(k_nop_mov_dpp, "s_nop 1\n v_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf")
CHAIN1(k_nop_add_dpp, "s_nop 1\n v_add_u32_dpp %0, %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf")
// a DPP consumer whose DPP operand was NOT written by the previous
// instruction (the chain runs through the non-DPP operand): no wait states
CHAIN1(k_add_dpp_k, "v_add_u32_dpp %0, %1, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf")
// two dependent ALU ops then a nop'd DPP, the pattern of a rotated row
CHAIN1(k_xor_rot_dpp, "v_xor_b32 %0, %0, %1\n v_alignbit_b32 %0, %0, %0, 12\n s_nop 1\n v_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf")
CHAIN1(k_s_nop1, "s_nop 1\n v_add_u32 %0, %0, %1")

// two independent chains interleaved: issue-bound if latency <= 2 x issue
__global__ __launch_bounds__(256) void k_add_x2(uint32_t *out, uint32_t iters,
                                                unsigned long long *clk) {
  uint32_t x = threadIdx.x, y = x + 7u, k = blockIdx.x | 1u;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i)
    asm volatile(R4(R4("v_add_u32 %0, %0, %2\n v_add_u32 %1, %1, %2\n")) : "+v"(x), "+v"(y) : "v"(k));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = x ^ y;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

// the BLAKE3 G function as one dependent chain (12 ops; 32 per REPS unit
// is not a multiple, so this one reports per G): a += b + m; d = rotr(d^a,16)
// c += d; b = rotr(b^c,12); a += b + m; d = rotr(d^a,8); c += d; b = rotr(b^c,7)
#define GASM                                         \
  "v_add3_u32 %0, %0, %1, %4\n"                      \
  "v_xor_b32 %3, %3, %0\n"                           \
  "v_alignbit_b32 %3, %3, %3, 16\n"                  \
  "v_add_u32 %2, %2, %3\n"                           \
  "v_xor_b32 %1, %1, %2\n"                           \
  "v_alignbit_b32 %1, %1, %1, 12\n"                  \
  "v_add3_u32 %0, %0, %1, %4\n"                      \
  "v_xor_b32 %3, %3, %0\n"                           \
  "v_alignbit_b32 %3, %3, %3, 8\n"                   \
  "v_add_u32 %2, %2, %3\n"                           \
  "v_xor_b32 %1, %1, %2\n"                           \
  "v_alignbit_b32 %1, %1, %1, 7\n"
__global__ __launch_bounds__(256) void k_g(uint32_t *out, uint32_t iters,
                                           unsigned long long *clk) {
  uint32_t a = threadIdx.x, b = a + 1u, c = a + 2u, d = a + 3u, m = blockIdx.x | 1u;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i)
    asm volatile(R4(GASM) : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(m));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

// dependent LDS reads (pointer chase: each address is the word just read)
__global__ __launch_bounds__(256) void k_ds_read(uint32_t *out, uint32_t iters,
                                                 unsigned long long *clk) {
  __shared__ uint32_t lds[256];
  lds[threadIdx.x] = ((threadIdx.x + 1u) & 255u) * 4u;
  __syncthreads();
  uint32_t p = threadIdx.x * 4u;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i)
    asm volatile(R32("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)\n") : "+v"(p) :: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = p;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = w1 - w0;
  }
}

typedef void (*KFn)(uint32_t *, uint32_t, unsigned long long *);

int main(int argc, char **argv) {
  const uint32_t iters = argc > 1 ? uint32_t(atoi(argv[1])) : 2000u;
  const int grid = argc > 2 ? atoi(argv[2]) : 256;  // 256 x 256 lanes: 1 wave / SIMD
  struct {
    const char *name;
    KFn fn;
    double per;  // instructions (or units) per loop iteration
  } ks[] = {
      {"v_add_u32", k_add, REPS},
      {"v_add3_u32", k_add3, REPS},
      {"v_xor_b32", k_xor, REPS},
      {"v_alignbit_b32 (7)", k_alignbit, REPS},
      {"v_alignbit_b32 (16)", k_alignbit16, REPS},
      {"v_perm_b32", k_perm, REPS},
      {"s_nop 1 + v_mov_b32_dpp (pair)", k_nop_mov_dpp, REPS},
      {"s_nop 1 + v_add_u32_dpp (pair)", k_nop_add_dpp, REPS},
      {"v_add_u32_dpp, chain through src1", k_add_dpp_k, REPS},
      {"xor + alignbit + s_nop 1 + mov_dpp (group)", k_xor_rot_dpp, REPS},
      {"s_nop 1 + v_add_u32 (pair)", k_s_nop1, REPS},
      {"v_add_u32, two chains (per instruction)", k_add_x2, 32},
      {"BLAKE3 G, 12 dependent ops (per G)", k_g, 4},
      {"ds_read_b32 pointer chase (per read)", k_ds_read, REPS},
  };
  uint32_t *out;
  unsigned long long *clk, h[2];
  CK(hipMalloc(&out, size_t(grid) * 256 * 4));
  CK(hipMalloc(&clk, 16));
  printf("{\"iters\": %u, \"grid\": %d, \"waves_per_simd\": %.2f, \"cycles\": {", iters, grid,
         grid * 4.0 / 1024.0);
  for (size_t i = 0; i < sizeof(ks) / sizeof(ks[0]); ++i) {
    hipLaunchKernelGGL(ks[i].fn, dim3(grid), dim3(256), 0, 0, out, 10u, clk);  // warm
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(ks[i].fn, dim3(grid), dim3(256), 0, 0, out, iters, clk);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    const double n = double(iters) * ks[i].per;
    printf("%s\"%s\": {\"cyc\": %.2f, \"ns\": %.3f, \"ghz\": %.3f}", i ? ", " : "", ks[i].name,
           double(h[0]) / n, double(h[1]) * 10.0 / n, double(h[0]) / (double(h[1]) * 10.0));
  }
  printf("}}\n");
  CK(hipFree(out));
  CK(hipFree(clk));
  return 0;
}
