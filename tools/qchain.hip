// qchain.hip -- the quad-layout BLAKE3 compression chain (post_kernels.hip
// quad_compress) in isolation, on gfx950 (not product code; VERDICT r5 next
// #4).  One wave per SIMD; each quad runs ITERS dependent compressions of its
// own 64-B LDS message slot (the CV of one feeds the next, like a chunk's 16
// blocks); thread 0 of workgroup 0 reads s_memtime around the loop.
// Variants (all must give the same CVs; main() checks them against v0):
//   v0  the product's quad_compress (C, compiler-scheduled; copied verbatim)
//   v1  v0 with the round's 4 message words read one round ahead
//   v2  each round as one hand-scheduled asm block: the three row rotations
//       as v_mov_b32_dpp placed in the chain's latency gaps, the first add
//       of the next step split as (a + m) then v_add_u32_dpp, one s_nop 0
//       per step change (DPP source written 2 instructions before)
//   v3  v2 with message words read one round ahead
//   hipcc -O3 --offload-arch=gfx950 tools/qchain.hip -o tools/qchain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                 \
  do {                                                        \
    hipError_t e = (x);                                       \
    if (e != hipSuccess) {                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));  \
      exit(2);                                                \
    }                                                         \
  } while (0)

struct Sched {
  int s[7][16];
};
constexpr Sched make_sched() {
  constexpr int perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  Sched t{};
  for (int i = 0; i < 16; ++i) t.s[0][i] = i;
  for (int r = 1; r < 7; ++r)
    for (int i = 0; i < 16; ++i) t.s[r][i] = t.s[r - 1][perm[i]];
  return t;
}
constexpr Sched kSched = make_sched();

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t qrot1(uint32_t x) {
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x39, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t qrot2(uint32_t x) {
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x4E, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t qrot3(uint32_t x) {
  return uint32_t(__builtin_amdgcn_mov_dpp(int(x), 0x93, 0xF, 0xF, true));
}
__device__ __forceinline__ uint32_t qsel(uint32_t q, uint32_t x0, uint32_t x1, uint32_t x2,
                                         uint32_t x3) {
  return q == 0 ? x0 : q == 1 ? x1 : q == 2 ? x2 : x3;
}
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t ldsw(uint32_t addr) {
  return *reinterpret_cast<const lds_u32 *>(addr);
}

#define QG(a, b, c, d, x, y) \
  a = a + b + (x);           \
  d = rotr(d ^ a, 16);       \
  c = c + d;                 \
  b = rotr(b ^ c, 12);       \
  a = a + b + (y);           \
  d = rotr(d ^ a, 8);        \
  c = c + d;                 \
  b = rotr(b ^ c, 7);

// v0: verbatim copy of the product's quad_compress
__device__ __forceinline__ void qc_v0(uint32_t &a, uint32_t &b, uint32_t c, uint32_t d,
                                      const uint32_t (&addr)[28]) {
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const uint32_t m0 = ldsw(addr[4 * r]);
    const uint32_t m1 = ldsw(addr[4 * r + 1]);
    const uint32_t m2 = ldsw(addr[4 * r + 2]);
    const uint32_t m3 = ldsw(addr[4 * r + 3]);
    QG(a, b, c, d, m0, m1);
    b = qrot1(b);
    c = qrot2(c);
    d = qrot3(d);
    QG(a, b, c, d, m2, m3);
    b = qrot3(b);
    c = qrot2(c);
    d = qrot1(d);
  }
  a ^= c;
  b ^= d;
}

// v1: round r+1's words read during round r
__device__ __forceinline__ void qc_v1(uint32_t &a, uint32_t &b, uint32_t c, uint32_t d,
                                      const uint32_t (&addr)[28]) {
  uint32_t m[4] = {ldsw(addr[0]), ldsw(addr[1]), ldsw(addr[2]), ldsw(addr[3])};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint32_t n[4] = {0, 0, 0, 0};
    if (r < 6) {
#pragma unroll
      for (int k = 0; k < 4; ++k) n[k] = ldsw(addr[4 * r + 4 + k]);
    }
    QG(a, b, c, d, m[0], m[1]);
    b = qrot1(b);
    c = qrot2(c);
    d = qrot3(d);
    QG(a, b, c, d, m[2], m[3]);
    b = qrot3(b);
    c = qrot2(c);
    d = qrot1(d);
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = n[k];
  }
  a ^= c;
  b ^= d;
}

// One round in asm.  In: a, b, c, d unrotated, t = a + m0 (the first add's
// message half, off the chain), m1, m2, m3.  Out: a, b, c, d unrotated and the
// dst of the last add folded: the caller's next round starts with
// a = rot?(b) + t.  The row rotations are v_mov_b32_dpp into the chain's
// latency gaps; a DPP read of a VGPR written by one of the two instructions
// before it needs wait states (one s_nop 0 per step change here).
//   quad_perm [1,2,3,0] = lane q <- q+1 (b of the diagonal step, d back)
//             [2,3,0,1] = q <- q+2 (c both ways)
//             [3,0,1,2] = q <- q+3 (d of the diagonal step, b back)
#define QROUND_ASM                                                              \
  /* column step: a = b + t (t = a + m0, its first add) */                      \
  "v_add_u32 %0, %1, %4\n"                                                      \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 12\n"                                             \
  "v_add3_u32 %0, %0, %1, %5\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_add_u32 %4, %0, %6\n"                          /* t = a + m2 (filler) */   \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_mov_b32_dpp %3, %3 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"       \
  "v_alignbit_b32 %1, %1, %1, 7\n"                                              \
  "v_mov_b32_dpp %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"       \
  "s_nop 0\n"                                                                   \
  /* diagonal step: a = rot1(b) + t, then b itself rotated in the gap */        \
  "v_add_u32_dpp %0, %1, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_mov_b32_dpp %1, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"       \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 12\n"                                             \
  "v_add3_u32 %0, %0, %1, %7\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_mov_b32_dpp %3, %3 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"       \
  "v_alignbit_b32 %1, %1, %1, 7\n"                                              \
  "v_mov_b32_dpp %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"       \
  "s_nop 0\n"                                                                   \
  "v_mov_b32_dpp %1, %1 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"

// v2: asm rounds, words read at the start of each round
__device__ __forceinline__ void qc_v2(uint32_t &a, uint32_t &b, uint32_t c, uint32_t d,
                                      const uint32_t (&addr)[28]) {
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const uint32_t m0 = ldsw(addr[4 * r]);
    const uint32_t m1 = ldsw(addr[4 * r + 1]);
    const uint32_t m2 = ldsw(addr[4 * r + 2]);
    const uint32_t m3 = ldsw(addr[4 * r + 3]);
    uint32_t t = a + m0;
    asm volatile(QROUND_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                 : "v"(m1), "v"(m2), "v"(m3));
  }
  a ^= c;
  b ^= d;
}

// v3: v2 with round r+1's words read during round r
__device__ __forceinline__ void qc_v3(uint32_t &a, uint32_t &b, uint32_t c, uint32_t d,
                                      const uint32_t (&addr)[28]) {
  uint32_t m[4] = {ldsw(addr[0]), ldsw(addr[1]), ldsw(addr[2]), ldsw(addr[3])};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint32_t n[4] = {0, 0, 0, 0};
    if (r < 6) {
#pragma unroll
      for (int k = 0; k < 4; ++k) n[k] = ldsw(addr[4 * r + 4 + k]);
    }
    uint32_t t = a + m[0];
    asm volatile(QROUND_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                 : "v"(m[1]), "v"(m[2]), "v"(m[3]));
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = n[k];
  }
  a ^= c;
  b ^= d;
}

// v4: every row rotation folded into its first consumer (v_add_u32_dpp /
// v_xor_b32_dpp, DPP on src0), the state left in the diagonal frame between
// steps: b, c, d go to lanes q+1, q+2, q+3 for the diagonal step and back
// in the next column step; a never moves.  Per round 26 ARX instructions,
// one filler add and two s_nop 0 (a DPP read of a VGPR written by one of
// the two instructions before it) instead of 33.
#define QCOL0_ASM                                                               \
  "v_add_u32 %0, %1, %4\n"                                                      \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 12\n"
#define QCOL_ASM                                                                \
  "s_nop 0\n"                                                                   \
  "v_add_u32_dpp %0, %1, %4 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %3, %3, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32_dpp %2, %2, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %1, %1, %2 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %1, %1, %1, 12\n"
#define QREST_ASM                                                               \
  "v_add3_u32 %0, %0, %1, %5\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 7\n"                                              \
  "v_add_u32 %4, %0, %6\n"                                                      \
  "s_nop 0\n"                                                                   \
  "v_add_u32_dpp %0, %1, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %3, %3, %0 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %3, %3, %3, 16\n"                                             \
  "v_add_u32_dpp %2, %2, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"   \
  "v_xor_b32_dpp %1, %1, %2 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"   \
  "v_alignbit_b32 %1, %1, %1, 12\n"                                             \
  "v_add3_u32 %0, %0, %1, %7\n"                                                 \
  "v_xor_b32 %3, %3, %0\n"                                                      \
  "v_alignbit_b32 %3, %3, %3, 8\n"                                              \
  "v_add_u32 %2, %2, %3\n"                                                      \
  "v_xor_b32 %1, %1, %2\n"                                                      \
  "v_alignbit_b32 %1, %1, %1, 7\n"

__device__ __forceinline__ void qc_v4(uint32_t &a, uint32_t &b, uint32_t c, uint32_t d,
                                      const uint32_t (&addr)[28]) {
  uint32_t m[4] = {ldsw(addr[0]), ldsw(addr[1]), ldsw(addr[2]), ldsw(addr[3])};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint32_t n[4] = {0, 0, 0, 0};
    if (r < 6) {
#pragma unroll
      for (int k = 0; k < 4; ++k) n[k] = ldsw(addr[4 * r + 4 + k]);
    }
    uint32_t t = a + m[0];
    if (r == 0)
      asm volatile(QCOL0_ASM QREST_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                   : "v"(m[1]), "v"(m[2]), "v"(m[3]));
    else
      asm volatile(QCOL_ASM QREST_ASM : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(t)
                   : "v"(m[1]), "v"(m[2]), "v"(m[3]));
#pragma unroll
    for (int k = 0; k < 4; ++k) m[k] = n[k];
  }
  // back from the diagonal frame: a ^= c_q, b = b_q ^ d_q
  uint32_t u;
  asm volatile("v_xor_b32_dpp %0, %2, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
               "s_nop 1\n"
               "v_mov_b32_dpp %4, %1 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"
               "v_xor_b32_dpp %1, %3, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
               : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "=&v"(u));
}

template <int V>
__global__ __launch_bounds__(256) void k_chain(const uint32_t *msg, uint32_t *out, uint32_t iters,
                                               unsigned long long *clk) {
  __shared__ uint32_t slots[64 * 16];  // 64 quads x 64 B
  const uint32_t tid = threadIdx.x, q = tid & 3u, quad = tid >> 2;
  for (uint32_t i = tid; i < 64 * 16; i += 256) slots[i] = msg[(blockIdx.x * 1024 + i) & 4095];
  __syncthreads();
  const uint32_t slot = uint32_t(reinterpret_cast<uintptr_t>(
      (const __attribute__((address_space(3))) void *)(slots + quad * 16)));
  uint32_t addr[28];
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    constexpr int kk[4] = {0, 1, 8, 9};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t w = qsel(q, kSched.s[r][kk[k]], kSched.s[r][kk[k] + 2],
                              kSched.s[r][kk[k] + 4], kSched.s[r][kk[k] + 6]);
      addr[4 * r + k] = slot + 4u * w;
    }
  }
  const uint32_t iv[4] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au};
  uint32_t cl = msg[q] ^ blockIdx.x, ch = msg[4 + q];
  const uint32_t ivq = qsel(q, iv[0], iv[1], iv[2], iv[3]);
  const uint32_t dq = qsel(q, quad, 0u, 64u, 3u);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; ++i) {
    // as in k_quad, where each block is stored into the slot before its
    // compression: the words must be read from LDS every time
    asm volatile("" ::: "memory");
    if constexpr (V == 0) qc_v0(cl, ch, ivq, dq, addr);
    if constexpr (V == 1) qc_v1(cl, ch, ivq, dq, addr);
    if constexpr (V == 2) qc_v2(cl, ch, ivq, dq, addr);
    if constexpr (V == 3) qc_v3(cl, ch, ivq, dq, addr);
    if constexpr (V == 4) qc_v4(cl, ch, ivq, dq, addr);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[(blockIdx.x * 256 + tid) * 2] = cl;
  out[(blockIdx.x * 256 + tid) * 2 + 1] = ch;
  if (blockIdx.x == 0 && tid == 0) clk[0] = t1 - t0;
}

int main(int argc, char **argv) {
  const uint32_t iters = argc > 1 ? uint32_t(atoi(argv[1])) : 256u;
  const int grid = argc > 2 ? atoi(argv[2]) : 1024;  // 1024 x 4 waves = 4/CU... see below
  // 256-lane workgroups; grid 1024 on 256 CUs = 4 waves per SIMD... use
  // grid 256 for one wave per SIMD (the index node's latency case)
  uint32_t *msg, *out;
  unsigned long long *clk;
  CK(hipMalloc(&msg, 4096 * 4));
  CK(hipMalloc(&out, size_t(grid) * 256 * 8));
  CK(hipMalloc(&clk, 8));
  uint32_t h[4096];
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 4096; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    h[i] = uint32_t(x);
  }
  CK(hipMemcpy(msg, h, sizeof h, hipMemcpyHostToDevice));
  void (*ks[5])(const uint32_t *, uint32_t *, uint32_t, unsigned long long *) = {
      k_chain<0>, k_chain<1>, k_chain<2>, k_chain<3>, k_chain<4>};
  uint32_t *ref = static_cast<uint32_t *>(malloc(size_t(grid) * 256 * 8));
  uint32_t *got = static_cast<uint32_t *>(malloc(size_t(grid) * 256 * 8));
  printf("{\"iters\": %u, \"grid\": %d, \"variants\": {", iters, grid);
  for (int v = 0; v < 5; ++v) {
    hipLaunchKernelGGL(ks[v], dim3(grid), dim3(256), 0, 0, msg, out, 4u, clk);
    CK(hipDeviceSynchronize());
    unsigned long long best = ~0ull;
    for (int rep = 0; rep < 3; ++rep) {
      hipLaunchKernelGGL(ks[v], dim3(grid), dim3(256), 0, 0, msg, out, iters, clk);
      CK(hipDeviceSynchronize());
      unsigned long long c;
      CK(hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost));
      if (c < best) best = c;
    }
    CK(hipMemcpy(v == 0 ? ref : got, out, size_t(grid) * 256 * 8, hipMemcpyDeviceToHost));
    const bool same = v == 0 || memcmp(ref, got, size_t(grid) * 256 * 8) == 0;
    printf("%s\"v%d\": {\"cycles_per_compression\": %.1f, \"same_as_v0\": %s}", v ? ", " : "",
           v, double(best) / iters, same ? "true" : "false");
  }
  printf("}}\n");
  return 0;
}
