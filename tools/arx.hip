// ARX forms on gfx950 (DESIGN.md "Rooflines"): the compiler form (v_add3_u32 /
// v_alignbit_b32, quarter-rate ops) against full-rate forms: rotate = lshr +
// lshl_or, add3 = two adds, rotate-16 = v_pk_add_u16 half swap.  Each kernel
// checks its result against the compiler form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){fprintf(stderr,"%s: %s\n",#x,hipGetErrorString(e)); exit(2);} } while(0)

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t d; asm("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint32_t xor2(uint32_t a, uint32_t b) {
  uint32_t d; asm("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
template <int N> __device__ __forceinline__ uint32_t rotr_lo(uint32_t x) {
  uint32_t h, d;
  asm("v_lshrrev_b32 %0, %1, %2" : "=v"(h) : "i"(N), "v"(x));
  asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(x), "i"(32 - N), "v"(h));
  return d;
}
__device__ __forceinline__ uint32_t rot16_pk(uint32_t x) {
  uint32_t d; asm("v_pk_add_u16 %0, %1, 0 op_sel:[1,0] op_sel_hi:[0,0]" : "=v"(d) : "v"(x)); return d; }
template <int N> __device__ __forceinline__ uint32_t rotr_c(uint32_t x) {
  return (x >> N) | (x << (32 - N)); }
// V: 0 compiler form, 1 full-rate (lshr+lshl_or, two adds), 2 = 1 with pk rot16
// 3: compiler form with rot16 = pk swap; 4: compiler form with add3 = two adds;
// 5: alignbit rotates as asm, two-add add3
template <int N> __device__ __forceinline__ uint32_t rotr_ab(uint32_t x) {
  uint32_t d; asm("v_alignbit_b32 %0, %1, %1, %2" : "=v"(d) : "v"(x), "i"(N)); return d; }
template <int V> __device__ __forceinline__ uint32_t R16(uint32_t x) {
  return (V == 0 || V == 4) ? rotr_c<16>(x) : V == 1 ? rotr_lo<16>(x) : (V == 5 || V == 9) ? rotr_ab<16>(x) : rot16_pk(x); }
template <int V, int N> __device__ __forceinline__ uint32_t R(uint32_t x) {
  return (V == 0 || V == 3 || V == 4) ? rotr_c<N>(x) : (V == 5 || V == 9) ? rotr_ab<N>(x) : rotr_lo<N>(x); }
__device__ __forceinline__ uint32_t add3a(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d; asm("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c)); return d; }
template <int V> __device__ __forceinline__ uint32_t A3(uint32_t a, uint32_t b, uint32_t c) {
  return (V == 0 || V == 3) ? a + b + c : V == 9 ? add3a(a, b, c) : add2(add2(a, b), c); }
template <int V> __device__ __forceinline__ uint32_t A2(uint32_t a, uint32_t b) {
  return (V == 0 || V == 3) ? a + b : add2(a, b); }
template <int V> __device__ __forceinline__ uint32_t X(uint32_t a, uint32_t b) {
  return (V == 0 || V == 3 || V == 4) ? a ^ b : xor2(a, b); }

// one asm block per QR: NOP = s_nop 0 after every instruction
#define NOPS0 ""
#define NOPS1 "s_nop 0\n"
template <int NOP>
__device__ __forceinline__ void QRblk(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  if (NOP)
    asm volatile(
      "v_add_u32 %0, %0, %1\n" NOPS1 "v_xor_b32 %3, %3, %0\n" NOPS1 "v_alignbit_b32 %3, %3, %3, 16\n" NOPS1
      "v_add_u32 %2, %2, %3\n" NOPS1 "v_xor_b32 %1, %1, %2\n" NOPS1 "v_alignbit_b32 %1, %1, %1, 20\n" NOPS1
      "v_add_u32 %0, %0, %1\n" NOPS1 "v_xor_b32 %3, %3, %0\n" NOPS1 "v_alignbit_b32 %3, %3, %3, 24\n" NOPS1
      "v_add_u32 %2, %2, %3\n" NOPS1 "v_xor_b32 %1, %1, %2\n" NOPS1 "v_alignbit_b32 %1, %1, %1, 25\n" NOPS1
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  else
    asm volatile(
      "v_add_u32 %0, %0, %1\n" "v_xor_b32 %3, %3, %0\n" "v_alignbit_b32 %3, %3, %3, 16\n"
      "v_add_u32 %2, %2, %3\n" "v_xor_b32 %1, %1, %2\n" "v_alignbit_b32 %1, %1, %1, 20\n"
      "v_add_u32 %0, %0, %1\n" "v_xor_b32 %3, %3, %0\n" "v_alignbit_b32 %3, %3, %3, 24\n"
      "v_add_u32 %2, %2, %3\n" "v_xor_b32 %1, %1, %2\n" "v_alignbit_b32 %1, %1, %1, 25\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
// the four QRs of a half round interleaved step by step, in one asm block
#define STEP4(op) op(0) op(1) op(2) op(3)
__device__ __forceinline__ void QR4blk(uint32_t &a0, uint32_t &b0, uint32_t &c0, uint32_t &d0,
                                       uint32_t &a1, uint32_t &b1, uint32_t &c1, uint32_t &d1,
                                       uint32_t &a2, uint32_t &b2, uint32_t &c2, uint32_t &d2,
                                       uint32_t &a3, uint32_t &b3, uint32_t &c3, uint32_t &d3) {
#define A_(i) "v_add_u32 %" #i "0, %" #i "0, %" #i "1\n"
  asm volatile(
    "v_add_u32 %0, %0, %1\n v_add_u32 %4, %4, %5\n v_add_u32 %8, %8, %9\n v_add_u32 %12, %12, %13\n"
    "v_xor_b32 %3, %3, %0\n v_xor_b32 %7, %7, %4\n v_xor_b32 %11, %11, %8\n v_xor_b32 %15, %15, %12\n"
    "v_alignbit_b32 %3, %3, %3, 16\n v_alignbit_b32 %7, %7, %7, 16\n v_alignbit_b32 %11, %11, %11, 16\n v_alignbit_b32 %15, %15, %15, 16\n"
    "v_add_u32 %2, %2, %3\n v_add_u32 %6, %6, %7\n v_add_u32 %10, %10, %11\n v_add_u32 %14, %14, %15\n"
    "v_xor_b32 %1, %1, %2\n v_xor_b32 %5, %5, %6\n v_xor_b32 %9, %9, %10\n v_xor_b32 %13, %13, %14\n"
    "v_alignbit_b32 %1, %1, %1, 20\n v_alignbit_b32 %5, %5, %5, 20\n v_alignbit_b32 %9, %9, %9, 20\n v_alignbit_b32 %13, %13, %13, 20\n"
    "v_add_u32 %0, %0, %1\n v_add_u32 %4, %4, %5\n v_add_u32 %8, %8, %9\n v_add_u32 %12, %12, %13\n"
    "v_xor_b32 %3, %3, %0\n v_xor_b32 %7, %7, %4\n v_xor_b32 %11, %11, %8\n v_xor_b32 %15, %15, %12\n"
    "v_alignbit_b32 %3, %3, %3, 24\n v_alignbit_b32 %7, %7, %7, 24\n v_alignbit_b32 %11, %11, %11, 24\n v_alignbit_b32 %15, %15, %15, 24\n"
    "v_add_u32 %2, %2, %3\n v_add_u32 %6, %6, %7\n v_add_u32 %10, %10, %11\n v_add_u32 %14, %14, %15\n"
    "v_xor_b32 %1, %1, %2\n v_xor_b32 %5, %5, %6\n v_xor_b32 %9, %9, %10\n v_xor_b32 %13, %13, %14\n"
    "v_alignbit_b32 %1, %1, %1, 25\n v_alignbit_b32 %5, %5, %5, 25\n v_alignbit_b32 %9, %9, %9, 25\n v_alignbit_b32 %13, %13, %13, 25\n"
    : "+v"(a0), "+v"(b0), "+v"(c0), "+v"(d0), "+v"(a1), "+v"(b1), "+v"(c1), "+v"(d1),
      "+v"(a2), "+v"(b2), "+v"(c2), "+v"(d2), "+v"(a3), "+v"(b3), "+v"(c3), "+v"(d3));
}

template <int V>
__device__ __forceinline__ void G(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                  uint32_t mx, uint32_t my) {
  a = A3<V>(a, b, mx); d = R16<V>(X<V>(d, a)); c = A2<V>(c, d); b = R<V, 12>(X<V>(b, c));
  a = A3<V>(a, b, my); d = R<V, 8>(X<V>(d, a)); c = A2<V>(c, d); b = R<V, 7>(X<V>(b, c));
}
template <int V>
__device__ __forceinline__ void QR(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  a = A2<V>(a, b); d = R16<V>(X<V>(d, a)); c = A2<V>(c, d); b = R<V, 20>(X<V>(b, c));
  a = A2<V>(a, b); d = R<V, 24>(X<V>(d, a)); c = A2<V>(c, d); b = R<V, 25>(X<V>(b, c));
}

template <int V>
__global__ __launch_bounds__(256) void k_blake(uint32_t *out, uint32_t iters) {
  uint32_t v[16], m[16];
  for (int i = 0; i < 16; ++i) { v[i] = threadIdx.x * 977u + i * 0x9e3779b9u; m[i] = blockIdx.x * 31u + i * 0x85ebca6bu; }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      G<V>(v[0], v[4], v[8], v[12], m[0], m[1]);  G<V>(v[1], v[5], v[9], v[13], m[2], m[3]);
      G<V>(v[2], v[6], v[10], v[14], m[4], m[5]); G<V>(v[3], v[7], v[11], v[15], m[6], m[7]);
      G<V>(v[0], v[5], v[10], v[15], m[8], m[9]); G<V>(v[1], v[6], v[11], v[12], m[10], m[11]);
      G<V>(v[2], v[7], v[8], v[13], m[12], m[13]); G<V>(v[3], v[4], v[9], v[14], m[14], m[15]);
      G<V>(v[0], v[4], v[8], v[12], m[15], m[14]);  G<V>(v[1], v[5], v[9], v[13], m[13], m[12]);
      G<V>(v[2], v[6], v[10], v[14], m[11], m[10]); G<V>(v[3], v[7], v[11], v[15], m[9], m[8]);
      G<V>(v[0], v[5], v[10], v[15], m[7], m[6]); G<V>(v[1], v[6], v[11], v[12], m[5], m[4]);
      G<V>(v[2], v[7], v[8], v[13], m[3], m[2]); G<V>(v[3], v[4], v[9], v[14], m[1], m[0]);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x = x * 31 + v[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int V>
__global__ __launch_bounds__(256) void k_chacha(uint32_t *out, uint32_t iters) {
  uint32_t v[16];
  for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 977u + i * 0x9e3779b9u + blockIdx.x;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
     if constexpr (V == 6 || V == 7) {
      QRblk<V - 6>(v[0], v[4], v[8], v[12]);  QRblk<V - 6>(v[1], v[5], v[9], v[13]);
      QRblk<V - 6>(v[2], v[6], v[10], v[14]); QRblk<V - 6>(v[3], v[7], v[11], v[15]);
      QRblk<V - 6>(v[0], v[5], v[10], v[15]); QRblk<V - 6>(v[1], v[6], v[11], v[12]);
      QRblk<V - 6>(v[2], v[7], v[8], v[13]);  QRblk<V - 6>(v[3], v[4], v[9], v[14]);
     } else if constexpr (V == 8) {
      QR4blk(v[0], v[4], v[8], v[12], v[1], v[5], v[9], v[13], v[2], v[6], v[10], v[14], v[3], v[7], v[11], v[15]);
      QR4blk(v[0], v[5], v[10], v[15], v[1], v[6], v[11], v[12], v[2], v[7], v[8], v[13], v[3], v[4], v[9], v[14]);
     } else {
      QR<V>(v[0], v[4], v[8], v[12]);  QR<V>(v[1], v[5], v[9], v[13]);
      QR<V>(v[2], v[6], v[10], v[14]); QR<V>(v[3], v[7], v[11], v[15]);
      QR<V>(v[0], v[5], v[10], v[15]); QR<V>(v[1], v[6], v[11], v[12]);
      QR<V>(v[2], v[7], v[8], v[13]);  QR<V>(v[3], v[4], v[9], v[14]);
     }
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x = x * 31 + v[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

typedef void (*Kf)(uint32_t *, uint32_t);
static int g_lds = 0;  // dynamic LDS per block: limits blocks (= waves per SIMD) per CU
static double run(const char *name, Kf k, uint32_t *out, int grid, uint32_t iters,
                  double units, int instr_per_unit, uint32_t *ref) {
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), g_lds, 0, out, iters); CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), g_lds, 0, out, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  static uint32_t h[1 << 22], hr[1 << 22];
  const size_t n = size_t(grid) * 256;
  CK(hipMemcpy(h, out, n * 4, hipMemcpyDeviceToHost));
  bool ok = true;
  if (ref) { CK(hipMemcpy(hr, ref, n * 4, hipMemcpyDeviceToHost)); ok = memcmp(h, hr, n * 4) == 0; }
  const double waves_per_simd = double(grid) * 4 / 1024;
  const double ns = best * 1e6 / (waves_per_simd * iters * units);
  printf("lds %6d %-16s grid %6d  %8.3f ms  %7.3f ns/unit/SIMD = %5.1f cyc at 2.1 GHz  (%d instr: %.2f cyc/instr)  %s\n",
         g_lds, name, grid, best, ns, ns * 2.1, instr_per_unit, ns * 2.1 / instr_per_unit,
         ref ? (ok ? "match" : "MISMATCH") : "ref");
  return best;
}

int main() {
  uint32_t *out[3];
  for (auto &o : out) CK(hipMalloc(&o, size_t(4) << 22));
  const uint32_t it = 256;
  for (int lds : {0}) {
  g_lds = lds;
  for (int grid : {256, 512, 16384}) {
    run("blake_asm_add3", k_blake<9>, out[1], grid, it, 32, 12, nullptr);
    run("blake_c", k_blake<0>, out[0], grid, it, 32, 12, nullptr);
    run("blake_fast", k_blake<1>, out[1], grid, it, 32, 18, out[0]);
    run("blake_fast_pk", k_blake<2>, out[2], grid, it, 32, 17, out[0]);
    run("blake_c_pk16", k_blake<3>, out[1], grid, it, 32, 12, out[0]);
    run("blake_c_2add", k_blake<4>, out[1], grid, it, 32, 14, out[0]);
    run("blake_asm_2add", k_blake<5>, out[1], grid, it, 32, 14, out[0]);
    run("chacha_c", k_chacha<0>, out[0], grid, it, 32, 12, nullptr);
    run("chacha_c_pk16", k_chacha<3>, out[1], grid, it, 32, 12, out[0]);
    run("chacha_asm", k_chacha<5>, out[1], grid, it, 32, 12, out[0]);
    run("chacha_blk", k_chacha<6>, out[1], grid, it, 32, 12, out[0]);
    run("chacha_blk_nop", k_chacha<7>, out[1], grid, it, 32, 12, out[0]);
    run("chacha_blk4", k_chacha<8>, out[1], grid, it, 32, 12, out[0]);
    run("chacha_fast", k_chacha<1>, out[1], grid, it, 32, 16, out[0]);
    run("chacha_fast_pk", k_chacha<2>, out[2], grid, it, 32, 15, out[0]);
  }
  }
  return 0;
}
