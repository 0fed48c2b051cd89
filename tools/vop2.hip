// Microbenchmark: does a BLAKE3 G / ChaCha20 quarter-round written only in
// 4-byte VOP2 instructions (v_add_u32, v_xor_b32, v_lshlrev_b32,
// v_lshrrev_b32, v_or_b32) beat the compiler's VOP3 form (v_add3_u32,
// v_alignbit_b32) on gfx950?  tools/pairs.hip measured pure VOP2 streams at
// ~2.15 cycles per wave64 instruction and any stream holding VOP3 at ~3.85;
// the VOP2 form needs 20 (ChaCha) / 22 (BLAKE3) instructions instead of 12.
//
// Each lane runs full 16-word states through rounds of 8 G (column + diagonal)
// with 16 message registers, so ILP and register pressure resemble the real
// kernels.  Every instruction is its own non-volatile asm statement, so the
// compiler still schedules and allocates, but cannot re-fuse them.
// Build: hipcc -O3 --offload-arch=gfx950 tools/vop2.hip -o tools/vop2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){fprintf(stderr,"%s: %s\n",#x,hipGetErrorString(e)); exit(2);} } while(0)

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t d; asm("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint32_t xor2(uint32_t a, uint32_t b) {
  uint32_t d; asm("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
template <int N> __device__ __forceinline__ uint32_t rotr_vop2(uint32_t x) {
  uint32_t h, l, d;
  asm("v_lshrrev_b32 %0, %1, %2" : "=v"(h) : "i"(N), "v"(x));
  asm("v_lshlrev_b32 %0, %1, %2" : "=v"(l) : "i"(32 - N), "v"(x));
  asm("v_or_b32 %0, %1, %2" : "=v"(d) : "v"(h), "v"(l));
  return d;
}
template <int N> __device__ __forceinline__ uint32_t rotr_c(uint32_t x) {
  return (x >> N) | (x << (32 - N)); }

// VARIANT 0: plain C (compiler: add3/alignbit).  1: pure VOP2.  2: VOP2
// rotates only (adds left to the compiler).
template <int V>
__device__ __forceinline__ void G(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                  uint32_t mx, uint32_t my) {
  if constexpr (V == 0) {
    a = a + b + mx; d = rotr_c<16>(d ^ a); c = c + d; b = rotr_c<12>(b ^ c);
    a = a + b + my; d = rotr_c<8>(d ^ a);  c = c + d; b = rotr_c<7>(b ^ c);
  } else if constexpr (V == 1) {
    a = add2(add2(a, b), mx); d = rotr_vop2<16>(xor2(d, a)); c = add2(c, d); b = rotr_vop2<12>(xor2(b, c));
    a = add2(add2(a, b), my); d = rotr_vop2<8>(xor2(d, a));  c = add2(c, d); b = rotr_vop2<7>(xor2(b, c));
  } else {
    a = a + b + mx; d = rotr_vop2<16>(d ^ a); c = c + d; b = rotr_vop2<12>(b ^ c);
    a = a + b + my; d = rotr_vop2<8>(d ^ a);  c = c + d; b = rotr_vop2<7>(b ^ c);
  }
}
// ChaCha QR (rotl 16,12,8,7 == rotr 16,20,24,25), no message words.
template <int V>
__device__ __forceinline__ void QR(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  if constexpr (V == 0) {
    a += b; d = rotr_c<16>(d ^ a); c += d; b = rotr_c<20>(b ^ c);
    a += b; d = rotr_c<24>(d ^ a); c += d; b = rotr_c<25>(b ^ c);
  } else {
    a = add2(a, b); d = rotr_vop2<16>(xor2(d, a)); c = add2(c, d); b = rotr_vop2<20>(xor2(b, c));
    a = add2(a, b); d = rotr_vop2<24>(xor2(d, a)); c = add2(c, d); b = rotr_vop2<25>(xor2(b, c));
  }
}

template <int V>
__global__ __launch_bounds__(256) void k_blake(uint32_t *out, uint32_t iters) {
  uint32_t v[16], m[16];
  for (int i = 0; i < 16; ++i) { v[i] = threadIdx.x * 977u + i * 0x9e3779b9u; m[i] = blockIdx.x * 31u + i; }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      G<V>(v[0], v[4], v[8], v[12], m[0], m[1]);  G<V>(v[1], v[5], v[9], v[13], m[2], m[3]);
      G<V>(v[2], v[6], v[10], v[14], m[4], m[5]); G<V>(v[3], v[7], v[11], v[15], m[6], m[7]);
      G<V>(v[0], v[5], v[10], v[15], m[8], m[9]); G<V>(v[1], v[6], v[11], v[12], m[10], m[11]);
      G<V>(v[2], v[7], v[8], v[13], m[12], m[13]); G<V>(v[3], v[4], v[9], v[14], m[14], m[15]);
      uint32_t t = m[0];
      for (int i = 0; i < 15; ++i) m[i] = m[i + 1];
      m[15] = t;
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int V>
__global__ __launch_bounds__(256) void k_chacha(uint32_t *out, uint32_t iters) {
  uint32_t v[16];
  for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 977u + i * 0x9e3779b9u + blockIdx.x;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      QR<V>(v[0], v[4], v[8], v[12]);  QR<V>(v[1], v[5], v[9], v[13]);
      QR<V>(v[2], v[6], v[10], v[14]); QR<V>(v[3], v[7], v[11], v[15]);
      QR<V>(v[0], v[5], v[10], v[15]); QR<V>(v[1], v[6], v[11], v[12]);
      QR<V>(v[2], v[7], v[8], v[13]);  QR<V>(v[3], v[4], v[9], v[14]);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x ^= v[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <typename K>
static void run(const char *name, K kern, uint32_t *out, int grid, uint32_t iters,
                double gs_per_iter_per_lane) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, iters); CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, iters);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  double waves = double(grid) * 4;             // 4 wave64 per 256-lane block
  double gs = waves * iters * gs_per_iter_per_lane;   // G (or QR) per wave
  // ns per G per wave per SIMD: 1024 SIMDs.
  double ns_per_g_simd = best * 1e6 * 1024.0 / gs;
  printf("%-14s grid %6d  %9.3f ms  %7.3f ns/G/wave/SIMD  (= %.1f cyc at 2.4 GHz, %.1f at 2.1)\n",
         name, grid, best, ns_per_g_simd, ns_per_g_simd * 2.4, ns_per_g_simd * 2.1);
}

int main() {
  uint32_t *out; CK(hipMalloc(&out, 65536 * 256 * 4));
  const uint32_t it = 64;
  for (int grid : {2048, 8192}) {
    run("blake_c", k_blake<0>, out, grid, it, 56.0);
    run("blake_vop2", k_blake<1>, out, grid, it, 56.0);
    run("blake_rotvop2", k_blake<2>, out, grid, it, 56.0);
    run("chacha_c", k_chacha<0>, out, grid, it, 80.0);
    run("chacha_vop2", k_chacha<1>, out, grid, it, 80.0);
  }
  return 0;
}
