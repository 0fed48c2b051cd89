// xor-then-rotate-by-16 as two 16-bit ops (gfx950): rotr16(d ^ a) =
//   lo <- d.hi ^ a.hi  (v_bitop3_b16 op_sel:[1,1,0,0])
//   hi <- d.lo ^ a.lo  (v_bitop3_b16 op_sel:[0,0,0,1], low half kept)
// against v_xor_b32 + v_alignbit_b32 (one full-rate + one half-rate op).
// Checks the identity on random words, then times BLAKE3 G / ChaCha20 QR
// chains in both forms (asm statements, as in post_kernels.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#define CK(x) do { hipError_t e=(x); if(e!=hipSuccess){fprintf(stderr,"%s: %s\n",#x,hipGetErrorString(e)); exit(2);} } while(0)

__device__ __forceinline__ uint32_t add2(uint32_t a, uint32_t b) {
  uint32_t d; asm("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d; asm("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c)); return d; }
__device__ __forceinline__ uint32_t xor2(uint32_t a, uint32_t b) {
  uint32_t d; asm("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b)); return d; }
template <int N> __device__ __forceinline__ uint32_t rot(uint32_t x) {
  uint32_t d; asm("v_alignbit_b32 %0, %1, %1, %2" : "=v"(d) : "v"(x), "i"(N)); return d; }
__device__ __forceinline__ uint32_t xrot16_b16(uint32_t d, uint32_t a) {
  uint32_t t;
  asm("v_bitop3_b16 %0, %1, %2, %2 bitop3:0x3c op_sel:[1,1,0,0]" : "=v"(t) : "v"(d), "v"(a));
  asm("v_bitop3_b16 %0, %1, %2, %2 bitop3:0x3c op_sel:[0,0,0,1]" : "+v"(t) : "v"(d), "v"(a));
  return t;
}
template <int V> __device__ __forceinline__ uint32_t XR16(uint32_t d, uint32_t a) {
  return V ? xrot16_b16(d, a) : rot<16>(xor2(d, a)); }

template <int V>
__device__ __forceinline__ void G(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d,
                                  uint32_t mx, uint32_t my) {
  a = add3(a, b, mx); d = XR16<V>(d, a); c = add2(c, d); b = rot<12>(xor2(b, c));
  a = add3(a, b, my); d = rot<8>(xor2(d, a)); c = add2(c, d); b = rot<7>(xor2(b, c));
}
template <int V>
__device__ __forceinline__ void QR(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t &d) {
  a = add2(a, b); d = XR16<V>(d, a); c = add2(c, d); b = rot<20>(xor2(b, c));
  a = add2(a, b); d = rot<24>(xor2(d, a)); c = add2(c, d); b = rot<25>(xor2(b, c));
}

__global__ void k_check(const uint32_t *x, const uint32_t *y, uint32_t *o0, uint32_t *o1) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  o0[i] = XR16<0>(x[i], y[i]);
  o1[i] = XR16<1>(x[i], y[i]);
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
      QR<V>(v[0], v[4], v[8], v[12]);  QR<V>(v[1], v[5], v[9], v[13]);
      QR<V>(v[2], v[6], v[10], v[14]); QR<V>(v[3], v[7], v[11], v[15]);
      QR<V>(v[0], v[5], v[10], v[15]); QR<V>(v[1], v[6], v[11], v[12]);
      QR<V>(v[2], v[7], v[8], v[13]);  QR<V>(v[3], v[4], v[9], v[14]);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 16; ++i) x = x * 31 + v[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}
typedef void (*Kf)(uint32_t *, uint32_t);
static void run(const char *name, Kf k, uint32_t *out, int grid, uint32_t iters,
                double units, uint32_t *ref) {
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, iters); CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, out, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
  }
  static uint32_t h[1 << 22], hr[1 << 22];
  const size_t n = size_t(grid) * 256;
  bool ok = true;
  if (ref) {
    CK(hipMemcpy(h, out, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr, ref, n * 4, hipMemcpyDeviceToHost));
    ok = memcmp(h, hr, n * 4) == 0;
  }
  const double waves_per_simd = double(grid) * 4 / 1024;
  const double ns = best * 1e6 / (waves_per_simd * iters * units);
  printf("%-12s grid %6d  %8.3f ms  %6.1f cyc/unit at 2.1 GHz  %s\n", name, grid, best, ns * 2.1,
         ref ? (ok ? "match" : "MISMATCH") : "ref");
}
int main() {
  const int n = 1 << 20;
  uint32_t *x, *y, *o0, *o1;
  CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4)); CK(hipMalloc(&o0, n * 4)); CK(hipMalloc(&o1, n * 4));
  static uint32_t hx[1 << 20], hy[1 << 20], h0[1 << 20], h1[1 << 20];
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17; hx[i] = uint32_t(s);
    s ^= s << 13; s ^= s >> 7; s ^= s << 17; hy[i] = uint32_t(s >> 32);
  }
  CK(hipMemcpy(x, hx, n * 4, hipMemcpyHostToDevice)); CK(hipMemcpy(y, hy, n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, x, y, o0, o1);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h0, o0, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(h1, o1, n * 4, hipMemcpyDeviceToHost));
  int bad0 = 0, bad1 = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t t = hx[i] ^ hy[i], want = (t >> 16) | (t << 16);
    bad0 += h0[i] != want; bad1 += h1[i] != want;
  }
  printf("identity: alignbit form %d bad, b16 form %d bad of %d\n", bad0, bad1, n);
  uint32_t *out[2];
  for (auto &o : out) CK(hipMalloc(&o, size_t(4) << 22));
  const uint32_t it = 256;
  for (int grid : {512, 16384}) {
    run("blake_ab", k_blake<0>, out[0], grid, it, 32, nullptr);
    run("blake_b16", k_blake<1>, out[1], grid, it, 32, out[0]);
    run("chacha_ab", k_chacha<0>, out[0], grid, it, 32, nullptr);
    run("chacha_b16", k_chacha<1>, out[1], grid, it, 32, out[0]);
    run("blake_ab", k_blake<0>, out[0], grid, it, 32, nullptr);
    run("blake_b16", k_blake<1>, out[1], grid, it, 32, out[0]);
  }
  return bad1 ? 1 : 0;
}
