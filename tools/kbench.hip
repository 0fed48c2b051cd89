// kbench.hip -- microbenchmarks for the DEK kernel design (not product code).
//
// Variants of the keyed-BLAKE3 pass over 1 MiB messages, timed with HIP
// events on one stream, outputs compared against the production kernel:
//   prod    : production k_pass<4,false,true>
//   noload  : same structure, message words synthesised in registers
//             (VALU ceiling of this code shape; output differs by design)
//   valu    : pure int-VALU loop (add3/xor/alignbit mix) -> practical peak
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kbench.hip -o tools/kbench
#include "../glfs_amd/csrc/post_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace glfsx;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e));        \
      exit(2);                                                             \
    }                                                                      \
  } while (0)

namespace {

// Pure VALU: 4 independent G-function chains per lane, ITER iterations.
__global__ __launch_bounds__(256) void k_valu(uint32_t *out, uint32_t iters) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 16 + i;
  for (uint32_t it = 0; it < iters; ++it) {
    B3G(v[0], v[4], v[8], v[12], it, v[1]);
    B3G(v[1], v[5], v[9], v[13], v[2], it);
    B3G(v[2], v[6], v[10], v[14], it, v[3]);
    B3G(v[3], v[7], v[11], v[15], v[0], it);
  }
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) x ^= v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// DEK-like pass without memory loads: each lane compresses 64 blocks of
// synthesised words (same compress/merge/LDS structure as k_pass<4>).
__global__ __launch_bounds__(256) void k_noload(KArgs a) {
  __shared__ uint32_t lds[256 * 8];
  const uint32_t t = threadIdx.x;
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = a.key[i];
  uint32_t cv[8], stk[2][8];
  uint32_t depth = 0;
  for (uint32_t jj = 0; jj < 4; ++jj) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = key[i];
    for (uint32_t b = 0; b < 16; ++b) {
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = (t << 8) ^ (b << 4) ^ i ^ jj;
      b3_compress(cv, m, t * 4 + jj, 0, 64, a.base | (b == 0) | ((b == 15) << 1));
    }
    const bool last = jj == 3;
    const uint32_t merges = last ? depth : uint32_t(__builtin_ctz(jj + 1));
    for (uint32_t i = 0; i < merges; ++i) {
      uint32_t m[16];
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        m[w] = stk[0][w];
        m[8 + w] = cv[w];
        cv[w] = key[w];
      }
#pragma unroll
      for (int w = 0; w < 8; ++w) stk[0][w] = stk[1][w];
      --depth;
      b3_compress(cv, m, 0u, 0u, 64u, a.base | kParent);
    }
    if (!last) {
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        stk[1][w] = stk[0][w];
        stk[0][w] = cv[w];
      }
      ++depth;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) lds[t * 8 + i] = cv[i];
  __syncthreads();
  uint32_t k = 256;
  uint32_t p[8];
  while (k > 1) {
    const uint32_t half = k >> 1;
    if (t < half) {
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        m[i] = lds[(2 * t) * 8 + i];
        m[8 + i] = lds[(2 * t + 1) * 8 + i];
        p[i] = key[i];
      }
      b3_compress(p, m, 0u, 0u, 64u, a.base | kParent | (k == 2 ? kRoot : 0u));
    }
    __syncthreads();
    if (t < half) {
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[t * 8 + i] = p[i];
    }
    __syncthreads();
    k = half;
  }
  if (t == 0) store_digest(a.refs + blockIdx.x * 64 + 32, p);
}

}  // namespace

int main(int argc, char **argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 8;
  const uint64_t bs = 1 << 20, total = gib << 30, n = total / bs;
  uint8_t *d_data, *d_refs, *d_refs2;
  uint32_t *d_out;
  CK(hipMalloc(&d_data, total));
  CK(hipMalloc(&d_refs, n * 64));
  CK(hipMalloc(&d_refs2, n * 64));
  CK(hipMalloc(&d_out, 1 << 24));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(launch_fill(d_data, 0, total, 7, s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto fn, double bytes, double ops) {
    fn();
    CK(hipStreamSynchronize(s));
    const int reps = 5;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) fn();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-10s %9.3f ms  %8.1f GB/s hashed  %6.2f Tops/s\n", name, ms,
           bytes / (ms * 1e-3) / 1e9, ops / (ms * 1e-3) / 1e12);
  };
  PostJob j{};
  j.src = d_data;
  j.stride = bs;
  j.msg_len = bs;
  j.last_len = bs;
  j.n = n;
  j.out = RefLayout{d_refs, ~0ull, 0};
  for (int i = 0; i < 8; ++i) j.salt[i] = 0x01010101u * i;
  const double ops_dek = double(total) / 64 * 16.0 / 16 * 700 * 1.06;
  timeit("prod", [&] { CK(launch_keyed_hash(j, 32, s)); }, double(total), ops_dek);
  KArgs a{};
  a.refs = d_refs2;
  a.n = n;
  for (int i = 0; i < 8; ++i) a.key[i] = j.salt[i];
  a.base = kKeyed;
  timeit("noload", [&] {
    hipLaunchKernelGGL(k_noload, dim3(n), dim3(256), 0, s, a);
  }, double(total), ops_dek);
  const uint32_t iters = 4096;
  const uint32_t grid = 256 * 8 * 4;  // 8 waves / SIMD worth of 256-thr WGs
  // per iteration per lane: 4 G = 48 VALU ops
  timeit("valu", [&] {
    hipLaunchKernelGGL(k_valu, dim3(grid), dim3(256), 0, s, d_out, iters);
  }, 0.0, double(grid) * 256 * iters * 48);
  std::vector<uint8_t> h(n * 64);
  CK(hipMemcpy(h.data(), d_refs, n * 64, hipMemcpyDeviceToHost));
  printf("dek[0] = ");
  for (int i = 32; i < 40; ++i) printf("%02x", h[i]);
  printf("\n");
  return 0;
}
