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
#include <cstring>

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
    B3G_A(v[0], v[4], v[8], v[12], it, v[1]);
    B3G_A(v[1], v[5], v[9], v[13], v[2], it);
    B3G_A(v[2], v[6], v[10], v[14], it, v[3]);
    B3G_A(v[3], v[7], v[11], v[15], v[0], it);
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


// DEK pass, G = 4, 1 MiB messages, all chunks full: loads staged through LDS
// with global_load_lds_dwordx4.  Per stage (2 blocks = 128 B per lane, 8 KiB
// per wave) glds instruction k loads the 128-B lines of lanes 8k..8k+7 (one
// full line per 8-lane group); pieces are XOR-swizzled by ((c>>1)&7) so the
// transposing ds_read_b128 of lane c is bank-conflict free.
__device__ __forceinline__ uint32_t swz(uint32_t c) { return (c >> 1) & 7u; }

__global__ __launch_bounds__(256) void k_dek_glds(KArgs a) {
  __shared__ uint4 smem[4 * 512];  // 4 waves x 8 KiB staging
  __shared__ uint32_t lds[256 * 8];
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  const uint64_t j = blockIdx.x;
  const uint8_t *msg = a.src + j * a.stride;
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = a.key[i];
  // per-lane source offsets inside a k-group, for k even / odd
  const uint32_t jj8 = l >> 3, p = l & 7;
  const uint32_t off0 = jj8 * 4096u + 16u * (p ^ ((jj8 >> 1) & 7u));
  const uint32_t off1 = jj8 * 4096u + 16u * (p ^ ((4u + (jj8 >> 1)) & 7u));
  const uint8_t *wbase = msg + uint64_t(w) * 64 * 4096;
  __attribute__((address_space(3))) uint4 *wst =
      (__attribute__((address_space(3))) uint4 *)(smem + w * 512);
  auto issue = [&](uint32_t s) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint8_t *src = wbase + k * 32768u + 128u * s + ((k & 1) ? off1 : off0);
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void *)src,
          (__attribute__((address_space(3))) void *)(wst + k * 64), 16, 0, 0);
    }
  };
  const uint32_t sw = swz(l);
  uint32_t cv[8], stk[2][8];
  uint32_t depth = 0;
  const uint32_t first = t * 4;
  issue(0);
  for (uint32_t s = 0; s < 32; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = smem[w * 512 + l * 8 + (i ^ sw)];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (s + 1 < 32) issue(s + 1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t m[16] = {q[4 * h].x, q[4 * h].y, q[4 * h].z, q[4 * h].w,
                        q[4 * h + 1].x, q[4 * h + 1].y, q[4 * h + 1].z, q[4 * h + 1].w,
                        q[4 * h + 2].x, q[4 * h + 2].y, q[4 * h + 2].z, q[4 * h + 2].w,
                        q[4 * h + 3].x, q[4 * h + 3].y, q[4 * h + 3].z, q[4 * h + 3].w};
      const uint32_t blk = 2 * s + h, b = blk & 15u, jj = blk >> 4;
      if (b == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[i] = key[i];
      }
      uint32_t fl = a.base | (b == 0 ? kChunkStart : 0u) | (b == 15 ? kChunkEnd : 0u);
      b3_compress(cv, m, first + jj, 0u, 64u, fl);
      if (b == 15) lane_merge<2>(cv, stk, depth, jj, jj == 3, false, key, a.base);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) lds[t * 8 + i] = cv[i];
  __syncthreads();
  uint32_t k = 256;
  uint32_t pp[8];
  while (k > 1) {
    const uint32_t half = k >> 1;
    if (t < half) {
      uint32_t m[16];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        m[i] = lds[(2 * t) * 8 + i];
        m[8 + i] = lds[(2 * t + 1) * 8 + i];
        pp[i] = key[i];
      }
      b3_compress(pp, m, 0u, 0u, 64u, a.base | kParent | (k == 2 ? kRoot : 0u));
    }
    __syncthreads();
    if (t < half) {
#pragma unroll
      for (int i = 0; i < 8; ++i) lds[t * 8 + i] = pp[i];
    }
    __syncthreads();
    k = half;
  }
  if (t == 0) store_digest(a.refs + blockIdx.x * 64 + 32, pp);
}
// Fast path: the lane's G chunks are all full (16*G consecutive 64-B blocks,
// 16-B aligned).  One loop over the blocks with the next block's four 16-B
// loads issued before the current compression, so the wave does not stall
// on HBM latency between blocks.
template <int G, bool CHACHA>
__device__ __forceinline__ void lane_subtree_full_v1(
    uint32_t (&cv)[8], const uint8_t *msg, uint8_t *cmsg, uint32_t first,
    bool whole, const uint32_t (&key)[8], uint32_t base,
    const uint32_t (&dek)[8]) {
  constexpr int D = ilog2(G);
  uint32_t stk[D > 0 ? D : 1][8];
  uint32_t depth = 0;
  const uint4 *q = reinterpret_cast<const uint4 *>(msg + (uint64_t(first) << 10));
  uint4 *cq = cmsg ? reinterpret_cast<uint4 *>(cmsg + (uint64_t(first) << 10))
                   : nullptr;
  uint4 n0 = q[0], n1 = q[1], n2 = q[2], n3 = q[3];
  for (uint32_t blk = 0; blk < 16u * G; ++blk) {
    uint32_t m[16] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w,
                      n2.x, n2.y, n2.z, n2.w, n3.x, n3.y, n3.z, n3.w};
    if (blk + 1 < 16u * G) {
      const uint4 *nq = q + 4 * (blk + 1);
      n0 = nq[0];
      n1 = nq[1];
      n2 = nq[2];
      n3 = nq[3];
    }
    const uint32_t b = blk & 15u, jj = blk >> 4;
    const uint32_t chunk = first + jj;
    if (b == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) cv[i] = key[i];
    }
    if constexpr (CHACHA) {
      uint32_t x[16];
      chacha_block(x, dek, (chunk << 4) + b);
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] ^= x[i];
      if (cq) {
        uint4 *o = cq + 4 * blk;
        o[0] = make_uint4(m[0], m[1], m[2], m[3]);
        o[1] = make_uint4(m[4], m[5], m[6], m[7]);
        o[2] = make_uint4(m[8], m[9], m[10], m[11]);
        o[3] = make_uint4(m[12], m[13], m[14], m[15]);
      }
    }
    uint32_t fl = base;
    if (b == 0) fl |= kChunkStart;
    if (b == 15) {
      fl |= kChunkEnd;
      if (whole && G == 1) fl |= kRoot;
    }
    b3_compress(cv, m, chunk, 0u, 64u, fl);
    if (b == 15) lane_merge<D>(cv, stk, depth, jj, jj + 1 == G, whole, key, base);
  }
}


template <int G, bool CHACHA>
__global__ __launch_bounds__(256) void k_pass_v1(KArgs a) {
  // production k_pass restricted to the fast path (all messages full), v1 loop
  __shared__ uint32_t lds[256 * 8];
  const uint64_t j = blockIdx.x;
  const uint8_t *msg = a.src + j * a.stride;
  uint8_t *cmsg = (CHACHA && a.ctext) ? a.ctext + j * a.stride : nullptr;
  uint8_t *ref = a.refs + j * 64;
  const uint32_t t = threadIdx.x;
  uint32_t key[8], dek[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = a.key[i];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    dek[i] = CHACHA ? __builtin_amdgcn_readfirstlane(reinterpret_cast<const uint32_t *>(ref + 32)[i]) : 0u;
  uint32_t cv[8];
  lane_subtree_full_v1<G, CHACHA>(cv, msg, cmsg, t * G, false, key, a.base, dek);
#pragma unroll
  for (int i = 0; i < 8; ++i) lds[t * 8 + i] = cv[i];
  __syncthreads();
  uint32_t k = 256, p[8];
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
  if (t == 0) store_digest(ref + (CHACHA ? 0 : 32), p);
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
  a.src = d_data;      // read by k_dek_glds (k_noload ignores it)
  a.stride = bs;
  a.msg_len = bs;
  a.last_len = bs;
  a.refs = d_refs2;
  a.n = n;
  for (int i = 0; i < 8; ++i) a.key[i] = j.salt[i];
  a.base = kKeyed;
  timeit("noload", [&] {
    hipLaunchKernelGGL(k_noload, dim3(n), dim3(256), 0, s, a);
  }, double(total), ops_dek);
  CK(hipMemset(d_refs2, 0, n * 64));
  timeit("dek_glds", [&] {
    hipLaunchKernelGGL(k_dek_glds, dim3(n), dim3(256), 0, s, a);
  }, double(total), ops_dek);
  {
    std::vector<uint8_t> h1(n * 64), h2(n * 64);
    CK(hipMemcpy(h1.data(), d_refs, n * 64, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), d_refs2, n * 64, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint64_t b = 0; b < n; ++b)
      if (memcmp(h1.data() + 64 * b + 32, h2.data() + 64 * b + 32, 32)) ++bad;
    printf("dek_glds vs prod: %zu / %llu DEKs differ\n", bad, (unsigned long long)n);
  }
  // interleaved A/B rounds in one process: production (v2 fast path) vs v1
  uint8_t *d_ct;
  CK(hipMalloc(&d_ct, total));
  PostJob jc = j;
  jc.ctext = d_ct;
  blake3_iv_words(jc.cid_key);  // unkeyed CID, as the C-ABI sets it
  jc.cid_keyed = false;
  KArgs a1 = a;
  a1.refs = d_refs;  // v1 reads the DEKs prod wrote
  a1.ctext = d_ct;
  const double ops_cid = double(total) / 64 * 1737;
  for (int r = 0; r < 3; ++r) {
    timeit("dek_v2", [&] { CK(launch_keyed_hash(j, 32, s)); }, double(total), ops_dek);
    timeit("dek_v1", [&] {
      hipLaunchKernelGGL((k_pass_v1<4, false>), dim3(n), dim3(256), 0, s, a);
    }, double(total), ops_dek);
    timeit("dek_glds", [&] {
      hipLaunchKernelGGL(k_dek_glds, dim3(n), dim3(256), 0, s, a);
    }, double(total), ops_dek);
    timeit("cid_v2", [&] { CK(launch_cid_pass(jc, s)); }, double(total), ops_cid);
    KArgs ac = a1;
    for (int i = 0; i < 8; ++i) ac.key[i] = kIV[i];
    ac.base = 0;
    ac.refs = d_refs2;
    timeit("cid_v1", [&] {
      hipLaunchKernelGGL((k_pass_v1<4, true>), dim3(n), dim3(256), 0, s, ac);
    }, double(total), ops_cid);
  }
  {
    // correctness of v1 CID vs production CID (same DEKs)
    CK(hipMemcpy(d_refs2, d_refs, n * 64, hipMemcpyDeviceToDevice));
    KArgs ac = a1;
    for (int i = 0; i < 8; ++i) ac.key[i] = kIV[i];
    ac.base = 0;
    ac.refs = d_refs2;
    hipLaunchKernelGGL((k_pass_v1<4, true>), dim3(n), dim3(256), 0, s, ac);
    CK(launch_cid_pass(jc, s));
    CK(hipStreamSynchronize(s));
    std::vector<uint8_t> h1(n * 64), h2(n * 64);
    CK(hipMemcpy(h1.data(), d_refs, n * 64, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), d_refs2, n * 64, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint64_t b = 0; b < n; ++b)
      if (memcmp(h1.data() + 64 * b, h2.data() + 64 * b, 64)) ++bad;
    printf("cid v1 vs v2: %zu / %llu refs differ\n", bad, (unsigned long long)n);
    // ctext fingerprint (compare across GLFSX_LDS_CTEXT builds)
    const size_t cn = size_t(1) << 28;
    std::vector<uint64_t> hc(cn / 8);
    uint64_t fp = 1469598103934665603ull;
    for (uint64_t off = 0; off < total; off += total / 4) {
      CK(hipMemcpy(hc.data(), d_ct + off, cn, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < hc.size(); ++i) fp = (fp ^ hc[i]) * 1099511628211ull;
    }
    printf("ctext fingerprint: %016llx\n", (unsigned long long)fp);
  }
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
