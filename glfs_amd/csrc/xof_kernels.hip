// xof_kernels.hip -- DeriveKey's full contract (bigblob/ref.go:152-161):
// BLAKE3 keyed with the salt over an input of any length, then len(out)
// bytes of the XOF (blake3.New(len(out), salt), h.XOF(), io.ReadFull).
//
// The write path only ever needs the 32-byte digest of a message of at most
// 4 GiB (post_kernels.hip).  DeriveKey as exported may ask for more output
// or a longer input, so this file hashes a stream of any length in one
// workgroup with state carried across launches in device memory (a slab of
// host input per launch):
//
//   k_b3_absorb: whole groups of 256 chunks (256 KiB) that are known not to
//     end the input.  Lane t compresses chunk t of the group (16 blocks), the
//     256 chunk CVs merge pairwise in LDS into the group's subtree CV (256 is
//     a power of two and groups start at multiples of 256 chunks, so the
//     group is a perfect subtree of the BLAKE3 tree), which is pushed on the
//     CV stack with BLAKE3's merge rule (merge while the group count has
//     trailing zeros).
//   k_b3_final: the last 1..256 chunks (or the empty input's one empty
//     chunk): their CVs merge into a left-complete subtree R exactly like a
//     fresh hasher's; the root is R itself (no stack) or the chain
//     parent(S0, parent(S1, ... parent(Sm, R))) down the stack.  The root's
//     compression inputs (chaining value, block, length, flags) are kept, and
//     64 lanes at a time produce XOF output blocks 0, 1, 2, ... (counter =
//     output block index, ROOT flag on each; BLAKE3 spec 2.6).
//
// Plain compiler-scheduled ARX: this is one workgroup on a utility path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace glfsx {
namespace {

constexpr uint32_t kIVx[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                              0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
enum : uint32_t { fStart = 1, fEnd = 2, fParent = 4, fRoot = 8 };

__device__ __forceinline__ uint32_t rr(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}

#define XG(a, b, c, d, x, y)        \
  v[a] = v[a] + v[b] + (x);         \
  v[d] = rr(v[d] ^ v[a], 16);       \
  v[c] = v[c] + v[d];               \
  v[b] = rr(v[b] ^ v[c], 12);       \
  v[a] = v[a] + v[b] + (y);         \
  v[d] = rr(v[d] ^ v[a], 8);        \
  v[c] = v[c] + v[d];               \
  v[b] = rr(v[b] ^ v[c], 7);

// The full 16-word compression output (spec 2.4): out[0..8) = v[0..8) ^
// v[8..16), out[8..16) = v[8..16) ^ cv.
__device__ void compress16(const uint32_t cv[8], const uint32_t m_in[16], uint64_t ctr,
                           uint32_t len, uint32_t flags, uint32_t out[16]) {
  uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    kIVx[0], kIVx[1], kIVx[2], kIVx[3],
                    uint32_t(ctr), uint32_t(ctr >> 32), len, flags};
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) m[i] = m_in[i];
  constexpr int P[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    XG(0, 4, 8, 12, m[0], m[1]);
    XG(1, 5, 9, 13, m[2], m[3]);
    XG(2, 6, 10, 14, m[4], m[5]);
    XG(3, 7, 11, 15, m[6], m[7]);
    XG(0, 5, 10, 15, m[8], m[9]);
    XG(1, 6, 11, 12, m[10], m[11]);
    XG(2, 7, 8, 13, m[12], m[13]);
    XG(3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      uint32_t t[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) t[i] = m[P[i]];
#pragma unroll
      for (int i = 0; i < 16; ++i) m[i] = t[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[i] = v[i] ^ v[i + 8];
    out[i + 8] = v[i + 8] ^ cv[i];
  }
}

__device__ void compress8(uint32_t cv[8], const uint32_t m[16], uint64_t ctr, uint32_t len,
                          uint32_t flags) {
  uint32_t o[16];
  compress16(cv, m, ctr, len, flags, o);
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = o[i];
}

// Message block `b` (<= 64 bytes at p, n valid, zero padded) as words.
__device__ void load_block(const uint8_t *p, uint32_t n, uint32_t m[16]) {
  if (n == 64 && (reinterpret_cast<uintptr_t>(p) & 3) == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = reinterpret_cast<const uint32_t *>(p)[i];
    return;
  }
  for (int i = 0; i < 16; ++i) {
    uint32_t w = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t o = uint32_t(4 * i + k);
      if (o < n) w |= uint32_t(p[o]) << (8 * k);
    }
    m[i] = w;
  }
}

// A chunk of n bytes (1..1024, or 0 for the empty input) with chunk index
// ctr: its CV (flags without ROOT), and the last block's compression inputs.
struct LastBlock {
  uint32_t cv[8], m[16], len, flags;
};
__device__ void chunk_cv(const uint8_t *p, uint32_t n, uint64_t ctr, const uint32_t key[8],
                         uint32_t base, uint32_t cv[8], LastBlock *lb) {
  const uint32_t nb = n ? (n + 63) / 64 : 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) cv[i] = key[i];
  for (uint32_t b = 0; b < nb; ++b) {
    const uint32_t blen = b + 1 < nb ? 64u : n - 64 * b;
    uint32_t m[16];
    load_block(p + 64 * b, blen, m);
    const uint32_t fl = base | (b == 0 ? fStart : 0u) | (b + 1 == nb ? fEnd : 0u);
    if (b + 1 == nb && lb) {
#pragma unroll
      for (int i = 0; i < 8; ++i) lb->cv[i] = cv[i];
#pragma unroll
      for (int i = 0; i < 16; ++i) lb->m[i] = m[i];
      lb->len = blen;
      lb->flags = fl;
    }
    compress8(cv, m, ctr, blen, fl);
  }
}

__device__ void parent_cv(const uint32_t l[8], const uint32_t r[8], const uint32_t key[8],
                          uint32_t base, uint32_t out[8]) {
  uint32_t m[16], cv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l[i];
    m[8 + i] = r[i];
    cv[i] = key[i];
  }
  compress8(cv, m, 0, 64, base | fParent);
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = cv[i];
}

// Pairwise left-complete merge of the k CVs in lds[0..8k) (tree_reduce in
// post_kernels.hip); stops at 2 left when keep2 (the root's children).
__device__ void merge_cvs(uint32_t *lds, uint32_t k, uint32_t t, const uint32_t key[8],
                          uint32_t base, bool keep2) {
  while (k > (keep2 ? 2u : 1u)) {
    const uint32_t half = k >> 1, odd = k & 1u;
    uint32_t p[8];
    if (t < half) parent_cv(lds + 16 * t, lds + 16 * t + 8, key, base, p);
    else if (odd && t == half)
      for (int i = 0; i < 8; ++i) p[i] = lds[(k - 1) * 8 + i];
    __syncthreads();
    if (t < half + odd)
      for (int i = 0; i < 8; ++i) lds[t * 8 + i] = p[i];
    __syncthreads();
    k = half + odd;
  }
}

}  // namespace

// 1 workgroup of 256 lanes; `groups` whole groups of 256 chunks at src.
__global__ __launch_bounds__(256) void k_b3_absorb(B3State *st, const uint8_t *src,
                                                   uint64_t groups) {
  __shared__ uint32_t lds[256 * 8];
  const uint32_t t = threadIdx.x;
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = st->key[i];
  const uint32_t base = st->base;
  for (uint64_t g = 0; g < groups; ++g) {
    uint32_t cv[8];
    chunk_cv(src + (g * 256 + t) * 1024, 1024, st->chunks + g * 256 + t, key, base, cv,
             nullptr);
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[t * 8 + i] = cv[i];
    __syncthreads();
    merge_cvs(lds, 256, t, key, base, false);
    if (t == 0) {  // push the group's subtree CV (BLAKE3's lazy merge rule)
      uint32_t c[8];
      for (int i = 0; i < 8; ++i) c[i] = lds[i];
      uint64_t total = (st->chunks >> 8) + g + 1;
      uint32_t d = st->depth;
      while ((total & 1) == 0) {
        --d;
        parent_cv(st->stack[d], c, key, base, c);
        total >>= 1;
      }
      for (int i = 0; i < 8; ++i) st->stack[d][i] = c[i];
      st->depth = d + 1;
    }
    __syncthreads();
  }
  if (t == 0) st->chunks += groups * 256;
}

// The last n bytes (0 <= n <= 256 KiB; n == 0 only for the empty input) and
// out_len bytes of XOF output to out.
__global__ __launch_bounds__(256) void k_b3_final(B3State *st, const uint8_t *src, uint64_t n,
                                                  uint8_t *out, uint64_t out_len) {
  __shared__ uint32_t lds[256 * 8];
  __shared__ uint32_t root_cv[8], root_m[16], root_len, root_flags;
  const uint32_t t = threadIdx.x;
  uint32_t key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = st->key[i];
  const uint32_t base = st->base;
  const uint32_t r = n ? uint32_t((n + 1023) / 1024) : 1u;
  if (t < r) {
    const uint32_t len = uint32_t(t + 1 < r ? 1024 : n - uint64_t(t) * 1024);
    uint32_t cv[8];
    LastBlock lb;
    chunk_cv(src + uint64_t(t) * 1024, len, st->chunks + t, key, base, cv, &lb);
    for (int i = 0; i < 8; ++i) lds[t * 8 + i] = cv[i];
    if (r == 1 && st->depth == 0) {  // the root is this one chunk's last block
      for (int i = 0; i < 8; ++i) root_cv[i] = lb.cv[i];
      for (int i = 0; i < 16; ++i) root_m[i] = lb.m[i];
      root_len = lb.len;
      root_flags = lb.flags | fRoot;
    }
  }
  __syncthreads();
  if (!(r == 1 && st->depth == 0)) {
    // R: the remainder's left-complete subtree; with no stack its last
    // parent is the root, so stop at its two children
    const bool r_is_root = st->depth == 0;
    merge_cvs(lds, r, t, key, base, r_is_root);
    if (t == 0) {
      uint32_t right[8], left[8];
      if (r_is_root) {
        for (int i = 0; i < 8; ++i) {
          left[i] = lds[i];
          right[i] = lds[8 + i];
        }
      } else {  // parent(S0, ... parent(Sm, R)): ROOT on the last
        for (int i = 0; i < 8; ++i) right[i] = lds[i];
        for (uint32_t d = st->depth; d-- > 1;) parent_cv(st->stack[d], right, key, base, right);
        for (int i = 0; i < 8; ++i) left[i] = st->stack[0][i];
      }
      for (int i = 0; i < 8; ++i) {
        root_cv[i] = key[i];
        root_m[i] = left[i];
        root_m[8 + i] = right[i];
      }
      root_len = 64;
      root_flags = base | fParent | fRoot;
    }
    __syncthreads();
  }
  // XOF: output block k = the root compression with counter k
  const uint64_t nblk = (out_len + 63) / 64;
  for (uint64_t k = t; k < nblk; k += 256) {
    uint32_t o[16], cv[8], m[16];
    for (int i = 0; i < 8; ++i) cv[i] = root_cv[i];
    for (int i = 0; i < 16; ++i) m[i] = root_m[i];
    compress16(cv, m, k, root_len, root_flags, o);
    const uint64_t take = out_len - 64 * k < 64 ? out_len - 64 * k : 64;
    for (uint64_t b = 0; b < take; ++b) out[64 * k + b] = uint8_t(o[b >> 2] >> (8 * (b & 3)));
  }
}

hipError_t launch_b3_absorb(B3State *st, const uint8_t *src, uint64_t groups, hipStream_t s) {
  if (groups == 0) return hipSuccess;
  hipLaunchKernelGGL(k_b3_absorb, dim3(1), dim3(256), 0, s, st, src, groups);
  return hipGetLastError();
}

hipError_t launch_b3_final(B3State *st, const uint8_t *src, uint64_t n, uint8_t *out,
                           uint64_t out_len, hipStream_t s) {
  if (n > (256ull << 10)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_b3_final, dim3(1), dim3(256), 0, s, st, src, n, out, out_len);
  return hipGetLastError();
}

}  // namespace glfsx
