// tree_kernels.hip -- gfx950 kernels for the glfs tree path (BASELINE config
// 4) and per-blob synthetic inputs.
//
// k_tree_len / k_tree_prefix / k_tree_write: TreeWriter.Put's JSON lines
// (tree.go:300-316, json.Encoder.Encode(TreeEntry)) for n entries whose refs
// are already in HBM (the roots glfsx_post_blobs_device wrote), so a tree of
// a million blobs is encoded and hashed without leaving the device.  Same
// bytes as the host encoder (tree.cpp) and glfs_amd/tree.py's
// entry_json_line: encoding/json's appendString with escapeHTML, decimal
// numbers, the cid as a hex string (parity unpinned at that one field, see
// tree.cpp).
//
// Layout: one thread per entry, kTreeWG entries per workgroup.  k_tree_len
// computes each line's length and a workgroup-inclusive scan; k_tree_prefix
// scans the workgroup totals (one workgroup); k_tree_write builds the
// workgroup's lines in LDS at the alignment of their destination (the two
// 64-digit hex fields, 55 % of a config-4 line, as 16-byte words computed
// four digits per instruction sequence and written with unaligned
// ds_write_b128) and stores them with aligned 16-byte stores (bytes at the two partial 16-byte granules of a
// workgroup's span, which it shares with its neighbours, are stored one by
// one).  A workgroup whose lines do not fit the LDS image stores bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace glfsx {
namespace {

struct TArgs {
  uint64_t n;
  const uint8_t *names;
  const uint64_t *name_offs;
  const uint32_t *modes;
  const uint8_t *types;
  const uint64_t *type_offs;
  const uint8_t *roots;
  const uint64_t *sizes, *block_sizes;
  uint64_t *local_end;  // per entry: inclusive end within its workgroup
  uint64_t *wg_total;   // per workgroup: total bytes, then (k_tree_prefix)
                        // the exclusive prefix
  uint64_t *line_ends;  // nullable: global inclusive line ends
  uint8_t *out;
  uint64_t cap;         // bytes at out; nothing is written if the total exceeds it
  const uint64_t *total;
  uint64_t *hex_pos;    // nullable: skip the hex digits, record where they go
  uint32_t prio;        // 1: the waves raise their issue priority
};

constexpr uint32_t kImg = 60 * 1024;  // LDS image per workgroup

// Go's utf8.DecodeRune (see tree.cpp)
__device__ __forceinline__ void decode_rune(const uint8_t *p, uint64_t n,
                                            uint32_t *r, uint32_t *sz) {
  const uint32_t b0 = p[0];
  *r = 0xFFFD;
  *sz = 1;
  auto cont = [&](uint64_t i) { return i < n && (p[i] & 0xC0) == 0x80; };
  if (b0 < 0x80) {
    *r = b0;
  } else if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (cont(1)) {
      *r = ((b0 & 0x1F) << 6) | (p[1] & 0x3F);
      *sz = 2;
    }
  } else if (b0 >= 0xE0 && b0 <= 0xEF) {
    if (cont(1) && cont(2) && !(b0 == 0xE0 && p[1] < 0xA0) &&
        !(b0 == 0xED && p[1] > 0x9F)) {
      *r = ((b0 & 0x0F) << 12) | (uint32_t(p[1] & 0x3F) << 6) | (p[2] & 0x3F);
      *sz = 3;
    }
  } else if (b0 >= 0xF0 && b0 <= 0xF4) {
    if (cont(1) && cont(2) && cont(3) && !(b0 == 0xF0 && p[1] < 0x90) &&
        !(b0 == 0xF4 && p[1] > 0x8F)) {
      *r = ((b0 & 0x07) << 18) | (uint32_t(p[1] & 0x3F) << 12) |
           (uint32_t(p[2] & 0x3F) << 6) | (p[3] & 0x3F);
      *sz = 4;
    }
  }
}

// Byte sinks.  `line` is instantiated once per sink, so the counting pass
// touches no output and reads only what lengths depend on, and the LDS
// writer compiles to ds_write_b8 (no flat stores through a generic pointer).
struct CountSink {
  uint32_t o = 0;
  __device__ __forceinline__ void put(uint8_t) { ++o; }
  static constexpr bool kWrites = false;
};
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
struct LdsSink {
  __attribute__((address_space(3))) uint8_t *p;
  uint32_t o;
  __device__ __forceinline__ void put(uint8_t c) { p[o++] = c; }
  // 16 bytes at any byte offset (LDS accesses may be unaligned on gfx950)
  __device__ __forceinline__ void put16(u32x4_t v) {
    typedef __attribute__((address_space(3))) u32x4_t lds_v4
        __attribute__((aligned(1)));
    *reinterpret_cast<lds_v4 *>(p + o) = v;
    o += 16;
  }
  static constexpr bool kWrites = true, kWide = true;
};
struct GlobalSink {
  uint8_t *p;
  uint32_t o;
  __device__ __forceinline__ void put(uint8_t c) { p[o++] = c; }
  static constexpr bool kWrites = true, kWide = false;
};

template <class S, int N>
__device__ __forceinline__ void lit(S &k, const char (&s)[N]) {
  if constexpr (!S::kWrites) {
    k.o += N - 1;
  } else {
#pragma unroll
    for (int i = 0; i + 1 < N; ++i) k.put(uint8_t(s[i]));
  }
}

__device__ __forceinline__ uint8_t hexd(uint32_t v) {
  return uint8_t(v < 10 ? '0' + v : 'a' - 10 + v);
}

// One ASCII byte of a JSON string (encoding/json appendString, escapeHTML).
template <class S>
__device__ __forceinline__ void put_ascii(S &k, uint32_t b) {
  if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
    k.put(uint8_t(b));
    return;
  }
  k.put('\\');
  switch (b) {
    case '"': case '\\': k.put(uint8_t(b)); break;
    case '\b': k.put('b'); break;
    case '\f': k.put('f'); break;
    case '\n': k.put('n'); break;
    case '\r': k.put('r'); break;
    case '\t': k.put('t'); break;
    default:
      k.put('u'); k.put('0'); k.put('0');
      k.put(hexd(b >> 4)); k.put(hexd(b & 15));
  }
}

template <class S>
__device__ void json_string(S &k, const uint8_t *s, uint64_t n) {
  // Short strings (names like config 4's "%07d", types): every byte's load
  // in flight at once, then the bytes from registers -- the general loop
  // below waits for each byte's load before the next (its step depends on
  // the byte), a chain of ~11 dependent global loads per line that left the
  // line kernels latency-bound at two workgroups per CU.
  if (n <= 16) {
    uint32_t b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) b[q] = uint64_t(q) < n ? s[q] : 0u;
    uint32_t hi = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) hi |= b[q];
    if (hi < 0x80) {  // ASCII: no rune decoding
      k.put('"');
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (uint64_t(q) < n) put_ascii(k, b[q]);
      k.put('"');
      return;
    }
  }
  k.put('"');
  for (uint64_t i = 0; i < n;) {
    const uint8_t b = s[i];
    if (b < 0x80) {
      put_ascii(k, b);
      ++i;
      continue;
    }
    uint32_t r, sz;
    decode_rune(s + i, n - i, &r, &sz);
    if (r == 0xFFFD && sz == 1) {
      lit(k, "\\ufffd");
    } else if (r == 0x2028 || r == 0x2029) {
      lit(k, "\\u202");
      k.put(hexd(r & 15));
    } else {
      for (uint32_t q = 0; q < sz; ++q) k.put(s[i + q]);
    }
    i += sz;
  }
  k.put('"');
}

// decimal digits of v (32-bit arithmetic while it fits)
template <class S>
__device__ void dec(S &k, uint64_t v) {
  uint8_t t[20];
  int c = 0;
  while (v >> 32) {
    t[c++] = uint8_t('0' + v % 10);
    v /= 10;
  }
  uint32_t w = uint32_t(v);
  do {
    t[c++] = uint8_t('0' + w % 10);
    w /= 10;
  } while (w);
  if constexpr (!S::kWrites) {
    k.o += c;
  } else {
    while (c) k.put(t[--c]);
  }
}

// Lower-case hex digits of bytes b0, b1 (bits 0-15 of x) as four ASCII bytes
// in output order (hi(b0) lo(b0) hi(b1) lo(b1)), little-endian.
__device__ __forceinline__ uint32_t hex4(uint32_t x) {
  const uint32_t n = ((x >> 4) & 0xFu) | ((x & 0xFu) << 8) |
                     ((x >> 12) & 0xFu) << 16 | ((x >> 8) & 0xFu) << 24;
  const uint32_t ge10 = ((n + 0x06060606u) >> 4) & 0x01010101u;  // nibble >= 10
  return n + 0x30303030u + ge10 * 39u;  // '0' + n, or 'a' - 10 + n
}

// "<64 hex digits>" of the 32 bytes at x (one 64-B ref holds two: aligned
// refs are read as 16-B words)
template <class S>
__device__ __forceinline__ void hex32(S &k, const uint8_t *x, bool aligned, bool skip = false) {
  if constexpr (!S::kWrites) {
    k.o += 66;
  } else if (skip) {  // the quotes only: the digits come from the CID pass
    k.put('"');
    k.o += 64;
    k.put('"');
  } else {
    uint32_t w[8];
    if (aligned) {
      const uint4 *q = reinterpret_cast<const uint4 *>(x);
      const uint4 a = q[0], b = q[1];
      w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
      w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        w[i] = uint32_t(x[4 * i]) | (uint32_t(x[4 * i + 1]) << 8) |
               (uint32_t(x[4 * i + 2]) << 16) | (uint32_t(x[4 * i + 3]) << 24);
    }
    k.put('"');
    if constexpr (S::kWide) {
#pragma unroll
      for (int i = 0; i < 8; i += 2)
        k.put16(u32x4_t{hex4(w[i]), hex4(w[i] >> 16), hex4(w[i + 1]), hex4(w[i + 1] >> 16)});
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t lo = hex4(w[i]), hi = hex4(w[i] >> 16);
#pragma unroll
        for (int b = 0; b < 4; ++b) k.put(uint8_t(lo >> (8 * b)));
#pragma unroll
        for (int b = 0; b < 4; ++b) k.put(uint8_t(hi >> (8 * b)));
      }
    }
    k.put('"');
  }
}

// *cid_at: the offset in the line of the cid's first hex digit
template <class S>
__device__ uint32_t line(const TArgs &a, uint64_t i, S k, uint32_t *cid_at = nullptr) {
  lit(k, "{\"name\":");
  json_string(k, a.names + a.name_offs[i], a.name_offs[i + 1] - a.name_offs[i]);
  lit(k, ",\"mode\":");
  dec(k, a.modes[i]);
  lit(k, ",\"ref\":{\"type\":");
  json_string(k, a.types + a.type_offs[i], a.type_offs[i + 1] - a.type_offs[i]);
  const bool al = (reinterpret_cast<uintptr_t>(a.roots) & 15) == 0;
  lit(k, ",\"cid\":");
  const bool skip = a.hex_pos != nullptr;
  if (cid_at) *cid_at = k.o + 1;
  hex32(k, a.roots + 64 * i, al, skip);
  lit(k, ",\"dek\":");
  hex32(k, a.roots + 64 * i + 32, al, skip);
  lit(k, ",\"size\":");
  dec(k, a.sizes[i]);
  lit(k, ",\"blockSize\":");
  dec(k, a.block_sizes[i]);
  lit(k, "}}\n");
  return k.o;
}

__global__ __launch_bounds__(kTreeWG) void k_tree_len(TArgs a) {
  __shared__ uint64_t s[kTreeWG];
  if (a.prio == 1) __builtin_amdgcn_s_setprio(3);
  const uint64_t i = uint64_t(blockIdx.x) * kTreeWG + threadIdx.x;
  uint64_t v = i < a.n ? line(a, i, CountSink{}) : 0;
  s[threadIdx.x] = v;
  __syncthreads();
  for (uint32_t d = 1; d < kTreeWG; d <<= 1) {  // Hillis-Steele inclusive scan
    const uint64_t add = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
    __syncthreads();
    v += add;
    s[threadIdx.x] = v;
    __syncthreads();
  }
  if (i < a.n) a.local_end[i] = v;
  if (threadIdx.x == kTreeWG - 1) a.wg_total[blockIdx.x] = v;
}

// One workgroup of T threads: wg_total[0..m) -> exclusive prefix, in chunks
// of T.  T = 256 (one wave per SIMD) runs beside the small-blob DEK pass,
// which leaves each SIMD room for one more wave; 1024 waits for a CU it
// cannot get there.
template <uint32_t T>
__global__ __launch_bounds__(T) void k_tree_prefix(uint64_t *t, uint64_t m, uint64_t *total,
                                                   uint32_t prio, uint64_t *host_out) {
  __shared__ uint64_t s[T];
  if (prio == 1) __builtin_amdgcn_s_setprio(3);
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < m; c0 += T) {
    const uint64_t i = c0 + threadIdx.x;
    const uint64_t x = i < m ? t[i] : 0;
    uint64_t v = x;
    s[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t d = 1; d < T; d <<= 1) {
      const uint64_t add = threadIdx.x >= d ? s[threadIdx.x - d] : 0;
      __syncthreads();
      v += add;
      s[threadIdx.x] = v;
      __syncthreads();
    }
    if (i < m) {
      t[i] = carry + v - x;
      // the host's copy (pinned), read once the launch's event completes
      if (host_out) __hip_atomic_store(host_out + i, carry + v - x, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
    }
    carry += s[T - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *total = carry;
    if (host_out) __hip_atomic_store(host_out + m, carry, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ __launch_bounds__(kTreeWG) void k_tree_write(TArgs a) {
  __shared__ uint4 img4[kImg / 16];
  uint8_t *img = reinterpret_cast<uint8_t *>(img4);
  const uint64_t wg = blockIdx.x;
  const uint64_t i = wg * kTreeWG + threadIdx.x;
  const uint64_t last = min<uint64_t>(wg * kTreeWG + kTreeWG - 1, a.n - 1);
  const uint64_t base = a.wg_total[wg];           // exclusive prefix
  const uint64_t span = a.local_end[last];        // this workgroup's bytes
  const uint32_t sh = uint32_t((reinterpret_cast<uintptr_t>(a.out) + base) & 15);
  if (*a.total > a.cap) {  // uniform: the caller reports the error
    // and the CID pass must not write digits anywhere
    if (a.hex_pos && i < a.n) a.hex_pos[i] = ~0ull;
    return;
  }
  const uint64_t end = i < a.n ? a.local_end[i] : 0;
  const uint64_t start = (i < a.n && threadIdx.x) ? a.local_end[i - 1] : 0;
  if (i < a.n && a.line_ends) a.line_ends[i] = base + end;
  uint32_t cid_at = 0;
  if (span + sh > kImg) {  // uniform: lines too long for the image
    if (i < a.n) {
      line(a, i, GlobalSink{a.out + base + start, 0}, &cid_at);
      if (a.hex_pos) a.hex_pos[i] = base + start + cid_at;
    }
    return;
  }
  if (i < a.n) {
    line(a, i, LdsSink{(__attribute__((address_space(3))) uint8_t *)img + sh + start, 0},
         &cid_at);
    if (a.hex_pos) a.hex_pos[i] = base + start + cid_at;
  }
  __syncthreads();
  // image byte x <-> out byte base - sh + x; granules [16g, 16g+16)
  uint8_t *dst = a.out + base - sh;
  const uint32_t tot = uint32_t(span) + sh;
  const uint32_t ng = (tot + 15) / 16;
  for (uint32_t g = threadIdx.x; g < ng; g += kTreeWG) {
    const uint32_t lo = 16 * g, hi = lo + 16;
    if (lo >= sh && hi <= tot) {
      *reinterpret_cast<uint4 *>(dst + lo) = img4[g];
    } else {
      for (uint32_t x = max(lo, sh); x < min(hi, tot); ++x) dst[x] = img[x];
    }
  }
}

// The static lines of glfsx_post_tree_device (hex_pos set: the digits come
// from the CID pass) in half workgroups: 128 threads for the entries [h *
// 128, h * 128 + 128) of layout workgroup wg (block 2 wg + h), a 30 KiB
// image.  Sized to run beside the small-blob DEK pass, whose persistent
// workgroups hold 4 x 32 KiB of each CU's 160 KiB LDS and 4 x 112 of each
// SIMD's 512 VGPRs per lane: this one (~50 VGPRs, one wave per SIMD) fits in
// what they leave, so the lines are written while the blobs hash instead
// of after (the 60 KiB form only got CUs as the DEK pass drained).
constexpr uint32_t kHalf = kTreeWG / 2;
constexpr uint32_t kHalfImg = 30 * 1024;
__global__ __launch_bounds__(kHalf) void k_tree_write_half(TArgs a) {
  __shared__ uint4 img4[kHalfImg / 16];
  // beside the DEK pass: issue ahead of its resident waves (the SIMD issues
  // oldest-first, so this youngest wave would otherwise take what is left)
  if (a.prio == 1) __builtin_amdgcn_s_setprio(3);
  uint8_t *img = reinterpret_cast<uint8_t *>(img4);
  const uint64_t wg = blockIdx.x >> 1, h = blockIdx.x & 1u;
  const uint64_t e0 = wg * kTreeWG + h * kHalf;  // this half's first entry
  const uint64_t i = e0 + threadIdx.x;
  if (e0 >= a.n) return;  // uniform: an empty second half
  if (*a.total > a.cap) {  // uniform: the caller reports the error
    if (i < a.n) a.hex_pos[i] = ~0ull;  // and the CID pass writes nothing
    return;
  }
  const uint64_t last = min<uint64_t>(e0 + kHalf, a.n) - 1;
  const uint64_t p0 = h ? a.local_end[e0 - 1] : 0;  // the half's start in its workgroup
  const uint64_t base = a.wg_total[wg] + p0;
  const uint64_t span = a.local_end[last] - p0;
  const uint32_t sh = uint32_t((reinterpret_cast<uintptr_t>(a.out) + base) & 15);
  const uint64_t start = (i < a.n && i > e0) ? a.local_end[i - 1] - p0 : 0;
  if (i < a.n && a.line_ends) a.line_ends[i] = base + a.local_end[i] - p0;
  uint32_t cid_at = 0;
  if (span + sh > kHalfImg) {  // uniform: lines too long for the image
    if (i < a.n) {
      line(a, i, GlobalSink{a.out + base + start, 0}, &cid_at);
      a.hex_pos[i] = base + start + cid_at;
    }
    return;
  }
  if (i < a.n) {
    line(a, i, LdsSink{(__attribute__((address_space(3))) uint8_t *)img + sh + start, 0},
         &cid_at);
    a.hex_pos[i] = base + start + cid_at;
  }
  __syncthreads();
  // image byte x <-> out byte base - sh + x; the partial granules at the
  // ends are shared with the neighbouring half and written byte by byte
  uint8_t *dst = a.out + base - sh;
  const uint32_t tot = uint32_t(span) + sh;
  const uint32_t ng = (tot + 15) / 16;
  for (uint32_t g = threadIdx.x; g < ng; g += kHalf) {
    const uint32_t lo = 16 * g, hi = lo + 16;
    if (lo >= sh && hi <= tot) {
      *reinterpret_cast<uint4 *>(dst + lo) = img4[g];
    } else {
      for (uint32_t x = max(lo, sh); x < min(hi, tot); ++x) dst[x] = img[x];
    }
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// n blobs of len bytes (len % 8 == 0) back to back: byte o of blob b =
// byte (o & 7) of splitmix64((seed0 + b) ^ (o >> 3)), i.e. blob b is the
// splitmix stream of seed seed0 + b (oracle_fill_splitmix_blobs).
__global__ __launch_bounds__(256) void k_fill_blobs(uint64_t *dst, uint64_t n,
                                                    uint64_t words, uint64_t seed0) {
  const uint64_t total = n * words;
  for (uint64_t w = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; w < total;
       w += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t b = w / words, k = w - b * words;
    dst[w] = splitmix64((seed0 + b) ^ k);
  }
}

}  // namespace

namespace {
TArgs tree_args(const TreeJob &j) {
  TArgs a{};
  a.n = j.n;
  a.names = j.names;
  a.name_offs = j.name_offs;
  a.modes = j.modes;
  a.types = j.types;
  a.type_offs = j.type_offs;
  a.roots = j.roots;
  a.sizes = j.sizes;
  a.block_sizes = j.block_sizes;
  a.local_end = j.scratch;
  a.wg_total = j.scratch + j.n;
  a.line_ends = j.line_ends;
  a.out = j.out;
  a.cap = j.cap;
  a.total = j.total;
  a.hex_pos = j.hex_pos;
  a.prio = j.prio;
  return a;
}
}  // namespace

hipError_t launch_tree_layout(const TreeJob &j, hipStream_t s) {
  if (j.n == 0) return hipSuccess;
  const TArgs a = tree_args(j);
  const uint64_t wgs = (j.n + kTreeWG - 1) / kTreeWG;
  hipLaunchKernelGGL(k_tree_len, dim3(uint32_t(wgs)), dim3(kTreeWG), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (j.prio)  // beside the DEK pass
    hipLaunchKernelGGL(k_tree_prefix<256>, dim3(1), dim3(256), 0, s, a.wg_total, wgs, j.total,
                       j.prio, j.prefix_host);
  else
    hipLaunchKernelGGL(k_tree_prefix<1024>, dim3(1), dim3(1024), 0, s, a.wg_total, wgs,
                       j.total, 0u, j.prefix_host);
  return hipGetLastError();
}

hipError_t launch_tree_static(const TreeJob &j, hipStream_t s) {
  if (j.n == 0 || !j.out || !j.hex_pos) return hipErrorInvalidValue;
  const uint64_t wgs = (j.n + kTreeWG - 1) / kTreeWG;
  hipLaunchKernelGGL(k_tree_write_half, dim3(uint32_t(2 * wgs)), dim3(kHalf), 0, s,
                     tree_args(j));
  return hipGetLastError();
}

hipError_t launch_tree_encode(const TreeJob &j, hipStream_t s) {
  if (j.n == 0) return hipSuccess;
  const TArgs a = tree_args(j);
  const uint64_t wgs = (j.n + kTreeWG - 1) / kTreeWG;
  hipLaunchKernelGGL(k_tree_len, dim3(uint32_t(wgs)), dim3(kTreeWG), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_tree_prefix<1024>, dim3(1), dim3(1024), 0, s, a.wg_total, wgs,
                     j.total, 0u, static_cast<uint64_t *>(nullptr));
  e = hipGetLastError();
  if (e != hipSuccess || !j.out) return e;
  hipLaunchKernelGGL(k_tree_write, dim3(uint32_t(wgs)), dim3(kTreeWG), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fill_blobs(uint8_t *dst, uint64_t n, uint64_t len, uint64_t seed0,
                             hipStream_t s) {
  if (n == 0 || len == 0) return hipSuccess;
  if (len % 8 || (reinterpret_cast<uintptr_t>(dst) & 7)) return hipErrorInvalidValue;
  const uint64_t words = n * (len / 8);
  uint64_t grid = (words + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(k_fill_blobs, dim3(uint32_t(grid)), dim3(256), 0, s,
                     reinterpret_cast<uint64_t *>(dst), n, len / 8, seed0);
  return hipGetLastError();
}

}  // namespace glfsx
