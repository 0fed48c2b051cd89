// tree_line.h -- device code for one TreeWriter.Put JSON line
// (tree.go:300-316, json.Encoder.Encode(TreeEntry)), shared by the tree-line
// kernels (tree_kernels.hip) and the small-blob DEK pass, which writes a
// line's static parts for the blob it has just hashed (post_kernels.hip).
// encoding/json's appendString with escapeHTML, decimal numbers, the cid
// and dek as hex strings (parity unpinned at the cid, see tree.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace glfsx {
namespace tree_line {

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
template <class S, class T>
__device__ uint32_t line(const T &a, uint64_t i, S k, uint32_t *cid_at = nullptr) {
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


}  // namespace tree_line
}  // namespace glfsx
