// tree.cpp -- host encoder of glfs tree blobs (tree.go:284-320 TreeWriter).
//
// A tree blob is JSON lines, one TreeEntry per Put (tree.go:300-316), written
// by Go's json.Encoder: struct fields in declaration order with their tags
// (TreeEntry tree.go:74-78, glfs.Ref glfs.go:35-38 with the embedded
// bigblob.Root promoted, Root blob.go:17-21, Ref ref.go:54-57, DEK as a hex
// string ref.go:28-33), strings escaped by encoding/json's appendString with
// escapeHTML on, numbers in decimal, each value followed by '\n'.
//
// The cid field is blobcache.CID's JSON form (blobcache module, absent here):
// it is written as a lower-case hex string, the same assumption as
// glfs_amd/tree.py (parity unpinned at that one field).
//
// Batched and multi-threaded: line lengths, an exclusive scan, then every
// thread writes its range of lines in place.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/glfsx.h"

namespace {

const char kHex[] = "0123456789abcdef";

// UTF-8 decode as Go's utf8.DecodeRune: returns the rune and its length, or
// (0xFFFD, 1) for an invalid / truncated / overlong / surrogate sequence.
inline void decode_rune(const uint8_t *p, size_t n, uint32_t *r, size_t *sz) {
  const uint8_t b0 = p[0];
  auto bad = [&] {
    *r = 0xFFFD;
    *sz = 1;
  };
  auto cont = [&](size_t i) { return i < n && (p[i] & 0xC0) == 0x80; };
  if (b0 < 0x80) {
    *r = b0;
    *sz = 1;
  } else if (b0 >= 0xC2 && b0 <= 0xDF) {
    if (!cont(1)) return bad();
    *r = (uint32_t(b0 & 0x1F) << 6) | (p[1] & 0x3F);
    *sz = 2;
  } else if (b0 >= 0xE0 && b0 <= 0xEF) {
    if (!cont(1) || !cont(2)) return bad();
    // E0: second byte A0..BF (no overlong); ED: 80..9F (no surrogates)
    if (b0 == 0xE0 && p[1] < 0xA0) return bad();
    if (b0 == 0xED && p[1] > 0x9F) return bad();
    *r = (uint32_t(b0 & 0x0F) << 12) | (uint32_t(p[1] & 0x3F) << 6) | (p[2] & 0x3F);
    *sz = 3;
  } else if (b0 >= 0xF0 && b0 <= 0xF4) {
    if (!cont(1) || !cont(2) || !cont(3)) return bad();
    if (b0 == 0xF0 && p[1] < 0x90) return bad();
    if (b0 == 0xF4 && p[1] > 0x8F) return bad();
    *r = (uint32_t(b0 & 0x07) << 18) | (uint32_t(p[1] & 0x3F) << 12) |
         (uint32_t(p[2] & 0x3F) << 6) | (p[3] & 0x3F);
    *sz = 4;
  } else {
    bad();
  }
}

// encoding/json appendString(escapeHTML = true).  out == nullptr: length only.
size_t json_string(const uint8_t *s, size_t n, uint8_t *out) {
  size_t o = 0;
  auto put = [&](uint8_t c) {
    if (out) out[o] = c;
    ++o;
  };
  put('"');
  for (size_t i = 0; i < n;) {
    const uint8_t b = s[i];
    if (b < 0x80) {
      // htmlSafeSet: printable ASCII except '"', '\\', '<', '>', '&'
      if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
        put(b);
      } else {
        put('\\');
        switch (b) {
          case '"': case '\\': put(b); break;
          case '\b': put('b'); break;
          case '\f': put('f'); break;
          case '\n': put('n'); break;
          case '\r': put('r'); break;
          case '\t': put('t'); break;
          default:
            put('u'); put('0'); put('0');
            put(uint8_t(kHex[b >> 4])); put(uint8_t(kHex[b & 15]));
        }
      }
      ++i;
      continue;
    }
    uint32_t r;
    size_t sz;
    decode_rune(s + i, n - i, &r, &sz);
    if (r == 0xFFFD && sz == 1) {  // invalid UTF-8: the 6-byte escape
      for (const char *e = "\\ufffd"; *e; ++e) put(uint8_t(*e));
    } else if (r == 0x2028 || r == 0x2029) {
      for (const char *e = "\\u202"; *e; ++e) put(uint8_t(*e));
      put(uint8_t(kHex[r & 15]));
    } else {
      for (size_t k = 0; k < sz; ++k) put(s[i + k]);
    }
    i += sz;
  }
  put('"');
  return o;
}

size_t u64_dec(uint64_t v, uint8_t *out) {
  uint8_t t[20];
  size_t k = 0;
  do {
    t[k++] = uint8_t('0' + v % 10);
    v /= 10;
  } while (v);
  if (out)
    for (size_t i = 0; i < k; ++i) out[i] = t[k - 1 - i];
  return k;
}

size_t lit(const char *s, uint8_t *out) {
  const size_t n = strlen(s);
  if (out) memcpy(out, s, n);
  return n;
}

size_t hex32(const uint8_t *x, uint8_t *out) {
  if (out) {
    out[0] = '"';
    for (int i = 0; i < 32; ++i) {
      out[1 + 2 * i] = uint8_t(kHex[x[i] >> 4]);
      out[2 + 2 * i] = uint8_t(kHex[x[i] & 15]);
    }
    out[65] = '"';
  }
  return 66;
}

struct Entries {
  const uint8_t *names;
  const uint64_t *name_offs;
  const uint32_t *modes;
  const uint8_t *types;
  const uint64_t *type_offs;
  const uint8_t *roots;
  const uint64_t *sizes, *block_sizes;
};

// One line (out == nullptr: its length).
size_t line(const Entries &e, uint64_t i, uint8_t *out) {
  size_t o = 0;
  auto at = [&]() { return out ? out + o : nullptr; };
  o += lit("{\"name\":", at());
  o += json_string(e.names + e.name_offs[i], e.name_offs[i + 1] - e.name_offs[i], at());
  o += lit(",\"mode\":", at());
  o += u64_dec(e.modes[i], at());
  o += lit(",\"ref\":{\"type\":", at());
  o += json_string(e.types + e.type_offs[i], e.type_offs[i + 1] - e.type_offs[i], at());
  o += lit(",\"cid\":", at());
  o += hex32(e.roots + 64 * i, at());
  o += lit(",\"dek\":", at());
  o += hex32(e.roots + 64 * i + 32, at());
  o += lit(",\"size\":", at());
  o += u64_dec(e.sizes[i], at());
  o += lit(",\"blockSize\":", at());
  o += u64_dec(e.block_sizes[i], at());
  o += lit("}}\n", at());
  return o;
}

template <class F>
void parallel_ranges(uint64_t n, F f) {
  unsigned hw = std::thread::hardware_concurrency();
  const uint64_t t = std::min<uint64_t>(std::min(16u, hw ? hw : 1u),
                                        std::max<uint64_t>(1, n / 4096));
  if (t <= 1) {
    f(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  for (uint64_t k = 0; k < t; ++k)
    th.emplace_back(f, k, n * k / t, n * (k + 1) / t);
  for (auto &x : th) x.join();
}

}  // namespace

extern "C" int glfsx_tree_encode(uint64_t n, const uint8_t *names,
                                 const uint64_t *name_offs, const uint32_t *modes,
                                 const uint8_t *types, const uint64_t *type_offs,
                                 const uint8_t *roots, const uint64_t *sizes,
                                 const uint64_t *block_sizes, uint8_t *out,
                                 uint64_t out_cap, uint64_t *out_len,
                                 uint64_t *line_ends) {
  if (!out_len || (n && (!name_offs || !modes || !type_offs || !roots || !sizes ||
                         !block_sizes)))
    return GLFSX_E_ARG;
  const Entries e{names, name_offs, modes, types, type_offs, roots, sizes, block_sizes};
  std::vector<uint64_t> ends(line_ends ? 0 : n);
  uint64_t *L = line_ends ? line_ends : ends.data();
  // pass 1: per-line lengths, then per-thread sums scanned into ends
  parallel_ranges(n, [&](uint64_t, uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) L[i] = line(e, i, nullptr);
  });
  uint64_t acc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    acc += L[i];
    L[i] = acc;
  }
  *out_len = acc;
  if (!out) return GLFSX_OK;
  if (out_cap < acc) return GLFSX_E_ARG;
  parallel_ranges(n, [&](uint64_t, uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) line(e, i, out + (i ? L[i - 1] : 0));
  });
  return GLFSX_OK;
}
