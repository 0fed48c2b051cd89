// store.cpp -- the store boundary of the write path.
//
// bigblob's post() hands every ctext to the store, whose Post computes the
// CID itself (ref.go:103 s.Post(ctx, ctext); blobcache MemStore hashes with
// BLAKE3-256 [ext]).  The GPU path already computed that CID, so a store that
// accepts it -- a pre-hashed Post -- removes the second host-side BLAKE3 pass
// over every byte.  glfsx_store is an in-memory content-addressed store
// (MemStore's role: CID -> ctext, MaxSize, Get, Exists) with both Posts:
//
//   GLFSX_STORE_TRUST  Post(ref, ctext) keeps the GPU CID; parity mode
//                      (verify_every = k > 0) re-hashes every k-th Post on the
//                      host and fails that Post on a mismatch;
//   GLFSX_STORE_HASH   Post hashes the ctext on the calling thread, as
//                      MemStore.Post does behind ref.go:103, and fails when
//                      the hash differs from the GPU CID.
//
// The host hash is the store's, not the write path's: it is the upstream
// BLAKE3 C implementation (1.8.2, AVX-512 dispatch) that ships inside the
// image's LLVM (libclang-cpp.so, llvm_blake3_*), loaded on first use.  When
// it is absent the hashing modes fail with GLFSX_E_UNSUPPORTED; nothing on
// the write path depends on it.
#include <dlfcn.h>
#include <sys/mman.h>

#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <algorithm>
#include <vector>

#include "../../include/glfsx.h"

namespace {

struct B3 {
  void (*init)(void *) = nullptr;
  void (*init_keyed)(void *, const uint8_t *) = nullptr;
  void (*update)(void *, const void *, size_t) = nullptr;
  void (*finalize)(const void *, uint8_t *, size_t) = nullptr;
  bool ok = false;
};

const B3 &host_blake3() {
  static B3 b;
  static std::once_flag once;
  std::call_once(once, [] {
    const char *paths[] = {"/opt/rocm/lib/llvm/lib/libclang-cpp.so", "libclang-cpp.so"};
    for (const char *p : paths) {
      void *h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
      if (!h) continue;
      b.init = reinterpret_cast<void (*)(void *)>(dlsym(h, "llvm_blake3_hasher_init"));
      b.init_keyed = reinterpret_cast<void (*)(void *, const uint8_t *)>(
          dlsym(h, "llvm_blake3_hasher_init_keyed"));
      b.update = reinterpret_cast<void (*)(void *, const void *, size_t)>(
          dlsym(h, "llvm_blake3_hasher_update"));
      b.finalize = reinterpret_cast<void (*)(const void *, uint8_t *, size_t)>(
          dlsym(h, "llvm_blake3_hasher_finalize"));
      b.ok = b.init && b.init_keyed && b.update && b.finalize;
      if (b.ok) break;
    }
  });
  return b;
}

struct CidHash {
  size_t operator()(const std::string &k) const {
    size_t h;
    memcpy(&h, k.data(), sizeof h);  // a CID is already uniform
    return h;
  }
};

}  // namespace

// Blob bytes live in large arenas (mmap'd, transparent huge pages where the
// kernel allows): one 1 MiB allocation plus 256 page faults per Post cost
// more than the write path's whole host round trip.
struct Arena {
  std::vector<std::pair<uint8_t *, size_t>> chunks;
  uint8_t *cur = nullptr;
  size_t left = 0;
  uint8_t *alloc(size_t n) {
    if (n > left) {
      const size_t sz = std::max<size_t>(n, size_t(256) << 20);
      void *p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (p == MAP_FAILED) return nullptr;
      (void)madvise(p, sz, MADV_HUGEPAGE);
      chunks.emplace_back(static_cast<uint8_t *>(p), sz);
      cur = static_cast<uint8_t *>(p);
      left = sz;
    }
    uint8_t *r = cur;
    const size_t a = (n + 63) & ~size_t(63);
    cur += std::min(a, left);
    left -= std::min(a, left);
    return r;
  }
  ~Arena() {
    for (auto &c : chunks) munmap(c.first, c.second);
  }
};

struct glfsx_store {
  uint64_t max_size = 0;
  int mode = GLFSX_STORE_TRUST;
  uint64_t verify_every = 0;
  bool keep_data = true;
  bool keyed = false;
  uint8_t key[32]{};
  std::mutex mu;
  std::unordered_map<std::string, std::pair<const uint8_t *, uint64_t>, CidHash> blobs;
  Arena arena;
  uint64_t posts = 0, bytes = 0, hashed = 0;
  std::string err;
};

namespace {
void hash_cid(const glfsx_store *s, const void *data, uint64_t n, uint8_t out[32]) {
  const B3 &b = host_blake3();
  alignas(64) uint8_t hasher[4096];  // upstream blake3_hasher is < 2 KiB
  if (s->keyed)
    b.init_keyed(hasher, s->key);
  else
    b.init(hasher);
  if (n) b.update(hasher, data, n);
  b.finalize(hasher, out, 32);
}
}  // namespace

extern "C" {

glfsx_store *glfsx_store_new(uint64_t max_size, int mode, uint64_t verify_every,
                             int keep_data, const uint8_t *cid_key) {
  if (mode != GLFSX_STORE_TRUST && mode != GLFSX_STORE_HASH) return nullptr;
  if ((mode == GLFSX_STORE_HASH || verify_every) && !host_blake3().ok) return nullptr;
  auto *s = new glfsx_store();
  s->max_size = max_size;
  s->mode = mode;
  s->verify_every = verify_every;
  s->keep_data = keep_data != 0;
  if (cid_key) {
    s->keyed = true;
    memcpy(s->key, cid_key, 32);
  }
  return s;
}

void glfsx_store_free(glfsx_store *s) { delete s; }

int glfsx_store_post(void *store, int kind, const uint8_t *ref, const void *ctext,
                     uint64_t len) {
  (void)kind;
  auto *s = static_cast<glfsx_store *>(store);
  if (!s || !ref || (len && !ctext)) return GLFSX_E_ARG;
  if (len > s->max_size) {  // MemStore: blob larger than MaxSize
    std::lock_guard<std::mutex> lk(s->mu);
    s->err = "blob too large";
    return GLFSX_E_ARG;
  }
  uint64_t seq;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    seq = s->posts++;
  }
  const bool rehash = s->mode == GLFSX_STORE_HASH ||
                      (s->verify_every && seq % s->verify_every == 0);
  if (rehash) {  // outside the lock: concurrent writers hash in parallel
    uint8_t cid[32];
    hash_cid(s, ctext, len, cid);
    if (memcmp(cid, ref, 32) != 0) {
      std::lock_guard<std::mutex> lk(s->mu);
      s->err = "store CID differs from the GPU CID";
      return GLFSX_E_STORE;
    }
  }
  std::lock_guard<std::mutex> lk(s->mu);
  s->bytes += len;
  s->hashed += rehash ? 1 : 0;
  std::string k(reinterpret_cast<const char *>(ref), 32);
  auto it = s->blobs.find(k);
  if (it == s->blobs.end()) {
    uint8_t *p = nullptr;
    if (s->keep_data && len) {
      p = s->arena.alloc(len);
      if (!p) {
        s->err = "store out of memory";
        return GLFSX_E_NOMEM;
      }
      memcpy(p, ctext, len);
    }
    s->blobs.emplace(std::move(k), std::make_pair(p, s->keep_data ? len : 0));
  }
  return 0;
}

int glfsx_store_exists(glfsx_store *s, const uint8_t cid[32]) {
  if (!s || !cid) return 0;
  std::lock_guard<std::mutex> lk(s->mu);
  return s->blobs.count(std::string(reinterpret_cast<const char *>(cid), 32)) ? 1 : 0;
}

int glfsx_store_get(glfsx_store *s, const uint8_t cid[32], const void **data,
                    uint64_t *len) {
  if (!s || !cid || !data || !len) return GLFSX_E_ARG;
  std::lock_guard<std::mutex> lk(s->mu);
  auto it = s->blobs.find(std::string(reinterpret_cast<const char *>(cid), 32));
  if (it == s->blobs.end()) return GLFSX_E_STORE;  // blobcache.ErrNotFound
  *data = it->second.first;
  *len = it->second.second;
  return 0;
}

uint64_t glfsx_store_stats(glfsx_store *s, uint64_t *posts, uint64_t *bytes,
                           uint64_t *hashed) {
  if (!s) return 0;
  std::lock_guard<std::mutex> lk(s->mu);
  if (posts) *posts = s->posts;
  if (bytes) *bytes = s->bytes;
  if (hashed) *hashed = s->hashed;
  return s->blobs.size();
}

// A copy per calling thread: concurrent Posts may replace s->err meanwhile.
const char *glfsx_store_error(glfsx_store *s) {
  if (!s) return "null store";
  static thread_local std::string copy;
  std::lock_guard<std::mutex> lk(s->mu);
  copy = s->err;
  return copy.c_str();
}

}  // extern "C"
