/*
 * oracle.c -- CPU restatement of the bigblob write path (TEST INFRASTRUCTURE).
 * See oracle.h for the reference citations and how this file is pinned.
 *
 * Deliberately written as a plain, recursive restatement of the published
 * specifications (BLAKE3 spec section 2.1-2.6; RFC 8439 section 2.3-2.4) and of
 * bigblob/blob.go's streaming writer, NOT as a copy of the GPU design, so
 * that the two implementations are independent.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ BLAKE3 */
/* Constants from the BLAKE3 specification, section 2.1 / 2.2. */
static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u,
                                  0xA54FF53Au, 0x510E527Fu, 0x9B05688Cu,
                                  0x1F83D9ABu, 0x5BE0CD19u};
static const int B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13,
                                1, 11, 12, 5, 9, 14, 15, 8};
enum {
  F_CHUNK_START = 1,
  F_CHUNK_END = 2,
  F_PARENT = 4,
  F_ROOT = 8,
  F_KEYED_HASH = 16,
};
#define B3_BLOCK 64
#define B3_CHUNK 1024

static inline uint32_t rotr32(uint32_t x, int n) {
  return (x >> n) | (x << (32 - n));
}
static inline uint32_t load32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}
static inline void store32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

static void b3_g(uint32_t *s, int a, int b, int c, int d, uint32_t x,
                 uint32_t y) {
  s[a] = s[a] + s[b] + x;
  s[d] = rotr32(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr32(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + y;
  s[d] = rotr32(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr32(s[b] ^ s[c], 7);
}

/* Full compression function (spec 2.2): 16-word output. */
static void b3_compress(uint32_t out[16], const uint32_t cv[8],
                        const uint32_t m_in[16], uint64_t counter,
                        uint32_t block_len, uint32_t flags) {
  uint32_t s[16], m[16], t[16];
  memcpy(m, m_in, sizeof m);
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  s[8] = B3_IV[0];
  s[9] = B3_IV[1];
  s[10] = B3_IV[2];
  s[11] = B3_IV[3];
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  for (int r = 0; r < 7; r++) {
    b3_g(s, 0, 4, 8, 12, m[0], m[1]);
    b3_g(s, 1, 5, 9, 13, m[2], m[3]);
    b3_g(s, 2, 6, 10, 14, m[4], m[5]);
    b3_g(s, 3, 7, 11, 15, m[6], m[7]);
    b3_g(s, 0, 5, 10, 15, m[8], m[9]);
    b3_g(s, 1, 6, 11, 12, m[10], m[11]);
    b3_g(s, 2, 7, 8, 13, m[12], m[13]);
    b3_g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
      memcpy(m, t, sizeof m);
    }
  }
  for (int i = 0; i < 8; i++) {
    out[i] = s[i] ^ s[i + 8];
    out[i + 8] = s[i + 8] ^ cv[i];
  }
}

/* The inputs of a node's final compression, before ROOT is known (spec 2.5:
 * "the root node's final compression gets the ROOT flag"). */
typedef struct {
  uint32_t cv[8];
  uint32_t block[16];
  uint64_t counter;
  uint32_t block_len;
  uint32_t flags;
} b3_node;

static void b3_node_cv(const b3_node *nd, uint32_t cv_out[8]) {
  uint32_t o[16];
  b3_compress(o, nd->cv, nd->block, nd->counter, nd->block_len, nd->flags);
  memcpy(cv_out, o, 32);
}

static void b3_words_from_bytes(uint32_t w[16], const uint8_t *p, size_t n) {
  uint8_t buf[B3_BLOCK];
  memset(buf, 0, sizeof buf);
  if (n) memcpy(buf, p, n);
  for (int i = 0; i < 16; i++) w[i] = load32(buf + 4 * i);
}

/* A chunk node (spec 2.4): up to 16 blocks, counter = chunk index. */
static void b3_chunk_node(b3_node *nd, const uint32_t key[8], uint32_t base,
                          const uint8_t *in, size_t n, uint64_t chunk_idx) {
  uint32_t cv[8];
  memcpy(cv, key, 32);
  size_t nblocks = n == 0 ? 1 : (n + B3_BLOCK - 1) / B3_BLOCK;
  for (size_t b = 0; b < nblocks; b++) {
    size_t off = b * B3_BLOCK;
    size_t len = n - off < B3_BLOCK ? n - off : B3_BLOCK;
    if (n == 0) len = 0;
    uint32_t flags = base;
    if (b == 0) flags |= F_CHUNK_START;
    if (b == nblocks - 1) flags |= F_CHUNK_END;
    uint32_t m[16];
    b3_words_from_bytes(m, in + off, len);
    if (b == nblocks - 1) {
      memcpy(nd->cv, cv, 32);
      memcpy(nd->block, m, 64);
      nd->counter = chunk_idx;
      nd->block_len = (uint32_t)len;
      nd->flags = flags;
    } else {
      uint32_t o[16];
      b3_compress(o, cv, m, chunk_idx, (uint32_t)len, flags);
      memcpy(cv, o, 32);
    }
  }
}

/* Any subtree (spec 2.5): the left subtree holds the largest power-of-two
 * number of chunks that leaves at least one byte for the right subtree. */
static void b3_subtree_node(b3_node *nd, const uint32_t key[8], uint32_t base,
                            const uint8_t *in, size_t n, uint64_t chunk0) {
  if (n <= B3_CHUNK) {
    b3_chunk_node(nd, key, base, in, n, chunk0);
    return;
  }
  size_t chunks = (n + B3_CHUNK - 1) / B3_CHUNK;
  size_t left_chunks = 1;
  while (left_chunks * 2 < chunks) left_chunks *= 2;
  size_t left_len = left_chunks * B3_CHUNK;
  b3_node l, r;
  b3_subtree_node(&l, key, base, in, left_len, chunk0);
  b3_subtree_node(&r, key, base, in + left_len, n - left_len,
                  chunk0 + left_chunks);
  uint32_t lcv[8], rcv[8];
  b3_node_cv(&l, lcv);
  b3_node_cv(&r, rcv);
  memcpy(nd->cv, key, 32);
  memcpy(nd->block, lcv, 32);
  memcpy(nd->block + 8, rcv, 32);
  nd->counter = 0;
  nd->block_len = B3_BLOCK;
  nd->flags = base | F_PARENT;
}

void oracle_blake3(uint8_t *out, size_t out_len, const uint8_t key[32],
                   const uint8_t *in, size_t n) {
  uint32_t kw[8];
  uint32_t base = 0;
  if (key) {
    for (int i = 0; i < 8; i++) kw[i] = load32(key + 4 * i);
    base = F_KEYED_HASH;
  } else {
    memcpy(kw, B3_IV, 32);
  }
  b3_node root;
  b3_subtree_node(&root, kw, base, in, n, 0);
  /* XOF (spec 2.6): output block t = root compression with counter t. */
  size_t done = 0;
  for (uint64_t t = 0; done < out_len; t++) {
    uint32_t o[16];
    b3_compress(o, root.cv, root.block, t, root.block_len, root.flags | F_ROOT);
    uint8_t ob[64];
    for (int i = 0; i < 16; i++) store32(ob + 4 * i, o[i]);
    size_t take = out_len - done < 64 ? out_len - done : 64;
    memcpy(out + done, ob, take);
    done += take;
  }
}

/* --------------------------------------------------------------- ChaCha20 */
/* RFC 8439 section 2.1-2.4. */
static inline uint32_t rotl32(uint32_t x, int n) {
  return (x << n) | (x >> (32 - n));
}
#define QR(a, b, c, d)        \
  do {                        \
    a += b;                   \
    d ^= a;                   \
    d = rotl32(d, 16);        \
    c += d;                   \
    b ^= c;                   \
    b = rotl32(b, 12);        \
    a += b;                   \
    d ^= a;                   \
    d = rotl32(d, 8);         \
    c += d;                   \
    b ^= c;                   \
    b = rotl32(b, 7);         \
  } while (0)

static void chacha20_block(uint8_t out[64], const uint32_t key[8],
                           uint32_t counter, const uint32_t nonce[3]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                     key[0],      key[1],      key[2],      key[3],
                     key[4],      key[5],      key[6],      key[7],
                     counter,     nonce[0],    nonce[1],    nonce[2]};
  uint32_t x[16];
  memcpy(x, in, sizeof x);
  for (int i = 0; i < 10; i++) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) store32(out + 4 * i, x[i] + in[i]);
}

void oracle_chacha20_xor(uint8_t *dst, const uint8_t *src, size_t n,
                         const uint8_t key[32], const uint8_t nonce[12],
                         uint32_t counter) {
  uint32_t kw[8], nw[3];
  for (int i = 0; i < 8; i++) kw[i] = load32(key + 4 * i);
  for (int i = 0; i < 3; i++) nw[i] = load32(nonce + 4 * i);
  uint8_t ks[64];
  for (size_t off = 0; off < n; off += 64, counter++) {
    chacha20_block(ks, kw, counter, nw);
    size_t take = n - off < 64 ? n - off : 64;
    for (size_t i = 0; i < take; i++) dst[off + i] = src[off + i] ^ ks[i];
  }
}

/* ---------------------------------------------------------- bigblob layer */
/* ref.go:152-161: blake3.New(len(out)=32, salt) keyed; first 32 XOF bytes. */
void oracle_derive_key(uint8_t out[32], const uint8_t salt[32],
                       const uint8_t *in, size_t n) {
  oracle_blake3(out, 32, salt, in, n);
}

/* ref.go:98-111 + 128-149: dek = DeriveKey(salt, ptext); ctext = ChaCha20(dek,
 * nonce 0^12, counter 0) ^ ptext; cid = store.Post(ctext). */
void oracle_post(uint8_t ref[64], uint8_t *ctext, const uint8_t salt[32],
                 const uint8_t *ptext, size_t n, const uint8_t *cid_key) {
  uint8_t dek[32];
  static const uint8_t zero_nonce[12] = {0};
  oracle_derive_key(dek, salt, ptext, n);
  uint8_t *ct = ctext;
  uint8_t *tmp = NULL;
  if (!ct) {
    tmp = (uint8_t *)malloc(n ? n : 1);
    ct = tmp;
  }
  oracle_chacha20_xor(ct, ptext, n, dek, zero_nonce, 0);
  oracle_blake3(ref, 32, cid_key, ct, n); /* CID */
  memcpy(ref + 32, dek, 32);              /* Ref = CID || DEK, ref.go:77-82 */
  free(tmp);
}

/* bigblob/blob.go:71-83 Writer state. */
struct oracle_writer {
  uint64_t bs, bf;
  uint8_t raw_salt[32], index_salt[32];
  uint8_t cid_key[32];
  int has_cid_key;
  oracle_sink_fn sink;
  void *sink_ctx;
  /* levels: indexes[i] is a bs-byte Index (index.go:12-14), counts[i] */
  uint8_t **indexes;
  uint64_t *counts;
  int nlevels, cap;
  uint64_t size;
  uint8_t *buf;
  uint64_t buflen;
  uint8_t *ct; /* scratch ctext, bs bytes */
};

static int w_post(oracle_writer *w, int kind, const uint8_t *salt,
                  const uint8_t *p, uint64_t n, uint8_t ref[64]) {
  oracle_post(ref, w->ct, salt, p, n, w->has_cid_key ? w->cid_key : NULL);
  if (w->sink) return w->sink(w->sink_ctx, kind, ref, w->ct, n);
  return 0;
}

static void w_grow(oracle_writer *w, int i) {
  while (w->nlevels <= i) {
    if (w->nlevels == w->cap) {
      w->cap = w->cap ? 2 * w->cap : 4;
      w->indexes = (uint8_t **)realloc(w->indexes, w->cap * sizeof(uint8_t *));
      w->counts = (uint64_t *)realloc(w->counts, w->cap * sizeof(uint64_t));
    }
    w->indexes[w->nlevels] = (uint8_t *)calloc(w->bs, 1);
    w->counts[w->nlevels] = 0;
    w->nlevels++;
  }
}

oracle_writer *oracle_writer_new(uint64_t block_size, uint64_t store_max,
                                 const uint8_t *salt, const uint8_t *cid_key,
                                 oracle_sink_fn sink, void *sink_ctx,
                                 int *err) {
  uint64_t bs = store_max; /* blob.go:86 */
  if (block_size > 0) bs = block_size;
  if (bs > store_max) { /* blob.go:90-92 panic */
    if (err) *err = -1;
    return NULL;
  }
  if (bs < 128) { /* blob.go:93-95 panic */
    if (err) *err = -2;
    return NULL;
  }
  static const uint8_t zero[32] = {0};
  if (!salt) salt = zero; /* blob.go:96-98 */
  oracle_writer *w = (oracle_writer *)calloc(1, sizeof *w);
  w->bs = bs;
  w->bf = bs / 64; /* blob.go:107 */
  oracle_derive_key(w->index_salt, salt, (const uint8_t *)"index", 5);
  oracle_derive_key(w->raw_salt, salt, (const uint8_t *)"raw", 3);
  if (cid_key) {
    memcpy(w->cid_key, cid_key, 32);
    w->has_cid_key = 1;
  }
  w->sink = sink;
  w->sink_ctx = sink_ctx;
  w_grow(w, 0);
  w->buf = (uint8_t *)malloc(bs);
  w->ct = (uint8_t *)malloc(bs);
  if (err) *err = 0;
  return w;
}

/* blob.go:165-182 */
static int w_add_ref(oracle_writer *w, int i, const uint8_t ref[64]) {
  w_grow(w, i);
  memcpy(w->indexes[i] + w->counts[i] * 64, ref, 64); /* index.go:33-38 */
  w->counts[i]++;
  if (w->counts[i] < w->bf) return 0;
  uint8_t r2[64];
  int e = w_post(w, 1, w->index_salt, w->indexes[i], w->bs, r2);
  if (e) return e;
  w->counts[i] = 0;
  memset(w->indexes[i], 0, w->bs); /* index.go:44-48 */
  return w_add_ref(w, i + 1, r2);
}

/* blob.go:152-163 */
static int w_post_buf(oracle_writer *w) {
  uint8_t ref[64];
  int e = w_post(w, 0, w->raw_salt, w->buf, w->buflen, ref);
  if (e) return e;
  e = w_add_ref(w, 0, ref);
  if (e) return e;
  w->size += w->buflen;
  w->buflen = 0;
  return 0;
}

/* blob.go:120-133 (the recursion unrolled into a loop) */
int oracle_writer_write(oracle_writer *w, const uint8_t *data, size_t n) {
  for (;;) {
    if (w->buflen + n < w->bs) {
      memcpy(w->buf + w->buflen, data, n);
      w->buflen += n;
      return 0;
    }
    size_t k = w->bs - w->buflen;
    memcpy(w->buf + w->buflen, data, k);
    w->buflen += k;
    int e = w_post_buf(w);
    if (e) return e;
    data += k;
    n -= k;
  }
}

/* blob.go:184-206 */
static int w_finish_indexes(oracle_writer *w, uint8_t out[64]) {
  for (int i = 0; i < w->nlevels; i++) {
    if (i == w->nlevels - 1) {
      if (w->counts[i] == 0) return w_post(w, 1, w->index_salt, NULL, 0, out);
      if (w->counts[i] == 1) {
        memcpy(out, w->indexes[i], 64);
        return 0;
      }
    }
    if (w->counts[i] > 0) {
      uint8_t r[64];
      int e = w_post(w, 1, w->index_salt, w->indexes[i], w->bs, r);
      if (e) return e;
      e = w_add_ref(w, i + 1, r);
      if (e) return e;
    }
  }
  return -100; /* "should not happen" panic */
}

/* blob.go:135-150 */
int oracle_writer_finish(oracle_writer *w, uint8_t root_ref[64],
                         uint64_t *size, uint64_t *block_size) {
  if (w->buflen > 0) {
    int e = w_post_buf(w);
    if (e) return e;
  }
  int e = w_finish_indexes(w, root_ref);
  if (e) return e;
  if (size) *size = w->size;
  if (block_size) *block_size = w->bs;
  return 0;
}

void oracle_writer_free(oracle_writer *w) {
  if (!w) return;
  for (int i = 0; i < w->nlevels; i++) free(w->indexes[i]);
  free(w->indexes);
  free(w->counts);
  free(w->buf);
  free(w->ct);
  free(w);
}

/* Closed form: n0 == 0 -> post(indexSalt, ""); n0 == 1 ->
 * ref0; else refs_{k+1}[j] = post(indexSalt, zeropad_bs(refs_k[j*bf..])).
 * Sink order differs from the streaming writer (level by level). */
int64_t oracle_create_closed(uint64_t bs, const uint8_t *salt,
                             const uint8_t *cid_key, const uint8_t *data,
                             uint64_t size, uint8_t root_ref[64],
                             oracle_sink_fn sink, void *sink_ctx) {
  static const uint8_t zero[32] = {0};
  if (!salt) salt = zero;
  uint8_t raw[32], idx[32];
  oracle_derive_key(idx, salt, (const uint8_t *)"index", 5);
  oracle_derive_key(raw, salt, (const uint8_t *)"raw", 3);
  uint64_t bf = bs / 64;
  uint64_t n = (size + bs - 1) / bs;
  int64_t posts = 0;
  uint8_t *ct = (uint8_t *)malloc(bs);
  if (n == 0) {
    oracle_post(root_ref, ct, idx, NULL, 0, cid_key);
    if (sink) sink(sink_ctx, 1, root_ref, ct, 0);
    free(ct);
    return 1;
  }
  uint8_t *refs = (uint8_t *)malloc(n * 64);
  for (uint64_t j = 0; j < n; j++) {
    uint64_t len = (j == n - 1) ? size - j * bs : bs;
    oracle_post(refs + 64 * j, ct, raw, data + j * bs, len, cid_key);
    if (sink) sink(sink_ctx, 0, refs + 64 * j, ct, len);
    posts++;
  }
  uint8_t *node = (uint8_t *)malloc(bs);
  while (n > 1) {
    uint64_t m = (n + bf - 1) / bf;
    uint8_t *up = (uint8_t *)malloc(m * 64);
    for (uint64_t j = 0; j < m; j++) {
      uint64_t cnt = n - j * bf < bf ? n - j * bf : bf;
      memset(node, 0, bs);
      memcpy(node, refs + j * bf * 64, cnt * 64);
      oracle_post(up + 64 * j, ct, idx, node, bs, cid_key);
      if (sink) sink(sink_ctx, 1, up + 64 * j, ct, bs);
      posts++;
    }
    free(refs);
    refs = up;
    n = m;
  }
  memcpy(root_ref, refs, 64);
  free(refs);
  free(node);
  free(ct);
  return posts;
}

/* blob.go:219-268 */
static uint64_t log2_ceil(uint64_t x) {
  int l = 64 - __builtin_clzll(x);
  if (__builtin_popcountll(x) > 1) l++;
  return (uint64_t)l - 1;
}
static uint64_t div_ceil(uint64_t a, uint64_t b) { return (a + b - 1) / b; }
int oracle_depth(uint64_t size, uint64_t bs) {
  if (size == 0) return 0;
  uint64_t blocks = div_ceil(size, bs);
  uint64_t bf = bs / 64;
  return (int)div_ceil(log2_ceil(blocks), log2_ceil(bf));
}

/* ------------------------------------------------- threaded CPU baseline */
typedef struct {
  uint8_t *refs, *ctext;
  const uint8_t *salt, *ptext, *cid_key;
  uint64_t total, chunk, first, last;
} batch_job;

static void *batch_worker(void *arg) {
  batch_job *j = (batch_job *)arg;
  uint8_t *scratch = j->ctext ? NULL : (uint8_t *)malloc(j->chunk);
  for (uint64_t b = j->first; b < j->last; b++) {
    uint64_t off = b * j->chunk;
    uint64_t len = j->total - off < j->chunk ? j->total - off : j->chunk;
    oracle_post(j->refs + 64 * b, j->ctext ? j->ctext + off : scratch, j->salt,
                j->ptext + off, len, j->cid_key);
  }
  free(scratch);
  return NULL;
}

void oracle_post_batch(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                       const uint8_t *ptext, uint64_t total, uint64_t chunk,
                       const uint8_t *cid_key, int threads) {
  uint64_t n = (total + chunk - 1) / chunk;
  if (threads < 1) threads = 1;
  if ((uint64_t)threads > n) threads = n ? (int)n : 1;
  pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
  batch_job *jobs = (batch_job *)malloc(sizeof(batch_job) * threads);
  for (int t = 0; t < threads; t++) {
    batch_job *j = &jobs[t];
    j->refs = refs;
    j->ctext = ctext;
    j->salt = salt;
    j->ptext = ptext;
    j->cid_key = cid_key;
    j->total = total;
    j->chunk = chunk;
    j->first = n * t / threads;
    j->last = n * (t + 1) / threads;
    pthread_create(&tid[t], NULL, batch_worker, j);
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  free(tid);
  free(jobs);
}

/* ------------------------------------------------------------- generator */
static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void oracle_fill_splitmix(uint8_t *dst, uint64_t offset, uint64_t n,
                          uint64_t seed) {
  for (uint64_t i = 0; i < n; i++) {
    uint64_t o = offset + i;
    uint64_t w = splitmix64(seed ^ (o >> 3));
    dst[i] = (uint8_t)(w >> (8 * (o & 7)));
  }
}

/* n blobs of len bytes back to back: blob b = oracle_fill_splitmix(seed0 + b)
 * at offset 0 (BASELINE config 4: distinct blobs, seed = blob index). */
void oracle_fill_splitmix_blobs(uint8_t *dst, uint64_t n, uint64_t len,
                                uint64_t seed0) {
  for (uint64_t b = 0; b < n; b++) oracle_fill_splitmix(dst + b * len, 0, len, seed0 + b);
}
