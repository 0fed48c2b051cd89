/*
 * cpu_simd.c -- a second CPU baseline for bench.py (TEST INFRASTRUCTURE: the
 * cpu_baseline leg only; never the checker, never the product).
 *
 * oracle.c restates the path in portable scalar C.  The reference's Go path
 * runs on assembly-backed primitives instead: lukechampine.com/blake3 v1.2.1
 * (AVX-512) for the DEK and blobcache's BLAKE3-256 for the CID [ext], and
 * x/crypto's ChaCha20 (generic Go on amd64 [ext]).  This file times the same
 * per-block sequence as oracle_post_batch (bigblob/ref.go:98-161: keyed
 * BLAKE3 -> ChaCha20 XOR -> BLAKE3 of the ctext) on the best SIMD
 * implementations present in the image: the upstream BLAKE3 C library
 * (1.8.2, AVX-512 dispatch) exported by libclang-cpp.so as llvm_blake3_*,
 * and OpenSSL's ChaCha20 (libcrypto EVP_chacha20, AVX-512).  It is an upper
 * bound on what the Go path's primitives can do per core, not the Go path.
 * Both libraries are loaded with dlopen; when either is absent the function
 * returns -1.
 *
 * oracle_post_batch_gomix is the Go path's primitive mix instead: the same
 * SIMD BLAKE3 for the DEK and the CID (as lukechampine's AVX-512 assembly,
 * go.mod:12) with the portable scalar ChaCha20 of oracle.c (as x/crypto's
 * generic Go ChaCha20, the one amd64 runs, go.mod:10; ref.go:137-144).
 * bench.py reports it as cpu_baseline.value.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  void (*init)(void *);
  void (*init_keyed)(void *, const uint8_t *);
  void (*update)(void *, const void *, size_t);
  void (*finalize)(const void *, uint8_t *, size_t);
  void *(*ctx_new)(void);
  void (*ctx_free)(void *);
  const void *(*chacha)(void);
  int (*enc_init)(void *, const void *, void *, const uint8_t *, const uint8_t *);
  int (*enc_update)(void *, uint8_t *, int *, const uint8_t *, int);
} simd_libs;

static int load(simd_libs *L) {
  void *b = dlopen("/opt/rocm/lib/llvm/lib/libclang-cpp.so", RTLD_NOW | RTLD_LOCAL);
  void *c = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
  if (!b || !c) return -1;
  L->init = (void (*)(void *))dlsym(b, "llvm_blake3_hasher_init");
  L->init_keyed = (void (*)(void *, const uint8_t *))dlsym(b, "llvm_blake3_hasher_init_keyed");
  L->update = (void (*)(void *, const void *, size_t))dlsym(b, "llvm_blake3_hasher_update");
  L->finalize = (void (*)(const void *, uint8_t *, size_t))dlsym(b, "llvm_blake3_hasher_finalize");
  L->ctx_new = (void *(*)(void))dlsym(c, "EVP_CIPHER_CTX_new");
  L->ctx_free = (void (*)(void *))dlsym(c, "EVP_CIPHER_CTX_free");
  L->chacha = (const void *(*)(void))dlsym(c, "EVP_chacha20");
  L->enc_init = (int (*)(void *, const void *, void *, const uint8_t *, const uint8_t *))
      dlsym(c, "EVP_EncryptInit_ex");
  L->enc_update = (int (*)(void *, uint8_t *, int *, const uint8_t *, int))
      dlsym(c, "EVP_EncryptUpdate");
  return (L->init && L->init_keyed && L->update && L->finalize && L->ctx_new &&
          L->ctx_free && L->chacha && L->enc_init && L->enc_update) ? 0 : -1;
}

typedef struct {
  const simd_libs *L;
  uint8_t *refs, *ctext;
  const uint8_t *salt, *ptext, *cid_key;
  uint64_t total, chunk, b0, b1;
  int scalar_chacha;
  int rc;
} job;

static void *run(void *arg) {
  job *j = arg;
  const simd_libs *L = j->L;
  uint8_t *h = aligned_alloc(64, 4096); /* upstream blake3_hasher < 2 KiB */
  void *cx = L->ctx_new();
  uint8_t *tmp = j->ctext ? NULL : malloc(j->chunk);
  static const uint8_t iv[16] = {0}; /* LE32 counter 0 || 12-byte zero nonce */
  for (uint64_t b = j->b0; b < j->b1 && !j->rc; b++) {
    const uint64_t off = b * j->chunk;
    const uint64_t n = (j->total - off < j->chunk) ? j->total - off : j->chunk;
    uint8_t *ref = j->refs + 64 * b;
    uint8_t *ct = j->ctext ? j->ctext + off : tmp;
    L->init_keyed(h, j->salt); /* DEK: ref.go:152-161 */
    L->update(h, j->ptext + off, n);
    L->finalize(h, ref + 32, 32);
    int outl = 0; /* ctext: ref.go:137-144 */
    if (j->scalar_chacha) {
      static const uint8_t zero_nonce[12] = {0};
      oracle_chacha20_xor(ct, j->ptext + off, n, ref + 32, zero_nonce, 0);
    } else if (L->enc_init(cx, L->chacha(), NULL, ref + 32, iv) != 1 ||
               (n && L->enc_update(cx, ct, &outl, j->ptext + off, (int)n) != 1)) {
      j->rc = -1;
      break;
    }
    if (j->cid_key) /* CID: the store's BLAKE3-256 of the ctext */
      L->init_keyed(h, j->cid_key);
    else
      L->init(h);
    L->update(h, ct, n);
    L->finalize(h, ref, 32);
  }
  L->ctx_free(cx);
  free(tmp);
  free(h);
  return NULL;
}

static int post_batch(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                      const uint8_t *ptext, uint64_t total, uint64_t chunk,
                      const uint8_t *cid_key, int threads, int scalar_chacha) {
  static simd_libs L;
  static int loaded = 0;
  if (!loaded) loaded = load(&L) == 0 ? 1 : -1;
  if (loaded < 0) return -1;
  const uint64_t nb = (total + chunk - 1) / chunk;
  if (threads < 1) threads = 1;
  job *jobs = calloc((size_t)threads, sizeof(job));
  pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
  for (int t = 0; t < threads; t++) {
    jobs[t] = (job){&L, refs, ctext, salt, ptext, cid_key, total, chunk,
                    nb * (uint64_t)t / (uint64_t)threads,
                    nb * (uint64_t)(t + 1) / (uint64_t)threads, scalar_chacha, 0};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  free(jobs);
  free(th);
  return rc;
}

int oracle_post_batch_simd(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                           const uint8_t *ptext, uint64_t total, uint64_t chunk,
                           const uint8_t *cid_key, int threads) {
  return post_batch(refs, ctext, salt, ptext, total, chunk, cid_key, threads, 0);
}

int oracle_post_batch_gomix(uint8_t *refs, uint8_t *ctext, const uint8_t salt[32],
                            const uint8_t *ptext, uint64_t total, uint64_t chunk,
                            const uint8_t *cid_key, int threads) {
  return post_batch(refs, ctext, salt, ptext, total, chunk, cid_key, threads, 1);
}
