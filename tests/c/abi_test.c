/*
 * abi_test.c -- a plain C consumer of include/glfsx.h (no ctypes, no torch):
 * what a cgo binding sees.  Built and run by tests/test_c_abi.py:
 *
 *   gcc -std=c11 -Wall -Wextra -Werror -Iinclude -Ioracle tests/c/abi_test.c \
 *       -Lglfs_amd -lglfsx -Loracle -loracle -lpthread -o abi_test
 *   ./abi_test layout     (no GPU needed: struct layout, status codes,
 *                          panics before any device work, no CPU fallback)
 *   ./abi_test gpu        (the Writer end to end against the oracle)
 *
 * The oracle (oracle/liboracle.so) is the checker only (test
 * infrastructure); every compute call goes through libglfsx.so.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "glfsx.h"
#include "oracle.h"

static int failures = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      failures++;                                                        \
    }                                                                    \
  } while (0)

/* ------------------------------------------------------------ post log */
typedef struct {
  int kind;
  uint8_t ref[64];
  uint64_t len;
  uint64_t sum; /* FNV-1a of the ctext */
} post_rec;

typedef struct {
  post_rec *v;
  size_t n, cap;
  size_t fail_at; /* 1-based Post that fails; 0 = never */
} post_log;

static uint64_t fnv(const uint8_t *p, uint64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

static int log_post(post_log *L, int kind, const uint8_t *ref, const void *ct,
                    uint64_t len) {
  if (L->n == L->cap) {
    L->cap = L->cap ? 2 * L->cap : 64;
    L->v = realloc(L->v, L->cap * sizeof(post_rec));
  }
  post_rec *r = &L->v[L->n++];
  r->kind = kind;
  memcpy(r->ref, ref, 64);
  r->len = len;
  r->sum = fnv((const uint8_t *)ct, len);
  return (L->fail_at && L->n == L->fail_at) ? 7 : 0;
}

/* the store.Post a cgo binding passes in (glfsx_post_fn) */
static int gpu_sink(void *ctx, int kind, const uint8_t *ref, const void *ctext,
                    uint64_t len) {
  return log_post((post_log *)ctx, kind, ref, ctext, len);
}
static int oracle_sink(void *ctx, int kind, const uint8_t ref[64],
                       const uint8_t *ctext, uint64_t len) {
  return log_post((post_log *)ctx, kind, ref, ctext, len);
}

static int same_logs(const post_log *a, const post_log *b) {
  if (a->n != b->n) return 0;
  for (size_t i = 0; i < a->n; i++)
    if (a->v[i].kind != b->v[i].kind || memcmp(a->v[i].ref, b->v[i].ref, 64) ||
        a->v[i].len != b->v[i].len || a->v[i].sum != b->v[i].sum)
      return 0;
  return 1;
}

/* ------------------------------------------------------- layout (no GPU) */
static void test_layout(void) {
  CHECK(sizeof(glfsx_root) == 80);
  CHECK(offsetof(glfsx_root, ref) == 0);
  CHECK(offsetof(glfsx_root, size) == 64);
  CHECK(offsetof(glfsx_root, block_size) == 72);
  CHECK(GLFSX_REF_SIZE == 64 && GLFSX_CID_SIZE == 32 && GLFSX_DEK_SIZE == 32);
  CHECK(GLFSX_MIN_BLOCK_SIZE == 128);
  CHECK(GLFSX_OK == 0 && GLFSX_E_BLOCKSIZE_GT_MAX == -1 && GLFSX_E_BLOCKSIZE_LT_MIN == -2 &&
        GLFSX_E_STORE == -3 && GLFSX_E_DEVICE == -4 && GLFSX_E_ARG == -5);
  /* blob.go:90-95 panics come back before any device work */
  int err = 0;
  glfsx_writer *w = glfsx_writer_new(2u << 20, 1u << 20, NULL, NULL, NULL, NULL, &err);
  CHECK(w == NULL && err == GLFSX_E_BLOCKSIZE_GT_MAX);
  CHECK(strstr(glfsx_last_error(), "blockSize 2097152 > maxSize 1048576") != NULL);
  w = glfsx_writer_new(100, 1u << 20, NULL, NULL, NULL, NULL, &err);
  CHECK(w == NULL && err == GLFSX_E_BLOCKSIZE_LT_MIN);
  CHECK(strstr(glfsx_last_error(), "blockSize cannot be < 128") != NULL);
  /* blob.go:256-268: pure shape math */
  CHECK(glfsx_depth(0, 1024) == 0 && glfsx_depth(1024, 1024) == 0 &&
        glfsx_depth(1025, 1024) == 1 && glfsx_depth(16 * 1024 + 1, 1024) == 2);
  CHECK(glfsx_branching_factor(1u << 20) == 16384);
}

static void test_no_fallback(void) {
  uint8_t out[32], salt[32] = {0};
  CHECK(glfsx_derive_key(out, 32, salt, "raw", 3) == GLFSX_E_DEVICE);
  CHECK(strstr(glfsx_last_error(), "no CPU") != NULL);
}

/* -------------------------------------------------------------- GPU part */
static uint8_t *fill(uint64_t n, uint64_t seed) {
  uint8_t *p = malloc(n ? n : 1); /* pageable, as Go memory is */
  oracle_fill_splitmix(p, 0, n, seed);
  return p;
}

/* the reference Writer (oracle) over `pieces`: index of the Write that
 * failed, n_pieces for Finish, -1 for none */
static int oracle_run(const uint8_t *data, const uint64_t *pieces, int np,
                      uint64_t bs, post_log *L, uint8_t root[64]) {
  int err = 0;
  oracle_writer *w = oracle_writer_new(bs, bs, NULL, NULL, oracle_sink, L, &err);
  uint64_t off = 0;
  int at = -1;
  for (int i = 0; i < np && at < 0; i++) {
    if (oracle_writer_write(w, data + off, pieces[i])) at = i;
    off += pieces[i];
  }
  uint64_t size, b;
  if (at < 0 && oracle_writer_finish(w, root, &size, &b)) at = np;
  oracle_writer_free(w);
  return at;
}

static int gpu_run(const uint8_t *data, const uint64_t *pieces, int np, uint64_t bs,
                   int strict, post_log *L, glfsx_root *root) {
  int err = 0;
  glfsx_writer *w = glfsx_writer_new(bs, bs, NULL, NULL, gpu_sink, L, &err);
  CHECK(w != NULL && err == 0);
  if (!w) return -2;
  CHECK(glfsx_writer_set_strict(w, strict) == 0);
  uint64_t off = 0;
  int at = -1;
  for (int i = 0; i < np && at < 0; i++) {
    int rc = glfsx_writer_write(w, data + off, pieces[i]);
    if (rc) {
      CHECK(rc == GLFSX_E_STORE);
      CHECK(strstr(glfsx_writer_error(w), "code 7") != NULL);
      at = i;
    }
    off += pieces[i];
  }
  if (at < 0) {
    int rc = glfsx_writer_finish(w, root);
    if (rc) {
      CHECK(rc == GLFSX_E_STORE);
      at = np;
    }
  }
  glfsx_writer_free(w);
  return at;
}

static void test_writer_vs_oracle(void) {
  const uint64_t bs = 1024; /* bf = 16: index nodes interleave with data */
  const uint64_t size = 300 * 1024 + 77;
  uint8_t *data = fill(size, 5);
  uint64_t pieces[] = {1, 1023, 5000, 64 * 1024, 7, 100 * 1024, 0};
  pieces[6] = size - (1 + 1023 + 5000 + 64 * 1024 + 7 + 100 * 1024);
  post_log a = {0}, b = {0};
  uint8_t want[64];
  glfsx_root got;
  CHECK(oracle_run(data, pieces, 7, bs, &a, want) == -1);
  CHECK(gpu_run(data, pieces, 7, bs, 0, &b, &got) == -1);
  CHECK(memcmp(got.ref, want, 64) == 0);
  CHECK(got.size == size && got.block_size == bs);
  CHECK(same_logs(&a, &b));
  /* strict error timing: the same Write fails after the same Posts */
  for (size_t k = 1; k < a.n; k += 37) {
    post_log c = {0, 0, 0, k}, d = {0, 0, 0, k};
    uint8_t r2[64];
    glfsx_root g2;
    int wa = oracle_run(data, pieces, 7, bs, &c, r2);
    int wb = gpu_run(data, pieces, 7, bs, 1, &d, &g2);
    CHECK(wa == wb);
    CHECK(same_logs(&c, &d));
    free(c.v);
    free(d.v);
  }
  /* glfsx_create == the same root */
  post_log e = {0};
  glfsx_root g3;
  CHECK(glfsx_create(bs, bs, NULL, NULL, data, size, gpu_sink, &e, &g3) == 0);
  CHECK(memcmp(g3.ref, want, 64) == 0 && same_logs(&a, &e));
  free(a.v);
  free(b.v);
  free(e.v);
  free(data);
}

static void test_primitives(void) {
  uint8_t salt[32], out[32], want[32];
  for (int i = 0; i < 32; i++) salt[i] = (uint8_t)(3 * i + 1);
  uint8_t *data = fill(5000, 9);
  CHECK(glfsx_derive_key(out, 32, salt, data, 5000) == 0);
  oracle_derive_key(want, salt, data, 5000);
  CHECK(memcmp(out, want, 32) == 0);
  uint8_t ref[64], wref[64];
  uint8_t *ct = malloc(5000), *wct = malloc(5000);
  CHECK(glfsx_post(salt, data, 5000, ct, ref, NULL) == 0);
  oracle_post(wref, wct, salt, data, 5000, NULL);
  CHECK(memcmp(ref, wref, 64) == 0 && memcmp(ct, wct, 5000) == 0);
  uint8_t *pt = malloc(5000);
  CHECK(glfsx_chacha20_xor(ref + 32, ct, pt, 5000) == 0);
  CHECK(memcmp(pt, data, 5000) == 0);
  free(data);
  free(ct);
  free(wct);
  free(pt);
}

/* a writer created on one thread, written on a second, finished on a third */
typedef struct {
  glfsx_writer *w;
  const uint8_t *p;
  uint64_t n;
  glfsx_root *root;
  int rc;
} thr_job;
static void *thr_new(void *x) {
  thr_job *j = x;
  int err;
  j->w = glfsx_writer_new(4096, 4096, NULL, NULL, NULL, NULL, &err);
  j->rc = err;
  return NULL;
}
static void *thr_write(void *x) {
  thr_job *j = x;
  j->rc = glfsx_writer_write(j->w, j->p, j->n);
  return NULL;
}
static void *thr_finish(void *x) {
  thr_job *j = x;
  j->rc = glfsx_writer_finish(j->w, j->root);
  glfsx_writer_free(j->w);
  return NULL;
}
static void test_threads(void) {
  const uint64_t size = 1000 * 4096 + 3;
  uint8_t *data = fill(size, 11);
  glfsx_root root;
  thr_job j = {0};
  j.root = &root;
  pthread_t t;
  pthread_create(&t, NULL, thr_new, &j);
  pthread_join(t, NULL);
  CHECK(j.rc == 0 && j.w);
  j.p = data;
  j.n = size / 2;
  pthread_create(&t, NULL, thr_write, &j);
  pthread_join(t, NULL);
  CHECK(j.rc == 0);
  j.p = data + size / 2;
  j.n = size - size / 2;
  pthread_create(&t, NULL, thr_write, &j);
  pthread_join(t, NULL);
  CHECK(j.rc == 0);
  pthread_create(&t, NULL, thr_finish, &j);
  pthread_join(t, NULL);
  CHECK(j.rc == 0);
  post_log a = {0};
  uint8_t want[64];
  uint64_t one[1] = {size};
  oracle_run(data, one, 1, 4096, &a, want);
  CHECK(memcmp(root.ref, want, 64) == 0);
  free(a.v);
  free(data);
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "layout";
  test_layout();
  if (strcmp(mode, "layout") == 0) {
    if (glfsx_device_count() == 0) test_no_fallback();
  } else {
    CHECK(glfsx_device_count() > 0);
    CHECK(glfsx_set_device(0) == 0);
    test_primitives();
    test_writer_vs_oracle();
    test_threads();
  }
  printf("abi_test %s: %s (%d failures)\n", mode, failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
