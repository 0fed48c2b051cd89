/* Concurrent per-call drop-in throughput (bench.py postblob_concurrency):
 * `threads` plain C threads, each posting its own `len`-byte blobs one call
 * at a time through glfsx_create as one glfs.PostBlob does (machine.go:64:
 * one Writer per blob, bs 2 MiB, the blob type salt, a counting sink that
 * receives every Post).  Measurement harness only -- not part of the
 * library; built by __graft_entry__.build() into tools/libpostbench.so.
 * The library's entry points come in as function pointers (the caller's
 * handle on libglfsx.so, or on a build variant for an A/B in one process).
 *
 * postbench_run: out[0] = calls completed, out[1] = wall seconds from the
 * first call to the last return (all threads released together), out[2] /
 * out[3] / out[4] = p50 / p90 / p99 per-call latency in microseconds.
 * Returns 0, or the first failing call's status. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/glfsx.h"

typedef int (*create_fn)(uint64_t, uint64_t, const uint8_t *, const uint8_t *, const void *,
                         uint64_t, glfsx_post_fn, void *, glfsx_root *);
typedef int (*set_device_fn)(int);
static create_fn create_p;
static set_device_fn set_device_p;
static glfsx_post_fn sink_p;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct {
  int id, dev, calls, rc;
  uint64_t len;
  const uint8_t *salt;
  double *lat;
  pthread_barrier_t *go;
  double t_end;
} job;

static void *worker(void *arg) {
  job *j = (job *)arg;
  uint8_t *data = (uint8_t *)malloc(j->len + 8);
  for (uint64_t i = 0; i < j->len + 8; i++) data[i] = (uint8_t)(i * 131 + 7 * j->id);
  uint64_t counts[2] = {0, 0};
  glfsx_root root;
  if (set_device_p(j->dev)) j->rc = -1;
  for (int i = 0; i < 3 && !j->rc; i++)  /* warm the thread's context */
    j->rc = create_p(2u << 20, 2u << 20, j->salt, NULL, data, j->len, sink_p, counts, &root);
  pthread_barrier_wait(j->go);
  for (int i = 0; i < j->calls && !j->rc; i++) {
    if (j->len >= 8) memcpy(data, &i, sizeof i); /* a distinct blob per call */
    const double t = now();
    j->rc = create_p(2u << 20, 2u << 20, j->salt, NULL, data, j->len, sink_p, counts, &root);
    j->lat[i] = now() - t;
  }
  j->t_end = now();
  free(data);
  return NULL;
}

static int cmp(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

int postbench_run(void *create, void *set_device, void *sink, int threads, uint64_t len,
                  int calls, const uint8_t *salt, int dev, double out[5]) {
  if (threads < 1 || calls < 1 || !create || !set_device || !sink) return -1;
  create_p = (create_fn)create;
  set_device_p = (set_device_fn)set_device;
  sink_p = (glfsx_post_fn)sink;
  pthread_t *th = (pthread_t *)calloc(threads, sizeof *th);
  job *jobs = (job *)calloc(threads, sizeof *jobs);
  double *lat = (double *)calloc((size_t)threads * calls, sizeof *lat);
  pthread_barrier_t go;
  pthread_barrier_init(&go, NULL, threads + 1);
  for (int k = 0; k < threads; k++) {
    jobs[k] = (job){k, dev, calls, 0, len, salt, lat + (size_t)k * calls, &go, 0};
    pthread_create(&th[k], NULL, worker, &jobs[k]);
  }
  pthread_barrier_wait(&go);
  const double t0 = now();
  double t1 = t0;
  int rc = 0;
  for (int k = 0; k < threads; k++) {
    pthread_join(th[k], NULL);
    if (jobs[k].rc && !rc) rc = jobs[k].rc;
    if (jobs[k].t_end > t1) t1 = jobs[k].t_end;
  }
  pthread_barrier_destroy(&go);
  if (!rc) {
    const size_t n = (size_t)threads * calls;
    qsort(lat, n, sizeof *lat, cmp);
    out[0] = (double)n;
    out[1] = t1 - t0;
    out[2] = lat[n / 2] * 1e6;
    out[3] = lat[n * 9 / 10] * 1e6;
    out[4] = lat[n * 99 / 100] * 1e6;
  }
  free(lat);
  free(jobs);
  free(th);
  return rc;
}
