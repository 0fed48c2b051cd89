/* Per-call latency and concurrent throughput of the drop-in's one-blob call
 * (a Go glfs.PostBlob is one Writer: glfsx_create with a store sink), driven
 * from plain C threads (no interpreter lock between calls).
 *   gcc -O2 -o gpurun_out/latency scripts/latency.c -Iinclude \
 *       -Lglfs_amd -lglfsx -Wl,-rpath,$PWD/glfs_amd -lpthread
 *   gpurun_out/latency [threads] [calls]
 * Prints one JSON line: per size, single-thread p50/p90 (us) and calls/s with
 * 1..threads threads. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "glfsx.h"

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static uint8_t salt[32];
static const uint64_t kBs = 2u << 20;

typedef struct {
  uint64_t size;
  int calls;
  double secs;
  int rc;
} job;

static int one(const uint8_t *data, uint64_t size) {
  uint64_t counts[2] = {0, 0};
  glfsx_root root;
  return glfsx_create(kBs, kBs, salt, NULL, data, size, glfsx_sink_count, counts, &root);
}

static void *run(void *arg) {
  job *j = arg;
  uint8_t *data = malloc(j->size + 1);
  for (uint64_t i = 0; i < j->size; i++) data[i] = (uint8_t)(i * 131 + 7);
  if (glfsx_set_device(0)) j->rc = -1;
  for (int i = 0; i < 5 && !j->rc; i++) j->rc = one(data, j->size);
  const double t0 = now();
  for (int i = 0; i < j->calls && !j->rc; i++) j->rc = one(data, j->size);
  j->secs = now() - t0;
  free(data);
  return NULL;
}

static int cmp(const void *a, const void *b) {
  const double x = *(const double *)a, y = *(const double *)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
  const int tmax = argc > 1 ? atoi(argv[1]) : 16;
  const int calls = argc > 2 ? atoi(argv[2]) : 400;
  for (int i = 0; i < 32; i++) salt[i] = (uint8_t)(3 * i + 1);
  const uint64_t sizes[] = {0, 9, 4096, 65536, 1u << 20, 2u << 20, 3u << 20};
  printf("{");
  for (size_t s = 0; s < sizeof sizes / sizeof sizes[0]; s++) {
    const uint64_t size = sizes[s];
    uint8_t *data = malloc(size + 1);
    memset(data, 0x5a, size + 1);
    double *ts = malloc(sizeof(double) * calls);
    for (int i = 0; i < 10; i++)
      if (one(data, size)) {
        fprintf(stderr, "glfsx_create: %s\n", glfsx_last_error());
        return 1;
      }
    for (int i = 0; i < calls; i++) {
      const double t = now();
      one(data, size);
      ts[i] = now() - t;
    }
    qsort(ts, calls, sizeof(double), cmp);
    printf("%s\"%llu\": {\"p50_us\": %.1f, \"p90_us\": %.1f", s ? ", " : "",
           (unsigned long long)size, ts[calls / 2] * 1e6, ts[calls * 9 / 10] * 1e6);
    for (int t = 1; t <= tmax; t *= 2) {
      pthread_t th[64];
      job jobs[64];
      for (int k = 0; k < t; k++) {
        jobs[k] = (job){size, calls, 0, 0};
        pthread_create(&th[k], NULL, run, &jobs[k]);
      }
      double worst = 0;
      for (int k = 0; k < t; k++) {
        pthread_join(th[k], NULL);
        if (jobs[k].rc) {
          fprintf(stderr, "thread: %d\n", jobs[k].rc);
          return 1;
        }
        if (jobs[k].secs > worst) worst = jobs[k].secs;
      }
      printf(", \"calls_per_s_%d\": %.0f", t, t * (double)calls / worst);
    }
    printf("}");
    fflush(stdout);
    free(ts);
    free(data);
  }
  printf("}\n");
  return 0;
}
