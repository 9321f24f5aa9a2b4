/* Throughput of the aggregation queue (f1) as its producers see it:
 * P threads submit Signature::verify requests (host memory, one 128-byte
 * triple each) as fast as the queue takes them; the callback counts verdicts
 * (all must be Ok).  One JSON line per run with requests/s, windows, the
 * wait-time percentiles and, for comparison, one host-pointer
 * coa_ed25519_verify_strict_many call over the same number of triples.
 * COA_QUEUE_SLOTS selects the windows in flight per GPU.
 *
 * Build (gcc, against the engine library; the run script does this):
 *   gcc -O2 -std=c11 -pthread -I include tools/queue_probe.c -o tools/queue_probe \
 *       -L xrpl-coa-prototype_amd/lib -lcoa_verify -Wl,-rpath,$PWD/xrpl-coa-prototype_amd/lib
 * usage: tools/queue_probe [signatures] [producers] [max_batch] [max_delay_us] [per_request]
 *        per_request > 1 submits groups through coa_queue_submit_verify_many. */
#define _POSIX_C_SOURCE 199309L
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "coa_verify.h"

#define NKEYS 8192

static uint8_t g_msgs[NKEYS * 32], g_pks[NKEYS * 32], g_sigs[NKEYS * 64];
static atomic_ulong g_done, g_bad;
static coa_queue* g_q;
static size_t g_per, g_group = 1;
static uint8_t* g_bm;  /* per-producer staging for groups */

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void cb(void* user, int status, const uint8_t* v, size_t n) {
  (void)user;
  size_t bad = status != COA_OK ? n : 0;
  for (size_t i = 0; status == COA_OK && i < n; i++) bad += v[i] != 0;
  if (bad) atomic_fetch_add(&g_bad, bad);
  atomic_fetch_add(&g_done, n);
}

static void* producer(void* arg) {
  const size_t id = (size_t)arg;
  if (g_group > 1) {  /* groups of g_group consecutive keys */
    uint8_t* m = g_bm + id * g_group * 128;
    uint8_t *p = m + g_group * 32, *sg = m + g_group * 64;
    for (size_t i = 0; i + g_group <= g_per; i += g_group) {
      for (size_t j = 0; j < g_group; j++) {
        const size_t k = (id * 7919 + i + j) % NKEYS;
        memcpy(m + 32 * j, g_msgs + 32 * k, 32);
        memcpy(p + 32 * j, g_pks + 32 * k, 32);
        memcpy(sg + 64 * j, g_sigs + 64 * k, 64);
      }
      if (coa_queue_submit_verify_many(g_q, m, p, sg, g_group, cb, NULL) != COA_OK) {
        atomic_fetch_add(&g_bad, g_group);
        atomic_fetch_add(&g_done, g_group);
      }
    }
    return NULL;
  }
  for (size_t i = 0; i < g_per; i++) {
    const size_t k = (id * 7919 + i) % NKEYS;
    if (coa_queue_submit_verify(g_q, g_msgs + 32 * k, g_pks + 32 * k, g_sigs + 64 * k, cb, NULL) != COA_OK) {
      atomic_fetch_add(&g_bad, 1);
      atomic_fetch_add(&g_done, 1);
    }
  }
  return NULL;
}

int main(int argc, char** argv) {
  const size_t total = argc > 1 ? strtoull(argv[1], NULL, 10) : 1u << 20;
  const size_t P = argc > 2 ? strtoull(argv[2], NULL, 10) : 8;
  const size_t max_batch = argc > 3 ? strtoull(argv[3], NULL, 10) : 65536;
  const unsigned delay = argc > 4 ? (unsigned)strtoul(argv[4], NULL, 10) : 200;
  g_group = argc > 5 ? strtoull(argv[5], NULL, 10) : 1;
  if (g_group < 1) g_group = 1;
  if (coa_init(1) != COA_OK) {
    fprintf(stderr, "coa_init: %s\n", coa_last_error());
    return 1;
  }
  uint8_t* seeds = malloc(NKEYS * 32);
  for (size_t i = 0; i < NKEYS * 32; i++) seeds[i] = (uint8_t)(i * 131 + 7);
  for (size_t i = 0; i < NKEYS * 32; i++) g_msgs[i] = (uint8_t)(i * 29 + 3);
  if (coa_ed25519_sign_many(seeds, g_msgs, 32, NKEYS, g_pks, g_sigs) != COA_OK) {
    fprintf(stderr, "sign: %s\n", coa_last_error());
    return 1;
  }
  g_per = total / P / g_group * g_group;
  const size_t n = g_per * P;
  g_bm = malloc(P * g_group * 128);
  g_q = coa_queue_create(max_batch, delay);
  pthread_t th[64];
  const double t0 = now_s();
  for (size_t p = 0; p < P; p++) pthread_create(&th[p], NULL, producer, (void*)p);
  for (size_t p = 0; p < P; p++) pthread_join(th[p], NULL);
  coa_queue_flush(g_q);
  const double deadline = now_s() + 60.0;
  while (atomic_load(&g_done) < n && now_s() < deadline) {
    struct timespec ts = {0, 20000};
    nanosleep(&ts, NULL);
  }
  const double el = now_s() - t0;
  coa_queue_metrics_t m;
  coa_queue_metrics(g_q, &m);
  coa_queue_destroy(g_q);
  /* the same triples through one host-pointer call */
  uint8_t *bm = malloc(n * 32), *bp = malloc(n * 32), *bs = malloc(n * 64), *out = malloc(n);
  for (size_t i = 0; i < n; i++) {
    const size_t k = i % NKEYS;
    memcpy(bm + 32 * i, g_msgs + 32 * k, 32);
    memcpy(bp + 32 * i, g_pks + 32 * k, 32);
    memcpy(bs + 64 * i, g_sigs + 64 * k, 64);
  }
  coa_ed25519_verify_strict_many(bm, 32, bp, bs, n, out);
  const double t1 = now_s();
  const int rc = coa_ed25519_verify_strict_many(bm, 32, bp, bs, n, out);
  const double el2 = now_s() - t1;
  size_t bad2 = 0;
  for (size_t i = 0; i < n; i++) bad2 += out[i] != 0;
  const char* slots = getenv("COA_QUEUE_SLOTS");
  printf("{\"signatures\": %zu, \"per_request\": %zu, \"producers\": %zu, \"max_batch\": %zu, \"max_delay_us\": %u, \"slots_per_gpu\": \"%s\", "
         "\"answered\": %lu, \"bad\": %lu, \"seconds\": %.4f, \"signatures_per_s\": %.1f, \"windows\": %llu, "
         "\"max_window\": %llu, \"max_in_flight\": %llu, \"wait_us_p50\": %.1f, \"wait_us_p99\": %.1f, "
         "\"one_call_host_pointers\": {\"rc\": %d, \"bad\": %zu, \"seconds\": %.4f, \"verify_per_s\": %.1f}}\n",
         n, g_group, P, max_batch, delay, slots ? slots : "default", (unsigned long)atomic_load(&g_done),
         (unsigned long)atomic_load(&g_bad), el, n / el, (unsigned long long)m.windows,
         (unsigned long long)m.max_window, (unsigned long long)m.max_in_flight, m.wait_us_p50, m.wait_us_p99, rc,
         bad2, el2, n / el2);
  return (atomic_load(&g_bad) || atomic_load(&g_done) < n || rc || bad2) ? 2 : 0;
}
