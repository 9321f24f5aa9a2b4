/*
 * queue_harness.c -- drives the aggregation queue (include/coa_verify.h,
 * coa_queue_*) the way the Rust VerifyService does (rust/crypto/src/service.rs):
 * several producer threads submit requests with a completion callback each,
 * and every callback checks its verdict bytes / digest against the golden
 * expectation it carries.  Built by tests/test_c_abi.py with
 * gcc -std=c11 -Wall -Wextra -Werror -pthread; run by tests/test_c_abi.py (no
 * GPU: every request must still be answered, with the engine error) and
 * tests/test_gpu_queue_harness.py (GPU: every verdict must match).
 *
 * usage: queue_harness <vectors.bin> <producers> <rounds> [max_batch] [max_delay_us]
 *
 * vectors.bin (written by test_c_abi.write_queue_vectors), little endian:
 *   u32 magic 0x51414F43, u32 n_verify, u32 n_batch, u32 n_digest
 *   n_verify x { msg[32] pk[32] sig[64] expect_u8 }        (0 = Ok, 1 = Err)
 *   n_batch  x { msg[32] u32 n expect_u8 n x { pk[32] sig[64] } }
 *   n_digest x { u32 len data[len] digest[32] }
 *
 * Per producer and round: the verify vectors go one request each on even
 * (producer + round) and in coa_queue_submit_verify_many groups of 8
 * otherwise; then every vote batch, then every digest.  `submitted` /
 * `answered` count vectors (a group of 8 counts 8).  The last stdout line is
 * one JSON object; exit status 0 only when every vector was answered once,
 * with status COA_OK and the expected bytes, and no window failed.
 */
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#include "coa_verify.h"

#define GROUP 8

typedef struct {
  uint8_t msg[32], pk[32], sig[64];
  uint8_t expect;
} verify_vec;

typedef struct {
  uint8_t msg[32];
  uint32_t n;
  uint8_t expect;
  uint8_t* pks;  /* n * 32 */
  uint8_t* sigs; /* n * 64 */
} batch_vec;

typedef struct {
  uint32_t len;
  uint8_t* data;
  uint8_t digest[32];
} digest_vec;

static verify_vec* g_v;
static batch_vec* g_b;
static digest_vec* g_d;
static uint32_t g_nv, g_nb, g_nd;
static coa_queue* g_q;
static int g_rounds;

static atomic_ullong g_submitted, g_answered, g_bad_status, g_wrong, g_callbacks, g_submit_err;

/* One request in flight: what its callback must see. */
typedef struct {
  size_t n_expect;     /* verdict bytes expected (or 32 for a digest) */
  uint8_t expect[32];  /* expected verdict bytes / digest */
  uint64_t weight;     /* vectors this request answers */
} request;

static void on_verdict(void* user, int status, const uint8_t* verdicts, size_t n) {
  request* r = (request*)user;
  atomic_fetch_add(&g_callbacks, 1);
  if (status != COA_OK) {
    atomic_fetch_add(&g_bad_status, r->weight);
  } else if (n != r->n_expect || !verdicts || memcmp(verdicts, r->expect, n) != 0) {
    atomic_fetch_add(&g_wrong, r->weight);
  }
  atomic_fetch_add(&g_answered, r->weight);
  free(r);
}

static request* new_request(size_t n_expect, const uint8_t* expect, uint64_t weight) {
  request* r = (request*)calloc(1, sizeof(request));
  if (!r) {
    fprintf(stderr, "out of memory\n");
    exit(2);
  }
  r->n_expect = n_expect;
  memcpy(r->expect, expect, n_expect);
  r->weight = weight;
  return r;
}

/* A submission the queue refused never gets a callback: answer it here. */
static void submit_result(int rc, request* r) {
  atomic_fetch_add(&g_submitted, r->weight);
  if (rc != COA_OK) {
    atomic_fetch_add(&g_submit_err, 1);
    atomic_fetch_add(&g_bad_status, r->weight);
    atomic_fetch_add(&g_answered, r->weight);
    free(r);
  }
}

static void* producer(void* arg) {
  const int p = (int)(intptr_t)arg;
  uint8_t gm[GROUP * 32], gp[GROUP * 32], gs[GROUP * 64], ge[GROUP];
  for (int round = 0; round < g_rounds; round++) {
    if ((p + round) % 2 == 0) {
      for (uint32_t i = 0; i < g_nv; i++) {
        const verify_vec* v = &g_v[i];
        request* r = new_request(1, &v->expect, 1);
        submit_result(coa_queue_submit_verify(g_q, v->msg, v->pk, v->sig, on_verdict, r), r);
      }
    } else {
      for (uint32_t i = 0; i < g_nv; i += GROUP) {
        const uint32_t k = g_nv - i < GROUP ? g_nv - i : GROUP;
        for (uint32_t j = 0; j < k; j++) {
          memcpy(gm + 32 * j, g_v[i + j].msg, 32);
          memcpy(gp + 32 * j, g_v[i + j].pk, 32);
          memcpy(gs + 64 * j, g_v[i + j].sig, 64);
          ge[j] = g_v[i + j].expect;
        }
        request* r = new_request(k, ge, k);
        submit_result(coa_queue_submit_verify_many(g_q, gm, gp, gs, k, on_verdict, r), r);
      }
    }
    for (uint32_t i = 0; i < g_nb; i++) {
      const batch_vec* b = &g_b[i];
      request* r = new_request(1, &b->expect, 1);
      submit_result(coa_queue_submit_batch(g_q, b->msg, b->pks, b->sigs, b->n, on_verdict, r), r);
    }
    for (uint32_t i = 0; i < g_nd; i++) {
      const digest_vec* d = &g_d[i];
      request* r = new_request(32, d->digest, 1);
      submit_result(coa_queue_submit_digest(g_q, d->data, d->len, on_verdict, r), r);
    }
  }
  return NULL;
}

/* ------------------------------------------------------------ vector file */
static const uint8_t* g_buf;
static size_t g_len, g_pos;

static const uint8_t* take(size_t n) {
  if (g_len - g_pos < n) {
    fprintf(stderr, "vector file truncated at %zu\n", g_pos);
    exit(2);
  }
  const uint8_t* p = g_buf + g_pos;
  g_pos += n;
  return p;
}

static uint32_t take_u32(void) {
  const uint8_t* p = take(4);
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

static void load_vectors(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    perror(path);
    exit(2);
  }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* buf = (uint8_t*)malloc(sz > 0 ? (size_t)sz : 1);
  if (!buf || fread(buf, 1, (size_t)sz, f) != (size_t)sz) {
    fprintf(stderr, "cannot read %s\n", path);
    exit(2);
  }
  fclose(f);
  g_buf = buf;
  g_len = (size_t)sz;
  if (take_u32() != 0x51414F43u) {
    fprintf(stderr, "bad magic\n");
    exit(2);
  }
  g_nv = take_u32();
  g_nb = take_u32();
  g_nd = take_u32();
  g_v = (verify_vec*)calloc(g_nv + 1, sizeof(verify_vec));
  g_b = (batch_vec*)calloc(g_nb + 1, sizeof(batch_vec));
  g_d = (digest_vec*)calloc(g_nd + 1, sizeof(digest_vec));
  for (uint32_t i = 0; i < g_nv; i++) {
    memcpy(g_v[i].msg, take(32), 32);
    memcpy(g_v[i].pk, take(32), 32);
    memcpy(g_v[i].sig, take(64), 64);
    g_v[i].expect = *take(1);
  }
  for (uint32_t i = 0; i < g_nb; i++) {
    batch_vec* b = &g_b[i];
    memcpy(b->msg, take(32), 32);
    b->n = take_u32();
    b->expect = *take(1);
    b->pks = (uint8_t*)malloc(32 * (size_t)b->n + 1);
    b->sigs = (uint8_t*)malloc(64 * (size_t)b->n + 1);
    for (uint32_t j = 0; j < b->n; j++) {
      memcpy(b->pks + 32 * (size_t)j, take(32), 32);
      memcpy(b->sigs + 64 * (size_t)j, take(64), 64);
    }
  }
  for (uint32_t i = 0; i < g_nd; i++) {
    digest_vec* d = &g_d[i];
    d->len = take_u32();
    d->data = (uint8_t*)malloc(d->len + 1);
    memcpy(d->data, take(d->len), d->len);
    memcpy(d->digest, take(32), 32);
  }
  if (g_pos != g_len) {
    fprintf(stderr, "%zu trailing bytes in vector file\n", g_len - g_pos);
    exit(2);
  }
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s vectors.bin producers rounds [max_batch] [max_delay_us]\n", argv[0]);
    return 2;
  }
  load_vectors(argv[1]);
  const int producers = atoi(argv[2]);
  g_rounds = atoi(argv[3]);
  const size_t max_batch = argc > 4 ? (size_t)strtoull(argv[4], NULL, 10) : 4096;
  const uint32_t max_delay = argc > 5 ? (uint32_t)strtoul(argv[5], NULL, 10) : 500;
  if (producers < 1 || producers > 256 || g_rounds < 1) {
    fprintf(stderr, "producers in 1..256, rounds >= 1\n");
    return 2;
  }

  g_q = coa_queue_create(max_batch, max_delay);
  if (!g_q) {
    fprintf(stderr, "coa_queue_create failed: %s\n", coa_last_error());
    return 2;
  }
  const double t0 = now_s();
  pthread_t th[256];
  for (int p = 0; p < producers; p++) pthread_create(&th[p], NULL, producer, (void*)(intptr_t)p);
  for (int p = 0; p < producers; p++) pthread_join(th[p], NULL);
  coa_queue_flush(g_q);
  /* the flush returns once every window is answered; allow the last
   * callbacks a bounded moment to finish their counters */
  const double deadline = now_s() + 60.0;
  while (atomic_load(&g_answered) < atomic_load(&g_submitted) && now_s() < deadline) {
    struct timespec ms = {0, 1000000};
    nanosleep(&ms, NULL);
  }
  const double wall = now_s() - t0;

  coa_queue_metrics_t m;
  memset(&m, 0, sizeof m);
  coa_queue_metrics(g_q, &m);
  coa_queue_destroy(g_q);

  const unsigned long long sub = atomic_load(&g_submitted), ans = atomic_load(&g_answered);
  const unsigned long long bad = atomic_load(&g_bad_status), wrong = atomic_load(&g_wrong);
  printf("{\"submitted\": %llu, \"answered\": %llu, \"bad_status\": %llu, \"wrong\": %llu, "
         "\"callbacks\": %llu, \"submit_errors\": %llu, \"requests\": %llu, \"windows\": %llu, "
         "\"max_window\": %llu, \"max_in_flight\": %llu, \"retried_windows\": %llu, "
         "\"recovered_windows\": %llu, \"failed_windows\": %llu, \"wait_us_p50\": %.1f, "
         "\"wait_us_p99\": %.1f, \"wall_s\": %.3f}\n",
         sub, ans, bad, wrong, (unsigned long long)atomic_load(&g_callbacks),
         (unsigned long long)atomic_load(&g_submit_err), (unsigned long long)m.requests,
         (unsigned long long)m.windows, (unsigned long long)m.max_window, (unsigned long long)m.max_in_flight,
         (unsigned long long)m.retried_windows, (unsigned long long)m.recovered_windows,
         (unsigned long long)m.failed_windows, m.wait_us_p50, m.wait_us_p99, wall);
  fflush(stdout);
  const int ok = ans == sub && bad == 0 && wrong == 0 && m.failed_windows == 0;
  return ok ? 0 : 1;
}
