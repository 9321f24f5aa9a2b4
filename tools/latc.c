/* Latency of the drop-in's one-item entry points as a compiled caller sees
 * them: the Rust crate calls coa_certificate_verify / coa_ed25519_verify_strict
 * through its extern "C" binding (rust/crypto/src/coa_ffi.rs), with no
 * per-call argument marshalling.  bench.py times the same calls through the
 * Python test binding (ctypes + numpy conversions) as well; this loop takes
 * that binding out of the clock.  Each sample is one blocking call: host
 * pointers in, verdict out.
 *
 * Built by xrpl-coa-prototype_amd/build.py into lib/liblatc.so (gcc, linked
 * against libcoa_verify.so).  Measurement infrastructure only. */
#define _POSIX_C_SOURCE 200809L
#include <stddef.h>
#include <stdint.h>
#include <time.h>

#include "coa_verify.h"

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec * 1e6 + (double)t.tv_nsec * 1e-3;
}

/* `samples` calls of coa_certificate_verify on one certificate; per-call
 * microseconds into out_us.  Returns 0, or the first non-zero result. */
int latc_certificate(const uint8_t* header_data, size_t header_len, const uint8_t* id, const uint8_t* origin,
                     const uint8_t* header_sig, uint64_t round, const uint8_t* vote_pks, const uint8_t* vote_sigs,
                     size_t n_votes, int samples, double* out_us) {
  for (int i = 0; i < samples; i++) {
    const double t0 = now_us();
    const int rc = coa_certificate_verify(header_data, header_len, id, origin, header_sig, round, vote_pks, vote_sigs,
                                          n_votes, 0);
    out_us[i] = now_us() - t0;
    if (rc != 0) return rc;
  }
  return 0;
}

/* `samples` calls of coa_ed25519_verify_strict cycling over n triples
 * (32-byte messages); per-call microseconds into out_us. */
int latc_verify(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, int n, int samples, double* out_us) {
  for (int i = 0; i < samples; i++) {
    const int j = i % n;
    const double t0 = now_us();
    const int rc = coa_ed25519_verify_strict(msgs + 32 * j, pks + 32 * j, sigs + 64 * j);
    out_us[i] = now_us() - t0;
    if (rc != 0) return rc;
  }
  return 0;
}

/* ------------------------------------------------------------------------
 * Paced arrivals through the aggregation queue (coa_queue_*): request i is
 * due arrive_s[i] seconds after the start; this thread sleeps until it is due
 * and submits it (a late request goes at once: its latency is measured from
 * the SCHEDULED arrival, so a producer or queue that falls behind shows up as
 * latency, not as a quietly lower rate).  kind[i]:
 *   0  Signature::verify of triple item[i] (vmsgs / vpks / vsigs)
 *   1  Certificate::verify of certificate item[i] (c_* arrays: header bytes
 *      with c_hoff offsets, ids, origins, header signatures, rounds, votes
 *      with c_voff offsets)
 *   2  Sha512 digest of message item[i] (d_data with d_off offsets)
 * Expected answers: v_expect[item] verdict byte, c_expect[item] status byte,
 * d_expect[32 * item] digest.  lat_us[i] = callback time - scheduled arrival.
 * Returns the number of wrong or failed answers (>= 0); queue metrics into
 * *m, wall time from the first arrival to the last answer into *elapsed_s. */
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  double due_us;
  double* out;
  const uint8_t* expect;
  size_t n_expect;
  atomic_int* wrong;
} PacedReq;

static double g_paced_t0;

static void paced_cb(void* user, int status, const uint8_t* v, size_t n) {
  PacedReq* r = (PacedReq*)user;
  *r->out = now_us() - g_paced_t0 - r->due_us;
  if (status != COA_OK || n != r->n_expect || memcmp(v, r->expect, n) != 0) atomic_fetch_add(r->wrong, 1);
}

static void sleep_until_us(double t_us) {
  for (;;) {
    const double left = t_us - (now_us() - g_paced_t0);
    if (left <= 0) return;
    if (left > 300.0) {
      struct timespec ts = {0, (long)((left - 150.0) * 1e3)};
      nanosleep(&ts, NULL);
    }
  }
}

int latc_paced(size_t max_batch, unsigned max_delay_us, size_t n, const double* arrive_s, const int* kind,
               const uint32_t* item, const uint8_t* vmsgs, const uint8_t* vpks, const uint8_t* vsigs,
               const uint8_t* v_expect, const uint8_t* c_hdata, const uint64_t* c_hoff, const uint8_t* c_ids,
               const uint8_t* c_origins, const uint8_t* c_hsigs, const uint64_t* c_rounds, const uint8_t* c_vpks,
               const uint8_t* c_vsigs, const uint64_t* c_voff, const uint8_t* c_expect, const uint8_t* d_data,
               const uint64_t* d_off, const uint8_t* d_expect, double* lat_us, double* elapsed_s,
               coa_queue_metrics_t* m) {
  coa_queue* q = coa_queue_create(max_batch, max_delay_us);
  if (!q) return -1;
  PacedReq* reqs = (PacedReq*)calloc(n ? n : 1, sizeof(PacedReq));
  atomic_int wrong = 0;
  /* warm-up, untimed: the schedule's first requests (up to 64, submitted at
   * once, answers checked), then the metrics are reset -- a node creates its
   * queue once, so the measured run starts from a queue that has already
   * answered, as tools/latc.c latc_stream_certificates does */
  {
    const size_t nw = n < 64 ? n : 64;
    double sink[64];
    g_paced_t0 = now_us();
    for (size_t i = 0; i < nw; i++) {
      PacedReq* r = &reqs[i];
      r->due_us = 0;
      r->out = &sink[i];
      r->wrong = &wrong;
      const size_t k = item[i];
      int rc;
      if (kind[i] == 0) {
        r->expect = v_expect + k;
        r->n_expect = 1;
        rc = coa_queue_submit_verify(q, vmsgs + 32 * k, vpks + 32 * k, vsigs + 64 * k, paced_cb, r);
      } else if (kind[i] == 1) {
        r->expect = c_expect + k;
        r->n_expect = 1;
        rc = coa_queue_submit_certificate(q, c_hdata + c_hoff[k], c_hoff[k + 1] - c_hoff[k], c_ids + 32 * k,
                                          c_origins + 32 * k, c_hsigs + 64 * k, c_rounds[k], c_vpks + 32 * c_voff[k],
                                          c_vsigs + 64 * c_voff[k], c_voff[k + 1] - c_voff[k], paced_cb, r);
      } else {
        r->expect = d_expect + 32 * k;
        r->n_expect = 32;
        rc = coa_queue_submit_digest(q, d_data + d_off[k], d_off[k + 1] - d_off[k], paced_cb, r);
      }
      if (rc != COA_OK) atomic_fetch_add(&wrong, 1);
    }
    coa_queue_flush(q);
    coa_queue_metrics_reset(q);
    memset(reqs, 0, (n ? n : 1) * sizeof(PacedReq));
  }
  g_paced_t0 = now_us();
  for (size_t i = 0; i < n; i++) {
    PacedReq* r = &reqs[i];
    r->due_us = arrive_s[i] * 1e6;
    r->out = &lat_us[i];
    r->wrong = &wrong;
    const size_t k = item[i];
    sleep_until_us(r->due_us);
    int rc;
    if (kind[i] == 0) {
      r->expect = v_expect + k;
      r->n_expect = 1;
      rc = coa_queue_submit_verify(q, vmsgs + 32 * k, vpks + 32 * k, vsigs + 64 * k, paced_cb, r);
    } else if (kind[i] == 1) {
      r->expect = c_expect + k;
      r->n_expect = 1;
      rc = coa_queue_submit_certificate(q, c_hdata + c_hoff[k], c_hoff[k + 1] - c_hoff[k], c_ids + 32 * k,
                                        c_origins + 32 * k, c_hsigs + 64 * k, c_rounds[k], c_vpks + 32 * c_voff[k],
                                        c_vsigs + 64 * c_voff[k], c_voff[k + 1] - c_voff[k], paced_cb, r);
    } else {
      r->expect = d_expect + 32 * k;
      r->n_expect = 32;
      rc = coa_queue_submit_digest(q, d_data + d_off[k], d_off[k + 1] - d_off[k], paced_cb, r);
    }
    if (rc != COA_OK) {
      lat_us[i] = -1.0;
      atomic_fetch_add(&wrong, 1);
    }
  }
  coa_queue_flush(q);
  *elapsed_s = (now_us() - g_paced_t0) * 1e-6;
  coa_queue_metrics(q, m);
  coa_queue_destroy(q);
  free(reqs);
  return atomic_load(&wrong);
}

/* ------------------------------------------------------------------------
 * End-to-end throughput of the host-pointer entry points, as the Rust
 * binding calls them: inputs in host memory, verdicts back in host memory,
 * H2D / D2H and packing inside the clock.  `threads` C threads each make
 * `calls` back-to-back calls over the same inputs (each thread its own
 * output); wall time from the first call to the last return into
 * *elapsed_s.  Returns the number of wrong outputs (all inputs valid:
 * verdict 0 / status 0), or a negative engine status. */
#include <pthread.h>

typedef struct {
  int what; /* 0 verify_strict_many, 1 certificate_verify_many */
  int calls;
  size_t n;
  const uint8_t *msgs, *pks, *sigs;
  const uint8_t *hdata, *ids, *origins, *hsigs, *vpks, *vsigs;
  const uint64_t *hoff, *rounds, *voff;
  const uint8_t* expect;
  uint8_t* out;
  int rc, wrong;
} ManyJob;

static void* many_thread(void* arg) {
  ManyJob* j = (ManyJob*)arg;
  for (int c = 0; c < j->calls && j->rc == 0; c++) {
    if (j->what == 0)
      j->rc = coa_ed25519_verify_strict_many(j->msgs, 32, j->pks, j->sigs, j->n, j->out);
    else
      j->rc = coa_certificate_verify_many(j->hdata, j->hoff, j->ids, j->origins, j->hsigs, j->rounds, j->vpks,
                                          j->vsigs, j->voff, j->n, 0, j->out);
    for (size_t i = 0; i < j->n && j->rc == 0; i++) j->wrong += j->out[i] != (j->expect ? j->expect[i] : 0);
  }
  return NULL;
}

static int run_many(ManyJob* proto, int threads, double* elapsed_s) {
  if (threads < 1 || threads > 64) return -1;
  ManyJob jobs[64];
  pthread_t th[64];
  for (int t = 0; t < threads; t++) {
    jobs[t] = *proto;
    jobs[t].out = (uint8_t*)malloc(proto->n ? proto->n : 1);
    jobs[t].rc = jobs[t].wrong = 0;
  }
  const double t0 = now_us();
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, many_thread, &jobs[t]);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  *elapsed_s = (now_us() - t0) * 1e-6;
  int rc = 0, wrong = 0;
  for (int t = 0; t < threads; t++) {
    if (jobs[t].rc < 0 && rc == 0) rc = jobs[t].rc;
    wrong += jobs[t].wrong;
    free(jobs[t].out);
  }
  return rc < 0 ? rc : wrong;
}

int latc_verify_many(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, size_t n, int calls, int threads,
                     double* elapsed_s) {
  ManyJob p;
  memset(&p, 0, sizeof(p));
  p.what = 0;
  p.calls = calls;
  p.n = n;
  p.msgs = msgs;
  p.pks = pks;
  p.sigs = sigs;
  return run_many(&p, threads, elapsed_s);
}

int latc_certificates_many(const uint8_t* hdata, const uint64_t* hoff, const uint8_t* ids, const uint8_t* origins,
                           const uint8_t* hsigs, const uint64_t* rounds, const uint8_t* vpks, const uint8_t* vsigs,
                           const uint64_t* voff, size_t n, const uint8_t* expect, int calls, int threads,
                           double* elapsed_s) {
  ManyJob p;
  memset(&p, 0, sizeof(p));
  p.what = 1;
  p.calls = calls;
  p.n = n;
  p.hdata = hdata;
  p.hoff = hoff;
  p.ids = ids;
  p.origins = origins;
  p.hsigs = hsigs;
  p.rounds = rounds;
  p.vpks = vpks;
  p.vsigs = vsigs;
  p.voff = voff;
  p.expect = expect;
  return run_many(&p, threads, elapsed_s);
}

/* A whole certificate round streamed through the aggregation queue, as
 * VerifyService::certificate submits it (coa_queue_submit_certificate, one
 * request per certificate): `producers` C threads submit certificates
 * p, p + producers, ... of the round, `rounds` times over, all at once; the
 * clock runs from the first submission to the last callback (flush).
 * Returns wrong answers (>= 0); queue metrics into *m. */
typedef struct {
  coa_queue* q;
  int p, producers, rounds, borrowed;
  double rate;   /* this producer's submissions per second (0: as fast as it can) */
  double t0_us;  /* its schedule's start */
  size_t n;
  const uint8_t *hdata, *ids, *origins, *hsigs, *vpks, *vsigs, *expect;
  const uint64_t *hoff, *rounds_of, *voff;
  atomic_int* wrong;
  atomic_long* answered;
} StreamJob;

typedef struct {
  const uint8_t* expect;
  atomic_int* wrong;
  atomic_long* answered;
} StreamReq;

static void stream_cb(void* user, int status, const uint8_t* v, size_t n) {
  StreamReq* r = (StreamReq*)user;
  if (status != COA_OK || n != 1 || v[0] != r->expect[0]) atomic_fetch_add(r->wrong, 1);
  atomic_fetch_add(r->answered, 1);
  free(r);
}

static void* stream_thread(void* arg) {
  StreamJob* j = (StreamJob*)arg;
  size_t sent = 0;
  for (int r = 0; r < j->rounds; r++)
    for (size_t k = (size_t)j->p; k < j->n; k += (size_t)j->producers, sent++) {
      if (j->rate > 0) {  /* paced: the i-th submission at t0 + i / rate */
        const double due = j->t0_us + (double)sent * 1e6 / j->rate;
        while (now_us() < due) {
        }
      }
      StreamReq* q = (StreamReq*)malloc(sizeof(StreamReq));
      q->expect = j->expect + k;
      q->wrong = j->wrong;
      q->answered = j->answered;
      const int rc = (j->borrowed ? coa_queue_submit_certificate_borrowed : coa_queue_submit_certificate)(
                                                  j->q, j->hdata + j->hoff[k], j->hoff[k + 1] - j->hoff[k],
                                                  j->ids + 32 * k, j->origins + 32 * k, j->hsigs + 64 * k,
                                                  j->rounds_of[k], j->vpks + 32 * j->voff[k],
                                                  j->vsigs + 64 * j->voff[k], j->voff[k + 1] - j->voff[k], stream_cb, q);
      if (rc != COA_OK) {
        atomic_fetch_add(j->wrong, 1);
        free(q);
      }
    }
  return NULL;
}

int latc_stream_certificates(size_t max_batch, unsigned max_delay_us, int producers, int rounds, int borrowed,
                             double rate_per_s,
                             const uint8_t* hdata, const uint64_t* hoff, const uint8_t* ids, const uint8_t* origins,
                             const uint8_t* hsigs, const uint64_t* rounds_of, const uint8_t* vpks,
                             const uint8_t* vsigs, const uint64_t* voff, size_t n, const uint8_t* expect,
                             double* elapsed_s, coa_queue_metrics_t* m) {
  if (producers < 1 || producers > 64) return -1;
  coa_queue* q = coa_queue_create(max_batch, max_delay_us);
  if (!q) return -1;
  atomic_int wrong = 0;
  atomic_long answered = 0;
  StreamJob jobs[64];
  pthread_t th[64];
  for (int p = 0; p < producers; p++) {
    StreamJob* j = &jobs[p];
    j->q = q;
    j->p = p;
    j->producers = producers;
    j->rounds = rounds;
    j->borrowed = borrowed;
    j->rate = 0;
    j->n = n;
    j->hdata = hdata;
    j->hoff = hoff;
    j->ids = ids;
    j->origins = origins;
    j->hsigs = hsigs;
    j->rounds_of = rounds_of;
    j->vpks = vpks;
    j->vsigs = vsigs;
    j->voff = voff;
    j->expect = expect;
    j->wrong = &wrong;
    j->answered = &answered;
  }
  // one untimed round first: a node's queue runs for hours, so its shards'
  // windows are recycled with their capacity and pages in place; a fresh
  // queue's first windows grow and fault in their vectors (steady state is
  // what the line reports; the metrics are reset after the warm-up)
  for (int p = 0; p < producers; p++) jobs[p].rounds = 1;
  for (int p = 0; p < producers; p++) pthread_create(&th[p], NULL, stream_thread, &jobs[p]);
  for (int p = 0; p < producers; p++) pthread_join(th[p], NULL);
  coa_queue_flush(q);
  coa_queue_metrics_reset(q);
  atomic_store(&answered, 0);
  const double t0 = now_us();
  for (int p = 0; p < producers; p++) {
    jobs[p].rounds = rounds;
    jobs[p].rate = rate_per_s / producers;
    jobs[p].t0_us = t0;
  }
  for (int p = 0; p < producers; p++) pthread_create(&th[p], NULL, stream_thread, &jobs[p]);
  for (int p = 0; p < producers; p++) pthread_join(th[p], NULL);
  coa_queue_flush(q);
  *elapsed_s = (now_us() - t0) * 1e-6;
  coa_queue_metrics(q, m);
  coa_queue_destroy(q);
  if (atomic_load(&answered) != (long)(n * (size_t)rounds)) atomic_fetch_add(&wrong, 1);
  return atomic_load(&wrong);
}
