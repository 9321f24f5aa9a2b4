/*
 * wire_queue_harness.c -- the pre-verification stage as a compiled caller
 * would run it on raw frames ("raw frames"): bincode
 * PrimaryMessage::Certificate frames, as PrimaryReceiverHandler::dispatch
 * receives them (primary/src/primary.rs:223-244), are scanned and decoded by
 * the engine's native decoder (coa_wire_scan / coa_wire_decode_certificates,
 * f4) straight into the certificate arrays, and every certificate is queued
 * through coa_queue_submit_certificate (what VerifyService::certificate does)
 * with a callback that checks its COA_CERT_* bits against the golden
 * expectation of tests/golden/wire_certificates.bin (oracle-computed by
 * tests/golden/make_wire_certificates.py).
 *
 * usage: wire_queue_harness <wire_certificates.bin> <register 0|1> <rounds>
 * The last stdout line is one JSON object; exit status 0 only when every
 * frame decoded as a certificate and every callback ran once with COA_OK and
 * the expected bits.  Without a GPU (tests/test_c_abi.py) the decode must
 * still succeed and every request must still be answered, with the engine's
 * error status.
 */
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "coa_verify.h"

typedef struct {
  uint8_t expect;
  atomic_int* wrong;
  atomic_int* bad_status;
  atomic_int* answered;
} Req;

static void on_status(void* user, int status, const uint8_t* v, size_t n) {
  Req* r = (Req*)user;
  if (status != COA_OK) {
    atomic_fetch_add(r->bad_status, 1);
  } else if (n != 1 || v[0] != r->expect) {
    atomic_fetch_add(r->wrong, 1);
  }
  atomic_fetch_add(r->answered, 1);
}

static uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <wire_certificates.bin> <register 0|1> <rounds>\n", argv[0]);
    return 2;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  fseek(f, 0, SEEK_END);
  const long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* buf = (uint8_t*)malloc((size_t)sz);
  if (!buf || fread(buf, 1, (size_t)sz, f) != (size_t)sz) return 2;
  fclose(f);
  if (sz < 12 || memcmp(buf, "CQWC", 4) != 0) return 2;
  const int do_register = atoi(argv[2]);
  const int rounds = atoi(argv[3]);
  size_t o = 4;
  const uint32_t n_keys = rd32(buf + o);
  o += 4;
  const uint8_t* keys = buf + o;
  o += 32 * (size_t)n_keys;
  const uint32_t n = rd32(buf + o);
  o += 4;
  uint8_t* frames = (uint8_t*)malloc((size_t)sz);
  uint64_t* foff = (uint64_t*)calloc(n + 1, 8);
  uint8_t* expect = (uint8_t*)malloc(n);
  size_t fb = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t len = rd32(buf + o);
    o += 4;
    memcpy(frames + fb, buf + o, len);
    o += len;
    fb += len;
    foff[i + 1] = fb;
    expect[i] = buf[o++];
  }
  /* the native decoder: scan, size, decode */
  int32_t* kinds = (int32_t*)malloc(n * 4);
  uint64_t* hbytes = (uint64_t*)malloc(n * 8);
  uint64_t* nvotes = (uint64_t*)malloc(n * 8);
  int rc = coa_wire_scan(frames, foff, n, kinds, hbytes, nvotes);
  int not_cert = 0;
  size_t hb = 0, nv = 0;
  for (uint32_t i = 0; i < n; i++) {
    not_cert += kinds[i] != COA_MSG_CERTIFICATE;
    hb += hbytes[i];
    nv += nvotes[i];
  }
  if (rc != COA_OK || not_cert) {
    printf("{\"decoded\": false, \"scan_rc\": %d, \"not_certificates\": %d}\n", rc, not_cert);
    return 1;
  }
  uint8_t* hdata = (uint8_t*)malloc(hb + 16);
  uint64_t* hoff = (uint64_t*)calloc(n + 1, 8);
  uint8_t *ids = (uint8_t*)malloc(n * 32), *origins = (uint8_t*)malloc(n * 32), *hsigs = (uint8_t*)malloc(n * 64);
  uint64_t* rnds = (uint64_t*)malloc(n * 8);
  uint8_t *vpks = (uint8_t*)malloc(nv * 32 + 32), *vsigs = (uint8_t*)malloc(nv * 64 + 64);
  uint64_t* voff = (uint64_t*)calloc(n + 1, 8);
  rc = coa_wire_decode_certificates(frames, foff, n, hdata, hoff, ids, origins, hsigs, rnds, vpks, vsigs, voff, NULL);
  if (rc != COA_OK) {
    printf("{\"decoded\": false, \"decode_rc\": %d}\n", rc);
    return 1;
  }
  int reg_rc = 0;
  if (do_register) reg_rc = coa_committee_register(keys, n_keys);
  /* the queue: one request per certificate, `rounds` times over */
  coa_queue* q = coa_queue_create(4096, 300);
  if (!q) return 1;
  atomic_int wrong = 0, bad_status = 0, answered = 0;
  Req* reqs = (Req*)malloc(sizeof(Req) * n * (size_t)rounds);
  int submit_fail = 0;
  for (int r = 0; r < rounds; r++)
    for (uint32_t i = 0; i < n; i++) {
      Req* q_ = &reqs[(size_t)r * n + i];
      q_->expect = expect[i];
      q_->wrong = &wrong;
      q_->bad_status = &bad_status;
      q_->answered = &answered;
      const int s = coa_queue_submit_certificate(q, hdata + hoff[i], hoff[i + 1] - hoff[i], ids + 32 * i,
                                                 origins + 32 * i, hsigs + 64 * i, rnds[i], vpks + 32 * voff[i],
                                                 vsigs + 64 * voff[i], voff[i + 1] - voff[i], on_status, q_);
      if (s != COA_OK) {
        submit_fail++;
        atomic_fetch_add(&answered, 1);
      }
    }
  coa_queue_flush(q);
  coa_queue_metrics_t m;
  coa_queue_metrics(q, &m);
  coa_queue_destroy(q);
  if (do_register && reg_rc >= 0) coa_committee_register(NULL, 0);
  const int total = (int)n * rounds;
  printf("{\"decoded\": true, \"frames\": %u, \"votes\": %zu, \"register_rc\": %d, \"submitted\": %d, "
         "\"answered\": %d, \"wrong\": %d, \"bad_status\": %d, \"submit_fail\": %d, \"windows\": %llu, "
         "\"failed_windows\": %llu}\n",
         n, nv, reg_rc, total, atomic_load(&answered), atomic_load(&wrong), atomic_load(&bad_status), submit_fail,
         (unsigned long long)m.windows, (unsigned long long)m.failed_windows);
  const int ok = atomic_load(&answered) == total && atomic_load(&wrong) == 0 && atomic_load(&bad_status) == 0 &&
                 submit_fail == 0 && reg_rc >= 0;
  return ok ? 0 : 1;
}
