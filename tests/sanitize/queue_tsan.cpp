// ThreadSanitizer run of the aggregation queue (xrpl-coa-prototype_amd/csrc/
// coa_queue.cpp) with many producer threads.  The queue's
// engine calls are served by a deterministic stub linked in their place (no
// GPU, no HIP): each verdict is a pure function of the request's bytes, so
// every callback can be checked against the request it answers.
//
// Build (tests/test_sanitizers.py): g++ -fsanitize=thread coa_queue.cpp
// queue_tsan.cpp.  usage: queue_tsan <producers> <requests per producer>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "coa_verify.h"

// ------------------------------------------------------------- stub engine
static std::atomic<long> g_engine_calls{0};
static void gpu_time() { std::this_thread::sleep_for(std::chrono::microseconds(50)); }
static uint8_t v_single(const uint8_t* msg, const uint8_t* sig) { return (uint8_t)((msg[0] ^ sig[0]) & 1u); }
static uint8_t v_group(const uint8_t* msg, size_t nvotes) { return (uint8_t)((msg[1] + nvotes) & 1u); }
static uint8_t v_cert(const uint8_t* id, size_t nvotes) { return (uint8_t)((id[2] + nvotes) & 7u); }
static uint8_t v_digest(const uint8_t* data, size_t len, int j) {
  return (uint8_t)((len ? data[0] : 0xa5) + 7 * j + (uint8_t)len);
}

extern "C" {
int coa_ed25519_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                   size_t n, uint8_t* verdicts_out) {
  (void)pks;
  g_engine_calls++;
  gpu_time();
  for (size_t i = 0; i < n; i++) verdicts_out[i] = v_single(msgs + i * msg_len, sigs + i * 64);
  return COA_OK;
}
int coa_ed25519_verify_batch_groups(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                    const uint64_t* group_offsets, size_t n_groups, uint8_t* group_verdicts_out,
                                    uint64_t rng_seed) {
  (void)pks;
  (void)sigs;
  (void)rng_seed;
  g_engine_calls++;
  gpu_time();
  for (size_t g = 0; g < n_groups; g++)
    group_verdicts_out[g] = v_group(msgs + g * 32, group_offsets[g + 1] - group_offsets[g]);
  return COA_OK;
}
int coa_certificate_verify_many(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                size_t n, uint64_t rng_seed, uint8_t* status_out) {
  (void)header_data;
  (void)header_offsets;
  (void)origins;
  (void)header_sigs;
  (void)rounds;
  (void)vote_pks;
  (void)vote_sigs;
  (void)rng_seed;
  g_engine_calls++;
  gpu_time();
  for (size_t c = 0; c < n; c++) status_out[c] = v_cert(ids + c * 32, vote_offsets[c + 1] - vote_offsets[c]);
  return COA_OK;
}
int coa_sha512_trunc32_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
  g_engine_calls++;
  gpu_time();
  for (size_t i = 0; i < n; i++)
    for (int j = 0; j < 32; j++) out32[i * 32 + j] = v_digest(data + offsets[i], offsets[i + 1] - offsets[i], j);
  return COA_OK;
}
}

// -------------------------------------------------------------- producers
struct Req {
  uint8_t expect[32];
  size_t n_expect;
  std::atomic<int> done{0};
  std::atomic<int> bad{0};
};

static void check_cb(void* user, int status, const uint8_t* verdicts, size_t n) {
  Req* r = static_cast<Req*>(user);
  if (status != COA_OK || n != r->n_expect || std::memcmp(verdicts, r->expect, n) != 0) r->bad++;
  r->done++;
}

int main(int argc, char** argv) {
  const int producers = argc > 1 ? std::atoi(argv[1]) : 8;
  const int per = argc > 2 ? std::atoi(argv[2]) : 400;
  coa_queue* q = coa_queue_create(64, 200);
  std::vector<std::vector<Req>> reqs(producers);
  for (auto& v : reqs) v = std::vector<Req>(per);
  std::vector<std::thread> th;
  for (int p = 0; p < producers; p++) {
    th.emplace_back([&, p] {
      std::mt19937 rng(1000 + p);
      for (int i = 0; i < per; i++) {
        Req& r = reqs[p][i];
        uint8_t a[32], b[64], c[32];
        for (auto& x : a) x = (uint8_t)rng();
        for (auto& x : b) x = (uint8_t)rng();
        for (auto& x : c) x = (uint8_t)rng();
        int rc = COA_OK;
        switch (rng() % 4) {
          case 0:
            r.n_expect = 1;
            r.expect[0] = v_single(a, b);
            rc = coa_queue_submit_verify(q, a, c, b, check_cb, &r);
            break;
          case 1: {
            const size_t nv = rng() % 5;
            std::vector<uint8_t> pks(nv * 32 + 1, 1), sigs(nv * 64 + 1, 2);
            r.n_expect = 1;
            r.expect[0] = v_group(a, nv);
            rc = coa_queue_submit_batch(q, a, pks.data(), sigs.data(), nv, check_cb, &r);
            break;
          }
          case 2: {
            const size_t nv = rng() % 4;
            std::vector<uint8_t> hdr(rng() % 100), pks(nv * 32 + 1, 3), sigs(nv * 64 + 1, 4);
            r.n_expect = 1;
            r.expect[0] = v_cert(a, nv);
            rc = coa_queue_submit_certificate(q, hdr.data(), hdr.size(), a, c, b, 9, pks.data(), sigs.data(), nv,
                                              check_cb, &r);
            break;
          }
          default: {
            std::vector<uint8_t> data(rng() % 300);
            for (auto& x : data) x = (uint8_t)rng();
            r.n_expect = 32;
            for (int j = 0; j < 32; j++) r.expect[j] = v_digest(data.data(), data.size(), j);
            rc = coa_queue_submit_digest(q, data.data(), data.size(), check_cb, &r);
            break;
          }
        }
        if (rc != COA_OK) r.bad++, r.done++;
        if (rng() % 97 == 0) coa_queue_flush(q);  // flushes race with submissions and the worker
        if (rng() % 53 == 0) {
          uint64_t l, it, g, d;
          coa_queue_stats(q, &l, &it, &g);
          coa_queue_digest_count(q, &d);
        }
      }
    });
  }
  for (auto& t : th) t.join();
  coa_queue_flush(q);
  long done = 0, bad = 0;
  for (auto& v : reqs)
    for (auto& r : v) {
      done += r.done.load();
      bad += r.bad.load();
    }
  uint64_t launches = 0, items = 0, groups = 0, digests = 0;
  coa_queue_stats(q, &launches, &items, &groups);
  coa_queue_digest_count(q, &digests);
  coa_queue_destroy(q);
  const long total = (long)producers * per;
  std::printf("queue tsan: %ld/%ld answered, %ld wrong, %llu launches, %ld engine calls\n", done, total, bad,
              (unsigned long long)launches, g_engine_calls.load());
  return (done == total && bad == 0 && items + groups + digests == (uint64_t)total) ? 0 : 1;
}
