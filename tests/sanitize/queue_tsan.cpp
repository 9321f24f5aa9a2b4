// ThreadSanitizer run of the aggregation queue (xrpl-coa-prototype_amd/csrc/
// coa_queue.cpp) with many producer threads.  The queue's
// launch backend (coa_queue.h) is a deterministic stub linked in place of the
// HIP one (no GPU, no HIP) with the same two-slot double buffering: each
// verdict is a pure function of the request's bytes, so every callback can be
// checked against the request it answers.
//
// Build (tests/test_sanitizers.py): g++ -fsanitize=thread coa_queue.cpp
// queue_tsan.cpp.  usage: queue_tsan <producers> <requests per producer>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "coa_queue.h"
#include "coa_verify.h"

// ------------------------------------------------------------ stub backend
// Two slots like the HIP backend: launch() blocks while both are busy and
// returns at once; complete() "runs" the launch (a short sleep) and writes
// every part's outputs.  Verdicts are pure functions of the request bytes.
// Fault injection (argv[3] = k): every k-th launch fails in complete() (no
// outputs, COA_EHIP), as a HIP error would; the queue must then re-run it
// through retry(), which succeeds -- unless argv[4] = 1, when every retry
// fails too and the callbacks must get the engine error.
static std::atomic<long> g_engine_calls{0}, g_injected{0}, g_resolver_passes{0}, g_resolved{0};
static unsigned long g_fault_every = 0;
static bool g_fault_all = false;
static uint8_t v_single(const uint8_t* msg, const uint8_t* sig) { return (uint8_t)((msg[0] ^ sig[0]) & 1u); }
static uint8_t v_group(const uint8_t* msg, size_t nvotes) { return (uint8_t)((msg[1] + nvotes) & 1u); }
static uint8_t v_cert(const uint8_t* id, size_t nvotes) { return (uint8_t)((id[2] + nvotes) & 7u); }
static uint8_t v_digest(const uint8_t* data, size_t len, int j) {
  return (uint8_t)((len ? data[0] : 0xa5) + 7 * j + (uint8_t)len);
}

namespace {
void run_launch(coa_q::Launch& L) {
  for (coa_q::Window* wp : L.parts) {
    coa_q::Window& w = *wp;
    for (size_t i = 0; i < w.nv; i++) w.v_out[i] = v_single(&w.v_msgs[i * 32], &w.v_sigs[i * 64]);
    // as the HIP backend does: bare vote batches, and the certificates the
    // "kernel" cannot decide alone (here: id[3] odd), are left to resolve()
    w.g_defer = w.ng > 0;
    for (size_t c = 0; c < w.nc; c++) {
      if (w.c_refs[c].id[3] & 1u)
        w.c_defer.push_back((uint32_t)c);
      else
        w.c_out[c] = v_cert(w.c_refs[c].id, w.c_refs[c].nv);
    }
    for (size_t i = 0; i < w.nd; i++)
      for (int j = 0; j < 32; j++)
        w.d_out[i * 32 + j] = v_digest(w.d_data.data() + w.d_offs[i], w.d_offs[i + 1] - w.d_offs[i], j);
  }
  L.rc = COA_OK;
}

class StubBackend : public coa_q::Backend {
 public:
  int slots() const override { return 2; }
  int devices() const override { return 2; }
  void launch(coa_q::Launch& L) override {
    std::unique_lock<std::mutex> l(m_);
    const int k = (int)(next_++ % 2);
    cv_.wait(l, [&] { return !busy_[k]; });
    busy_[k] = true;
    L.slot = k;
    fail_[k] = g_fault_every && next_ % g_fault_every == 0;
  }
  // as the HIP backend: the collector waits here before it closes a window
  // while both slots are busy (the backlog window, coa_queue.cpp)
  bool wait_free_slot() override {
    std::unique_lock<std::mutex> l(m_);
    if (!busy_[0] || !busy_[1]) return false;
    cv_.wait(l, [&] { return !busy_[0] || !busy_[1]; });
    return true;
  }
  void complete(coa_q::Launch& L) override {
    g_engine_calls++;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
    bool failed;
    {
      std::lock_guard<std::mutex> l(m_);
      failed = fail_[L.slot];
    }
    if (failed) {
      g_injected++;
      L.rc = COA_EHIP;  // outputs stay at their "failed" values
    } else {
      run_launch(L);
    }
    std::lock_guard<std::mutex> l(m_);
    busy_[L.slot] = false;
    cv_.notify_all();
  }
  void retry(coa_q::Launch& L, int attempt) override {
    if (attempt < 1 || attempt > devices()) std::abort();
    if (g_fault_all) {
      L.rc = COA_EHIP;
      return;
    }
    run_launch(L);
  }
  int resolve(const std::vector<coa_q::Window*>& ws) override {
    g_resolver_passes++;
    std::this_thread::sleep_for(std::chrono::microseconds(200));  // slower than a window: the rest must not wait
    for (coa_q::Window* w : ws) {
      for (uint32_t c : w->c_defer) {
        w->c_out[c] = v_cert(w->c_refs[c].id, w->c_refs[c].nv);
        g_resolved++;
      }
      if (w->g_defer)
        for (size_t g = 0; g < w->ng; g++) {
          w->g_out[g] = v_group(&w->g_msgs[g * 32], w->g_offs[g + 1] - w->g_offs[g]);
          g_resolved++;
        }
    }
    return COA_OK;
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  bool busy_[2] = {false, false};
  bool fail_[2] = {false, false};
  unsigned long next_ = 0;
};
}  // namespace

coa_q::Backend* coa_q::make_backend(int) { return new StubBackend(); }

// -------------------------------------------------------------- producers
struct Req {
  uint8_t expect[32];
  size_t n_expect;
  std::vector<uint8_t> hold;  // a borrowed certificate's bytes, valid until the end of the run
  std::atomic<int> done{0};
  std::atomic<int> bad{0};
};

static std::atomic<long> g_engine_errors{0};
static void check_cb(void* user, int status, const uint8_t* verdicts, size_t n) {
  Req* r = static_cast<Req*>(user);
  if (status == COA_EHIP) {
    g_engine_errors++;
    if (!g_fault_all) r->bad++;
  } else if (status != COA_OK || n != r->n_expect || std::memcmp(verdicts, r->expect, n) != 0) {
    r->bad++;
  }
  r->done++;
}

int main(int argc, char** argv) {
  const int producers = argc > 1 ? std::atoi(argv[1]) : 8;
  const int per = argc > 2 ? std::atoi(argv[2]) : 400;
  g_fault_every = argc > 3 ? std::strtoul(argv[3], nullptr, 10) : 0;
  g_fault_all = argc > 4 && std::atoi(argv[4]) == 1;
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
            if (rng() % 2) {
              rc = coa_queue_submit_certificate(q, hdr.data(), hdr.size(), a, c, b, 9, pks.data(), sigs.data(), nv,
                                                check_cb, &r);
            } else {  // borrowed: the queue reads the caller's arrays until the callback
              r.hold.resize(32 + 32 + 64 + hdr.size() + nv * 96);
              uint8_t* h = r.hold.data();
              auto put = [](uint8_t* d, const uint8_t* src, size_t len) {
                if (len) std::memcpy(d, src, len);
              };
              put(h, a, 32);
              put(h + 32, c, 32);
              put(h + 64, b, 64);
              put(h + 128, hdr.data(), hdr.size());
              put(h + 128 + hdr.size(), pks.data(), nv * 32);
              put(h + 128 + hdr.size() + nv * 32, sigs.data(), nv * 64);
              rc = coa_queue_submit_certificate_borrowed(q, h + 128, hdr.size(), h, h + 32, h + 64, 9, h + 128 + hdr.size(),
                                                         h + 128 + hdr.size() + nv * 32, nv, check_cb, &r);
            }
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
          coa_queue_metrics_t mm;
          coa_queue_metrics(q, &mm);
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
  coa_queue_metrics_t m;
  coa_queue_metrics(q, &m);
  coa_queue_destroy(q);
  const long total = (long)producers * per;
  std::printf("queue tsan: %ld/%ld answered, %ld wrong, %llu launches, %ld windows completed, max in flight %llu, "
              "wait p50 %.0f us p99 %.0f us, injected %ld, retried %llu, recovered %llu, failed %llu, engine errors %ld, "
              "deferred %llu in %llu passes\n",
              done, total, bad, (unsigned long long)launches, g_engine_calls.load(),
              (unsigned long long)m.max_in_flight, m.wait_us_p50, m.wait_us_p99, g_injected.load(),
              (unsigned long long)m.retried_windows, (unsigned long long)m.recovered_windows,
              (unsigned long long)m.failed_windows, g_engine_errors.load(), (unsigned long long)m.deferred_requests,
              (unsigned long long)m.resolver_passes);
  // every injected failure was retried; retries succeed unless told not to
  const bool recovery_ok =
      m.retried_windows == (uint64_t)g_injected.load() &&
      (g_fault_all ? (m.recovered_windows == 0 && m.failed_windows == m.retried_windows &&
                      (g_injected.load() == 0 || g_engine_errors.load() > 0))
                   : (m.recovered_windows == m.retried_windows && m.failed_windows == 0 && g_engine_errors.load() == 0));
  // every deferred request was answered by a resolver pass (none when every
  // window failed), and the passes the queue counted are the backend's
  const bool defer_ok = m.deferred_requests == (uint64_t)g_resolved.load() &&
                        m.resolver_passes == (uint64_t)g_resolver_passes.load() &&
                        m.deferred_requests > 0;
  const bool metrics_ok = m.requests == (uint64_t)total && m.batches + m.certificates + m.digests <= (uint64_t)total &&
                          m.windows == launches && recovery_ok && defer_ok;
  return (done == total && bad == 0 && items + groups + digests == (uint64_t)total && metrics_ok) ? 0 : 1;
}
