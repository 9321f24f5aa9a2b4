// Host-side cost of the aggregation queue's certificate intake, on the CPU:
// coa_queue.cpp with a stub backend that packs each launch into a staging
// block (as coa_queue_hip.cpp does, one memcpy per part array) and "runs"
// it for a fixed time.  Producers submit C3-shaped certificates (3,336-byte
// header input, 67 votes: 9,920 bytes each) as fast as they can, like
// tools/latc.c latc_stream_certificates; prints certificates/s and the
// queue's per-stage time per window (COA_QSTAGE_*).
//
// build: g++ -O2 -std=c++17 -pthread -I include -I xrpl-coa-prototype_amd/csrc \
//          xrpl-coa-prototype_amd/csrc/coa_queue.cpp tools/queue_host_bench.cpp -o /tmp/qhb
// usage: qhb <producers> [certs per producer] [device_us] [borrowed 0|1]
// (one untimed round first, then the metrics are reset: steady state)
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "coa_queue.h"
#include "coa_verify.h"

static int g_device_us = 300;

namespace {
class PackStub : public coa_q::Backend {
 public:
  int slots() const override { return 4; }
  int devices() const override { return 1; }
  void launch(coa_q::Launch& L) override {
    std::unique_lock<std::mutex> l(m_);
    int k = -1;
    cv_.wait(l, [&] {
      for (int i = 0; i < 4; i++)
        if (!busy_[i]) return (k = i) >= 0;
      return false;
    });
    busy_[k] = true;
    L.slot = k;
    l.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    const size_t bytes = (L.hbytes + L.nc * 136 + L.nvotes * 96) + 64;
    std::vector<uint8_t>& st = stage_[k];
    if (st.size() < bytes) st.resize(2 * bytes);
    size_t o = 0;
    for (const coa_q::Window* w : L.parts)
      for (const coa_q::Window::CertRef& r : w->c_refs) {
        for (auto f : {std::make_pair(r.hdr, r.hlen), std::make_pair(r.id, (uint64_t)32),
                       std::make_pair(r.origin, (uint64_t)32), std::make_pair(r.hsig, (uint64_t)64),
                       std::make_pair(r.vpks, r.nv * 32), std::make_pair(r.vsigs, r.nv * 64)}) {
          std::memcpy(st.data() + o, f.first, f.second);
          o += f.second;
        }
      }
    L.stage_ns[COA_QSTAGE_PACK] +=
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    done_at_[k] = std::chrono::steady_clock::now() + std::chrono::microseconds(g_device_us);
  }
  void complete(coa_q::Launch& L) override {
    std::this_thread::sleep_until(done_at_[L.slot]);
    for (coa_q::Window* w : L.parts) w->c_out.assign(w->nc, 0);
    std::lock_guard<std::mutex> l(m_);
    busy_[L.slot] = false;
    cv_.notify_all();
  }
  void retry(coa_q::Launch& L, int) override { L.rc = COA_EHIP; }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  bool busy_[4] = {};
  std::chrono::steady_clock::time_point done_at_[4];
  std::vector<uint8_t> stage_[4];
};
}  // namespace

coa_q::Backend* coa_q::make_backend(int) { return new PackStub(); }

static std::atomic<long> g_answered{0};
static void cb(void*, int, const uint8_t*, size_t) { g_answered++; }

int main(int argc, char** argv) {
  const int producers = argc > 1 ? atoi(argv[1]) : 4;
  const int per = argc > 2 ? atoi(argv[2]) : 7500;
  g_device_us = argc > 3 ? atoi(argv[3]) : 300;
  const bool borrowed = argc > 4 && atoi(argv[4]) == 1;
  const size_t hlen = 3336, nv = 67, ncert = 2500;
  // a pool of distinct certificates (cold in cache, like a round's)
  std::vector<uint8_t> hdr(ncert * hlen, 1), pks(ncert * nv * 32, 2), sigs(ncert * nv * 64, 3), ids(ncert * 32, 4);
  coa_queue* q = coa_queue_create(65536, 500);
  auto round = [&] {
    std::vector<std::thread> th;
    for (int p = 0; p < producers; p++)
      th.emplace_back([&, p] {
        for (int i = 0; i < per; i++) {
          const size_t c = (size_t)(p * per + i) % ncert;
          (borrowed ? coa_queue_submit_certificate_borrowed : coa_queue_submit_certificate)(
              q, &hdr[c * hlen], hlen, &ids[c * 32], &ids[c * 32], &sigs[c * nv * 64], 1, &pks[c * nv * 32],
              &sigs[c * nv * 64], nv, cb, nullptr);
        }
      });
    for (auto& t : th) t.join();
    coa_queue_flush(q);
  };
  round();
  coa_queue_metrics_reset(q);
  g_answered = 0;
  const auto t0 = std::chrono::steady_clock::now();
  round();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  coa_queue_metrics_t m;
  coa_queue_metrics(q, &m);
  coa_queue_destroy(q);
  const char* names[] = {"intake", "gather", "slot_wait", "pack", "enqueue", "device_wait", "scatter", "callbacks",
                         "resolve"};
  std::printf("%s producers %d: %.0f certs/s, %llu windows, wait p99 %.0f us; per window:", borrowed ? "borrowed" : "copied", producers,
              (double)g_answered.load() / s, (unsigned long long)m.windows, m.wait_us_p99);
  for (int k = 0; k < COA_QSTAGES; k++) std::printf(" %s %.1f", names[k], m.stage_us[k] / (double)m.windows);
  std::printf("\n");
  return g_answered.load() == (long)producers * per ? 0 : 1;
}
