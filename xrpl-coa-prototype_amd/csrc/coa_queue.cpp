// Aggregation queue: the pre-verification stage between
// PrimaryReceiverHandler::dispatch (primary/src/primary.rs:223-244) and
// Core (primary/src/core.rs:349-389).  Core verifies one message at a time;
// this stage collects pending header/vote signatures, vote batches, whole
// certificates and worker batch digests from any number of producer threads
// and launches them as a few large GPU calls.  Modelled on the reference's
// SignatureService (crypto/src/lib.rs:222-250): a request channel in, a
// per-request reply (here a C callback, which the Rust side maps onto a
// oneshot channel).
//
// Pipeline (double buffering):
//   producers   copy each request straight into the open window (packed by
//               kind: the arrays the engine's batched entry points take)
//   collector   closes the window when `max_batch` items are pending, when
//               the oldest request is `max_delay_us` old, or on flush, and
//               hands it to the backend, which stages it in a free device
//               slot and enqueues its copies and kernels on that slot's
//               stream -- WITHOUT waiting for them; it then collects the next
//               window, which is packed and launched while the previous one
//               is still on the GPU
//   completer   waits for the windows in launch order and answers every
//               request of a window through its callback
// The backend (coa_queue.h) is the HIP one (coa_queue_hip.cpp, two slots
// per opened GPU) or, in the ThreadSanitizer build, a stub.
//
// Metrics (coa_queue_metrics): per-kind request counts, window sizes,
// windows in flight, pending depth, and the submit -> callback wait time of
// every request (mean, max, p50/p99 from a log-spaced histogram) -- the
// numbers needed to tune max_batch / max_delay_us against the serial
// Core::run.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "coa_queue.h"

namespace {

using clock_t_ = std::chrono::steady_clock;

enum Kind : uint8_t { K_VERIFY, K_BATCH, K_CERT, K_DIGEST };

struct Req {
  Kind kind;
  uint32_t idx;  // index among the window's requests of this kind
  coa_verdict_cb cb;
  void* user;
  clock_t_::time_point t0;
};

struct Flight {
  std::unique_ptr<coa_q::Window> w;
  std::vector<Req> reqs;
};

// Wait-time histogram: bucket b covers [2^(b/8), 2^((b+1)/8)) microseconds.
constexpr int HB = 8 * 40;
int wait_bucket(double us) {
  if (us < 1.0) return 0;
  return std::min(HB - 1, (int)(8.0 * std::log2(us)) + 1);
}
double bucket_mid(int b) { return b == 0 ? 0.5 : std::exp2((b - 0.5) / 8.0); }

}  // namespace

struct coa_queue {
  size_t max_batch = 65536;
  std::chrono::microseconds max_delay{500};
  std::unique_ptr<coa_q::Backend> be;

  std::mutex mu;
  std::condition_variable cv;         // collector: requests arrived / flush / stop
  std::condition_variable flight_cv;  // completer: a window was launched / stop
  std::condition_variable idle_cv;    // flush: everything answered
  std::unique_ptr<coa_q::Window> open{new coa_q::Window()};
  std::vector<Req> open_reqs;
  size_t pending = 0;  // items in the open window
  clock_t_::time_point oldest;
  std::deque<Flight> flight;  // launched, not yet answered (launch order)
  size_t busy = 0;            // windows taken by the collector and not yet answered
  bool flush = false, stop = false, collector_done = false;

  // metrics (under mu)
  uint64_t m_requests = 0, m_windows = 0, m_sig = 0, m_batch = 0, m_cert = 0, m_dig = 0;
  uint64_t m_max_window = 0, m_max_in_flight = 0, m_max_pending = 0;
  double m_wait_sum = 0.0, m_wait_max = 0.0;
  uint64_t m_hist[HB] = {};

  std::thread collector, completer;

  void start() {
    open->g_offs.push_back(0);
    open->c_hoff.push_back(0);
    open->c_voff.push_back(0);
    open->d_offs.push_back(0);
    collector = std::thread([this] { collect(); });
    completer = std::thread([this] { answer(); });
  }

  // under mu: a request of `items` items joined the open window
  void arrived(Req r, size_t items) {
    if (pending == 0) oldest = clock_t_::now();
    r.t0 = clock_t_::now();
    open_reqs.push_back(r);
    const bool first = pending == 0;
    pending += items;
    m_max_pending = std::max<uint64_t>(m_max_pending, pending);
    if (first || pending >= max_batch) cv.notify_one();  // arm the deadline / launch a full window
  }

  void collect() {
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      cv.wait(l, [&] { return stop || pending > 0; });
      if (pending == 0) break;  // stop with nothing pending
      // window is open: close it when full, at the deadline, on flush or stop
      while (!stop && !flush && pending < max_batch) {
        if (cv.wait_until(l, oldest + max_delay) == std::cv_status::timeout) break;
      }
      Flight f;
      f.w = std::move(open);
      f.reqs.swap(open_reqs);
      m_max_window = std::max<uint64_t>(m_max_window, pending);
      pending = 0;
      flush = false;
      open.reset(new coa_q::Window());
      open->g_offs.push_back(0);
      open->c_hoff.push_back(0);
      open->c_voff.push_back(0);
      open->d_offs.push_back(0);
      busy++;
      l.unlock();
      be->launch(*f.w);  // stages and enqueues; blocks only while every slot is busy
      l.lock();
      m_windows++;
      flight.push_back(std::move(f));
      m_max_in_flight = std::max<uint64_t>(m_max_in_flight, flight.size());
      flight_cv.notify_one();
    }
    collector_done = true;
    flight_cv.notify_one();
  }

  void answer() {
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      flight_cv.wait(l, [&] { return !flight.empty() || collector_done; });
      if (flight.empty()) return;
      Flight f = std::move(flight.front());
      flight.pop_front();
      l.unlock();
      be->complete(*f.w);
      const coa_q::Window& w = *f.w;
      std::vector<double> waits;
      waits.reserve(f.reqs.size());
      for (const Req& r : f.reqs) {
        const auto now = clock_t_::now();
        waits.push_back(std::chrono::duration<double, std::micro>(now - r.t0).count());
        switch (r.kind) {
          case K_VERIFY: r.cb(r.user, w.rc, w.v_out.data() + r.idx, 1); break;
          case K_BATCH: r.cb(r.user, w.rc, w.g_out.data() + r.idx, 1); break;
          case K_CERT: r.cb(r.user, w.rc, w.c_out.data() + r.idx, 1); break;
          case K_DIGEST: r.cb(r.user, w.rc, w.d_out.data() + (size_t)r.idx * 32, 32); break;
        }
      }
      l.lock();
      for (double us : waits) {
        m_wait_sum += us;
        m_wait_max = std::max(m_wait_max, us);
        m_hist[wait_bucket(us)]++;
      }
      m_requests += f.reqs.size();
      m_sig += w.nv;
      m_batch += w.ng;
      m_cert += w.nc;
      m_dig += w.nd;
      busy--;
      if (busy == 0 && pending == 0) idle_cv.notify_all();
    }
  }

  double percentile(double q) const {  // under mu
    uint64_t total = 0;
    for (uint64_t c : m_hist) total += c;
    if (total == 0) return 0.0;
    const double want = q * (double)total;
    uint64_t run = 0;
    for (int b = 0; b < HB; b++) {
      run += m_hist[b];
      if ((double)run >= want) return bucket_mid(b);
    }
    return bucket_mid(HB - 1);
  }
};

extern "C" {

coa_queue* coa_queue_create(size_t max_batch, uint32_t max_delay_us) {
  coa_queue* q = new coa_queue();
  q->max_batch = max_batch ? max_batch : 65536;
  q->max_delay = std::chrono::microseconds(max_delay_us);
  q->be.reset(coa_q::make_backend());
  q->start();
  return q;
}

int coa_queue_submit_verify(coa_queue* q, const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64],
                            coa_verdict_cb cb, void* user) {
  if (!q || !msg || !pk || !sig || !cb) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  coa_q::Window& w = *q->open;
  w.v_msgs.insert(w.v_msgs.end(), msg, msg + 32);
  w.v_pks.insert(w.v_pks.end(), pk, pk + 32);
  w.v_sigs.insert(w.v_sigs.end(), sig, sig + 64);
  q->arrived({K_VERIFY, (uint32_t)w.nv++, cb, user, {}}, 1);
  return COA_OK;
}

int coa_queue_submit_batch(coa_queue* q, const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                           coa_verdict_cb cb, void* user) {
  if (!q || !msg || (n && (!pks || !sigs)) || !cb) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  coa_q::Window& w = *q->open;
  w.g_msgs.insert(w.g_msgs.end(), msg, msg + 32);
  if (n) {
    w.g_pks.insert(w.g_pks.end(), pks, pks + n * 32);
    w.g_sigs.insert(w.g_sigs.end(), sigs, sigs + n * 64);
  }
  w.g_offs.push_back(w.g_offs.back() + n);
  q->arrived({K_BATCH, (uint32_t)w.ng++, cb, user, {}}, n ? n : 1);
  return COA_OK;
}

int coa_queue_submit_certificate(coa_queue* q, const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                                 const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                                 const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, coa_verdict_cb cb,
                                 void* user) {
  if (!q || (header_len && !header_data) || !id || !origin || !header_sig || (n_votes && (!vote_pks || !vote_sigs)) ||
      !cb)
    return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  coa_q::Window& w = *q->open;
  if (header_len) w.c_hdata.insert(w.c_hdata.end(), header_data, header_data + header_len);
  w.c_hoff.push_back(w.c_hdata.size());
  w.c_ids.insert(w.c_ids.end(), id, id + 32);
  w.c_origins.insert(w.c_origins.end(), origin, origin + 32);
  w.c_hsigs.insert(w.c_hsigs.end(), header_sig, header_sig + 64);
  w.c_rounds.push_back(round);
  if (n_votes) {
    w.c_pks.insert(w.c_pks.end(), vote_pks, vote_pks + n_votes * 32);
    w.c_sigs.insert(w.c_sigs.end(), vote_sigs, vote_sigs + n_votes * 64);
  }
  w.c_voff.push_back(w.c_voff.back() + n_votes);
  q->arrived({K_CERT, (uint32_t)w.nc++, cb, user, {}}, 1 + n_votes);
  return COA_OK;
}

int coa_queue_submit_digest(coa_queue* q, const uint8_t* data, size_t len, coa_verdict_cb cb, void* user) {
  if (!q || (len && !data) || !cb) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  if (q->stop) return COA_EINVAL;
  coa_q::Window& w = *q->open;
  if (len) w.d_data.insert(w.d_data.end(), data, data + len);
  w.d_offs.push_back(w.d_data.size());
  q->arrived({K_DIGEST, (uint32_t)w.nd++, cb, user, {}}, 1);
  return COA_OK;
}

int coa_queue_flush(coa_queue* q) {
  if (!q) return COA_EINVAL;
  std::unique_lock<std::mutex> l(q->mu);
  if (q->pending == 0 && q->busy == 0) return COA_OK;
  if (q->pending) {
    q->flush = true;
    q->cv.notify_one();
  }
  q->idle_cv.wait(l, [&] { return q->pending == 0 && q->busy == 0; });
  return COA_OK;
}

int coa_queue_stats(coa_queue* q, uint64_t* launches, uint64_t* items, uint64_t* groups) {
  if (!q) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  if (launches) *launches = q->m_windows;
  if (items) *items = q->m_sig;
  if (groups) *groups = q->m_batch + q->m_cert;
  return COA_OK;
}

int coa_queue_digest_count(coa_queue* q, uint64_t* digests) {
  if (!q || !digests) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  *digests = q->m_dig;
  return COA_OK;
}

int coa_queue_metrics(coa_queue* q, coa_queue_metrics_t* out) {
  if (!q || !out) return COA_EINVAL;
  std::lock_guard<std::mutex> l(q->mu);
  out->requests = q->m_requests;
  out->windows = q->m_windows;
  out->signatures = q->m_sig;
  out->batches = q->m_batch;
  out->certificates = q->m_cert;
  out->digests = q->m_dig;
  out->max_window = q->m_max_window;
  out->max_in_flight = q->m_max_in_flight;
  out->max_pending = q->m_max_pending;
  out->wait_us_mean = q->m_requests ? q->m_wait_sum / (double)q->m_requests : 0.0;
  out->wait_us_p50 = q->percentile(0.50);
  out->wait_us_p99 = q->percentile(0.99);
  out->wait_us_max = q->m_wait_max;
  return COA_OK;
}

int coa_queue_destroy(coa_queue* q) {
  if (!q) return COA_EINVAL;
  coa_queue_flush(q);
  {
    std::lock_guard<std::mutex> l(q->mu);
    q->stop = true;
    q->cv.notify_one();
  }
  q->collector.join();
  q->completer.join();
  delete q;
  return COA_OK;
}

}  // extern "C"
