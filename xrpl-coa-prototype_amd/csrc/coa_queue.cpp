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
//   producers   copy each request into their own intake shard (one per
//               producer thread and queue, packed by kind: the arrays the
//               engine's batched entry points take), under that shard's lock
//               only -- with one shared window, eight producers contended
//               down to ~1 M requests/s against ~4 M/s for one
//               (tools/queue_probe.c)
//   collector   closes the window when `max_batch` items are pending, when
//               the oldest request is `max_delay_us` old, or on flush, takes
//               every shard's requests into it (the first by swapping, the
//               others appended with their indices rebased) and hands it to
//               the backend, which stages it in a free device
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
#include <atomic>
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
  uint32_t n = 1;  // K_VERIFY: consecutive signatures of the request
};

struct Flight {
  std::unique_ptr<coa_q::Window> w;
  std::vector<Req> reqs;
};

// One producer thread's intake for one queue.
struct Shard {
  std::mutex mu;
  std::unique_ptr<coa_q::Window> w{new coa_q::Window()};
  std::unique_ptr<coa_q::Window> next;  // a reset window for the next swap
  std::vector<Req> reqs;
  size_t items = 0;
  Shard() { w->reset(); }
};

template <class T>
void append(std::vector<T>& dst, const std::vector<T>& src) {
  dst.insert(dst.end(), src.begin(), src.end());
}
// offsets array src (starting at 0) appended after dst's last entry
void append_offs(std::vector<uint64_t>& dst, const std::vector<uint64_t>& src) {
  const uint64_t base = dst.back();
  for (size_t i = 1; i < src.size(); i++) dst.push_back(base + src[i]);
}

// Window `src` with requests `reqs` joins window `dst` with requests `dreqs`.
void merge(coa_q::Window& dst, std::vector<Req>& dreqs, const coa_q::Window& src, const std::vector<Req>& reqs) {
  const uint32_t bv = (uint32_t)dst.nv, bg = (uint32_t)dst.ng, bc = (uint32_t)dst.nc, bd = (uint32_t)dst.nd;
  append(dst.v_msgs, src.v_msgs);
  append(dst.v_pks, src.v_pks);
  append(dst.v_sigs, src.v_sigs);
  append(dst.g_msgs, src.g_msgs);
  append(dst.g_pks, src.g_pks);
  append(dst.g_sigs, src.g_sigs);
  append_offs(dst.g_offs, src.g_offs);
  append(dst.c_hdata, src.c_hdata);
  append_offs(dst.c_hoff, src.c_hoff);
  append(dst.c_ids, src.c_ids);
  append(dst.c_origins, src.c_origins);
  append(dst.c_hsigs, src.c_hsigs);
  append(dst.c_rounds, src.c_rounds);
  append(dst.c_pks, src.c_pks);
  append(dst.c_sigs, src.c_sigs);
  append_offs(dst.c_voff, src.c_voff);
  append(dst.d_data, src.d_data);
  append_offs(dst.d_offs, src.d_offs);
  dst.nv += src.nv;
  dst.ng += src.ng;
  dst.nc += src.nc;
  dst.nd += src.nd;
  for (Req r : reqs) {
    r.idx += r.kind == K_VERIFY ? bv : r.kind == K_BATCH ? bg : r.kind == K_CERT ? bc : bd;
    dreqs.push_back(r);
  }
}

std::atomic<uint64_t> g_queue_ids{1};

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
  const uint64_t id = g_queue_ids.fetch_add(1);

  std::mutex mu;
  std::condition_variable cv;         // collector: requests arrived / flush / stop
  std::condition_variable flight_cv;  // completer: a window was launched / stop
  std::condition_variable idle_cv;    // flush: everything answered
  std::vector<std::unique_ptr<coa_q::Window>> spare;  // answered windows, recycled (capacity kept)
  std::atomic<int64_t> pend{0};  // items submitted and not yet taken (briefly < 0 while a take races an arrival)
  std::atomic<bool> stop{false};
  clock_t_::time_point oldest;
  std::deque<Flight> flight;  // launched, not yet answered (launch order)
  size_t busy = 0;            // windows taken by the collector and not yet answered
  bool flush = false, collector_done = false;

  std::mutex shards_mu;
  std::vector<std::unique_ptr<Shard>> shards;

  // metrics (under mu, except m_max_pending)
  uint64_t m_requests = 0, m_windows = 0, m_sig = 0, m_batch = 0, m_cert = 0, m_dig = 0;
  uint64_t m_max_window = 0, m_max_in_flight = 0;
  std::atomic<int64_t> m_max_pending{0};
  double m_wait_sum = 0.0, m_wait_max = 0.0;
  uint64_t m_hist[HB] = {};

  std::thread collector, completer;

  void start() {
    collector = std::thread([this] { collect(); });
    completer = std::thread([this] { answer(); });
  }

  // The calling thread's shard (created on its first submission).
  Shard* my_shard() {
    struct Entry {
      uint64_t qid;
      Shard* sh;
    };
    thread_local Entry cache[4] = {};
    thread_local unsigned next_slot = 0;
    for (const Entry& e : cache)
      if (e.qid == id) return e.sh;
    std::lock_guard<std::mutex> l(shards_mu);
    shards.emplace_back(new Shard());
    Shard* sh = shards.back().get();
    cache[next_slot++ & 3] = {id, sh};
    return sh;
  }

  // A request of `items` items joined a shard (its lock released).  Wakes the
  // collector only on the two edges it waits for: the first pending item
  // (arms the deadline) and max_batch reached.
  void arrived(size_t items) {
    const int64_t old = pend.fetch_add((int64_t)items), now_pend = old + (int64_t)items;
    int64_t mx = m_max_pending.load(std::memory_order_relaxed);
    while (now_pend > mx && !m_max_pending.compare_exchange_weak(mx, now_pend, std::memory_order_relaxed)) {
    }
    const bool first = old <= 0 && now_pend > 0;
    const bool crossed = old < (int64_t)max_batch && now_pend >= (int64_t)max_batch;
    if (first || crossed) {
      std::lock_guard<std::mutex> l(mu);
      if (first) oldest = clock_t_::now();
      cv.notify_one();
    }
  }

  // Shards' pending requests into f (the collector, no queue lock): whole
  // shards, starting one shard further each window, until f holds max_batch
  // items; the rest waits for the next window (which the collector then
  // closes at once: pend is still >= max_batch).
  size_t rr = 0;
  void gather(Flight& f) {
    std::vector<Shard*> snap;
    {
      std::lock_guard<std::mutex> l(shards_mu);
      for (auto& s : shards) snap.push_back(s.get());
    }
    const size_t ns = snap.size(), start = ns ? rr++ % ns : 0;
    size_t taken = 0;
    for (size_t k = 0; k < ns && taken < max_batch; k++) {
      Shard* sh = snap[(start + k) % ns];
      std::unique_ptr<coa_q::Window> w;
      std::vector<Req> reqs;
      size_t items;
      {
        std::lock_guard<std::mutex> l(sh->mu);
        if (sh->items == 0) continue;
        w = std::move(sh->w);
        if (sh->next) {
          sh->w = std::move(sh->next);
        } else {
          sh->w.reset(new coa_q::Window());
          sh->w->reset();
        }
        reqs.swap(sh->reqs);
        items = sh->items;
        sh->items = 0;
      }
      pend.fetch_sub((int64_t)items);
      taken += items;
      if (f.reqs.empty()) {  // the first shard's window becomes the launch window
        std::swap(f.w, w);
        f.reqs.swap(reqs);
      } else {
        merge(*f.w, f.reqs, *w, reqs);
      }
      w->reset();
      std::lock_guard<std::mutex> l(sh->mu);
      if (!sh->next) sh->next = std::move(w);
    }
  }

  void collect() {
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      cv.wait(l, [&] { return stop.load() || pend.load() > 0; });
      if (stop.load() && pend.load() <= 0) break;  // stop with nothing pending
      // window is open: close it when full, at the deadline, on flush or stop
      while (!stop.load() && !flush && pend.load() < (int64_t)max_batch) {
        if (cv.wait_until(l, oldest + max_delay) == std::cv_status::timeout) break;
      }
      flush = false;
      busy++;  // before the take: flush must not see pend == 0 and busy == 0 meanwhile
      Flight f;
      if (spare.empty()) {
        f.w.reset(new coa_q::Window());
      } else {
        f.w = std::move(spare.back());
        spare.pop_back();
      }
      f.w->reset();
      l.unlock();
      gather(f);
      l.lock();
      if (f.reqs.empty()) {  // every pending item was taken by an earlier window
        busy--;
        spare.push_back(std::move(f.w));
        if (busy == 0 && pend.load() <= 0) idle_cv.notify_all();
        continue;
      }
      m_max_window = std::max<uint64_t>(m_max_window, f.w->nv + f.w->c_voff.back() + f.w->g_offs.back() + f.w->nd);
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
          case K_VERIFY: r.cb(r.user, w.rc, w.v_out.data() + r.idx, r.n); break;
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
      if (spare.size() < 8) spare.push_back(std::move(f.w));
      busy--;
      if (busy == 0 && pend.load() <= 0) idle_cv.notify_all();
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

// The submissions: the request goes into the calling thread's shard under
// that shard's lock; then the queue's pending count (and, on an edge, the
// collector) learns of it.
#define COA_Q_INTAKE(q)                         \
  Shard* sh = (q)->my_shard();                  \
  std::unique_lock<std::mutex> sl(sh->mu);      \
  if ((q)->stop.load()) return COA_EINVAL;      \
  coa_q::Window& w = *sh->w;

namespace {
void submitted(coa_queue* q, Shard* sh, std::unique_lock<std::mutex>& sl, Req r, size_t items) {
  r.t0 = clock_t_::now();
  sh->reqs.push_back(r);
  sh->items += items;
  sl.unlock();
  q->arrived(items);
}
}  // namespace

int coa_queue_submit_verify(coa_queue* q, const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64],
                            coa_verdict_cb cb, void* user) {
  if (!q || !msg || !pk || !sig || !cb) return COA_EINVAL;
  COA_Q_INTAKE(q)
  w.v_msgs.insert(w.v_msgs.end(), msg, msg + 32);
  w.v_pks.insert(w.v_pks.end(), pk, pk + 32);
  w.v_sigs.insert(w.v_sigs.end(), sig, sig + 64);
  submitted(q, sh, sl, {K_VERIFY, (uint32_t)w.nv++, cb, user, {}}, 1);
  return COA_OK;
}

int coa_queue_submit_verify_many(coa_queue* q, const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, size_t n,
                                 coa_verdict_cb cb, void* user) {
  if (!q || !cb || n == 0 || n > UINT32_MAX || !msgs || !pks || !sigs) return COA_EINVAL;
  COA_Q_INTAKE(q)
  w.v_msgs.insert(w.v_msgs.end(), msgs, msgs + n * 32);
  w.v_pks.insert(w.v_pks.end(), pks, pks + n * 32);
  w.v_sigs.insert(w.v_sigs.end(), sigs, sigs + n * 64);
  Req r{K_VERIFY, (uint32_t)w.nv, cb, user, {}};
  r.n = (uint32_t)n;
  w.nv += n;
  submitted(q, sh, sl, r, n);
  return COA_OK;
}

int coa_queue_submit_batch(coa_queue* q, const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                           coa_verdict_cb cb, void* user) {
  if (!q || !msg || (n && (!pks || !sigs)) || !cb) return COA_EINVAL;
  COA_Q_INTAKE(q)
  w.g_msgs.insert(w.g_msgs.end(), msg, msg + 32);
  if (n) {
    w.g_pks.insert(w.g_pks.end(), pks, pks + n * 32);
    w.g_sigs.insert(w.g_sigs.end(), sigs, sigs + n * 64);
  }
  w.g_offs.push_back(w.g_offs.back() + n);
  submitted(q, sh, sl, {K_BATCH, (uint32_t)w.ng++, cb, user, {}}, n ? n : 1);
  return COA_OK;
}

int coa_queue_submit_certificate(coa_queue* q, const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                                 const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                                 const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, coa_verdict_cb cb,
                                 void* user) {
  if (!q || (header_len && !header_data) || !id || !origin || !header_sig || (n_votes && (!vote_pks || !vote_sigs)) ||
      !cb)
    return COA_EINVAL;
  COA_Q_INTAKE(q)
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
  submitted(q, sh, sl, {K_CERT, (uint32_t)w.nc++, cb, user, {}}, 1 + n_votes);
  return COA_OK;
}

int coa_queue_submit_digest(coa_queue* q, const uint8_t* data, size_t len, coa_verdict_cb cb, void* user) {
  if (!q || (len && !data) || !cb) return COA_EINVAL;
  COA_Q_INTAKE(q)
  if (len) w.d_data.insert(w.d_data.end(), data, data + len);
  w.d_offs.push_back(w.d_data.size());
  submitted(q, sh, sl, {K_DIGEST, (uint32_t)w.nd++, cb, user, {}}, 1);
  return COA_OK;
}

int coa_queue_flush(coa_queue* q) {
  if (!q) return COA_EINVAL;
  std::unique_lock<std::mutex> l(q->mu);
  if (q->pend.load() <= 0 && q->busy == 0) return COA_OK;
  if (q->pend.load() > 0) {
    q->flush = true;
    q->cv.notify_one();
  }
  q->idle_cv.wait(l, [&] { return q->pend.load() <= 0 && q->busy == 0; });
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
  out->max_pending = (uint64_t)std::max<int64_t>(0, q->m_max_pending.load());
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
