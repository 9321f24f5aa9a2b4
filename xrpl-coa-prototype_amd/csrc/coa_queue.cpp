// Aggregation queue: the pre-verification stage between
// PrimaryReceiverHandler::dispatch (primary/src/primary.rs:223-244) and
// Core (primary/src/core.rs:349-389).  Core verifies one message at a time;
// this stage collects pending header/vote signatures, vote batches, whole
// certificates and worker batch digests from any number of producer threads
// and launches them as a few large GPU calls.  Modelled on the reference's
// SignatureService (crypto/src/lib.rs:222-250): a request channel in, a
// per-request reply (here a C callback, which the Rust side maps onto a
// oneshot channel: rust/crypto/src/service.rs).
//
// Pipeline:
//   producers   copy each request into an intake shard under that shard's
//               lock only.  A queue has a fixed pool of kShards shards; a
//               thread always uses shard (thread ordinal mod kShards), so
//               memory is bounded whatever the number of threads or queues.
//               The queue-wide pending count is told in steps (a shard's
//               first item, then every kReport items), so producers do not
//               share a written cache line per request
//   collector   closes the window when `max_batch` items are pending, when
//               the oldest request is `max_delay_us` old, on flush, or --
//               with COA_QUEUE_IDLE_LAUNCH=k -- as soon as fewer than k
//               windows are in flight (a lone request on an idle device
//               launches at once; under load the arrivals still coalesce
//               behind the windows in flight), takes
//               every non-empty shard's window (a swap per shard -- the
//               parts are never merged on the host: the backend packs them
//               straight into its pinned staging) and hands the parts to the
//               backend, which enqueues their copies and kernels on a free
//               device slot's stream WITHOUT waiting; it then collects the
//               next window, which is packed and launched while the previous
//               one is still on the GPU
//   completer   waits for the launches in order and answers every request
//               through its callback.  A failed launch is retried on the
//               backend's recovery context of each device in turn (its slot
//               rebuilt meanwhile); only when every attempt failed do the
//               callbacks get the engine error -- the reference's verify
//               never fails for a reason other than the signature, and
//               Core::run logs every error and continues
//               (primary/src/core.rs:390-398).
// Lanes: all of the above exists twice -- one lane for signatures, vote
// batches and certificates, one for worker-batch digests -- each with its own
// shards, collector, backend slots and completer.  A digest window is a 14 ms
// serial SHA-512 chain per batch; in a shared window, slot or completion
// order it would hold every verdict behind it for that long.
// The backend (coa_queue.h) is the HIP one (coa_queue_hip.cpp) or, in the
// sanitizer and CPU tests, a stub.
//
// Metrics (coa_queue_metrics): per-kind request counts, window sizes,
// windows in flight, pending depth, retried / recovered / failed windows, the
// submit -> callback wait time of every request (mean, max, p50/p99 from a
// log-spaced histogram), and where a tail comes from: the slowest window's
// launch -> completion time with its size and kinds, the longest wait for a
// free slot, staging reallocations -- the numbers needed to tune max_batch /
// max_delay_us against the serial Core::run.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "coa_queue.h"

namespace {

using coa_q::Launch;
using coa_q::Window;

enum Kind : uint8_t { K_VERIFY, K_BATCH, K_CERT, K_DIGEST };

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#else
  std::this_thread::yield();
#endif
}

inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Req {
  coa_verdict_cb cb;
  void* user;
  int64_t t0;      // submission time, ns
  uint32_t idx;    // index among the part's requests of this kind
  uint32_t n;      // K_VERIFY: consecutive signatures of the request
  Kind kind;
};

constexpr size_t kShards = 64;  // intake shards per queue
// bounded spins around a shard's lock: the collector's pause-spin on try_lock
// before it yields between tries (~tens of microseconds), and a producer's
// yields to a `taking` collector before it queues on the lock anyway
constexpr int kGatherSpins = 4096;
constexpr int kTakingYields = 2000;
constexpr size_t kReport = 64;  // a shard tells the pending count every kReport items
constexpr size_t kSpares = 4;   // recycled windows kept per shard

// One intake shard.  `reported` is the part of `items` already added to the
// queue's pending count.
struct alignas(64) Shard {
  std::mutex mu;
  // set while the collector waits to take the shard: a producer submitting
  // in a tight loop re-takes the (unfair) mutex within nanoseconds of
  // releasing it, and a round-4 take waited 60-310 us per window for a gap;
  // producers hold off while it is set, so a take waits for one copy at most
  std::atomic<bool> taking{false};
  std::unique_ptr<Window> w;
  std::vector<Req> reqs;
  size_t items = 0, reported = 0;
  // recycled windows and request vectors for the next takes (capacity kept):
  // up to kSpares each, because with several windows in flight a shard's
  // windows come back later than it needs the next one -- a fresh Window
  // grows its vectors from nothing, on new pages (round 4's streamed C3:
  // producers copied at ~3 GB/s, the collector's take cost 60-190 us)
  std::vector<std::unique_ptr<Window>> spares;
  std::vector<std::vector<Req>> spare_reqs;
};

// One shard's requests inside a launch.
struct Part {
  std::unique_ptr<Window> w;
  std::vector<Req> reqs;
  uint32_t shard;
};

struct Flight {
  std::vector<Part> parts;
  Launch L;
  int64_t t_launch = 0;  // ns, when the collector handed the window to the backend
};

// A part's requests the backend left open (Window::c_defer, g_defer), with
// the part's window (moved out of the flight, not recycled): the resolver
// thread decides them and answers their callbacks.
struct Deferred {
  std::unique_ptr<Window> w;
  std::vector<Req> reqs;
  uint32_t shard;  // the window goes back to this shard's pool once answered
};

inline bool is_deferred(const Req& r, const Window& w) {
  return (r.kind == K_CERT && w.is_deferred_cert(r.idx)) || (r.kind == K_BATCH && w.g_defer);
}

std::atomic<uint64_t> g_queue_ids{1};
std::atomic<uint32_t> g_thread_ord{0};

uint32_t thread_ordinal() {
  static thread_local const uint32_t ord = g_thread_ord.fetch_add(1, std::memory_order_relaxed);
  return ord;
}

// Wait-time histogram: bucket 0 is < 1 us; bucket 8e + m + 1 covers
// [2^e (1 + m/8), 2^e (1 + (m+1)/8)) microseconds (the exponent and the top
// three mantissa bits of the double: no log per request).
constexpr int HB = 8 * 40;
int wait_bucket(double us) {
  if (!(us >= 1.0)) return 0;
  uint64_t bits;
  std::memcpy(&bits, &us, 8);
  const int e = (int)((bits >> 52) & 0x7ff) - 1023, m = (int)((bits >> 49) & 7);
  return std::min(HB - 1, 8 * e + m + 1);
}
double bucket_mid(int b) {
  if (b == 0) return 0.5;
  const int e = (b - 1) / 8, m = (b - 1) % 8;
  return std::ldexp(1.0 + (m + 0.5) / 8.0, e);
}

// Callback helpers: the completion thread answers a large launch together
// with kHelpers threads, each taking contiguous runs of requests (a launch
// of 10^5 single signatures is 10^5 callbacks: on one thread they, not the
// GPU, set the queue's rate).  Launches still complete in order: the next
// one starts only when every run of this one has been answered.
constexpr int kHelpersDefault = 3;         // COA_QUEUE_HELPERS overrides (0..15; read at queue creation)
constexpr size_t kParallelAnswer = 8192;  // requests per launch from which the helpers join
constexpr size_t kRun = 4096;             // requests per run

// True on the queue's own completion, helper and resolver threads: a
// callback that submits must not launch from there (a launch can wait for a
// free slot, and only those threads free slots).
thread_local bool t_queue_thread = false;

struct AnswerPool {
  std::mutex m;
  std::condition_variable cv, done_cv;
  std::function<void(size_t)> job;
  size_t runs = 0, next = 0, done = 0;
  uint64_t gen = 0;
  bool stop = false;
  std::vector<std::thread> th;

  void start(int n) {
    for (int i = 0; i < n; i++)
      th.emplace_back([this] {
        t_queue_thread = true;
        loop();
      });
  }
  ~AnswerPool() {
    {
      std::lock_guard<std::mutex> l(m);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  // Runs f(0..n-1) on the helpers and the calling thread; returns when all ran.
  void run(size_t n, std::function<void(size_t)> f) {
    {
      std::lock_guard<std::mutex> l(m);
      job = std::move(f);
      runs = n;
      next = 0;
      done = 0;
      gen++;
    }
    cv.notify_all();
    work();
    std::unique_lock<std::mutex> l(m);
    done_cv.wait(l, [&] { return done == runs; });
    job = nullptr;
  }

 private:
  // takes runs until none is left (caller or helper)
  void work() {
    for (;;) {
      size_t i;
      std::function<void(size_t)>* f;
      {
        std::lock_guard<std::mutex> l(m);
        if (next >= runs) return;
        i = next++;
        f = &job;
      }
      (*f)(i);
      std::lock_guard<std::mutex> l(m);
      if (++done == runs) done_cv.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return stop || (gen != seen && next < runs); });
        if (stop) return;
        seen = gen;
      }
      work();
    }
  }
};

// One lane of a queue: intake shards, collector, backend slots, completer.
struct Lane {
  size_t max_batch = 65536;
  // A window closed while every slot is busy waits for a slot first; if a
  // backlog of at least backlog_min windows (of max_batch items) built up
  // meanwhile, the window takes up to backlog_batch items of it instead of
  // max_batch.  Round 6's paced C3 stream (max_batch 16,384: windows of ~240
  // certificates) was slot-bound at ~2.4 M certificates/s, so 3 M/s offered
  // built a backlog (p99 7.4-8.7 ms); with backlog windows of 32,768 items
  // it keeps up (2.93 M/s achieved, p99 1.5-1.7 ms, profiles/
  // r06_backlog_ab.txt).  Windows grown further (65,536) serialise the
  // backlog on one slot's quarter of the CUs and fell behind again (2.2-2.7
  // M/s); grown at a backlog of one window they raised the 2 M/s p99 from
  // 0.86 to 1.5-5.9 ms.  COA_QUEUE_BACKLOG_BATCH (read at creation; 0 = off)
  // and COA_QUEUE_BACKLOG_MIN override; default min(2 x max_batch, 65,536)
  // (never below max_batch) on the verify lane, off on the digest lane.
  size_t backlog_batch = 65536;
  double backlog_min = 2.0;
  size_t reserve_items = 131072;  // Window::reserve_for's items (coa_queue_create)
  bool digest_lane = false;
  std::atomic<bool> prepared{false};  // slots' streams and staging set up (coa_queue_create or the first window)
  std::chrono::microseconds max_delay{500};
  std::unique_ptr<coa_q::Backend> be;
  std::unique_ptr<Shard[]> shards{new Shard[kShards]};

  std::mutex mu;
  std::condition_variable cv;         // collector: requests arrived / flush / stop
  std::condition_variable flight_cv;  // completer: a window was launched / stop
  std::condition_variable idle_cv;    // flush: everything answered
  std::condition_variable resolve_cv; // resolver: open requests deferred / stop
  std::atomic<int64_t> pend{0};  // reported items not yet taken (briefly < 0 while a take races a report)
  std::atomic<bool> stop{false};
  std::chrono::steady_clock::time_point oldest;
  std::deque<Flight> flight;  // launched, not yet answered (launch order)
  size_t busy = 0;            // windows taken by the collector and not yet answered
  bool flush = false, collector_done = false;
  int collectors_live = 0;  // collector threads not yet exited
  std::deque<Deferred> open;  // deferred parts waiting for the resolver
  size_t resolving = 0;       // deferred parts not yet answered (queued or in a pass)
  bool resolver_stop = false;
  bool idle() const { return pend.load() <= 0 && busy == 0 && resolving == 0; }

  // metrics (under mu, except m_max_pending)
  uint64_t m_requests = 0, m_windows = 0, m_sig = 0, m_batch = 0, m_cert = 0, m_dig = 0;
  uint64_t m_max_window = 0, m_max_in_flight = 0;
  uint64_t m_retried = 0, m_recovered = 0, m_failed = 0;
  std::atomic<int64_t> m_max_pending{0};
  double m_wait_sum = 0.0, m_wait_max = 0.0;
  uint64_t m_hist[HB] = {};
  // the slowest window (launch call -> outputs in host memory) and the
  // longest wait for a free slot
  double m_window_us_max = 0.0, m_slot_wait_us_max = 0.0;
  uint64_t m_window_max_items = 0;
  int64_t m_epoch_ns = now_ns();  // creation or the last reset_metrics
  double m_window_max_at_ms = 0.0, m_window_max_dev_us = 0.0;
  uint32_t m_window_max_kinds = 0;
  uint64_t m_deferred = 0, m_passes = 0;
  double m_resolve_us_max = 0.0;
  double m_stage_us[COA_QSTAGES] = {};

  // COA_QUEUE_COLLECTORS (1..4, default 2; read at creation): collector
  // threads.  A window's pack (its requests' bytes into the slot's
  // page-locked staging, ~13 MB for a streamed C3 window) runs on the thread
  // that closed the window, so with one collector the next window could not
  // be gathered until that pack was done: the streamed C3 path's bound
  // (gather + pack + enqueue ~300 us per window of ~1,300 certificates, one
  // thread).  A second collector closes and packs the next window meanwhile.
  std::vector<std::thread> collectors;
  std::thread completer, resolver;
  std::mutex prep_mu;  // one prepare() (cold lane) at a time
  AnswerPool helpers;  // started lazily by the first large launch
  int n_helpers = kHelpersDefault;
  bool helpers_on = false;
  // COA_QUEUE_IDLE_LAUNCH (read at creation; 0 = off, the default): a window
  // closes at once while fewer than this many windows are in flight
  size_t idle_launch = 0;
  // With idle launch, a request that finds the engine idle is launched by
  // the submitting thread itself (COA_QUEUE_DIRECT=0: by the collector, as
  // before): no wake-up of the collector thread on a lone request's path
  bool direct_ok = true;
  std::mutex gather_mu;  // one gather at a time (the collector, or a submitter launching directly)
  double trace_slow_us = 0;  // COA_QUEUE_TRACE_SLOW_US (read at creation): report slower windows on stderr

  Lane() {
    for (size_t i = 0; i < kShards; i++) {
      shards[i].w.reset(new Window());
      shards[i].w->reset();
    }
  }

  void start() {
    int n = 2;
    if (const char* e = getenv("COA_QUEUE_COLLECTORS")) n = std::max(1, std::min(4, atoi(e)));
    collectors_live = n;
    for (int i = 0; i < n; i++) collectors.emplace_back([this] { collect(); });
    completer = std::thread([this] { answer(); });
    resolver = std::thread([this] { resolve_loop(); });
  }

  // The calling thread's shard, locked into `sl`; a shard whose window already
  // holds max_batch items sends the request on to the next one (the
  // collector takes whole shards, so one busy producer thread would otherwise
  // build a window of any size behind a backlog: 254,184 items of streamed
  // certificates, 920 worker batches at 4,000 batches/s).  The last shard
  // tried takes the overflow.
  Shard& intake(std::unique_lock<std::mutex>& sl) {
    const size_t home = thread_ordinal() % kShards;
    for (size_t k = 0;; k++) {
      Shard& sh = shards[(home + k) % kShards];
      // the collector is taking this shard: let it have the lock first (a
      // producer that takes it back at once starves the collector: a bounded
      // pause-spin here cut the 1-producer C3 stream from 3.7 to 1.2 M/s), by
      // yielding -- bounded, so a descheduled collector cannot park the
      // shard's producers for long
      for (int y = 0; y < kTakingYields && sh.taking.load(std::memory_order_acquire); y++) std::this_thread::yield();
      sl = std::unique_lock<std::mutex>(sh.mu);
      if (sh.items < max_batch || k + 1 == kShards) return sh;
    }
  }

  // `items` more items were reported by a shard (its lock released).  Wakes
  // the collector only on the two edges it waits for: the first pending item
  // (arms the deadline) and max_batch reached.
  void arrived(size_t items) {
    const int64_t old = pend.fetch_add((int64_t)items), now_pend = old + (int64_t)items;
    int64_t mx = m_max_pending.load(std::memory_order_relaxed);
    while (now_pend > mx && !m_max_pending.compare_exchange_weak(mx, now_pend, std::memory_order_relaxed)) {
    }
    const bool first = old <= 0 && now_pend > 0;
    const bool crossed = old < (int64_t)max_batch && now_pend >= (int64_t)max_batch;
    if (first || crossed) {
      std::unique_lock<std::mutex> l(mu);
      if (first) oldest = std::chrono::steady_clock::now();
      // idle launch on an idle engine: this thread takes the window and
      // launches it at once (the collector's wake-up was most of a lone
      // request's queueing at low rates, where its thread has gone to sleep)
      if (first && direct_ok && !t_queue_thread && busy < idle_launch && busy < (size_t)be->slots() && !stop.load() &&
          !flush && prepared.load() && pend.load() > 0) {
        busy++;
        launch_window(l);
        return;
      }
      cv.notify_one();
    }
  }

  // Non-empty shards' windows into f (the collector, no queue lock): whole
  // shards, starting one shard further each window, until f holds `cap`
  // items (max_batch, or backlog_batch after a wait for a slot); the rest waits for the next window (which the collector then
  // closes at once: pend is still >= max_batch).
  size_t rr = 0;
  void gather(Flight& f, size_t cap) {
    const size_t start = rr++ % kShards;
    size_t taken = 0;
    for (size_t k = 0; k < kShards && taken < cap; k++) {
      const uint32_t si = (uint32_t)((start + k) % kShards);
      Shard& sh = shards[si];
      Part p;
      size_t items, rep;
      {
        // spin, not sleep: the holder is inside one copy and will not re-take
        // the lock while `taking` is set (a futex sleep here cost a scheduling
        // round trip per shard under load) -- for a bounded number of tries,
        // then yield between tries: gather may run on a submitting thread
        // (direct launch), which must not burn a core while the holder is
        // descheduled.  Never a blocking lock(): a producer that got the
        // mutex back first would starve the collector
        sh.taking.store(true, std::memory_order_release);
        for (int spin = 0; !sh.mu.try_lock(); spin++) {
          if (spin < kGatherSpins)
            cpu_relax();
          else
            std::this_thread::yield();
        }
        std::lock_guard<std::mutex> l(sh.mu, std::adopt_lock);
        sh.taking.store(false, std::memory_order_release);
        if (sh.items == 0) continue;
        p.w = std::move(sh.w);
        p.reqs.swap(sh.reqs);
        if (!sh.spares.empty()) {
          sh.w = std::move(sh.spares.back());
          sh.spares.pop_back();
        } else {
          sh.w.reset(new Window());
          sh.w->reset();
        }
        if (!sh.spare_reqs.empty()) {
          sh.reqs.swap(sh.spare_reqs.back());
          sh.spare_reqs.pop_back();
        }
        items = sh.items;
        rep = sh.reported;
        sh.items = sh.reported = 0;
      }
      pend.fetch_sub((int64_t)rep);
      taken += items;
      p.shard = si;
      f.parts.push_back(std::move(p));
    }
    f.L.parts.clear();
    for (Part& p : f.parts) {
      p.w->bind();
      f.L.parts.push_back(p.w.get());
      f.L.stage_ns[COA_QSTAGE_INTAKE] += p.w->intake_ns;
    }
    f.L.tally();
  }

  void collect() {
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      cv.wait(l, [&] { return stop.load() || pend.load() > 0; });
      if (stop.load() && pend.load() <= 0) break;  // stop with nothing pending
      // window is open: close it when full, at the deadline, on flush or
      // stop, or (idle launch) while fewer than idle_launch windows are in
      // flight -- the completer wakes the collector when one is answered
      while (!stop.load() && !flush && pend.load() < (int64_t)max_batch && busy >= idle_launch) {
        if (cv.wait_until(l, oldest + max_delay) == std::cv_status::timeout) break;
      }
      flush = false;
      busy++;  // before the take: flush must not see pend == 0 and busy == 0 meanwhile
      launch_window(l);
    }
    if (--collectors_live == 0) {  // the last collector out (under mu)
      collector_done = true;
      flight_cv.notify_one();
    }
  }

  // Takes the pending requests as one window and launches it: the collector,
  // or (idle launch) a submitting thread that found the engine idle.  Called
  // with `l` holding mu and busy already counting the window; returns with
  // `l` held.
  void launch_window(std::unique_lock<std::mutex>& l) {
    Flight f;
    l.unlock();
    // every slot busy: wait for one before taking the window, which grows to
    // backlog_batch items if a backlog built up meanwhile (see backlog_batch)
    size_t cap = max_batch;
    const int64_t tw = now_ns();
    if (be->wait_free_slot()) {
      if ((double)pend.load() >= backlog_min * (double)max_batch) cap = backlog_batch;
      f.L.stage_ns[COA_QSTAGE_SLOT_WAIT] += now_ns() - tw;
    }
    const int64_t tg = now_ns();
    {
      std::lock_guard<std::mutex> g(gather_mu);
      gather(f, cap);
    }
    f.L.stage_ns[COA_QSTAGE_GATHER] += now_ns() - tg;
    l.lock();
    if (f.parts.empty()) {  // every pending item was taken by an earlier window
      busy--;
      if (idle()) idle_cv.notify_all();
      return;
    }
    m_max_window = std::max<uint64_t>(m_max_window, f.L.items());
    l.unlock();
    f.L.reset_outputs();
    f.L.attempts = 1;
    f.t_launch = now_ns();
    if (!prepared.load()) {  // a lane COA_QUEUE_LANES left cold: set up by its first window (the collector's)
      std::lock_guard<std::mutex> p(prep_mu);
      if (!prepared.load()) {
        be->prepare(backlog_batch);
        prepared.store(true);
      }
    }
    be->launch(f.L);  // stages and enqueues; blocks only while every slot is busy
    f.L.stage_ns[COA_QSTAGE_SLOT_WAIT] += f.L.slot_wait_ns;
    l.lock();
    m_windows++;
    flight.push_back(std::move(f));
    m_max_in_flight = std::max<uint64_t>(m_max_in_flight, flight.size());
    flight_cv.notify_one();
  }

  // A launch that failed on the device (a HIP error or an allocation
  // failure; not "no device" or bad arguments): retried on the recovery
  // context of each device in turn (the first retry on the next device),
  // until one succeeds.
  static bool recoverable(int rc) { return rc == COA_EHIP || rc == COA_ENOMEM; }
  void recover(Launch& L) {
    const int n = std::max(1, be->devices());
    for (int a = 1; a <= n && recoverable(L.rc); a++) {
      L.reset_outputs();
      L.attempts++;
      be->retry(L, a);
    }
  }

  void answer() {
    t_queue_thread = true;
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      flight_cv.wait(l, [&] { return !flight.empty() || collector_done; });
      if (flight.empty()) return;
      Flight f = std::move(flight.front());
      flight.pop_front();
      l.unlock();
      be->complete(f.L);
      const double window_us = (double)(now_ns() - f.t_launch) * 1e-3;
      if (trace_slow_us > 0 && window_us > trace_slow_us) {  // COA_QUEUE_TRACE_SLOW_US (diagnostics)
        fprintf(stderr,
                "[coa queue] slow window %.0f us at t=%.6f s: %zu items kinds %u slot %d; slot_wait %.0f pack %.0f "
                "enqueue %.0f (pin %.0f h2d %.0f launch %.0f d2h %.0f event %.0f) device_wait %.0f scatter %.0f us\n",
                window_us, (double)f.t_launch * 1e-9, f.L.items(), f.L.kinds(), f.L.slot,
                f.L.stage_ns[COA_QSTAGE_SLOT_WAIT] * 1e-3, f.L.stage_ns[COA_QSTAGE_PACK] * 1e-3,
                f.L.stage_ns[COA_QSTAGE_ENQUEUE] * 1e-3, f.L.enq_ns[Launch::ENQ_PIN] * 1e-3,
                f.L.enq_ns[Launch::ENQ_H2D] * 1e-3, f.L.enq_ns[Launch::ENQ_LAUNCH] * 1e-3,
                f.L.enq_ns[Launch::ENQ_D2H] * 1e-3, f.L.enq_ns[Launch::ENQ_EVENT] * 1e-3,
                f.L.stage_ns[COA_QSTAGE_DEVICE_WAIT] * 1e-3, f.L.stage_ns[COA_QSTAGE_SCATTER] * 1e-3);
      }
      const bool retried = recoverable(f.L.rc);
      if (retried) recover(f.L);
      const int rc = f.L.rc;
      // requests the backend left open go to the resolver, the rest are
      // answered now (a failed window leaves nothing open: every request
      // gets the error)
      bool any_defer = false;
      for (Part& p : f.parts) {
        if (rc != COA_OK) {
          p.w->c_defer.clear();
          p.w->g_defer = false;
        }
        any_defer = any_defer || p.w->deferred();
      }
      const int64_t tcb = now_ns();
      // callbacks, in runs of contiguous requests (helpers join for large
      // launches); wait times from a clock read every 32 requests
      struct Seg {
        const Part* p;
        size_t lo, hi;
      };
      std::vector<Seg> segs;
      size_t nreq = 0;
      for (const Part& p : f.parts) {
        for (size_t lo = 0; lo < p.reqs.size(); lo += kRun) segs.push_back({&p, lo, std::min(p.reqs.size(), lo + kRun)});
        nreq += p.reqs.size();
      }
      struct Tally {
        uint64_t hist[HB] = {};
        double wsum = 0.0, wmax = 0.0;
      };
      std::vector<Tally> tallies(segs.size());
      auto answer_seg = [&](size_t si) {
        const Seg& g = segs[si];
        const Window& w = *g.p->w;
        Tally& t = tallies[si];
        int64_t tnow = now_ns();
        for (size_t k = g.lo; k < g.hi; k++) {
          const Req& r = g.p->reqs[k];
          if (any_defer && is_deferred(r, w)) continue;  // the resolver answers it
          if (((k - g.lo) & 31) == 31) tnow = now_ns();
          const double us = (double)(tnow - r.t0) * 1e-3;
          t.wsum += us;
          t.wmax = std::max(t.wmax, us);
          t.hist[wait_bucket(us)]++;
          switch (r.kind) {
            case K_VERIFY: r.cb(r.user, rc, w.v_out.data() + r.idx, r.n); break;
            case K_BATCH: r.cb(r.user, rc, w.g_out.data() + r.idx, 1); break;
            case K_CERT: r.cb(r.user, rc, w.c_out.data() + r.idx, 1); break;
            case K_DIGEST: r.cb(r.user, rc, w.d_out.data() + (size_t)r.idx * 32, 32); break;
          }
        }
      };
      if (n_helpers > 0 && nreq >= kParallelAnswer && segs.size() > 1) {
        if (!helpers_on) {
          helpers.start(n_helpers);
          helpers_on = true;
        }
        helpers.run(segs.size(), answer_seg);
      } else {
        for (size_t si = 0; si < segs.size(); si++) answer_seg(si);
      }
      f.L.stage_ns[COA_QSTAGE_CALLBACKS] += now_ns() - tcb;
      uint64_t hist[HB] = {};
      double wsum = 0.0, wmax = 0.0;
      for (const Tally& t : tallies) {
        for (int b = 0; b < HB; b++) hist[b] += t.hist[b];
        wsum += t.wsum;
        wmax = std::max(wmax, t.wmax);
      }
      // the open requests, with their windows, for the resolver
      std::vector<Deferred> jobs;
      size_t ndef = 0;
      if (any_defer) {
        for (Part& p : f.parts) {
          if (!p.w->deferred()) continue;
          Deferred d;
          for (const Req& r : p.reqs)
            if (is_deferred(r, *p.w)) d.reqs.push_back(r);
          ndef += d.reqs.size();
          d.w = std::move(p.w);
          d.shard = p.shard;
          jobs.push_back(std::move(d));
        }
      }
      // recycle each part's window (unless the resolver has it) and request
      // vector into its shard
      for (Part& p : f.parts) {
        if (p.w) p.w->reset();
        p.reqs.clear();
        Shard& sh = shards[p.shard];
        std::lock_guard<std::mutex> g(sh.mu);
        if (p.w && sh.spares.size() < kSpares) sh.spares.push_back(std::move(p.w));
        if (sh.spare_reqs.size() < kSpares) sh.spare_reqs.push_back(std::move(p.reqs));
      }
      l.lock();
      for (int b = 0; b < HB; b++) m_hist[b] += hist[b];
      m_wait_sum += wsum;
      m_wait_max = std::max(m_wait_max, wmax);
      m_requests += nreq - ndef;
      for (int k = 0; k < COA_QSTAGES; k++) m_stage_us[k] += (double)f.L.stage_ns[k] * 1e-3;
      m_sig += f.L.nv;
      m_batch += f.L.ng;
      m_cert += f.L.nc;
      m_dig += f.L.nd;
      if (retried) {
        m_retried++;
        if (rc == COA_OK) m_recovered++;
      }
      if (window_us > m_window_us_max) {
        m_window_us_max = window_us;
        m_window_max_items = f.L.items();
        m_window_max_kinds = f.L.kinds();
        m_window_max_at_ms = (double)(f.t_launch - m_epoch_ns) * 1e-6;
        m_window_max_dev_us = (double)f.L.stage_ns[COA_QSTAGE_DEVICE_WAIT] * 1e-3;
      }
      m_slot_wait_us_max = std::max(m_slot_wait_us_max, (double)f.L.slot_wait_ns * 1e-3);
      if (rc != COA_OK) m_failed++;
      if (!jobs.empty()) {
        resolving += jobs.size();
        for (Deferred& d : jobs) open.push_back(std::move(d));
        resolve_cv.notify_one();
      }
      busy--;
      if (idle()) idle_cv.notify_all();
      if (idle_launch && busy < idle_launch && pend.load() > 0) cv.notify_one();
    }
  }

  // The resolver: takes every deferred part queued so far, has the backend
  // decide them in one pass (one engine call per kind for all of them), and
  // answers their callbacks -- off the completion thread, so the windows
  // behind an open certificate are answered while it is being decided.
  void resolve_loop() {
    t_queue_thread = true;
    std::unique_lock<std::mutex> l(mu);
    for (;;) {
      resolve_cv.wait(l, [&] { return !open.empty() || resolver_stop; });
      if (open.empty()) return;
      std::vector<Deferred> jobs;
      while (!open.empty()) {
        jobs.push_back(std::move(open.front()));
        open.pop_front();
      }
      l.unlock();
      const int64_t t0 = now_ns();
      std::vector<Window*> ws;
      for (Deferred& d : jobs) ws.push_back(d.w.get());
      const int rc = be->resolve(ws);
      if (rc != COA_OK) {
        for (Window* w : ws) {  // "failed" outputs with the engine error
          for (uint32_t c : w->c_defer) w->c_out[c] = 7;
          if (w->g_defer) w->g_out.assign(w->ng, 1);
        }
      }
      const int64_t t1 = now_ns();
      uint64_t hist[HB] = {};
      double wsum = 0.0, wmax = 0.0;
      size_t n = 0;
      for (const Deferred& d : jobs) {
        const Window& w = *d.w;
        for (const Req& r : d.reqs) {
          const double us = (double)(now_ns() - r.t0) * 1e-3;
          wsum += us;
          wmax = std::max(wmax, us);
          hist[wait_bucket(us)]++;
          if (r.kind == K_CERT)
            r.cb(r.user, rc, w.c_out.data() + r.idx, 1);
          else
            r.cb(r.user, rc, w.g_out.data() + r.idx, 1);
          n++;
        }
      }
      const int64_t t2 = now_ns();
      for (Deferred& d : jobs) {  // the answered windows back to their shards' pools
        d.w->reset();
        Shard& sh = shards[d.shard];
        std::lock_guard<std::mutex> g(sh.mu);
        if (sh.spares.size() < kSpares) sh.spares.push_back(std::move(d.w));
      }
      l.lock();
      for (int b = 0; b < HB; b++) m_hist[b] += hist[b];
      m_wait_sum += wsum;
      m_wait_max = std::max(m_wait_max, wmax);
      m_requests += n;
      m_deferred += n;
      m_passes++;
      m_resolve_us_max = std::max(m_resolve_us_max, (double)(t1 - t0) * 1e-3);
      m_stage_us[COA_QSTAGE_RESOLVE] += (double)(t1 - t0) * 1e-3;
      m_stage_us[COA_QSTAGE_CALLBACKS] += (double)(t2 - t1) * 1e-3;
      resolving -= jobs.size();
      if (idle()) idle_cv.notify_all();
    }
  }

  void reset_metrics() {
    std::lock_guard<std::mutex> l(mu);
    m_requests = m_windows = m_sig = m_batch = m_cert = m_dig = 0;
    m_max_window = m_max_in_flight = 0;
    m_retried = m_recovered = m_failed = 0;
    m_max_pending.store(0);
    m_wait_sum = m_wait_max = 0.0;
    std::fill(m_hist, m_hist + HB, 0);
    m_window_us_max = m_slot_wait_us_max = 0.0;
    m_window_max_items = 0;
    m_window_max_kinds = 0;
    m_epoch_ns = now_ns();
    m_window_max_at_ms = m_window_max_dev_us = 0.0;
    m_deferred = m_passes = 0;
    m_resolve_us_max = 0.0;
    std::fill(m_stage_us, m_stage_us + COA_QSTAGES, 0.0);
    be->reset_grows();
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
      cv.notify_all();
    }
    for (std::thread& c : collectors) c.join();
    completer.join();
    {
      std::lock_guard<std::mutex> l(mu);
      resolver_stop = true;
      resolve_cv.notify_one();
    }
    resolver.join();
  }

  int flush_all() {
    std::unique_lock<std::mutex> l(mu);
    if (idle()) return COA_OK;
    if (pend.load() > 0) {
      flush = true;
      cv.notify_one();
    }
    idle_cv.wait(l, [&] { return idle(); });
    return COA_OK;
  }
};

double hist_percentile(const uint64_t* hist, double q) {
  uint64_t total = 0;
  for (int b = 0; b < HB; b++) total += hist[b];
  if (total == 0) return 0.0;
  const double want = q * (double)total;
  uint64_t run = 0;
  for (int b = 0; b < HB; b++) {
    run += hist[b];
    if ((double)run >= want) return bucket_mid(b);
  }
  return bucket_mid(HB - 1);
}

}  // namespace

struct coa_queue {
  const uint64_t id = g_queue_ids.fetch_add(1);
  Lane lanes[coa_q::LANES];
  Lane& lane_of(Kind k) { return lanes[k == K_DIGEST ? coa_q::LANE_DIGEST : coa_q::LANE_VERIFY]; }
};

namespace {
void submitted(Lane* q, Shard& sh, std::unique_lock<std::mutex>& sl, Kind kind, uint32_t idx, uint32_t n,
               coa_verdict_cb cb, void* user, size_t items, int64_t t_in) {
  sh.reqs.push_back(Req{cb, user, t_in, idx, n, kind});
  sh.w->intake_ns += now_ns() - t_in;
  sh.items += items;
  size_t delta = 0;
  if (sh.reported == 0 || sh.items - sh.reported >= kReport) {
    delta = sh.items - sh.reported;
    sh.reported = sh.items;
  }
  sl.unlock();
  if (delta) q->arrived(delta);
}

template <size_t N>
inline void put(std::vector<uint8_t>& v, const uint8_t* src) {
  v.insert(v.end(), src, src + N);  // one copy (resize would zero the bytes first)
}
}  // namespace

extern "C" {

coa_queue* coa_queue_create(size_t max_batch, uint32_t max_delay_us) {
  coa_queue* q = new coa_queue();
  for (int k = 0; k < coa_q::LANES; k++) {
    Lane& L = q->lanes[k];
    L.max_batch = max_batch ? max_batch : 65536;
    if (k == coa_q::LANE_DIGEST) {
      // Digest windows hold whole ~500 KB worker batches: at most
      // COA_QUEUE_DIGEST_MAX (default 96, ~49 MB) per window, so a backlog
      // is split over the lane's slots and the staging warmed at creation
      // (2 x 32 MB per slot) is never regrown on the launch path.  Unbounded,
      // a backlog at 4,000 batches/s became windows of up to 920 batches
      // (467 MB) whose page-locked regrowth held a window 218-234 ms.
      const char* e = getenv("COA_QUEUE_DIGEST_MAX");
      const size_t cap = e ? (size_t)std::max(1, atoi(e)) : 96;
      L.max_batch = std::min(L.max_batch, cap);
    }
    L.max_delay = std::chrono::microseconds(max_delay_us);
    L.digest_lane = k == coa_q::LANE_DIGEST;
    // windows reserve their capacity on first use (a shard no producer
    // thread maps to never does): twice max_batch items, capped at 2 x 65,536
    // -- a larger max_batch's windows grow past it on demand
    L.reserve_items = 2 * std::min<size_t>(L.max_batch, 65536);
    L.backlog_batch = k == coa_q::LANE_DIGEST ? L.max_batch
                                              : std::max<size_t>(L.max_batch, std::min<size_t>(2 * L.max_batch, 65536));
    if (const char* e = getenv("COA_QUEUE_BACKLOG_BATCH")) {
      const long long v = atoll(e);
      L.backlog_batch = v <= 0 ? L.max_batch : std::max<size_t>(L.max_batch, (size_t)v);
    }
    if (const char* e = getenv("COA_QUEUE_BACKLOG_MIN")) L.backlog_min = std::max(0.0, atof(e));
    if (const char* e = getenv("COA_QUEUE_HELPERS")) L.n_helpers = std::max(0, std::min(15, atoi(e)));
    if (const char* e = getenv("COA_QUEUE_IDLE_LAUNCH")) L.idle_launch = (size_t)std::max(0, std::min(64, atoi(e)));
    if (const char* e = getenv("COA_QUEUE_DIRECT")) L.direct_ok = e[0] != '0';
    if (const char* e = getenv("COA_QUEUE_TRACE_SLOW_US")) L.trace_slow_us = atof(e);
    L.be.reset(coa_q::make_backend(k));
    // COA_QUEUE_LANES=verify|digest|verify,digest (read at creation; default
    // both): the lanes set up now -- streams, their first dispatch, staging
    // (a verify slot ~23 MB page-locked + ~320 MB of HBM at max_batch 65,536,
    // a digest slot 64 + 64 MB; four verify and eight digest slots per GPU).  A primary that never
    // hashes worker batches, or a worker that never verifies, names its lane;
    // the other is set up by its first window (which then waits ~25-75 ms).
    const char* lanes = getenv("COA_QUEUE_LANES");
    const bool warm = !lanes || std::strstr(lanes, k == coa_q::LANE_DIGEST ? "digest" : "verify") != nullptr;
    if (warm) {
      L.be->prepare(L.backlog_batch);
      L.prepared.store(true);
    }
    L.start();
  }
  return q;
}

// The submissions: the request goes into the calling thread's shard of the
// kind's lane under that shard's lock; then the lane's pending count (and, on
// an edge, its collector) learns of it.
#define COA_Q_INTAKE(q, kind)                                                \
  const int64_t t_in = now_ns();                                             \
  Lane* ln = &(q)->lane_of(kind);                                            \
  std::unique_lock<std::mutex> sl;                                           \
  Shard& sh = ln->intake(sl);                                                \
  if (ln->stop.load()) return COA_EINVAL;                                    \
  Window& w = *sh.w;                                                         \
  if (!w.reserved) w.reserve_for(ln->reserve_items, ln->digest_lane);


int coa_queue_submit_verify(coa_queue* q, const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64],
                            coa_verdict_cb cb, void* user) {
  if (!q || !msg || !pk || !sig || !cb) return COA_EINVAL;
  COA_Q_INTAKE(q, K_VERIFY)
  put<32>(w.v_msgs, msg);
  put<32>(w.v_pks, pk);
  put<64>(w.v_sigs, sig);
  submitted(ln, sh, sl, K_VERIFY, (uint32_t)w.nv++, 1, cb, user, 1, t_in);
  return COA_OK;
}

int coa_queue_submit_verify_many(coa_queue* q, const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, size_t n,
                                 coa_verdict_cb cb, void* user) {
  if (!q || !cb || n == 0 || n > UINT32_MAX || !msgs || !pks || !sigs) return COA_EINVAL;
  COA_Q_INTAKE(q, K_VERIFY)
  w.v_msgs.insert(w.v_msgs.end(), msgs, msgs + n * 32);
  w.v_pks.insert(w.v_pks.end(), pks, pks + n * 32);
  w.v_sigs.insert(w.v_sigs.end(), sigs, sigs + n * 64);
  const uint32_t idx = (uint32_t)w.nv;
  w.nv += n;
  submitted(ln, sh, sl, K_VERIFY, idx, (uint32_t)n, cb, user, n, t_in);
  return COA_OK;
}

int coa_queue_submit_batch(coa_queue* q, const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                           coa_verdict_cb cb, void* user) {
  if (!q || !msg || (n && (!pks || !sigs)) || !cb) return COA_EINVAL;
  COA_Q_INTAKE(q, K_BATCH)
  put<32>(w.g_msgs, msg);
  if (n) {
    w.g_pks.insert(w.g_pks.end(), pks, pks + n * 32);
    w.g_sigs.insert(w.g_sigs.end(), sigs, sigs + n * 64);
  }
  w.g_offs.push_back(w.g_offs.back() + n);
  submitted(ln, sh, sl, K_BATCH, (uint32_t)w.ng++, 1, cb, user, n ? n : 1, t_in);
  return COA_OK;
}

int coa_queue_submit_certificate(coa_queue* q, const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                                 const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                                 const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, coa_verdict_cb cb,
                                 void* user) {
  if (!q || (header_len && !header_data) || !id || !origin || !header_sig || (n_votes && (!vote_pks || !vote_sigs)) ||
      !cb)
    return COA_EINVAL;
  COA_Q_INTAKE(q, K_CERT)
  // one append per field into the window's own buffer; the ref keeps offsets
  // (bind() turns them into pointers at the take)
  std::vector<uint8_t>& o = w.c_own;
  auto at = [&o] { return reinterpret_cast<const uint8_t*>(static_cast<uintptr_t>(o.size())); };
  Window::CertRef r;
  r.hdr = at();
  if (header_len) o.insert(o.end(), header_data, header_data + header_len);
  r.id = at();
  put<32>(o, id);
  r.origin = at();
  put<32>(o, origin);
  r.hsig = at();
  put<64>(o, header_sig);
  r.vpks = at();
  if (n_votes) o.insert(o.end(), vote_pks, vote_pks + n_votes * 32);
  r.vsigs = at();
  if (n_votes) o.insert(o.end(), vote_sigs, vote_sigs + n_votes * 64);
  r.hlen = header_len;
  r.round = round;
  r.nv = n_votes;
  r.owned = true;
  w.c_refs.push_back(r);
  w.c_votes += n_votes;
  w.c_hbytes += header_len;
  submitted(ln, sh, sl, K_CERT, (uint32_t)w.nc++, 1, cb, user, 1 + n_votes, t_in);
  return COA_OK;
}

int coa_queue_submit_certificate_borrowed(coa_queue* q, const uint8_t* header_data, size_t header_len,
                                          const uint8_t id[32], const uint8_t origin[32], const uint8_t header_sig[64],
                                          uint64_t round, const uint8_t* vote_pks, const uint8_t* vote_sigs,
                                          size_t n_votes, coa_verdict_cb cb, void* user) {
  if (!q || (header_len && !header_data) || !id || !origin || !header_sig || (n_votes && (!vote_pks || !vote_sigs)) ||
      !cb)
    return COA_EINVAL;
  COA_Q_INTAKE(q, K_CERT)
  Window::CertRef r;
  r.hdr = header_data;
  r.id = id;
  r.origin = origin;
  r.hsig = header_sig;
  r.vpks = vote_pks;
  r.vsigs = vote_sigs;
  r.hlen = header_len;
  r.round = round;
  r.nv = n_votes;
  r.owned = false;
  w.c_refs.push_back(r);
  w.c_votes += n_votes;
  w.c_hbytes += header_len;
  submitted(ln, sh, sl, K_CERT, (uint32_t)w.nc++, 1, cb, user, 1 + n_votes, t_in);
  return COA_OK;
}

int coa_queue_submit_digest(coa_queue* q, const uint8_t* data, size_t len, coa_verdict_cb cb, void* user) {
  if (!q || (len && !data) || !cb) return COA_EINVAL;
  COA_Q_INTAKE(q, K_DIGEST)
  if (len) w.d_data.insert(w.d_data.end(), data, data + len);
  w.d_offs.push_back(w.d_data.size());
  submitted(ln, sh, sl, K_DIGEST, (uint32_t)w.nd++, 1, cb, user, 1, t_in);
  return COA_OK;
}

int coa_queue_flush(coa_queue* q) {
  if (!q) return COA_EINVAL;
  for (Lane& L : q->lanes) L.flush_all();
  return COA_OK;
}

int coa_queue_set_idle_launch(coa_queue* q, uint32_t windows_in_flight) {
  if (!q || windows_in_flight > 64) return COA_EINVAL;
  for (Lane& L : q->lanes) {
    std::lock_guard<std::mutex> l(L.mu);
    L.idle_launch = windows_in_flight;
    L.cv.notify_one();  // an open window may close now
  }
  return COA_OK;
}

int coa_queue_stats(coa_queue* q, uint64_t* launches, uint64_t* items, uint64_t* groups) {
  if (!q) return COA_EINVAL;
  uint64_t w = 0, it = 0, g = 0;
  for (Lane& L : q->lanes) {
    std::lock_guard<std::mutex> l(L.mu);
    w += L.m_windows;
    it += L.m_sig;
    g += L.m_batch + L.m_cert;
  }
  if (launches) *launches = w;
  if (items) *items = it;
  if (groups) *groups = g;
  return COA_OK;
}

int coa_queue_digest_count(coa_queue* q, uint64_t* digests) {
  if (!q || !digests) return COA_EINVAL;
  Lane& L = q->lanes[coa_q::LANE_DIGEST];
  std::lock_guard<std::mutex> l(L.mu);
  *digests = L.m_dig;
  return COA_OK;
}

int coa_queue_metrics(coa_queue* q, coa_queue_metrics_t* out) {
  if (!q || !out) return COA_EINVAL;
  std::memset(out, 0, sizeof(*out));
  uint64_t hist[HB] = {};
  double wsum = 0.0;
  for (int k = 0; k < coa_q::LANES; k++) {
    Lane& L = q->lanes[k];
    std::lock_guard<std::mutex> l(L.mu);
    out->requests += L.m_requests;
    out->windows += L.m_windows;
    out->signatures += L.m_sig;
    out->batches += L.m_batch;
    out->certificates += L.m_cert;
    out->digests += L.m_dig;
    out->max_window = std::max<uint64_t>(out->max_window, L.m_max_window);
    out->max_in_flight = std::max<uint64_t>(out->max_in_flight, L.m_max_in_flight);
    out->max_pending = std::max<uint64_t>(out->max_pending, (uint64_t)std::max<int64_t>(0, L.m_max_pending.load()));
    for (int b = 0; b < HB; b++) hist[b] += L.m_hist[b];
    wsum += L.m_wait_sum;
    out->wait_us_max = std::max(out->wait_us_max, L.m_wait_max);
    out->retried_windows += L.m_retried;
    out->recovered_windows += L.m_recovered;
    out->failed_windows += L.m_failed;
    if (L.m_window_us_max > out->window_us_max) {
      out->window_us_max = L.m_window_us_max;
      out->window_max_items = L.m_window_max_items;
      out->window_max_kinds = L.m_window_max_kinds;
      out->window_max_at_ms = L.m_window_max_at_ms;
      out->window_max_device_us = L.m_window_max_dev_us;
    }
    out->slot_wait_us_max = std::max(out->slot_wait_us_max, L.m_slot_wait_us_max);
    out->staging_grows += L.be->grows();
    out->stream_kind = std::max(out->stream_kind, (int32_t)L.be->stream_kind());
    (k == coa_q::LANE_DIGEST ? out->slots_digest : out->slots_verify) = (uint32_t)L.be->slots();
    out->deferred_requests += L.m_deferred;
    out->resolver_passes += L.m_passes;
    out->resolve_us_max = std::max(out->resolve_us_max, L.m_resolve_us_max);
    for (int s = 0; s < COA_QSTAGES; s++) out->stage_us[s] += L.m_stage_us[s];
  }
  out->wait_us_mean = out->requests ? wsum / (double)out->requests : 0.0;
  out->wait_us_p50 = hist_percentile(hist, 0.50);
  out->wait_us_p99 = hist_percentile(hist, 0.99);
  return COA_OK;
}

int coa_queue_metrics_reset(coa_queue* q) {
  if (!q) return COA_EINVAL;
  for (Lane& L : q->lanes) L.reset_metrics();
  return COA_OK;
}

int coa_queue_destroy(coa_queue* q) {
  if (!q) return COA_EINVAL;
  coa_queue_flush(q);
  for (Lane& L : q->lanes) L.shutdown();
  delete q;
  return COA_OK;
}

}  // extern "C"
