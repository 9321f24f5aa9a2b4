// Host runtime behind include/coa_verify.h.
//
// * One context per GPU: a non-blocking HIP stream, the fixed-base B table
//   (built on the device by k_build_btable at coa_init), growable device
//   buffers and its own host worker thread ("each GPU has its
//   own host thread, context and streams").  Each context has its own mutex; a
//   shard holds its context's mutex until the context's stream drains.
// * Host-pointer "many" calls shard items by contiguous index range over the
//   opened contexts: every shard runs on its context's worker
//   thread, so the shards' copies, launches and waits proceed concurrently; no
//   cross-GPU exchange, verdict bytes land in place in the caller's output
//   slice.  A call with one shard runs on the caller's thread (no hop).
// * Device-pointer calls enqueue on the caller's stream and return.
// * No CPU fallback anywhere: without a usable GPU, calls fail with
//   COA_ENODEVICE.
#include "../../include/coa_verify.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "coa_batch.h"
#include "coa_msm.h"
#include "coa_committee.h"
#include "coa_halved.h"
#include "coa_kernels.h"
#include "coa_latency.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                              \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return fail(COA_EHIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  // exact: no 25 % growth headroom (multi-GB tables)
  hipError_t ensure(size_t bytes, bool exact = false) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = exact ? bytes : std::max<size_t>(bytes + bytes / 4, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Page-locked host staging (hipHostMalloc), growable: one H2D copy per call
// on the certificate path.
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// True on a context worker thread: nested sharded calls then run inline
// (a worker never waits for its own queue).
thread_local bool t_in_worker = false;

// Result of a task run on another thread: return code + that thread's error.
using TaskResult = std::pair<int, std::string>;

// One host thread per device context, running submitted tasks in order.
class Worker {
 public:
  Worker() : th_([this] { loop(); }) {}
  ~Worker() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  std::future<TaskResult> submit(std::function<int()> f) {
    auto task = std::make_shared<std::packaged_task<TaskResult()>>([f = std::move(f)] {
      g_err.clear();
      const int rc = f();
      return TaskResult(rc, rc == COA_OK ? std::string() : g_err);
    });
    std::future<TaskResult> fut = task->get_future();
    {
      std::lock_guard<std::mutex> l(m_);
      q_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  void loop() {
    t_in_worker = true;
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;  // last: starts after the members above exist
};

// One committee's key tables on one device (f2): sorted keys, flags, a
// radix-256 comb of -A per key and (within the HBM budget) the wide combs.
// Immutable once built and shared by every context open on the device; a
// registration builds the next generation beside it (DevShared).
struct KeySet {
  int dev = -1;
  DevBuf ckeys, kflags, ktabs, kwtabs;
  uint32_t nkeys = 0;
  bool kwide = false;  // kwtabs holds the committee's wide combs
  bool kw20 = false;   // ... in the radix-2^20 layout (COA_KWCOMB20_*)
  KeySet() = default;
  KeySet(const KeySet&) = delete;
  KeySet& operator=(const KeySet&) = delete;
  ~KeySet() {
    if (dev >= 0) (void)hipSetDevice(dev);
    for (DevBuf* b : {&ckeys, &kflags, &ktabs, &kwtabs}) b->release();
  }
};
using KeySetP = std::shared_ptr<const KeySet>;

// What the contexts open on one HIP device share: B's wide comb (8.9 GB,
// built once per device, not once per context) and the current key-cache
// generation.  coa_committee_register builds a new generation on `build`
// (no context's lock, stream or buffers), swaps it in under `mu`, and frees
// the old one once no call or queue window holds it.
struct DevShared {
  int id = -1;
  uint32_t* wcomb = nullptr;  // wide B comb, COA_WCOMB_POS x 2^(W-1) entries (8.9 GB at W = 24)
  hipStream_t build = nullptr;
  std::mutex mu;  // guards `keys`
  KeySetP keys;   // never null while the device is open
  std::mutex reg_mu;  // one registration at a time per device
  // (under reg_mu) a generation's buffers no call holds any more, kept for
  // the next registration: a 65 GB allocation clears its memory on the
  // device, which held live windows back 2.4-7.6 ms (profiles/r04_register_ab.txt)
  std::shared_ptr<KeySet> spare;
  // Generations read by kernels a device-pointer call enqueued on a caller's
  // stream and returned from (the call's own pin is gone): each held until
  // its event completes.  The registrar waits for these instead of a
  // hipDeviceSynchronize, which blocked every other thread's kernel launches
  // for its whole wait (a queue window's launch 13.2 ms, exactly the
  // registrar's sync: profiles/r06_regtrace.txt).
  std::mutex trail_mu;
  std::vector<std::pair<hipEvent_t, KeySetP>> trailing;
  std::vector<hipEvent_t> trail_events;  // completed ones, for reuse
  // (under reg_mu) page-locked staging of the committee's keys: a copy from
  // pageable memory is staged by HIP itself, synchronously
  void* kstage = nullptr;
  size_t kstage_cap = 0;
};

// Host copies split over a few persistent threads: packing a round of
// certificates (68 MB at C3) into page-locked staging runs at one core's
// memcpy rate (~8 GB/s) on one thread -- slower than PCIe.  COA_PACK_THREADS
// (default 8, at most 16) threads including the caller.
class CopyPool {
 public:
  struct Seg {
    void* dst;
    const void* src;
    size_t bytes;
  };
  static CopyPool& get() {
    static CopyPool pool;
    return pool;
  }
  // Copies every segment, pieces of at most kPiece bytes spread over the pool.
  void copy(const std::vector<Seg>& segs) {
    // Below kInline bytes the caller copies alone: waking the pool
    // (notify_all of 7 threads + a done_cv wait) cost one C3 certificate
    // (~10 KB in 7 segments) ~27 us of its 0.12 ms p50 in round 4.
    size_t total = 0;
    for (const Seg& g : segs) total += g.bytes;
    if (total < kInline) {
      for (const Seg& g : segs) std::memcpy(g.dst, g.src, g.bytes);
      return;
    }
    std::vector<Seg> pieces;
    for (const Seg& g : segs)
      for (size_t o = 0; o < g.bytes; o += kPiece)
        pieces.push_back({static_cast<uint8_t*>(g.dst) + o, static_cast<const uint8_t*>(g.src) + o,
                          std::min(kPiece, g.bytes - o)});
    // chunks of consecutive pieces of >= kChunk bytes, claimed with one atomic
    // add each: a queue window of C3 certificates is ~2,000 segments of a few
    // KB, and a mutex per segment made eight threads copy at 3 GB/s
    std::vector<size_t> cuts{0};
    size_t acc = 0;
    for (size_t k = 0; k < pieces.size(); k++) {
      acc += pieces[k].bytes;
      if (acc >= kChunk) {
        cuts.push_back(k + 1);
        acc = 0;
      }
    }
    if (cuts.back() != pieces.size()) cuts.push_back(pieces.size());
    const size_t nchunks = cuts.size() - 1;
    if (nchunks <= 1 || th_.empty()) {
      for (const Seg& g : pieces) std::memcpy(g.dst, g.src, g.bytes);
      return;
    }
    // Several jobs may be in progress at once (two collectors' windows, a
    // host call): each has its own counters, the workers take chunks of the
    // oldest job that has some left, and every caller works on its own job
    // until it is claimed, then waits for the rest of it.  (Round 5 ran one
    // job at a time and a second caller copied alone, at one core's rate.)
    auto job = std::make_shared<Job>();
    job->pieces = pieces.data();
    job->cuts = cuts.data();
    job->n = nchunks;
    {
      std::lock_guard<std::mutex> l(m_);
      jobs_.push_back(job);
    }
    cv_.notify_all();
    work(*job);
    std::unique_lock<std::mutex> l(m_);
    done_cv_.wait(l, [&] { return job->done.load(std::memory_order_acquire) == nchunks; });
    jobs_.erase(std::find(jobs_.begin(), jobs_.end(), job));
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  struct Job {
    const Seg* pieces = nullptr;
    const size_t* cuts = nullptr;  // chunk k = pieces [cuts[k], cuts[k + 1])
    size_t n = 0;                  // chunks
    std::atomic<size_t> next{0}, done{0};
  };
  static constexpr size_t kPiece = 1 << 20;
  static constexpr size_t kChunk = 256 << 10;
  static constexpr size_t kInline = 512 << 10;  // ~50 us of one core's memcpy
  CopyPool() {
    const char* e = getenv("COA_PACK_THREADS");
    const int n = std::max(1, std::min(16, e ? atoi(e) : 8));
    for (int i = 1; i < n; i++) th_.emplace_back([this] { loop(); });
  }
  void work(Job& j) {
    for (;;) {
      const size_t k = j.next.fetch_add(1, std::memory_order_relaxed);
      if (k >= j.n) return;
      for (size_t i = j.cuts[k]; i < j.cuts[k + 1]; i++) std::memcpy(j.pieces[i].dst, j.pieces[i].src, j.pieces[i].bytes);
      if (j.done.fetch_add(1, std::memory_order_acq_rel) + 1 == j.n) {
        std::lock_guard<std::mutex> l(m_);
        done_cv_.notify_all();
      }
    }
  }
  // the oldest job with unclaimed chunks (under m_), or null
  std::shared_ptr<Job> open_job() const {
    for (const auto& j : jobs_)
      if (j->next.load(std::memory_order_relaxed) < j->n) return j;
    return nullptr;
  }
  void loop() {
    for (;;) {
      std::shared_ptr<Job> j;
      {
        // the job is taken by the predicate itself: chunks are claimed without
        // the lock, so a second open_job() here could find none left
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || (j = open_job()) != nullptr; });
        if (stop_) return;
      }
      work(*j);
    }
  }
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::shared_ptr<Job>> jobs_;  // in progress, oldest first
  bool stop_ = false;
  std::vector<std::thread> th_;
};

struct Dev {
  int id = 0;
  DevShared* sh = nullptr;
  std::unique_ptr<Worker> worker;
  hipStream_t stream = nullptr;
  hipStream_t cstreams[3] = {};  // further streams of the pipelined certificate path (created on first use)
  uint32_t* btab = nullptr;  // 128 x (j+1)B, radix-256 fixed-base table (12 KiB)
  uint32_t* comb = nullptr;  // 32 x 128 x (v+1)256^j B comb for k_verify_halved (384 KiB)
  DevBuf msgs, pks, sigs, kbuf, rec, verdicts, scratch, aux, rbuf, seeds, offs, data, out, idx, zs, terms, flags;
  DevBuf cert, cscr;
  DevBuf certc[4], cscrc[4];  // pipelined certificate path: up to four chunks in flight
  PinBuf pinc[4];
  DevBuf msm;  // Pippenger workspace (one large verify_batch group)
  DevBuf lat;  // single-signature latency path: inputs beyond the inline ones
  uint32_t* lat_res = nullptr;  // page-locked result words the latency kernels write
  size_t lat_res_cap = 0;
  uint32_t lat_tag = 0;
  uint32_t* lat_ctr = nullptr;  // device block counter of k_cert_verify_lat (0 between calls)
  PinBuf pin;
  std::mutex mu;
  std::vector<DevBuf*> all() {
    return {&msgs, &pks,  &sigs,  &kbuf, &rec, &verdicts, &scratch,  &aux,     &rbuf,     &seeds,   &offs, &data,
            &out,  &idx,  &zs,    &terms, &flags, &cert,   &cscr,   &certc[0], &certc[1], &certc[2], &certc[3],
            &cscrc[0], &cscrc[1], &cscrc[2], &cscrc[3], &msm, &lat};
  }
};

// COA_VERIFY_IMPL=full selects the full-length k_verify_strict kernel (A/B
// and parity runs; read per call); the default is the halved-scalar path.
bool full_impl() {
  const char* impl = getenv("COA_VERIFY_IMPL");
  return impl && std::string(impl) == "full";
}
bool env_is(const char* name, const char* value) {
  const char* v = getenv(name);
  return v && std::string(v) == value;
}
// The wide comb is built at device open unless COA_WCOMB=0 then; COA_WCOMB=0
// at call time selects the radix-256 comb (A/B runs; read per call).
const uint32_t* wcomb_of(const Dev& d) { return env_is("COA_WCOMB", "0") ? nullptr : d.sh->wcomb; }
// Bytes of HBM the committee's wide key combs may take (COA_KEY_WCOMB_MB,
// default 16 GiB: committees up to 341 keys; 0 disables them).
double key_wcomb_budget() {
  const char* v = getenv("COA_KEY_WCOMB_MB");
  return (v ? atof(v) : 16384.0) * 1048576.0;
}
// Bytes of HBM the radix-2^20 key combs (654 MB per key) of one key-cache
// generation may take on one device (COA_KEY_WCOMB20_MB, default 128 GiB of
// the MI355X's 288 GB: committees up to ~210 keys; 0 disables them).  The
// generation is shared by the device's contexts; while a registration
// builds the next one both are resident for a moment (the new one falls
// back to the radix-2^16 combs, or to none, when that does not fit).
double key_wcomb20_budget() {
  const char* v = getenv("COA_KEY_WCOMB20_MB");
  return (v ? atof(v) : 131072.0) * 1048576.0;
}
// Bytes of HBM the wide key combs of ALL key-cache generations resident on
// one device at once may take (COA_KEY_RESIDENT_MB, default 224 GiB of the
// MI355X's 288 GB, beside B's 8.9 GB comb and the contexts' workspaces): the
// current generation, the one a registration builds beside it, and the
// spare kept for the next registration.  A new generation takes wide combs
// only when they fit beside the current one; a spare is kept only when it
// fits beside the current generation (the per-generation budget
// alone let two 65 GB generations plus a spare approach the HBM size).
double key_resident_budget() {
  const char* v = getenv("COA_KEY_RESIDENT_MB");
  return (v ? atof(v) : 229376.0) * 1048576.0;
}
// COA_VERIFY_WAVES=3 selects the 168-VGPR instance of k_verify_halved.
int verify_waves() {
  const char* w = getenv("COA_VERIFY_WAVES");
  return (w && std::string(w) == "3") ? 3 : 2;
}

std::mutex g_init_mu;
std::vector<std::unique_ptr<Dev>> g_devs;
bool g_inited = false;

// Engine-failure recovery counters (coa_engine_recoveries).
std::atomic<uint64_t> g_ctx_rebuilt{0}, g_shards_rerun{0};

std::vector<std::unique_ptr<DevShared>> g_shared;  // one per opened HIP device id

DevShared* shared_of(int id) {
  for (auto& p : g_shared)
    if (p->id == id) return p.get();
  return nullptr;
}

// The key-cache generation a call or launch on context d reads: the one this
// thread pinned (coa_keycache_use, the aggregation queue's windows) or the
// device's current one.  Holding the returned pointer keeps it alive.
thread_local const KeySetP* t_keys_pinned = nullptr;
KeySetP keys_now(const Dev& d) {
  if (t_keys_pinned && *t_keys_pinned && (*t_keys_pinned)->dev == d.id) return *t_keys_pinned;
  std::lock_guard<std::mutex> l(d.sh->mu);
  return d.sh->keys;
}

// Drops the trailing generations whose kernels have completed (an event in
// error counts as complete: nothing more will read through it).
void reap_trailing(DevShared& sh) {
  std::lock_guard<std::mutex> l(sh.trail_mu);
  for (size_t i = 0; i < sh.trailing.size();) {
    if (hipEventQuery(sh.trailing[i].first) != hipErrorNotReady) {
      sh.trail_events.push_back(sh.trailing[i].first);
      sh.trailing[i] = std::move(sh.trailing.back());
      sh.trailing.pop_back();
    } else {
      i++;
    }
  }
  (void)hipGetLastError();
}

// A device-pointer call that read generation `ks` in kernels it enqueued on
// `s` and returns before they complete: `ks` stays held until they have (an
// event on `s`).  Windows of the aggregation queue pin their generation until
// complete() and need none.  If no event can be recorded, the call waits for
// its stream instead.
int trail_keys(Dev& d, const KeySetP& ks, hipStream_t s) {
  if (t_keys_pinned && *t_keys_pinned) return COA_OK;
  DevShared& sh = *d.sh;
  reap_trailing(sh);
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> l(sh.trail_mu);
    if (!sh.trail_events.empty()) {
      ev = sh.trail_events.back();
      sh.trail_events.pop_back();
    }
  }
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
  if (!ev || hipEventRecord(ev, s) != hipSuccess) {
    if (ev) (void)hipEventDestroy(ev);
    (void)hipGetLastError();
    HIP_TRY(hipStreamSynchronize(s));
    return COA_OK;
  }
  std::lock_guard<std::mutex> l(sh.trail_mu);
  sh.trailing.emplace_back(ev, ks);
  return COA_OK;
}

int open_device(int d) {
  auto dev = std::make_unique<Dev>();
  dev->id = d;
  HIP_TRY(hipSetDevice(d));
  HIP_TRY(hipStreamCreateWithFlags(&dev->stream, hipStreamNonBlocking));
  HIP_TRY(hipMalloc(&dev->btab, COA_BTAB_DWORDS * sizeof(uint32_t)));
  HIP_TRY(coa_launch_build_btable(dev->btab, dev->stream));
  HIP_TRY(hipMalloc(&dev->comb, COA_COMB_DWORDS * sizeof(uint32_t)));
  HIP_TRY(coa_launch_build_comb(dev->comb, dev->btab, dev->stream));
  DevShared* sh = shared_of(d);
  if (!sh) {  // first context on this device: its shared tables
    g_shared.push_back(std::make_unique<DevShared>());
    sh = g_shared.back().get();
    sh->id = d;
    auto empty = std::make_shared<KeySet>();
    empty->dev = d;
    sh->keys = std::move(empty);
    // the wide comb only speeds things up: without the memory for it the
    // radix-256 comb serves every call
    if (!env_is("COA_WCOMB", "0")) {
      if (hipMalloc(&sh->wcomb, COA_WCOMB_DWORDS * sizeof(uint32_t)) == hipSuccess) {
        HIP_TRY(coa_launch_build_wcomb(sh->wcomb, dev->comb, dev->stream));
      } else {
        sh->wcomb = nullptr;
        (void)hipGetLastError();
      }
    }
  }
  dev->sh = sh;
  HIP_TRY(hipStreamSynchronize(dev->stream));
  dev->worker = std::make_unique<Worker>();
  g_devs.push_back(std::move(dev));
  return COA_OK;
}

// Opens the listed devices (ids == nullptr: the first n, n <= 0: all).
int init_locked(const int* ids, int n) {
  if (g_inited) return COA_OK;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0)
    return fail(COA_ENODEVICE, "no HIP device available (this engine has no CPU fallback)");
  std::vector<int> want;
  if (ids) {
    // a device listed k times gets k contexts (k index-range shards on one
    // GPU: rehearses an N-GPU split, e.g. tests/test_gpu_c5.py)
    for (int i = 0; i < n; i++) {
      if (ids[i] < 0 || ids[i] >= count) return fail(COA_EINVAL, "device id out of range");
      want.push_back(ids[i]);
    }
    if (want.empty()) return fail(COA_EINVAL, "empty device list");
  } else {
    if (n <= 0 || n > count) n = count;
    for (int d = 0; d < n; d++) want.push_back(d);
  }
  for (int d : want) {
    const int rc = open_device(d);
    if (rc != COA_OK) {
      g_devs.clear();
      return rc;
    }
  }
  g_inited = true;
  return COA_OK;
}
int init_locked(int n_gpus) { return init_locked(nullptr, n_gpus); }

int ensure_init() {
  std::lock_guard<std::mutex> g(g_init_mu);
  return init_locked(0);
}

Dev* dev_by_id(int device) {
  for (auto& d : g_devs)
    if (d->id == device) return d.get();
  return nullptr;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint32_t verify_lanes(size_t n) {
  const size_t lanes = align_up(std::max<size_t>(n, 1), COA_VERIFY_BLOCK);
  return (uint32_t)std::min<size_t>(lanes, COA_VERIFY_MAX_LANES);
}

struct Range {
  Dev* dev;
  size_t lo, hi;
};

// Items per shard below which a call uses fewer contexts (COA_MIN_SHARD,
// default 65,536 = one lane per item, one wave per SIMD on an MI355X: a
// smaller shard leaves SIMDs idle in the one-wave main kernel, and a call
// spread over every context cannot overlap with another caller's).
size_t min_shard() {
  const char* e = getenv("COA_MIN_SHARD");
  return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)65536;
}
std::atomic<uint32_t> g_shard_rr{0};

// Contiguous index ranges [g*n/G', (g+1)*n/G') over G' of the opened
// contexts: all of them when every shard keeps min_shard() items (a C5 set
// over the 8 GPUs of a node), else n / min_shard() of them (at least one),
// idle ones first, starting one further each call -- so host threads calling
// at once land on different contexts and their calls run side by side.
// `work`: the call's size in the min_shard() unit (signatures; a
// certificate counts its votes too).
std::vector<Range> shard(size_t n, size_t work) {
  std::vector<Range> r;
  const size_t G = g_devs.size();
  const size_t ms = min_shard();
  const size_t want = ms ? std::max<size_t>(1, std::min(G, work / ms)) : G;
  std::vector<Dev*> pick;
  if (want == G) {
    for (auto& d : g_devs) pick.push_back(d.get());
  } else {
    const size_t start = g_shard_rr.fetch_add(1, std::memory_order_relaxed) % G;
    std::vector<bool> taken(G, false);
    for (size_t k = 0; k < G && pick.size() < want; k++) {
      const size_t i = (start + k) % G;
      if (g_devs[i]->mu.try_lock()) {  // idle now
        g_devs[i]->mu.unlock();
        pick.push_back(g_devs[i].get());
        taken[i] = true;
      }
    }
    for (size_t k = 0; k < G && pick.size() < want; k++)
      if (!taken[(start + k) % G]) pick.push_back(g_devs[(start + k) % G].get());
  }
  const size_t P = pick.size();
  for (size_t g = 0; g < P; g++) {
    const size_t lo = n * g / P, hi = n * (g + 1) / P;
    if (hi > lo) r.push_back({pick[g], lo, hi});
  }
  return r;
}

// Workspace layout for n items: k [n][32] | rec [n][128] | scratch [lanes][2 KiB]
struct Workspace {
  uint32_t* k;
  uint32_t* rec;
  uint8_t* flags;  // split path: pre-check verdicts, two bytes (A, R) per item
  uint32_t* ebp;   // split path: [e]B per item (cached form, 128 B)
  uint32_t* scratch;
};
size_t ws_bytes(size_t n) {
  n = std::max<size_t>(n, 1);
  // scratch: per-lane slabs (single-kernel path) or per-item slabs of one
  // split chunk, whichever is larger (the path is chosen per call)
  const size_t slabs = std::max<size_t>(verify_lanes(n), std::min<size_t>(n, COA_SPLIT_CHUNK));
  return align_up(n * 32, 256) + align_up(n * COA_HALVE_REC_BYTES, 256) + align_up(2 * n, 256) + n * 128 +
         slabs * COA_HALVED_SCRATCH_PER_LANE;
}
Workspace ws_carve(void* base, size_t n) {
  n = std::max<size_t>(n, 1);
  uint8_t* p = static_cast<uint8_t*>(base);
  Workspace w;
  w.k = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * 32, 256);
  w.rec = reinterpret_cast<uint32_t*>(p);
  p += align_up(n * COA_HALVE_REC_BYTES, 256);
  w.flags = p;
  p += align_up(2 * n, 256);
  w.ebp = reinterpret_cast<uint32_t*>(p);
  p += n * 128;
  w.scratch = reinterpret_cast<uint32_t*>(p);
  return w;
}

// COA_VERIFY_SPLIT=0 selects the single-kernel k_halve + k_verify_halved path
// (A/B runs; read per call); the default is the split path.
bool split_impl() { return !env_is("COA_VERIFY_SPLIT", "0"); }

// Split path in chunks of at most COA_SPLIT_CHUNK items (one slab each).
// k from d_k, or hashed in k_pre_halve from d_msgs (msg_len bytes per item)
// when d_k is null.  [e]B is summed by k_pre_halve's hash/halving role after
// the halving (that role ends early beside the two decompression roles:
// the 13 comb additions fill its idle tail instead of k_verify_main's lone
// wave); COA_SPLIT_EB=0 leaves it to k_verify_main (A/B, parity tests).
int enqueue_split(Dev& d, const uint8_t* d_msgs, size_t msg_len, const uint32_t* d_k, const uint8_t* d_pks,
                  const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, const Workspace& w, hipStream_t s) {
  for (size_t lo = 0; lo < n; lo += COA_SPLIT_CHUNK) {
    const uint32_t cnt = (uint32_t)std::min<size_t>(COA_SPLIT_CHUNK, n - lo);
    HIP_TRY(coa_launch_verify_split(d_pks + lo * 32, d_sigs + lo * 64, d_k ? nullptr : d_msgs + lo * msg_len,
                                    (uint32_t)msg_len, d_k ? d_k + lo * 8 : nullptr, cnt, w.rec + lo * 32,
                                    w.flags + 2 * lo, d_verdicts + lo, w.scratch,
                                    env_is("COA_SPLIT_EB", "0") ? nullptr : w.ebp, d.comb, wcomb_of(d), s));
  }
  return COA_OK;
}

// Verify with k already in w.k: halved path (k_halve + k_verify_halved) or
// the full-length k_verify_strict.
int enqueue_verify_prehashed(Dev& d, const uint8_t* d_pks, const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts,
                             const uint32_t* d_k, const Workspace& w, hipStream_t s) {
  const uint32_t lanes = verify_lanes(n);
  if (full_impl()) {
    HIP_TRY(coa_launch_verify_strict(d_pks, d_sigs, d_k, (uint32_t)n, d_verdicts, w.scratch, lanes, d.btab, s));
    return COA_OK;
  }
  if (split_impl()) return enqueue_split(d, nullptr, 0, d_k, d_pks, d_sigs, n, d_verdicts, w, s);
  HIP_TRY(coa_launch_halve(d_k, d_sigs, (uint32_t)n, w.rec, s));
  HIP_TRY(coa_launch_verify_halved(d_pks, d_sigs, w.rec, (uint32_t)n, d_verdicts, w.scratch, lanes, d.comb,
                                   wcomb_of(d), verify_waves(), s));
  return COA_OK;
}

// Enqueue k = H(R||A||M) then the verification for device-resident inputs.
int enqueue_verify(Dev& d, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks, const uint8_t* d_sigs,
                   size_t n, uint8_t* d_verdicts, const Workspace& w, hipStream_t s) {
  if (split_impl() && !full_impl() && !env_is("COA_SPLIT_HRAM", "kernel") && (d_msgs || msg_len == 0))
    return enqueue_split(d, d_msgs ? d_msgs : d_pks, msg_len, nullptr, d_pks, d_sigs, n, d_verdicts, w, s);
  HIP_TRY(coa_launch_hram(d_msgs, (uint32_t)msg_len, msg_len, nullptr, d_pks, d_sigs, (uint32_t)n, w.k, s));
  return enqueue_verify_prehashed(d, d_pks, d_sigs, n, d_verdicts, w.k, w, s);
}

// Calls of at most lat_max() signatures with 32-byte messages take the
// single-signature latency kernel (coa_latency.hip, one workgroup per
// signature: faster than the split kernels up to ~2k signatures,
// tools/lat_probe.py); COA_LAT_MAX overrides (0 = never).
size_t lat_max() {
  const char* e = getenv("COA_LAT_MAX");
  return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)2048;
}

// n <= lat_max() triples with 32-byte messages through k_verify_lat on device
// d (its lock held, device set).  Up to COA_LAT_INLINE signatures travel in
// the kernel arguments (no H2D copy); the kernel writes tagged verdict words
// into page-locked host memory and this thread polls for the tag (no D2H copy,
// no stream synchronisation on the latency path).
// Page-locked result words for n items and the call's tag (device d, its
// lock held).
int lat_res_prepare(Dev& d, size_t n, uint32_t& tag) {
  if (n > d.lat_res_cap) {
    if (d.lat_res) (void)hipHostFree(d.lat_res);
    d.lat_res = nullptr;
    d.lat_res_cap = 0;
    const size_t cap = std::max<size_t>(n, 64);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&d.lat_res), cap * 4, hipHostMallocCoherent));
    d.lat_res_cap = cap;
  }
  // the words this call waits for start at 0, which no tag matches: a word
  // left over from an earlier call can never pass for this call's result,
  // however the 24-bit tag wraps
  std::memset(d.lat_res, 0, n * 4);
  d.lat_tag = (d.lat_tag + 1) & 0xffffffu;
  if (d.lat_tag == 0) d.lat_tag = 1;
  tag = d.lat_tag;
  return COA_OK;
}

// The context a latency call runs on: the first idle one (its lock free),
// starting one further on each call; when every context is busy, the next
// one in turn (the call then waits for its lock).  Concurrent one-message
// calls (Core and the two Processors) thus spread over every opened context
// instead of queueing on the first.
std::atomic<uint32_t> g_lat_rr{0};
Dev& lat_dev(std::unique_lock<std::mutex>& lk) {
  const size_t n = g_devs.size();
  const size_t start = g_lat_rr.fetch_add(1, std::memory_order_relaxed) % n;
  for (size_t k = 0; k < n; k++) {
    Dev& d = *g_devs[(start + k) % n];
    std::unique_lock<std::mutex> l(d.mu, std::try_to_lock);
    if (l.owns_lock()) {
      lk = std::move(l);
      return d;
    }
  }
  Dev& d = *g_devs[start];
  lk = std::unique_lock<std::mutex>(d.mu);
  return d;
}

// Waits until the n result words carry `tag` (written by the kernel just
// launched on s); the low byte of each goes to out[i] (out may be null).  A
// kernel that ends without publishing (a fault) ends the wait through the
// stream's status; a bound stops a hang.
int lat_res_wait(Dev& d, hipStream_t s, size_t n, uint32_t tag, uint32_t* out) {
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < n; i++) {
    const volatile uint32_t* w = d.lat_res + i;
    for (uint64_t spin = 0; (*w >> 8) != tag; spin++) {
      if ((spin & 1023) == 1023) {
        const hipError_t q = hipStreamQuery(s);
        if (q != hipSuccess && q != hipErrorNotReady)
          return fail(COA_EHIP, std::string("latency kernel: ") + hipGetErrorString(q));
        if (q == hipSuccess && (*w >> 8) != tag)
          return fail(COA_EHIP, "latency kernel finished without publishing a result");
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
          return fail(COA_EHIP, "latency kernel timed out");
      }
    }
    if (out) out[i] = *w & 0xffu;
  }
  return COA_OK;
}

// msg_of: item i's message is msgs + msg_of[i] * 32 (null: item i's own).
// batch_n: items [0, batch_n) take the verify_batch prefilter (LatArgs::batch_n).
// cd_in / n_cd: Certificate::digest inputs (72 bytes each, LatArgs::cd_in);
// a prefilter item's message is then its certificate's index (first dword).
int lat_verify(Dev& d, const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, size_t n, uint8_t* out,
               const uint32_t* msg_of = nullptr, size_t batch_n = 0, const uint8_t* cd_in = nullptr,
               size_t n_cd = 0) {
  uint32_t tag = 0;
  int rc = lat_res_prepare(d, n, tag);
  if (rc != COA_OK) return rc;
  LatArgs a;
  std::memset(&a, 0, sizeof(a));
  hipStream_t s = d.stream;
  a.n = (uint32_t)n;
  a.batch_n = (uint32_t)batch_n;
  a.n_inline = (uint32_t)std::min<size_t>(n, COA_LAT_INLINE);
  auto msg = [&](size_t i) { return msgs + (msg_of ? (size_t)msg_of[i] : i) * 32; };
  for (size_t i = 0; i < a.n_inline; i++) {
    std::memcpy(&a.inl[i][0], msg(i), 32);
    std::memcpy(&a.inl[i][8], pks + i * 32, 32);
    std::memcpy(&a.inl[i][16], sigs + i * 64, 64);
  }
  // the records past the inline ones, then the certificate digest inputs,
  // through one pinned staging buffer and one H2D
  const size_t rec_end = n > COA_LAT_INLINE ? n * 128 : 0;
  const size_t cd_off = align_up(std::max<size_t>(rec_end, COA_LAT_INLINE * 128), 256);
  const size_t in_bytes = n_cd ? cd_off + n_cd * 72 : rec_end;
  if (in_bytes) {
    HIP_TRY(d.pin.ensure(in_bytes));
    HIP_TRY(d.lat.ensure(in_bytes));
    uint8_t* h = static_cast<uint8_t*>(d.pin.p);
    for (size_t i = COA_LAT_INLINE; i < n; i++) {
      std::memcpy(h + i * 128, msg(i), 32);
      std::memcpy(h + i * 128 + 32, pks + i * 32, 32);
      std::memcpy(h + i * 128 + 64, sigs + i * 64, 64);
    }
    if (n_cd) std::memcpy(h + cd_off, cd_in, n_cd * 72);
    const size_t from = rec_end ? (size_t)COA_LAT_INLINE * 128 : cd_off;
    HIP_TRY(hipMemcpyAsync(d.lat.as<uint8_t>() + from, h + from, in_bytes - from, hipMemcpyHostToDevice, s));
    a.in = d.lat.as<uint32_t>();
    if (n_cd) a.cd_in = reinterpret_cast<const uint32_t*>(d.lat.as<uint8_t>() + cd_off);
  }
  a.tag = tag;
  a.res = d.lat_res;
  const KeySetP ks = keys_now(d);  // held until the verdicts are in
  a.keys = ks->ckeys.as<uint32_t>();
  a.kflags = ks->kflags.as<uint32_t>();
  a.ktabs = ks->ktabs.as<uint32_t>();
  a.nk = ks->nkeys;
  a.comb = d.comb;
  HIP_TRY(coa_launch_verify_lat(a, s));
  std::vector<uint32_t> words(n);
  rc = lat_res_wait(d, s, n, tag, words.data());
  if (rc != COA_OK) return rc;
  for (size_t i = 0; i < n; i++) out[i] = (uint8_t)words[i];
  return COA_OK;
}

int check_n(size_t n) {
  if (n > 0xffffffffull / 2) return fail(COA_EINVAL, "n too large for one call");
  return COA_OK;
}

// Runs tasks that each own one context: concurrently on the contexts' worker
// threads, or inline on this thread when they all use one context (no thread
// hop on the latency path) or when this is already a worker.  Returns the
// first failure (its message in this thread's coa_last_error).
int run_tasks(std::vector<std::pair<Dev*, std::function<int()>>>& tasks) {
  bool one_ctx = true;
  for (auto& t : tasks) one_ctx = one_ctx && t.first == tasks[0].first;
  if (one_ctx || t_in_worker) {
    for (auto& t : tasks) {
      const int rc = t.second();
      if (rc != COA_OK) return rc;
    }
    return COA_OK;
  }
  std::vector<std::future<TaskResult>> futs;
  futs.reserve(tasks.size());
  for (auto& t : tasks) futs.push_back(t.first->worker->submit(t.second));
  int rc = COA_OK;
  std::string msg;
  for (auto& f : futs) {
    TaskResult r = f.get();  // wait for every task: they reference the caller's buffers
    if (r.first != COA_OK && rc == COA_OK) {
      rc = r.first;
      msg = r.second;
    }
  }
  if (rc != COA_OK) g_err = msg;
  return rc;
}

// COA_FAULT_SHARD=<k>: every k-th shard of a sharded call fails with
// COA_EHIP after its work has run (fault injection for the recovery tests;
// never set in production).  COA_FAULT_SHARD=all: every attempt fails,
// re-runs on the other contexts included, so the call itself fails (the
// caller's failure policy is then what answers: tests/test_gpu_recovery.py).
// Read per call.
bool fault_every_attempt() {
  const char* e = getenv("COA_FAULT_SHARD");
  return e && std::strcmp(e, "all") == 0;
}
bool inject_shard_fault() {
  static std::atomic<unsigned long long> count{0};
  if (fault_every_attempt()) return true;
  const char* e = getenv("COA_FAULT_SHARD");
  const unsigned long long every = e ? strtoull(e, nullptr, 10) : 0ull;
  return every && (count.fetch_add(1) + 1) % every == 0;
}

// Rebuilds a context after a HIP failure (its lock held): drains and
// replaces its stream and releases its per-call buffers (they regrow on
// demand).  The fixed-base and committee tables are kept: they were built
// and checked before and no call writes them.  Same process, no exec.
int rebuild_context(Dev& d) {
  (void)hipSetDevice(d.id);
  (void)hipStreamSynchronize(d.stream);
  (void)hipStreamDestroy(d.stream);
  d.stream = nullptr;
  for (hipStream_t& cs : d.cstreams)
    if (cs) {
      (void)hipStreamSynchronize(cs);
      (void)hipStreamDestroy(cs);
      cs = nullptr;
    }
  for (DevBuf* b : d.all()) b->release();  // per-call buffers (the tables live in DevShared)
  (void)hipGetLastError();
  HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  g_ctx_rebuilt++;
  return COA_OK;
}

// Run `body` for every shard with its context's lock held, then drain the
// context's stream.  body(Dev&, lo, hi) enqueues work and returns COA_OK or an
// error.  The shards run concurrently, one per context worker.
// Engine-failure recovery: a shard that fails with a device error
// (COA_EHIP / COA_ENOMEM) has its context rebuilt and is re-run on the next
// contexts in turn (the rebuilt one last); the call fails only when every
// context failed it.  body must therefore be re-runnable for its range: it
// writes only its own slice of the caller's outputs.
template <class F>
int for_shards(size_t n, F body, size_t work = 0) {
  std::vector<std::pair<Dev*, std::function<int()>>> tasks;
  const std::vector<Range> ranges = shard(n, work ? work : n);
  std::vector<int> rcs(ranges.size(), COA_OK);
  std::vector<std::string> msgs(ranges.size());
  auto run_on = [&body](Dev& d, size_t lo, size_t hi, bool inject) -> int {
    std::lock_guard<std::mutex> l(d.mu);
    if (hipSetDevice(d.id) != hipSuccess) return fail(COA_EHIP, "hipSetDevice failed");
    int rc = body(d, lo, hi);
    const hipError_t e = hipStreamSynchronize(d.stream);
    if (e != hipSuccess && rc == COA_OK) rc = fail(COA_EHIP, std::string("stream sync: ") + hipGetErrorString(e));
    if (rc == COA_OK && inject) rc = fail(COA_EHIP, "injected shard fault (COA_FAULT_SHARD)");
    if (rc == COA_EHIP || rc == COA_ENOMEM) (void)rebuild_context(d);
    return rc;
  };
  for (size_t i = 0; i < ranges.size(); i++) {
    const Range r = ranges[i];
    const bool inject = inject_shard_fault();
    tasks.emplace_back(r.dev, [r, inject, i, &rcs, &msgs, &run_on]() -> int {
      rcs[i] = run_on(*r.dev, r.lo, r.hi, inject);
      if (rcs[i] != COA_OK) msgs[i] = g_err;
      // recoverable failures are re-run below, so the other shards finish
      return (rcs[i] == COA_EHIP || rcs[i] == COA_ENOMEM) ? COA_OK : rcs[i];
    });
  }
  int rc = run_tasks(tasks);
  if (rc != COA_OK) return rc;
  for (size_t i = 0; i < ranges.size(); i++) {
    if (rcs[i] == COA_OK) continue;
    size_t at = 0;
    for (size_t g = 0; g < g_devs.size(); g++)
      if (g_devs[g].get() == ranges[i].dev) at = g;
    int r = rcs[i];
    const std::string first = msgs[i];
    for (size_t k = 1; k <= g_devs.size() && (r == COA_EHIP || r == COA_ENOMEM); k++) {
      r = run_on(*g_devs[(at + k) % g_devs.size()], ranges[i].lo, ranges[i].hi, fault_every_attempt());
      g_shards_rerun++;
    }
    if (r != COA_OK) return fail(r, "shard failed on every context: " + first + " / " + g_err);
  }
  return COA_OK;
}

uint64_t os_entropy_seed() {
  std::random_device rd;
  uint64_t s = 0;
  while (s == 0) s = ((uint64_t)rd() << 32) ^ rd();
  return s;
}

// Groups of at least msm_min() signatures take the Pippenger path
// (coa_msm.hip), and so do the groups of a call with at most two; COA_MSM_MIN
// overrides (0 = never).
size_t msm_min() {
  const char* e = getenv("COA_MSM_MIN");
  return e ? (size_t)strtoull(e, nullptr, 10) : (size_t)16384;
}

// One group through the Pippenger kernels, device buffers resident.
// d_zs: caller weights (16 B per signature) or NULL = derive from seed.
int enqueue_msm(Dev& d, const uint8_t* d_msg, const uint8_t* d_pks, const uint8_t* d_sigs, size_t n,
                const uint8_t* d_zs, uint64_t seed, uint32_t group, uint8_t* d_verdict, void* ws_base,
                hipStream_t s) {
  const MsmWs ws = coa_msm_ws_carve(ws_base, n);
  HIP_TRY(coa_launch_hram(d_msg, 32, 0, nullptr, d_pks, d_sigs, (uint32_t)n, ws.k, s));
  if (d_zs) HIP_TRY(hipMemcpyAsync(ws.z, d_zs, n * 16, hipMemcpyDeviceToDevice, s));
  else HIP_TRY(coa_launch_batch_z(ws.k, d_sigs, nullptr, group, (uint32_t)n, seed, ws.z, s));
  HIP_TRY(coa_launch_msm(d_pks, d_sigs, (uint32_t)n, ws, d_verdict, s));
  return COA_OK;
}

// Host-pointer form for one group on device d (lock held by the caller).
int msm_group(Dev& d, const uint8_t* msg, const uint8_t* pks, const uint8_t* sigs, size_t n, const uint8_t* zs_in,
              uint64_t seed, uint32_t group, uint8_t* verdict_out) {
  hipStream_t s = d.stream;
  HIP_TRY(d.msgs.ensure(32));
  HIP_TRY(d.pks.ensure(n * 32 + 32));
  HIP_TRY(d.sigs.ensure(n * 64 + 64));
  HIP_TRY(d.verdicts.ensure(16));
  HIP_TRY(d.msm.ensure(coa_msm_ws_bytes(n)));
  if (zs_in) HIP_TRY(d.zs.ensure(n * 16 + 16));
  HIP_TRY(hipMemcpyAsync(d.msgs.p, msg, 32, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d.pks.p, pks, n * 32, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(d.sigs.p, sigs, n * 64, hipMemcpyHostToDevice, s));
  if (zs_in) HIP_TRY(hipMemcpyAsync(d.zs.p, zs_in, n * 16, hipMemcpyHostToDevice, s));
  const int rc = enqueue_msm(d, d.msgs.as<uint8_t>(), d.pks.as<uint8_t>(), d.sigs.as<uint8_t>(), n,
                             zs_in ? d.zs.as<uint8_t>() : nullptr, seed, group, d.verdicts.as<uint8_t>(), d.msm.p, s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipMemcpyAsync(verdict_out, d.verdicts.p, 1, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}

int batch_groups_impl(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, const uint64_t* group_offsets,
                      size_t n_groups, const uint8_t* zs_in, uint64_t seed, uint8_t* verdicts_out,
                      uint32_t gbase = 0, bool prefilter = true);

// Large groups through the Pippenger path, dealt round-robin to the contexts
// and run concurrently on their workers; runs of small groups through the
// per-vote path (sharded over the contexts) meanwhile.
// gbase: the global index of this call's first group (the z_i hash binds it).
int batch_groups_split(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, const uint64_t* group_offsets,
                       size_t n_groups, const uint8_t* zs_in, uint64_t seed, uint8_t* verdicts_out, size_t mmin,
                       uint32_t gbase) {
  std::vector<std::vector<size_t>> large(g_devs.size());
  std::vector<std::pair<size_t, size_t>> small_runs;
  size_t nlarge = 0;
  for (size_t g = 0; g < n_groups;) {
    size_t e = g;
    while (e < n_groups && group_offsets[e + 1] - group_offsets[e] < mmin) e++;
    if (e > g) {
      small_runs.emplace_back(g, e);
      g = e;
    } else {
      large[nlarge++ % g_devs.size()].push_back(g++);
    }
  }
  std::vector<std::pair<Dev*, std::function<int()>>> tasks;
  for (size_t di = 0; di < g_devs.size(); di++) {
    if (large[di].empty()) continue;
    Dev* d = g_devs[di].get();
    const std::vector<size_t>* mine = &large[di];
    tasks.emplace_back(d, [=]() -> int {
      std::lock_guard<std::mutex> l(d->mu);
      HIP_TRY(hipSetDevice(d->id));
      for (size_t g : *mine) {
        const uint64_t v0 = group_offsets[g], nv = group_offsets[g + 1] - v0;
        const int rc = msm_group(*d, msgs + g * 32, pks + v0 * 32, sigs + v0 * 64, nv,
                                 zs_in ? zs_in + v0 * 16 : nullptr, seed, gbase + (uint32_t)g, verdicts_out + g);
        if (rc != COA_OK) return rc;
      }
      return COA_OK;
    });
  }
  // the large groups go to the workers first when there are several
  // contexts; with one context (or inside a worker) everything runs here
  bool one_ctx = g_devs.size() == 1 || t_in_worker;
  std::vector<std::future<TaskResult>> futs;
  if (!one_ctx)
    for (auto& t : tasks) futs.push_back(t.first->worker->submit(t.second));
  int rc = COA_OK;
  for (auto& r : small_runs) {
    const size_t g = r.first, e = r.second;
    const uint64_t v0 = group_offsets[g];
    std::vector<uint64_t> offs(e - g + 1);
    for (size_t k = 0; k <= e - g; k++) offs[k] = group_offsets[g + k] - v0;
    rc = batch_groups_impl(msgs + g * 32, pks + v0 * 32, sigs + v0 * 64, offs.data(), e - g,
                           zs_in ? zs_in + v0 * 16 : nullptr, seed, verdicts_out + g, gbase + (uint32_t)g, false);
    if (rc != COA_OK) break;
  }
  std::string msg = rc != COA_OK ? g_err : std::string();
  if (one_ctx) {
    if (rc == COA_OK) rc = run_tasks(tasks);
    return rc;
  }
  for (auto& f : futs) {
    TaskResult t = f.get();
    if (t.first != COA_OK && rc == COA_OK) {
      rc = t.first;
      msg = t.second;
    }
  }
  if (rc != COA_OK) g_err = msg;
  return rc;
}

// Calls of at most lat_max() signatures first go through the latency kernel
// as a prefilter (LatArgs::batch): a group whose votes all pass it (verify_strict
// and [l]A == O) is accepted by dalek's batch equation for every z, so its
// verdict is Ok without the batch kernels; the other groups -- some vote
// failing its own equation, a key with torsion, an encoding error -- are
// resolved exactly below, each with its own global group index (the z_i
// derivation binds it).  One launch of one workgroup per vote, the groups'
// votes side by side: ~0.2 ms for one certificate's 67 votes against ~0.4 ms
// through the Pippenger kernels.  COA_BATCH_LAT=0 disables it.
int batch_prefilter(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, const uint64_t* group_offsets,
                    size_t n_groups, uint8_t* verdicts_out, std::vector<uint8_t>& pass) {
  const size_t total = group_offsets[n_groups];
  std::vector<uint32_t> msg_of(total);
  for (size_t g = 0; g < n_groups; g++)
    for (uint64_t i = group_offsets[g]; i < group_offsets[g + 1]; i++) msg_of[i] = (uint32_t)g;
  std::vector<uint8_t> v(total);
  {
    std::unique_lock<std::mutex> l;
    Dev& d = lat_dev(l);
    HIP_TRY(hipSetDevice(d.id));
    const int rc = lat_verify(d, msgs, pks, sigs, total, v.data(), msg_of.data(), total);
    if (rc != COA_OK) return rc;
  }
  pass.assign(n_groups, 1);
  for (size_t g = 0; g < n_groups; g++) {
    for (uint64_t i = group_offsets[g]; i < group_offsets[g + 1]; i++) pass[g] &= v[i] == 0 ? 1 : 0;
    if (pass[g]) verdicts_out[g] = 0;
  }
  return COA_OK;
}

int batch_groups_impl(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs, const uint64_t* group_offsets,
                      size_t n_groups, const uint8_t* zs_in, uint64_t seed, uint8_t* verdicts_out, uint32_t gbase,
                      bool prefilter) {
  if (n_groups == 0) return COA_OK;
  if (!msgs || !group_offsets || !verdicts_out) return fail(COA_EINVAL, "null argument");
  if (group_offsets[0] != 0) return fail(COA_EINVAL, "group_offsets[0] must be 0");
  for (size_t g = 0; g < n_groups; g++)
    if (group_offsets[g + 1] < group_offsets[g]) return fail(COA_EINVAL, "group_offsets not monotone");
  const size_t total = group_offsets[n_groups];
  if (total && (!pks || !sigs)) return fail(COA_EINVAL, "null pks/sigs");
  if (check_n(total) != COA_OK) return COA_EINVAL;
  const uint64_t eff_seed = zs_in ? 0 : (seed ? seed : os_entropy_seed());
  if (prefilter && total > 0 && total <= lat_max() && !env_is("COA_BATCH_LAT", "0")) {
    std::vector<uint8_t> pass;
    int rc = batch_prefilter(msgs, pks, sigs, group_offsets, n_groups, verdicts_out, pass);
    if (rc != COA_OK) return rc;
    // runs of groups the prefilter did not accept, through the exact path
    for (size_t g = 0; g < n_groups;) {
      if (pass[g]) {
        g++;
        continue;
      }
      size_t e = g;
      while (e < n_groups && !pass[e]) e++;
      const uint64_t v0 = group_offsets[g];
      std::vector<uint64_t> offs(e - g + 1);
      for (size_t k = 0; k <= e - g; k++) offs[k] = group_offsets[g + k] - v0;
      rc = batch_groups_impl(msgs + g * 32, pks + v0 * 32, sigs + v0 * 64, offs.data(), e - g,
                             zs_in ? zs_in + v0 * 16 : nullptr, eff_seed, verdicts_out + g, gbase + (uint32_t)g, false);
      if (rc != COA_OK) return rc;
      g = e;
    }
    return COA_OK;
  }
  // One or two groups take the Pippenger path at any size: the per-vote path
  // waits for one lane's whole joint scalar multiplication (~1.4 ms however
  // few groups), the Pippenger kernels spread a group over the chip (~0.5 ms
  // at 67 votes, tools/batch_route_probe.py); from three groups one per-vote
  // launch is faster than the groups one after another.
  size_t mmin = msm_min();
  if (mmin && n_groups <= 2) mmin = 1;
  if (mmin) {
    for (size_t g = 0; g < n_groups; g++)
      if (group_offsets[g + 1] - group_offsets[g] >= mmin)
        return batch_groups_split(msgs, pks, sigs, group_offsets, n_groups, zs_in, eff_seed, verdicts_out, mmin,
                                  gbase);
  }
  // shard by group index (sized by the votes)
  return for_shards(n_groups, [&](Dev& d, size_t glo, size_t ghi) -> int {
    const size_t vlo = group_offsets[glo], vhi = group_offsets[ghi];
    const size_t nv = vhi - vlo, ng = ghi - glo;
    std::vector<uint64_t> offs(ng + 1);
    std::vector<uint32_t> group_of(std::max<size_t>(nv, 1));
    for (size_t g = 0; g <= ng; g++) offs[g] = group_offsets[glo + g] - vlo;
    for (size_t g = 0; g < ng; g++)
      for (uint64_t i = offs[g]; i < offs[g + 1]; i++) group_of[i] = (uint32_t)(glo + g);
    const uint32_t lanes = verify_lanes(nv);
    hipStream_t s = d.stream;
    HIP_TRY(d.msgs.ensure(ng * 32));
    HIP_TRY(d.pks.ensure(nv * 32 + 32));
    HIP_TRY(d.sigs.ensure(nv * 64 + 64));
    HIP_TRY(d.kbuf.ensure(nv * 32 + 32));
    HIP_TRY(d.zs.ensure(nv * 16 + 16));
    HIP_TRY(d.idx.ensure(group_of.size() * 4));
    HIP_TRY(d.offs.ensure((ng + 1) * 8));
    HIP_TRY(d.terms.ensure(nv * 128 + 128));
    HIP_TRY(d.flags.ensure(nv + 16));
    HIP_TRY(d.scratch.ensure((size_t)lanes * COA_BATCH_SCRATCH_PER_LANE));
    HIP_TRY(d.verdicts.ensure(ng + 16));
    HIP_TRY(hipMemcpyAsync(d.msgs.p, msgs + glo * 32, ng * 32, hipMemcpyHostToDevice, s));
    if (nv) {
      HIP_TRY(hipMemcpyAsync(d.pks.p, pks + vlo * 32, nv * 32, hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(d.sigs.p, sigs + vlo * 64, nv * 64, hipMemcpyHostToDevice, s));
    }
    // group ids are relative to this shard's message slice
    for (auto& gid : group_of) gid -= (uint32_t)glo;
    HIP_TRY(hipMemcpyAsync(d.idx.p, group_of.data(), group_of.size() * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.offs.p, offs.data(), (ng + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(coa_launch_hram(d.msgs.as<uint8_t>(), 32, 32, d.idx.as<uint32_t>(), d.pks.as<uint8_t>(),
                            d.sigs.as<uint8_t>(), (uint32_t)nv, d.kbuf.as<uint32_t>(), s));
    if (zs_in) {
      if (nv) HIP_TRY(hipMemcpyAsync(d.zs.p, zs_in + vlo * 16, nv * 16, hipMemcpyHostToDevice, s));
    } else {
      // z derivation binds the global group index: restore it for the hash
      std::vector<uint32_t> gabs(group_of.size());
      for (size_t i = 0; i < group_of.size(); i++) gabs[i] = group_of[i] + (uint32_t)glo + gbase;
      HIP_TRY(hipMemcpyAsync(d.idx.p, gabs.data(), gabs.size() * 4, hipMemcpyHostToDevice, s));
      HIP_TRY(coa_launch_batch_z(d.kbuf.as<uint32_t>(), d.sigs.as<uint8_t>(), d.idx.as<uint32_t>(), 0, (uint32_t)nv,
                                 eff_seed, d.zs.as<uint32_t>(), s));
      HIP_TRY(hipStreamSynchronize(s));  // gabs lifetime
    }
    HIP_TRY(coa_launch_batch_terms(d.pks.as<uint8_t>(), d.sigs.as<uint8_t>(), d.kbuf.as<uint32_t>(),
                                   d.zs.as<uint32_t>(), (uint32_t)nv, d.terms.as<uint32_t>(), d.flags.as<uint8_t>(),
                                   d.scratch.as<uint32_t>(), lanes, d.btab, s));
    HIP_TRY(coa_launch_batch_reduce(d.offs.as<uint64_t>(), (uint32_t)ng, d.terms.as<uint32_t>(),
                                    d.flags.as<uint8_t>(), d.verdicts.as<uint8_t>(), s));
    HIP_TRY(hipMemcpyAsync(verdicts_out + glo, d.verdicts.p, ng, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));  // offs / group_of host vectors die here
    return COA_OK;
  }, group_offsets[n_groups]);
}

// ------------------------------------------------------------------------
// Certificate::verify crypto (f2 + f3).  Inputs of a shard [lo, hi) are
// packed into the device's pinned staging buffer and copied with ONE H2D; the
// status words come back with one D2H.
struct CertIn {
  const uint8_t* hdr_data;
  const uint64_t* hdr_off;
  const uint8_t* ids;
  const uint8_t* origins;
  const uint8_t* hsigs;
  const uint64_t* rounds;
  const uint8_t* vpks;
  const uint8_t* vsigs;
  const uint64_t* voff;
};

// COA_CERT_LANES=1|64 forces the lanes-per-signature variant.
int cert_lanes(size_t jobs) {
  const char* e = getenv("COA_CERT_LANES");
  if (e && std::string(e) == "1") return 1;
  if (e && std::string(e) == "64") return 64;
  return jobs <= 2048 ? 64 : 1;
}

struct CertPack {
  size_t status, hoff, ids, origins, hsigs, rounds, voff, vpks, vsigs, hdata, total;
};
CertPack cert_layout(size_t nc, size_t nv, size_t hbytes) {
  CertPack p;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 256);
    return at;
  };
  p.status = take(nc * 4);
  p.hoff = take((nc + 1) * 8);
  p.ids = take(nc * 32);
  p.origins = take(nc * 32);
  p.hsigs = take(nc * 64);
  p.rounds = take(nc * 8);
  p.voff = take((nc + 1) * 8);
  p.vpks = take(nv * 32);
  p.vsigs = take(nv * 64);
  p.hdata = take(hbytes + 16);
  p.total = o;
  return p;
}

CertArgs cert_args(Dev& d, const KeySet& ks, uint8_t* base, const CertPack& p, size_t nc, size_t nv) {
  CertArgs a;
  a.hdr_data = base + p.hdata;
  a.hdr_off = reinterpret_cast<const uint64_t*>(base + p.hoff);
  a.ids = reinterpret_cast<const uint32_t*>(base + p.ids);
  a.origins = reinterpret_cast<const uint32_t*>(base + p.origins);
  a.hsigs = reinterpret_cast<const uint32_t*>(base + p.hsigs);
  a.rounds = reinterpret_cast<const uint64_t*>(base + p.rounds);
  a.vpks = reinterpret_cast<const uint32_t*>(base + p.vpks);
  a.vsigs = reinterpret_cast<const uint32_t*>(base + p.vsigs);
  a.voff = reinterpret_cast<const uint64_t*>(base + p.voff);
  a.nc = (uint32_t)nc;
  a.nv = (uint32_t)nv;
  a.hdr_blocks = 0;
  a.keys = ks.ckeys.as<uint32_t>();
  a.kflags = ks.kflags.as<uint32_t>();
  a.ktabs = ks.ktabs.as<uint32_t>();
  a.nk = ks.nkeys;
  a.comb = d.comb;
  a.wcomb = wcomb_of(d);
  a.kwtabs = (ks.kwide && !env_is("COA_KEY_WCOMB", "0")) ? ks.kwtabs.as<uint32_t>() : nullptr;
  a.kw20 = ks.kw20 ? 1u : 0u;
  a.status = reinterpret_cast<uint32_t*>(base + p.status);
  return a;
}

// Fast path for certificates [lo, hi) on one device: raw status words out.
// publish: the latency variant writes its status words straight into
// page-locked host memory (no D2H copy, no stream synchronisation).
// The latency launch with the certificates inline in the kernel arguments
// (no pinned staging copy, no H2D transfer): for calls whose arrays fit
// COA_CERT_INLINE_BYTES.  Returns 1 when they do not fit (nothing launched).
// Certificates [lo, hi) of `in` into ci's buffer; false when they do not fit.
bool cert_inl_build(CertInl& ci, const CertIn& in, size_t lo, size_t hi) {
  const size_t nc = hi - lo;
  const uint64_t h0 = in.hdr_off[lo], hb = in.hdr_off[hi] - h0;
  const uint64_t v0 = in.voff[lo], nv = in.voff[hi] - v0;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o = align_up(o + bytes, 16);
    return (uint32_t)at;
  };
  ci.off_hoff = take((nc + 1) * 8);
  ci.off_voff = take((nc + 1) * 8);
  ci.off_ids = take(nc * 32);
  ci.off_origins = take(nc * 32);
  ci.off_hsigs = take(nc * 64);
  ci.off_rounds = take(nc * 8);
  ci.off_vpks = take(nv * 32);
  ci.off_vsigs = take(nv * 64);
  ci.off_hdr = take(hb + 16);
  if (o > COA_CERT_INLINE_BYTES || nc > 64) return false;
  uint8_t* b = ci.buf;
  uint64_t* ho = reinterpret_cast<uint64_t*>(b + ci.off_hoff);
  uint64_t* vo = reinterpret_cast<uint64_t*>(b + ci.off_voff);
  for (size_t i = 0; i <= nc; i++) {
    ho[i] = in.hdr_off[lo + i] - h0;
    vo[i] = in.voff[lo + i] - v0;
  }
  std::memcpy(b + ci.off_ids, in.ids + lo * 32, nc * 32);
  std::memcpy(b + ci.off_origins, in.origins + lo * 32, nc * 32);
  std::memcpy(b + ci.off_hsigs, in.hsigs + lo * 64, nc * 64);
  std::memcpy(b + ci.off_rounds, in.rounds + lo, nc * 8);
  if (nv) {
    std::memcpy(b + ci.off_vpks, in.vpks + v0 * 32, nv * 32);
    std::memcpy(b + ci.off_vsigs, in.vsigs + v0 * 64, nv * 64);
  }
  if (hb) std::memcpy(b + ci.off_hdr, in.hdr_data + h0, hb);
  std::memset(b + ci.off_hdr + hb, 0, 16);
  return true;
}

int cert_inline(Dev& d, const CertIn& in, size_t lo, size_t hi, uint32_t* status_out) {
  const size_t nc = hi - lo;
  const uint64_t nv = in.voff[hi] - in.voff[lo];
  static thread_local CertInl ci;  // ~3 KB, staged on the host; copied into the launch
  if (!cert_inl_build(ci, in, lo, hi)) return 1;
  hipStream_t s = d.stream;
  if (!d.lat_ctr) {  // [0] block counter, [1..64] status words; the kernel re-zeroes both
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d.lat_ctr), 65 * 4));
    HIP_TRY(hipMemsetAsync(d.lat_ctr, 0, 65 * 4, s));
  }
  uint32_t tag = 0;
  int rc = lat_res_prepare(d, nc, tag);
  if (rc != COA_OK) return rc;
  CertArgs& a = ci.a;
  const KeySetP ks = keys_now(d);  // held until the status words are in
  a = cert_args(d, *ks, nullptr, CertPack{}, nc, nv);
  a.status = d.lat_ctr + 1;
  a.host_res = d.lat_res;
  a.done_ctr = d.lat_ctr;
  a.tag = tag;
  HIP_TRY(coa_launch_cert_verify_inl(ci, s));
  return lat_res_wait(d, s, nc, tag, status_out + lo);
}

// Packs certificates [lo, hi) into page-locked staging h laid out as p (the
// copies spread over the CopyPool).
void cert_pack(uint8_t* h, const CertPack& p, const CertIn& in, size_t lo, size_t hi) {
  const size_t nc = hi - lo;
  const uint64_t h0 = in.hdr_off[lo], hb = in.hdr_off[hi] - h0;
  const uint64_t v0 = in.voff[lo], nv = in.voff[hi] - v0;
  std::memset(h + p.status, 0, nc * 4);
  uint64_t* ho = reinterpret_cast<uint64_t*>(h + p.hoff);
  uint64_t* vo = reinterpret_cast<uint64_t*>(h + p.voff);
  for (size_t i = 0; i <= nc; i++) {
    ho[i] = in.hdr_off[lo + i] - h0;
    vo[i] = in.voff[lo + i] - v0;
  }
  std::vector<CopyPool::Seg> segs = {{h + p.ids, in.ids + lo * 32, nc * 32},
                                     {h + p.origins, in.origins + lo * 32, nc * 32},
                                     {h + p.hsigs, in.hsigs + lo * 64, nc * 64},
                                     {h + p.rounds, in.rounds + lo, nc * 8}};
  if (nv) {
    segs.push_back({h + p.vpks, in.vpks + v0 * 32, nv * 32});
    segs.push_back({h + p.vsigs, in.vsigs + v0 * 64, nv * 64});
  }
  if (hb) segs.push_back({h + p.hdata, in.hdr_data + h0, hb});
  CopyPool::get().copy(segs);
}

// Jobs (header + votes) per chunk of the pipelined certificate path
// (COA_CERT_CHUNK_JOBS, read per call; default 2^17: ~1,900 C3
// certificates, ~19 MB of staging, enough jobs for the persistent
// certificate grid to fill the chip) and chunks in flight
// (COA_CERT_BUFFERS, 2..4, default 3).
size_t cert_chunk_jobs() {
  const char* e = getenv("COA_CERT_CHUNK_JOBS");
  const long v = e ? atol(e) : 0;
  return v >= (1 << 12) ? (size_t)v : ((size_t)1 << 17);
}
// The first chunks of a pipelined call are smaller (COA_CERT_RAMP = r, read
// per call, default 1: chunk k < r takes chunk_jobs >> (r - k) jobs), so the
// GPU starts after a half chunk's pack and copy instead of a full one's.
// Host C3 round, same box, 8 alternating pairs: r = 1 +1.4 to +6.7 % over
// r = 0; r = 2 and 3 slower (more chunks); profiles/r05_c3_host_ramp_ab.txt.
int cert_ramp() {
  const char* e = getenv("COA_CERT_RAMP");
  const int v = e ? atoi(e) : 1;
  return v < 0 ? 0 : (v > 4 ? 4 : v);
}
// COA_CERT_PIPE_KEYSORT=1: the pipelined host path's chunks also take
// their jobs in key order (A/B; see coa_committee.hip k_job_count)
bool pipe_keysort() { return env_is("COA_CERT_PIPE_KEYSORT", "1"); }
int cert_buffers() {
  const char* e = getenv("COA_CERT_BUFFERS");
  const int v = e ? atoi(e) : 3;
  return v < 2 ? 2 : (v > 4 ? 4 : v);
}

// Certificates [lo, hi) on one device in chunks, up to cert_buffers() in
// flight on as many streams, each with its own page-locked staging and
// device buffers: while the GPU runs chunk k's kernel, chunk k + 1's copy
// crosses PCIe and the host packs chunk k + 2 (CopyPool).  With two buffer
// sets the host could only pack chunk k + 2 once chunk k had finished, so a
// round took about (pack + copy + kernel) / 2 per chunk.  Raw status words
// out.  COA_CERT_TRACE=1 prints the host's pack and wait time per call.
int cert_shard_pipelined(Dev& d, const CertIn& in, size_t lo, size_t hi, uint32_t* status_out) {
  const size_t chunk_jobs = cert_chunk_jobs();
  const int nb = cert_buffers();
  const int ramp = cert_ramp();
  std::vector<size_t> cuts{lo};
  size_t jobs = 0;
  for (size_t c = lo; c < hi; c++) {
    jobs += 1 + (in.voff[c + 1] - in.voff[c]);
    const int k = (int)cuts.size() - 1;  // the chunk being cut
    if (jobs >= (chunk_jobs >> std::max(0, ramp - k)) && c + 1 < hi) {
      cuts.push_back(c + 1);
      jobs = 0;
    }
  }
  cuts.push_back(hi);
  hipStream_t st[4] = {d.stream, nullptr, nullptr, nullptr};
  for (int b = 1; b < nb; b++) {
    if (!d.cstreams[b - 1]) HIP_TRY(hipStreamCreateWithFlags(&d.cstreams[b - 1], hipStreamNonBlocking));
    st[b] = d.cstreams[b - 1];
  }
  const KeySetP ks = keys_now(d);  // held until every chunk is done
  struct Pending {
    bool busy = false;
    size_t lo = 0, hi = 0, status = 0;
  } pend[4];
  const bool trace = env_is("COA_CERT_TRACE", "1");
  double t_pack = 0, t_wait = 0;
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  auto drain = [&](int b) -> int {
    if (!pend[b].busy) return COA_OK;
    const double t0 = trace ? now() : 0;
    HIP_TRY(hipStreamSynchronize(st[b]));
    if (trace) t_wait += now() - t0;
    std::memcpy(status_out + pend[b].lo, static_cast<uint8_t*>(d.pinc[b].p) + pend[b].status,
                (pend[b].hi - pend[b].lo) * 4);
    pend[b].busy = false;
    return COA_OK;
  };
  for (size_t k = 0; k + 1 < cuts.size(); k++) {
    const int b = (int)(k % nb);
    int rc = drain(b);  // this buffer set's previous chunk
    if (rc != COA_OK) return rc;
    const size_t clo = cuts[k], chi = cuts[k + 1], nc = chi - clo;
    const uint64_t nv = in.voff[chi] - in.voff[clo], hb = in.hdr_off[chi] - in.hdr_off[clo];
    const CertPack p = cert_layout(nc, nv, hb);
    HIP_TRY(d.pinc[b].ensure(p.total));
    HIP_TRY(d.certc[b].ensure(p.total));
    HIP_TRY(d.cscrc[b].ensure(coa_cert_scratch_bytes(nc + nv, pipe_keysort())));
    uint8_t* h = static_cast<uint8_t*>(d.pinc[b].p);
    const double t0 = trace ? now() : 0;
    cert_pack(h, p, in, clo, chi);
    if (trace) t_pack += now() - t0;
    HIP_TRY(hipMemcpyAsync(d.certc[b].p, h, p.total, hipMemcpyHostToDevice, st[b]));
    CertArgs a = cert_args(d, *ks, d.certc[b].as<uint8_t>(), p, nc, nv);
    a.key_order = pipe_keysort() ? 1u : 0u;
    HIP_TRY(coa_launch_cert_verify(a, 1, d.cscrc[b].as<uint32_t>(), st[b]));
    HIP_TRY(hipMemcpyAsync(h + p.status, d.certc[b].as<uint8_t>() + p.status, nc * 4, hipMemcpyDeviceToHost, st[b]));
    pend[b] = {true, clo, chi, p.status};
  }
  for (size_t k = 0; k < (size_t)nb; k++) {
    const int rc = drain((int)((cuts.size() - 1 + k) % nb));  // oldest first
    if (rc != COA_OK) return rc;
  }
  if (trace)
    fprintf(stderr, "[coa] cert pipeline: %zu chunks x %d buffers, pack %.3f ms, wait %.3f ms\n", cuts.size() - 1, nb,
            t_pack * 1e3, t_wait * 1e3);
  return COA_OK;
}

int cert_shard(Dev& d, const CertIn& in, size_t lo, size_t hi, uint32_t* status_out, bool publish = false) {
  const size_t nc = hi - lo;
  const uint64_t h0 = in.hdr_off[lo], hb = in.hdr_off[hi] - h0;
  const uint64_t v0 = in.voff[lo], nv = in.voff[hi] - v0;
  if (publish && cert_lanes(nc + nv) == 64 && !env_is("COA_CERT_INLINE", "0")) {
    const int rc = cert_inline(d, in, lo, hi, status_out);
    if (rc != 1) return rc;
  }
  if (!publish && nc + nv >= 2 * cert_chunk_jobs() && !env_is("COA_CERT_PIPELINE", "0"))
    return cert_shard_pipelined(d, in, lo, hi, status_out);
  const CertPack p = cert_layout(nc, nv, hb);
  HIP_TRY(d.pin.ensure(p.total));
  HIP_TRY(d.cert.ensure(p.total));
  uint8_t* h = static_cast<uint8_t*>(d.pin.p);
  cert_pack(h, p, in, lo, hi);
  hipStream_t s = d.stream;
  HIP_TRY(hipMemcpyAsync(d.cert.p, h, p.total, hipMemcpyHostToDevice, s));
  const KeySetP ks = keys_now(d);  // held until the status words are in
  CertArgs a = cert_args(d, *ks, d.cert.as<uint8_t>(), p, nc, nv);
  const int lanes = cert_lanes(nc + nv);
  if (lanes == 64 && publish) {  // the last block writes the status words to host memory
    if (!d.lat_ctr) {
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d.lat_ctr), 65 * 4));
      HIP_TRY(hipMemsetAsync(d.lat_ctr, 0, 65 * 4, s));
    }
    uint32_t tag = 0;
    int rc = lat_res_prepare(d, nc, tag);
    if (rc != COA_OK) return rc;
    a.host_res = d.lat_res;
    a.done_ctr = d.lat_ctr;
    a.tag = tag;
    HIP_TRY(coa_launch_cert_verify(a, lanes, nullptr, s));
    return lat_res_wait(d, s, nc, tag, status_out + lo);
  }
  if (lanes == 1) HIP_TRY(d.cscr.ensure(coa_cert_scratch_bytes(nc + nv, a.key_order != 0)));
  HIP_TRY(coa_launch_cert_verify(a, lanes, d.cscr.as<uint32_t>(), s));
  HIP_TRY(hipMemcpyAsync(h + p.status, d.cert.as<uint8_t>() + p.status, nc * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::memcpy(status_out + lo, h + p.status, nc * 4);
  return COA_OK;
}

// Exact (non-cached) resolution of certificates `idx`: header signatures by
// verify_strict (only when `hdr_too`), votes by the RLC kernels over
// Certificate::digest.  ORs COA_CST_BAD_* into status.
int cert_resolve(const CertIn& in, const std::vector<size_t>& idx, bool hdr_too, uint64_t seed, uint32_t* status) {
  if (idx.empty()) return COA_OK;
  const size_t m = idx.size();
  // Certificate::digest inputs: id || round LE || origin (72 B)
  std::vector<uint8_t> cin(m * 72);
  for (size_t j = 0; j < m; j++) {
    const size_t c = idx[j];
    std::memcpy(&cin[j * 72], in.ids + c * 32, 32);
    std::memcpy(&cin[j * 72 + 32], &in.rounds[c], 8);
    std::memcpy(&cin[j * 72 + 40], in.origins + c * 32, 32);
  }
  // the digests of certificates `sel` (indices into idx) into gm
  std::vector<uint8_t> gm(m * 32), gv(m), vp, vs;
  auto digests = [&](const std::vector<size_t>& sel) -> int {
    if (sel.empty()) return COA_OK;
    std::vector<uint8_t> sin(sel.size() * 72), dig(sel.size() * 64);
    std::vector<uint64_t> soff(sel.size() + 1);
    for (size_t k = 0; k < sel.size(); k++) {
      std::memcpy(&sin[k * 72], &cin[sel[k] * 72], 72);
      soff[k] = k * 72;
    }
    soff[sel.size()] = sel.size() * 72;
    const int r = coa_sha512_many(sin.data(), soff.data(), sel.size(), dig.data());
    for (size_t k = 0; r == COA_OK && k < sel.size(); k++) std::memcpy(&gm[sel[k] * 32], &dig[k * 64], 32);
    return r;
  };
  std::vector<uint64_t> goff(m + 1, 0);
  for (size_t j = 0; j < m; j++) {
    const size_t c = idx[j];
    const uint64_t a = in.voff[c], b = in.voff[c + 1];
    vp.insert(vp.end(), in.vpks + a * 32, in.vpks + b * 32);
    vs.insert(vs.end(), in.vsigs + a * 64, in.vsigs + b * 64);
    goff[j + 1] = goff[j] + (b - a);
  }
  std::vector<uint8_t> hv(m, 0);
  const size_t nvotes = goff[m];
  int rc;
  if (hdr_too && nvotes + m <= lat_max() && !env_is("COA_BATCH_LAT", "0") && !env_is("COA_RESOLVE_ONE_LAUNCH", "0")) {
    // ONE latency launch for the votes (the verify_batch prefilter: items
    // [0, nvotes), each message Certificate::digest hashed in the kernel from
    // cin, LatArgs::cd_in) and the header signatures (plain verify_strict:
    // items [nvotes, nvotes + m)): a certificate with keys outside the
    // committee took a digest launch, a prefilter launch and a header launch,
    // one after the other
    std::vector<uint8_t> msgs(m * 32, 0), pks(vp), sigs(vs);
    std::vector<uint32_t> msg_of(nvotes + m);
    for (size_t j = 0; j < m; j++) {
      const uint32_t jj = (uint32_t)j;
      std::memcpy(&msgs[j * 32], &jj, 4);  // the certificate's index: its digest input in cin
      for (uint64_t i = goff[j]; i < goff[j + 1]; i++) msg_of[i] = (uint32_t)j;
      msg_of[nvotes + j] = (uint32_t)(m + j);
      const size_t c = idx[j];
      msgs.insert(msgs.end(), in.ids + c * 32, in.ids + c * 32 + 32);
      pks.insert(pks.end(), in.origins + c * 32, in.origins + c * 32 + 32);
      sigs.insert(sigs.end(), in.hsigs + c * 64, in.hsigs + c * 64 + 64);
    }
    std::vector<uint8_t> v(nvotes + m);
    {
      std::unique_lock<std::mutex> l;
      Dev& d = lat_dev(l);
      HIP_TRY(hipSetDevice(d.id));
      rc = lat_verify(d, msgs.data(), pks.data(), sigs.data(), nvotes + m, v.data(), msg_of.data(), nvotes,
                      cin.data(), m);
      if (rc != COA_OK) return rc;
    }
    // a group every vote of which passed is Ok for every z; the others take
    // the exact path with their own weights (as batch_groups_impl's prefilter)
    std::vector<size_t> open;
    for (size_t j = 0; j < m; j++) {
      bool pass = true;
      for (uint64_t i = goff[j]; i < goff[j + 1]; i++) pass = pass && v[i] == 0;
      gv[j] = pass ? 0 : 1;
      if (!pass) open.push_back(j);
      hv[j] = v[nvotes + j] ? 1 : 0;
    }
    rc = digests(open);  // only the groups the prefilter did not accept need their digest on the host
    if (rc != COA_OK) return rc;
    for (size_t j : open) {
      const uint64_t a = goff[j], n = goff[j + 1] - a;
      const uint64_t offs[2] = {0, n};
      rc = batch_groups_impl(&gm[j * 32], vp.data() + a * 32, vs.data() + a * 64, offs, 1, nullptr, seed, &gv[j], 0,
                             false);
      if (rc != COA_OK) return rc;
    }
    for (size_t j = 0; j < m; j++)
      status[idx[j]] |= (gv[j] ? COA_CST_BAD_VOTES : 0u) | (hv[j] ? COA_CST_BAD_HEADER_SIG : 0u);
    return COA_OK;
  }
  std::vector<size_t> all(m);
  for (size_t j = 0; j < m; j++) all[j] = j;
  rc = digests(all);
  if (rc != COA_OK) return rc;
  rc = batch_groups_impl(gm.data(), vp.data(), vs.data(), goff.data(), m, nullptr, seed, gv.data());
  if (rc != COA_OK) return rc;
  if (hdr_too) {
    std::vector<uint8_t> hm(m * 32), hp(m * 32), hs(m * 64);
    for (size_t j = 0; j < m; j++) {
      const size_t c = idx[j];
      std::memcpy(&hm[j * 32], in.ids + c * 32, 32);
      std::memcpy(&hp[j * 32], in.origins + c * 32, 32);
      std::memcpy(&hs[j * 64], in.hsigs + c * 64, 64);
    }
    rc = coa_ed25519_verify_strict_many(hm.data(), 32, hp.data(), hs.data(), m, hv.data());
    if (rc != COA_OK) return rc;
  }
  for (size_t j = 0; j < m; j++) {
    status[idx[j]] |= (gv[j] ? COA_CST_BAD_VOTES : 0u) | (hv[j] ? COA_CST_BAD_HEADER_SIG : 0u);
  }
  return COA_OK;
}

// Raw status words of the fused kernel -> exact verdicts: a certificate with
// a key outside the registered committee is re-decided entirely (header
// signature by verify_strict, votes by the RLC kernels; its digest check does
// not use the cache and stands), one whose votes were inconclusive (a vote
// failed its own equation, or a key has torsion) by the RLC kernels alone.
// Shared by certificates_impl and the queue's resolver
// (coa_certificate_resolve_raw), which hands over the words of the
// certificates its window could not answer at once.
int resolve_raw(const CertIn& in, size_t n, uint32_t* st, uint64_t rng_seed) {
  std::vector<size_t> uncached, rlc;
  for (size_t i = 0; i < n; i++) {
    if (st[i] & COA_CST_UNCACHED) {
      st[i] &= COA_CST_BAD_HEADER_ID;  // the digest check does not use the cache
      uncached.push_back(i);
    } else if ((st[i] & COA_CST_VOTES_INCONCLUSIVE) && !(st[i] & COA_CST_BAD_VOTES)) {
      rlc.push_back(i);
    }
  }
  // weights for the exact re-decision only: OS entropy is a syscall, and the
  // common call (every certificate decided by the cached kernel) needs none
  const uint64_t seed = rng_seed || (uncached.empty() && rlc.empty()) ? rng_seed : os_entropy_seed();
  int rc = cert_resolve(in, uncached, true, seed, st);
  if (rc != COA_OK) return rc;
  return cert_resolve(in, rlc, false, seed, st);
}

int certificates_impl(const CertIn& in, size_t n, uint64_t rng_seed, uint8_t* status_out) {
  if (n == 0) return COA_OK;
  if (!in.hdr_off || !in.ids || !in.origins || !in.hsigs || !in.rounds || !in.voff || !status_out)
    return fail(COA_EINVAL, "null argument");
  for (size_t i = 0; i < n; i++)
    if (in.hdr_off[i + 1] < in.hdr_off[i] || in.voff[i + 1] < in.voff[i])
      return fail(COA_EINVAL, "offsets not monotone");
  if (in.voff[0] != 0) return fail(COA_EINVAL, "vote_offsets[0] must be 0");
  if (in.hdr_off[n] > in.hdr_off[0] && !in.hdr_data) return fail(COA_EINVAL, "null header data");
  if (in.voff[n] && (!in.vpks || !in.vsigs)) return fail(COA_EINVAL, "null vote arrays");
  if (check_n(n + in.voff[n]) != COA_OK) return COA_EINVAL;
  std::vector<uint32_t> st(n, 0);
  int rc;
  if (cert_lanes(n + in.voff[n]) == 64) {  // latency path: one idle context, no stream sync
    std::unique_lock<std::mutex> l;
    Dev& d = lat_dev(l);
    HIP_TRY(hipSetDevice(d.id));
    rc = cert_shard(d, in, 0, n, st.data(), true);
  } else {
    rc = for_shards(
        n, [&](Dev& d, size_t lo, size_t hi) -> int { return cert_shard(d, in, lo, hi, st.data()); },
        n + in.voff[n]);
  }
  if (rc != COA_OK) return rc;
  rc = resolve_raw(in, n, st.data(), rng_seed);
  if (rc != COA_OK) return rc;
  for (size_t i = 0; i < n; i++) status_out[i] = (uint8_t)(st[i] & 7u);
  return COA_OK;
}

int sign_enqueue(Dev& d, const uint8_t* d_seeds, const uint8_t* d_msgs, size_t msg_len, size_t n, uint8_t* d_pks,
                 uint8_t* d_sigs, hipStream_t s) {
  HIP_TRY(d.aux.ensure(n * 64 + 64));
  HIP_TRY(d.rbuf.ensure(n * 32 + 32));
  HIP_TRY(d.kbuf.ensure(n * 32 + 32));
  HIP_TRY(coa_launch_keygen(d_seeds, (uint32_t)n, d_pks, d.aux.as<uint32_t>(), d.btab, s));
  HIP_TRY(coa_launch_sign_r(d.aux.as<uint32_t>(), d_msgs, (uint32_t)msg_len, (uint32_t)n, d_sigs,
                            d.rbuf.as<uint32_t>(), d.btab, s));
  HIP_TRY(coa_launch_hram(d_msgs, (uint32_t)msg_len, msg_len, nullptr, d_pks, d_sigs, (uint32_t)n,
                          d.kbuf.as<uint32_t>(), s));
  HIP_TRY(coa_launch_sign_s(d.aux.as<uint32_t>(), d.rbuf.as<uint32_t>(), d.kbuf.as<uint32_t>(), (uint32_t)n, d_sigs,
                            s));
  return COA_OK;
}

// Builds the next key-cache generation of device sh on its build stream
// while every call and queue window keeps the current one, swaps it in, then
// frees the old generation once nothing holds it: no call or window waits
// for a registration, and none is held back (the round-3 write gate stalled
// the queue's certificate windows for the whole 0.6-2.7 s build).
int build_keyset(DevShared& sh, const std::vector<std::array<uint32_t, 8>>& keys) {
  std::lock_guard<std::mutex> r(sh.reg_mu);
  HIP_TRY(hipSetDevice(sh.id));
  if (!sh.build) {
    // the build runs beside live windows (a committee-100 build is 65 GB of
    // comb entries, ~0.6 s on the whole GPU): on a plain stream at the least
    // priority, so the hardware queue scheduler dispatches the windows'
    // workgroups first.  tools/regab.sh, a C3 certificate stream at 5,000/s
    // with two re-registrations (profiles/r04_register_ab.txt): request
    // latency p99 during the build 0.89 ms (max 1.3 ms), registration 0.61 s;
    // a CU-masked stream over half the CUs (COA_REGISTER_CUS=128) left the
    // windows 17 ms (bounded resident grid) to 1.4 s (one workgroup per 256
    // entries) behind.
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, sh.id));
    const char* e = getenv("COA_REGISTER_CUS");
    const int want = e ? atoi(e) : 0;
    if (want <= 0) {
      int least = 0, greatest = 0;
      HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIP_TRY(hipStreamCreateWithPriority(&sh.build, hipStreamNonBlocking, least));
    } else {
      const int use = std::min(cus, want);
      std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
      for (int c = cus - use; c < cus; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
      HIP_TRY(hipExtStreamCreateWithCUMask(&sh.build, (uint32_t)mask.size(), mask.data()));
    }
  }
  const size_t nk = keys.size();
  // the buffers of the generation before the current one, when kept
  // (COA_KEY_SPARE=0: none kept, every registration allocates)
  const bool keep_spare = !env_is("COA_KEY_SPARE", "0");
  std::shared_ptr<KeySet> ks = keep_spare && sh.spare ? std::move(sh.spare) : std::make_shared<KeySet>();
  sh.spare.reset();
  // wide-comb bytes the current generation keeps resident while this one is
  // built (charged against COA_KEY_RESIDENT_MB)
  double cur_wide = 0.0;
  {
    std::lock_guard<std::mutex> l(sh.mu);
    if (sh.keys) cur_wide = (double)sh.keys->kwtabs.cap;
  }
  const double resident_room = key_resident_budget() - cur_wide;
  ks->dev = sh.id;
  ks->nkeys = 0;
  ks->kwide = ks->kw20 = false;
  hipStream_t s = sh.build;
  // COA_REGISTER_TRACE=1: phase times of this registration on stderr
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  clk::time_point t_alloc = t0, t_built = t0;
  if (nk) {
    HIP_TRY(ks->ckeys.ensure(nk * 32));
    HIP_TRY(ks->kflags.ensure(nk * 4));
    HIP_TRY(ks->ktabs.ensure(nk * (size_t)COA_KEY_TAB_DWORDS * 4));
    if (env_is("COA_REGISTER_PAGEABLE", "1")) {  // A/B: the keys straight from the caller's (pageable) vector
      HIP_TRY(hipMemcpyAsync(ks->ckeys.p, keys.data(), nk * 32, hipMemcpyHostToDevice, s));
    } else {
      if (sh.kstage_cap < nk * 32) {
        if (sh.kstage) HIP_TRY(hipHostFree(sh.kstage));
        sh.kstage = nullptr;
        sh.kstage_cap = 0;
        HIP_TRY(hipHostMalloc(&sh.kstage, nk * 32, hipHostMallocDefault));
        sh.kstage_cap = nk * 32;
      }
      std::memcpy(sh.kstage, keys.data(), nk * 32);
      HIP_TRY(hipMemcpyAsync(ks->ckeys.p, sh.kstage, nk * 32, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(coa_launch_key_flags(ks->ckeys.as<uint32_t>(), (uint32_t)nk, ks->kflags.as<uint32_t>(), s));
    HIP_TRY(coa_launch_key_tables(ks->ckeys.as<uint32_t>(), (uint32_t)nk, ks->ktabs.as<uint32_t>(), s));
    // wide combs when the committee fits the budget: radix 2^20 (654 MB per
    // key, 13 additions per [k](-A)) within COA_KEY_WCOMB20_MB, else radix
    // 2^16 (48 MiB per key, 16 additions) within COA_KEY_WCOMB_MB (speed
    // only: without the memory the radix-256 key combs serve)
    KeySet& k = *ks;
    // an exact fit is reused as it is; a different size is reallocated
    auto fit = [](DevBuf& b, size_t bytes) {
      if (b.cap != bytes) b.release();
      return b.ensure(bytes, true);
    };
    const double w20 = (double)nk * COA_KWCOMB20_DWORDS * 4, w16 = (double)nk * COA_KWCOMB_DWORDS * 4;
    if (w20 <= key_wcomb20_budget() && w20 <= resident_room) {
      if (fit(k.kwtabs, nk * (size_t)COA_KWCOMB20_DWORDS * 4) == hipSuccess) {
        t_alloc = clk::now();
        HIP_TRY(coa_launch_key_wcombs20(k.ktabs.as<uint32_t>(), (uint32_t)nk, k.kwtabs.as<uint32_t>(), s));
        k.kwide = k.kw20 = true;
      } else {
        k.kwtabs.release();
        (void)hipGetLastError();
      }
    }
    if (!k.kw20 && w16 <= key_wcomb_budget() && w16 <= resident_room) {
      if (fit(k.kwtabs, nk * (size_t)COA_KWCOMB_DWORDS * 4) == hipSuccess) {
        HIP_TRY(coa_launch_key_wcombs(k.ktabs.as<uint32_t>(), (uint32_t)nk, k.kwtabs.as<uint32_t>(), s));
        k.kwide = true;
      } else {
        k.kwtabs.release();
        (void)hipGetLastError();
      }
    }
    if (!k.kwide) k.kwtabs.release();  // a reused spare's wide combs no budget admits
    HIP_TRY(hipStreamSynchronize(s));
    k.nkeys = (uint32_t)nk;
    t_built = clk::now();
  }
  KeySetP old;
  {
    std::lock_guard<std::mutex> l(sh.mu);
    old = std::move(sh.keys);
    sh.keys = std::move(ks);
  }
  // the old generation: calls and windows that took it still hold it (their
  // kernels read it until they complete), and a device-pointer call on a
  // caller's stream left it in `trailing` with an event after its kernels
  // (trail_keys).  Only this thread waits -- no hipDeviceSynchronize, which
  // held every other thread's launches for its whole wait.
  const auto t_swap = clk::now();
  while (old.use_count() > 1) {
    reap_trailing(sh);
    if (old.use_count() > 1) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  const auto t_unpinned = clk::now();
  const auto t_synced = t_unpinned;
  // the replaced generation's buffers become the spare of the next
  // registration; after the first registration of a device (nothing to
  // replace yet) a spare of the same size is allocated now, while the
  // committee is being set up rather than under load later
  if (keep_spare && nk) {
    const KeySet& cur = *sh.keys;
    // the next registration of a committee this size finds its buffers ready
    auto fits = [&](const KeySet& k) {
      return k.ckeys.cap >= nk * 32 && k.kflags.cap >= nk * 4 && k.ktabs.cap >= nk * (size_t)COA_KEY_TAB_DWORDS * 4 &&
             k.kwtabs.cap == cur.kwtabs.cap;
    };
    // a spare only beside the current generation within COA_KEY_RESIDENT_MB
    // (without one, the next registration allocates its wide combs while
    // windows run: 2.4-7.6 ms held back, profiles/r04_register_ab.txt)
    const bool room = 2.0 * (double)cur.kwtabs.cap <= key_resident_budget();
    if (!room) {
      old.reset();
    } else if (old && fits(*old)) {
      sh.spare = std::const_pointer_cast<KeySet>(old);
    } else {
      old.reset();  // another size: freed now, and a spare of this size made
      auto sp = std::make_shared<KeySet>();
      sp->dev = sh.id;
      if (sp->ckeys.ensure(cur.ckeys.cap, true) == hipSuccess && sp->kflags.ensure(cur.kflags.cap, true) == hipSuccess &&
          sp->ktabs.ensure(cur.ktabs.cap, true) == hipSuccess &&
          (!cur.kwtabs.cap || sp->kwtabs.ensure(cur.kwtabs.cap, true) == hipSuccess))
        sh.spare = std::move(sp);
      else
        (void)hipGetLastError();  // no spare: the next registration allocates
    }
  } else if (keep_spare && !nk && old && old->nkeys && !sh.spare) {
    // a committee cleared: its generation's buffers stay as the spare instead
    // of being freed.  Freeing a 65 GB generation here, and allocating one
    // again at the next registration, each held the HIP runtime while other
    // threads enqueued: a signature window of the queue spent 7.9 ms in
    // `enqueue` (profiles/r05_register_gc.txt:19) while
    // test_register_while_queue_saturated_with_certificates cleared and
    // re-registered the committee in a loop
    sh.spare = std::const_pointer_cast<KeySet>(old);
  }
  old.reset();
  if (env_is("COA_REGISTER_TRACE", "1"))
    fprintf(stderr,
            "coa_committee_register dev %d keys %zu at t=%.6f s: alloc %.1f build %.1f swap %.1f unpinned %.1f sync "
            "%.1f free %.1f ms\n",
            sh.id, nk, std::chrono::duration<double>(t0.time_since_epoch()).count(), ms(t0, t_alloc),
            ms(t_alloc, t_built), ms(t_built, t_swap), ms(t_swap, t_unpinned),
            ms(t_unpinned, t_synced), ms(t_synced, clk::now()));
  return COA_OK;
}

}  // namespace

extern "C" {

const char* coa_last_error(void) { return g_err.c_str(); }
const char* coa_version(void) { return "coa_verify 0.1.0 gfx950"; }

int coa_init(int n_gpus) {
  std::lock_guard<std::mutex> g(g_init_mu);
  return init_locked(n_gpus);
}

int coa_init_devices(const int* device_ids, int n) {
  if (!device_ids || n <= 0) return fail(COA_EINVAL, "empty device list");
  std::lock_guard<std::mutex> g(g_init_mu);
  return init_locked(device_ids, n);
}

int coa_shutdown(void) {
  std::lock_guard<std::mutex> g(g_init_mu);
  for (auto& d : g_devs) {
    std::lock_guard<std::mutex> l(d->mu);
    (void)hipSetDevice(d->id);
    (void)hipStreamSynchronize(d->stream);
    for (DevBuf* b : d->all()) b->release();
    d->pin.release();
    for (PinBuf& p : d->pinc) p.release();
    for (hipStream_t& cs : d->cstreams)
      if (cs) {
        (void)hipStreamSynchronize(cs);
        (void)hipStreamDestroy(cs);
        cs = nullptr;
      }
    if (d->lat_res) (void)hipHostFree(d->lat_res);
    d->lat_res = nullptr;
    d->lat_res_cap = 0;
    if (d->lat_ctr) (void)hipFree(d->lat_ctr);
    d->lat_ctr = nullptr;
    if (d->btab) (void)hipFree(d->btab);
    if (d->comb) (void)hipFree(d->comb);
    (void)hipStreamDestroy(d->stream);
  }
  g_devs.clear();
  for (auto& sh : g_shared) {
    (void)hipSetDevice(sh->id);
    if (sh->wcomb) (void)hipFree(sh->wcomb);
    if (sh->build) (void)hipStreamDestroy(sh->build);
    if (sh->kstage) (void)hipHostFree(sh->kstage);
    {
      std::lock_guard<std::mutex> t(sh->trail_mu);
      for (auto& e : sh->trailing) {
        (void)hipEventSynchronize(e.first);
        (void)hipEventDestroy(e.first);
      }
      for (hipEvent_t e : sh->trail_events) (void)hipEventDestroy(e);
      sh->trailing.clear();
      sh->trail_events.clear();
    }
    std::lock_guard<std::mutex> l(sh->mu);
    sh->keys.reset();
  }
  g_shared.clear();
  g_inited = false;
  return COA_OK;
}

int coa_device_count(void) {
  const int r = ensure_init();
  if (r != COA_OK) return r;
  return (int)g_devs.size();
}

int coa_device_ids(int* ids_out, int cap) {
  const int r = ensure_init();
  if (r != COA_OK) return r;
  if (cap > 0 && !ids_out) return fail(COA_EINVAL, "null argument");
  for (int i = 0; i < (int)g_devs.size() && i < cap; i++) ids_out[i] = g_devs[i]->id;
  return (int)g_devs.size();
}

int coa_self_test(int device, uint64_t* bad_entries) {
  if (!bad_entries) return fail(COA_EINVAL, "null output");
  *bad_entries = 0;
  const int r = ensure_init();
  if (r != COA_OK) return r;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  std::lock_guard<std::mutex> l(d->mu);
  if (!d->sh->wcomb) return COA_OK;
  HIP_TRY(hipSetDevice(d->id));
  uint32_t* dbad = nullptr;
  HIP_TRY(hipMalloc(&dbad, sizeof(uint32_t)));
  uint32_t hbad = 0;
  hipError_t e = hipMemsetAsync(dbad, 0, sizeof(uint32_t), d->stream);
  if (e == hipSuccess) e = coa_launch_check_wcomb(d->sh->wcomb, dbad, d->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(&hbad, dbad, sizeof(uint32_t), hipMemcpyDeviceToHost, d->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
  (void)hipFree(dbad);
  HIP_TRY(e);
  *bad_entries = hbad;
  return COA_OK;
}

int coa_fe_rows_check_device(int device, const uint8_t* d_in, size_t n, uint32_t* d_out, void* stream) {
  const int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n && (!d_in || !d_out)) return fail(COA_EINVAL, "null argument");
  if (n > (1u << 24)) return fail(COA_EINVAL, "n too large");
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_fe_rows_check(d_in, (uint32_t)n, d_out, s));
  if (!stream) HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}

size_t coa_verify_workspace_bytes(size_t n) { return ws_bytes(n); }

int coa_ed25519_verify_strict_many(const uint8_t* msgs, size_t msg_len, const uint8_t* pks, const uint8_t* sigs,
                                   size_t n, uint8_t* verdicts_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if ((!msgs && msg_len) || !pks || !sigs || !verdicts_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  if (msg_len == 32 && n <= lat_max()) {  // few signatures: the latency kernel on an idle context
    std::unique_lock<std::mutex> l;
    Dev& d = lat_dev(l);
    HIP_TRY(hipSetDevice(d.id));
    return lat_verify(d, msgs, pks, sigs, n, verdicts_out);
  }
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    hipStream_t s = d.stream;
    HIP_TRY(d.msgs.ensure(cnt * msg_len + 4));
    HIP_TRY(d.pks.ensure(cnt * 32));
    HIP_TRY(d.sigs.ensure(cnt * 64));
    HIP_TRY(d.scratch.ensure(ws_bytes(cnt)));
    HIP_TRY(d.verdicts.ensure(cnt));
    if (msg_len) HIP_TRY(hipMemcpyAsync(d.msgs.p, msgs + lo * msg_len, cnt * msg_len, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.pks.p, pks + lo * 32, cnt * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.sigs.p, sigs + lo * 64, cnt * 64, hipMemcpyHostToDevice, s));
    int r = enqueue_verify(d, d.msgs.as<uint8_t>(), msg_len, d.pks.as<uint8_t>(), d.sigs.as<uint8_t>(), cnt,
                           d.verdicts.as<uint8_t>(), ws_carve(d.scratch.p, cnt), s);
    if (r != COA_OK) return r;
    HIP_TRY(hipMemcpyAsync(verdicts_out + lo, d.verdicts.p, cnt, hipMemcpyDeviceToHost, s));
    return COA_OK;
  });
}

int coa_ed25519_verify_strict(const uint8_t msg[32], const uint8_t pk[32], const uint8_t sig[64]) {
  uint8_t v = 1;
  const int rc = coa_ed25519_verify_strict_many(msg, 32, pk, sig, 1, &v);
  if (rc != COA_OK) return rc;
  return v ? COA_REJECT : COA_OK;
}

int coa_ed25519_verify_strict_many_device(int device, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks,
                                          const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, void* workspace,
                                          void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if ((!d_msgs && msg_len) || !d_pks || !d_sigs || !d_verdicts) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (workspace) return enqueue_verify(*d, d_msgs, msg_len, d_pks, d_sigs, n, d_verdicts, ws_carve(workspace, n), s);
  std::lock_guard<std::mutex> l(d->mu);
  HIP_TRY(d->scratch.ensure(ws_bytes(n)));
  rc = enqueue_verify(*d, d_msgs, msg_len, d_pks, d_sigs, n, d_verdicts, ws_carve(d->scratch.p, n), s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));  // engine-owned workspace: drain before release
  return COA_OK;
}

int coa_ed25519_challenge_many_device(int device, const uint8_t* d_msgs, size_t msg_len, const uint8_t* d_pks,
                                      const uint8_t* d_sigs, size_t n, uint8_t* d_k_out, void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if ((!d_msgs && msg_len) || !d_pks || !d_sigs || !d_k_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_hram(d_msgs, (uint32_t)msg_len, msg_len, nullptr, d_pks, d_sigs, (uint32_t)n,
                          reinterpret_cast<uint32_t*>(d_k_out), s));
  return COA_OK;
}

int coa_ed25519_verify_prehashed_many_device(int device, const uint8_t* d_k, const uint8_t* d_pks,
                                             const uint8_t* d_sigs, size_t n, uint8_t* d_verdicts, void* workspace,
                                             void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_k || !d_pks || !d_sigs || !d_verdicts) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  const uint32_t* k = reinterpret_cast<const uint32_t*>(d_k);
  if (workspace) return enqueue_verify_prehashed(*d, d_pks, d_sigs, n, d_verdicts, k, ws_carve(workspace, n), s);
  std::lock_guard<std::mutex> l(d->mu);
  HIP_TRY(d->scratch.ensure(ws_bytes(n)));
  rc = enqueue_verify_prehashed(*d, d_pks, d_sigs, n, d_verdicts, k, ws_carve(d->scratch.p, n), s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}

int coa_ed25519_verify_batch_groups(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                    const uint64_t* group_offsets, size_t n_groups, uint8_t* group_verdicts_out,
                                    uint64_t rng_seed) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  return batch_groups_impl(msgs, pks, sigs, group_offsets, n_groups, nullptr, rng_seed, group_verdicts_out);
}

int coa_ed25519_verify_batch_groups_z(const uint8_t* msgs, const uint8_t* pks, const uint8_t* sigs,
                                      const uint64_t* group_offsets, size_t n_groups, const uint8_t* zs,
                                      uint8_t* group_verdicts_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (!zs && n_groups && group_offsets && group_offsets[n_groups]) return fail(COA_EINVAL, "null zs");
  static const uint8_t zero16[16] = {0};
  return batch_groups_impl(msgs, pks, sigs, group_offsets, n_groups, zs ? zs : zero16, 0, group_verdicts_out);
}

size_t coa_verify_batch_workspace_bytes(size_t n) { return coa_msm_ws_bytes(n); }

int coa_ed25519_verify_batch_device(int device, const uint8_t* d_msg, const uint8_t* d_pks, const uint8_t* d_sigs,
                                    size_t n, const uint8_t* d_zs, uint64_t rng_seed, uint8_t* d_verdict,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (!d_msg || !d_verdict || (n && (!d_pks || !d_sigs))) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  if (n == 0) {  // empty batch: the equation is [0]B = O, Ok (as dalek)
    HIP_TRY(hipMemsetAsync(d_verdict, 0, 1, s));
    return COA_OK;
  }
  const uint64_t seed = d_zs ? 0 : (rng_seed ? rng_seed : os_entropy_seed());
  if (workspace) {
    // the chunk count (and so the layout) depends on the bucket run length of
    // this call: refuse a buffer sized for another one
    if (workspace_bytes < coa_msm_ws_bytes(n))
      return fail(COA_EINVAL, "workspace smaller than coa_verify_batch_workspace_bytes(n)");
    return enqueue_msm(*d, d_msg, d_pks, d_sigs, n, d_zs, seed, 0, d_verdict, workspace, s);
  }
  std::lock_guard<std::mutex> l(d->mu);
  HIP_TRY(d->msm.ensure(coa_msm_ws_bytes(n)));
  rc = enqueue_msm(*d, d_msg, d_pks, d_sigs, n, d_zs, seed, 0, d_verdict, d->msm.p, s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}

int coa_ed25519_verify_batch(const uint8_t msg[32], const uint8_t* pks, const uint8_t* sigs, size_t n,
                             uint64_t rng_seed) {
  const uint64_t offs[2] = {0, (uint64_t)n};
  uint8_t v = 1;
  const int rc = coa_ed25519_verify_batch_groups(msg, pks, sigs, offs, 1, &v, rng_seed);
  if (rc != COA_OK) return rc;
  return v ? COA_REJECT : COA_OK;
}

int coa_sha512_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out64) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!offsets || !out64) return fail(COA_EINVAL, "null argument");
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i]) return fail(COA_EINVAL, "offsets not monotone");
  if (offsets[n] > offsets[0] && !data) return fail(COA_EINVAL, "null data");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    const uint64_t base = offsets[lo], bytes = offsets[hi] - base;
    std::vector<uint64_t> rel(cnt + 1);
    for (size_t i = 0; i <= cnt; i++) rel[i] = offsets[lo + i] - base;
    hipStream_t s = d.stream;
    HIP_TRY(d.data.ensure(bytes + 16));
    HIP_TRY(d.offs.ensure((cnt + 1) * 8));
    HIP_TRY(d.out.ensure(cnt * 64));
    if (bytes) HIP_TRY(hipMemcpyAsync(d.data.p, data + base, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d.offs.p, rel.data(), (cnt + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(coa_launch_sha512_many(d.data.as<uint8_t>(), d.offs.as<uint64_t>(), (uint32_t)cnt,
                                   d.out.as<uint32_t>(), s));
    HIP_TRY(hipMemcpyAsync(out64 + lo * 64, d.out.p, cnt * 64, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));  // rel dies here
    return COA_OK;
  });
}

int coa_sha512_trunc32_many(const uint8_t* data, const uint64_t* offsets, size_t n, uint8_t* out32) {
  if (n == 0) return ensure_init();
  if (!out32) return fail(COA_EINVAL, "null argument");
  std::vector<uint8_t> full(n * 64);
  const int rc = coa_sha512_many(data, offsets, n, full.data());
  if (rc != COA_OK) return rc;
  for (size_t i = 0; i < n; i++) std::memcpy(out32 + i * 32, full.data() + i * 64, 32);
  return COA_OK;
}

int coa_sha512_many_device(int device, const uint8_t* d_data, const uint64_t* d_offsets, size_t n, uint8_t* d_out64,
                           void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_data || !d_offsets || !d_out64) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_sha512_many(d_data, d_offsets, (uint32_t)n, reinterpret_cast<uint32_t*>(d_out64), s));
  return COA_OK;
}

int coa_ed25519_sign_many(const uint8_t* seeds, const uint8_t* msgs, size_t msg_len, size_t n, uint8_t* pks_out,
                          uint8_t* sigs_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!seeds || (!msgs && msg_len) || !pks_out || !sigs_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    hipStream_t s = d.stream;
    HIP_TRY(d.seeds.ensure(cnt * 32));
    HIP_TRY(d.msgs.ensure(cnt * msg_len + 4));
    HIP_TRY(d.pks.ensure(cnt * 32));
    HIP_TRY(d.sigs.ensure(cnt * 64));
    HIP_TRY(hipMemcpyAsync(d.seeds.p, seeds + lo * 32, cnt * 32, hipMemcpyHostToDevice, s));
    if (msg_len) HIP_TRY(hipMemcpyAsync(d.msgs.p, msgs + lo * msg_len, cnt * msg_len, hipMemcpyHostToDevice, s));
    int r = sign_enqueue(d, d.seeds.as<uint8_t>(), d.msgs.as<uint8_t>(), msg_len, cnt, d.pks.as<uint8_t>(),
                         d.sigs.as<uint8_t>(), s);
    if (r != COA_OK) return r;
    HIP_TRY(hipMemcpyAsync(pks_out + lo * 32, d.pks.p, cnt * 32, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(sigs_out + lo * 64, d.sigs.p, cnt * 64, hipMemcpyDeviceToHost, s));
    return COA_OK;
  });
}

int coa_ed25519_public_keys(const uint8_t* seeds, size_t n, uint8_t* pks_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!seeds || !pks_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  return for_shards(n, [&](Dev& d, size_t lo, size_t hi) -> int {
    const size_t cnt = hi - lo;
    hipStream_t s = d.stream;
    HIP_TRY(d.seeds.ensure(cnt * 32));
    HIP_TRY(d.pks.ensure(cnt * 32));
    HIP_TRY(d.aux.ensure(cnt * 64));
    HIP_TRY(hipMemcpyAsync(d.seeds.p, seeds + lo * 32, cnt * 32, hipMemcpyHostToDevice, s));
    HIP_TRY(coa_launch_keygen(d.seeds.as<uint8_t>(), (uint32_t)cnt, d.pks.as<uint8_t>(), d.aux.as<uint32_t>(),
                              d.btab, s));
    HIP_TRY(hipMemcpyAsync(pks_out + lo * 32, d.pks.p, cnt * 32, hipMemcpyDeviceToHost, s));
    return COA_OK;
  });
}

int coa_ed25519_sign_many_device(int device, const uint8_t* d_seeds, const uint8_t* d_msgs, size_t msg_len, size_t n,
                                 uint8_t* d_pks_out, uint8_t* d_sigs_out, void* stream) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_seeds || (!d_msgs && msg_len) || !d_pks_out || !d_sigs_out) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  std::lock_guard<std::mutex> l(d->mu);
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  rc = sign_enqueue(*d, d_seeds, d_msgs, msg_len, n, d_pks_out, d_sigs_out, s);
  if (rc != COA_OK) return rc;
  HIP_TRY(hipStreamSynchronize(s));
  return COA_OK;
}


int coa_committee_register(const uint8_t* pks, size_t n) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n && !pks) return fail(COA_EINVAL, "null argument");
  if (n > (1u << 20)) return fail(COA_EINVAL, "committee too large");
  std::vector<std::array<uint32_t, 8>> keys(n);
  for (size_t i = 0; i < n; i++) std::memcpy(keys[i].data(), pks + i * 32, 32);
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  // one generation per device (shared by its contexts), the devices built
  // concurrently on the worker of each device's first context
  std::vector<std::pair<Dev*, std::function<int()>>> tasks;
  for (auto& shp : g_shared) {
    DevShared* sh = shp.get();
    Dev* first = nullptr;
    for (auto& dp : g_devs)
      if (dp->id == sh->id && !first) first = dp.get();
    if (!first) continue;
    tasks.emplace_back(first, [sh, &keys]() -> int { return build_keyset(*sh, keys); });
  }
  rc = run_tasks(tasks);
  if (rc != COA_OK) return rc;
  return (int)keys.size();
}

void* coa_keycache_pin(int device) {
  DevShared* sh = shared_of(device);
  if (!sh) return nullptr;
  std::lock_guard<std::mutex> l(sh->mu);
  return new KeySetP(sh->keys);
}

void coa_keycache_unpin(void* pin) { delete static_cast<KeySetP*>(pin); }

void coa_keycache_use(void* pin) { t_keys_pinned = static_cast<const KeySetP*>(pin); }

void coa_copy_segments(const CoaCopySeg* segs, size_t n) {
  std::vector<CopyPool::Seg> v;
  v.reserve(n);
  for (size_t i = 0; i < n; i++) v.push_back({segs[i].dst, segs[i].src, segs[i].bytes});
  CopyPool::get().copy(v);
}

size_t coa_lat_max(void) { return lat_max(); }

int coa_lat_verify_device(int device, const uint8_t* d_in, size_t n, uint32_t* d_res, void* stream) {
  const int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_in || !d_res) return fail(COA_EINVAL, "null argument");
  if (check_n(n) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  LatArgs a;
  std::memset(&a, 0, sizeof(a));
  a.n = (uint32_t)n;
  a.n_inline = 0;
  a.in = reinterpret_cast<const uint32_t*>(d_in);
  a.res = d_res;
  a.tag = 1;
  // the pinned generation (the queue) or the current one: a registration
  // frees a replaced generation only after the device has drained
  const KeySetP ks = keys_now(*d);
  a.keys = ks->ckeys.as<uint32_t>();
  a.kflags = ks->kflags.as<uint32_t>();
  a.ktabs = ks->ktabs.as<uint32_t>();
  a.nk = ks->nkeys;
  a.comb = d->comb;
  const hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_verify_lat(a, s));
  return trail_keys(*d, ks, s);
}

int coa_lat_verify_inline(int device, const uint8_t* h_records, size_t n, uint32_t* res, uint32_t tag, void* stream) {
  const int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!h_records || !res || tag == 0) return fail(COA_EINVAL, "null argument or zero tag");
  if (n > COA_LAT_INLINE) return fail(COA_EINVAL, "more records than the kernel arguments hold");
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  LatArgs a;
  std::memset(&a, 0, sizeof(a));
  a.n = a.n_inline = (uint32_t)n;
  std::memcpy(a.inl, h_records, n * 128);  // msg | pk | R | s, as the device records
  a.res = res;
  a.tag = tag;
  const KeySetP ks = keys_now(*d);  // pinned (the queue) or current; see coa_lat_verify_device
  a.keys = ks->ckeys.as<uint32_t>();
  a.kflags = ks->kflags.as<uint32_t>();
  a.ktabs = ks->ktabs.as<uint32_t>();
  a.nk = ks->nkeys;
  a.comb = d->comb;
  const hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  HIP_TRY(coa_launch_verify_lat(a, s));
  return trail_keys(*d, ks, s);
}

int coa_certificate_verify_publish(int device, const uint8_t* h_base, uint8_t* d_base, size_t in_bytes,
                                   const CoaCertOffsets* off, size_t n, size_t n_votes, uint32_t* d_ctr,
                                   uint32_t* host_res, uint32_t tag, void* stream) {
  const int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (n > 64 || cert_lanes(n + n_votes) != 64) return 1;  // not the latency kernel's size: nothing enqueued
  if (!h_base || !d_base || !off || !d_ctr || !host_res || tag == 0) return fail(COA_EINVAL, "null argument");
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  const CertIn in{h_base + off->hdr,
                  reinterpret_cast<const uint64_t*>(h_base + off->hoff),
                  h_base + off->ids,
                  h_base + off->origins,
                  h_base + off->hsigs,
                  reinterpret_cast<const uint64_t*>(h_base + off->rounds),
                  h_base + off->vpks,
                  h_base + off->vsigs,
                  reinterpret_cast<const uint64_t*>(h_base + off->voff)};
  const KeySetP ks = keys_now(*d);  // pinned (the queue) or current; see coa_lat_verify_device
  static thread_local CertInl ci;
  if (!env_is("COA_CERT_INLINE", "0") && cert_inl_build(ci, in, 0, n)) {
    CertArgs& a = ci.a;
    a = cert_args(*d, *ks, nullptr, CertPack{}, n, n_votes);
    a.status = d_ctr + 1;
    a.host_res = host_res;
    a.done_ctr = d_ctr;
    a.tag = tag;
    HIP_TRY(coa_launch_cert_verify_inl(ci, s));
    return trail_keys(*d, ks, s);
  }
  HIP_TRY(hipMemcpyAsync(d_base, h_base, in_bytes, hipMemcpyHostToDevice, s));
  CertPack p{};
  p.hdata = off->hdr;
  p.hoff = off->hoff;
  p.ids = off->ids;
  p.origins = off->origins;
  p.hsigs = off->hsigs;
  p.rounds = off->rounds;
  p.vpks = off->vpks;
  p.vsigs = off->vsigs;
  p.voff = off->voff;
  CertArgs a = cert_args(*d, *ks, d_base, p, n, n_votes);
  a.status = d_ctr + 1;
  a.host_res = host_res;
  a.done_ctr = d_ctr;
  a.tag = tag;
  HIP_TRY(coa_launch_cert_verify(a, 64, nullptr, s));
  return trail_keys(*d, ks, s);
}

int coa_engine_recoveries(uint64_t* contexts_rebuilt, uint64_t* shards_rerun) {
  if (contexts_rebuilt) *contexts_rebuilt = g_ctx_rebuilt.load();
  if (shards_rerun) *shards_rerun = g_shards_rerun.load();
  return COA_OK;
}

int coa_committee_key_flags(uint32_t* flags_out, size_t cap) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  Dev& d = *g_devs[0];
  std::lock_guard<std::mutex> l(d.mu);
  const KeySetP ks = keys_now(d);
  const size_t nk = std::min<size_t>(ks->nkeys, cap);
  if (nk == 0) return (int)ks->nkeys;
  if (!flags_out) return fail(COA_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(d.id));
  HIP_TRY(hipMemcpyAsync(flags_out, ks->kflags.p, nk * 4, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(hipStreamSynchronize(d.stream));
  return (int)ks->nkeys;
}

int coa_certificate_verify_many(const uint8_t* header_data, const uint64_t* header_offsets, const uint8_t* ids,
                                const uint8_t* origins, const uint8_t* header_sigs, const uint64_t* rounds,
                                const uint8_t* vote_pks, const uint8_t* vote_sigs, const uint64_t* vote_offsets,
                                size_t n, uint64_t rng_seed, uint8_t* status_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  const CertIn in{header_data, header_offsets, ids, origins, header_sigs, rounds, vote_pks, vote_sigs, vote_offsets};
  return certificates_impl(in, n, rng_seed, status_out);
}

int coa_certificate_verify(const uint8_t* header_data, size_t header_len, const uint8_t id[32],
                           const uint8_t origin[32], const uint8_t header_sig[64], uint64_t round,
                           const uint8_t* vote_pks, const uint8_t* vote_sigs, size_t n_votes, uint64_t rng_seed) {
  const uint64_t hoff[2] = {0, (uint64_t)header_len};
  const uint64_t voff[2] = {0, (uint64_t)n_votes};
  uint8_t st = 0;
  const int rc = coa_certificate_verify_many(header_data, hoff, id, origin, header_sig, &round, vote_pks, vote_sigs,
                                             voff, 1, rng_seed, &st);
  return rc != COA_OK ? rc : (int)st;
}

int coa_certificate_resolve_raw(const uint8_t* ids, const uint8_t* origins, const uint8_t* header_sigs,
                                const uint64_t* rounds, const uint8_t* vote_pks, const uint8_t* vote_sigs,
                                const uint64_t* vote_offsets, size_t n, uint32_t* raw, uint8_t* status_out) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!ids || !origins || !header_sigs || !rounds || !vote_offsets || !raw || !status_out ||
      (vote_offsets[n] && (!vote_pks || !vote_sigs)))
    return fail(COA_EINVAL, "null argument");
  // the exact path never reads the header bytes (Header::digest was checked
  // by the fused kernel and its bit stands)
  const CertIn in{nullptr, nullptr, ids, origins, header_sigs, rounds, vote_pks, vote_sigs, vote_offsets};
  rc = resolve_raw(in, n, raw, 0);
  if (rc != COA_OK) return rc;
  for (size_t i = 0; i < n; i++) status_out[i] = (uint8_t)(raw[i] & 7u);
  return COA_OK;
}

size_t coa_certificate_workspace_bytes(size_t n, size_t n_votes) {
  return coa_cert_scratch_bytes(n + n_votes, true);  // the public device call sorts by key
}

int coa_certificate_verify_many_device(int device, const uint8_t* d_header_data, const uint64_t* d_header_offsets,
                                       const uint8_t* d_ids, const uint8_t* d_origins, const uint8_t* d_header_sigs,
                                       const uint64_t* d_rounds, const uint8_t* d_vote_pks,
                                       const uint8_t* d_vote_sigs, const uint64_t* d_vote_offsets, size_t n,
                                       size_t n_votes, uint32_t* d_status, void* workspace, void* stream) {
  // one device-resident round: jobs in key order
  return coa_certificate_verify_many_device_order(device, d_header_data, d_header_offsets, d_ids, d_origins,
                                                  d_header_sigs, d_rounds, d_vote_pks, d_vote_sigs, d_vote_offsets, n,
                                                  n_votes, d_status, workspace, stream, 1);
}

int coa_certificate_verify_many_device_order(int device, const uint8_t* d_header_data,
                                             const uint64_t* d_header_offsets, const uint8_t* d_ids,
                                             const uint8_t* d_origins, const uint8_t* d_header_sigs,
                                             const uint64_t* d_rounds, const uint8_t* d_vote_pks,
                                             const uint8_t* d_vote_sigs, const uint64_t* d_vote_offsets, size_t n,
                                             size_t n_votes, uint32_t* d_status, void* workspace, void* stream,
                                             int key_order) {
  int rc = ensure_init();
  if (rc != COA_OK) return rc;
  if (n == 0) return COA_OK;
  if (!d_header_offsets || !d_ids || !d_origins || !d_header_sigs || !d_rounds || !d_vote_offsets || !d_status ||
      (n_votes && (!d_vote_pks || !d_vote_sigs)))
    return fail(COA_EINVAL, "null argument");
  if (check_n(n + n_votes) != COA_OK) return COA_EINVAL;
  Dev* d = dev_by_id(device);
  if (!d) return fail(COA_EINVAL, "device not opened by coa_init");
  HIP_TRY(hipSetDevice(device));
  hipStream_t s = stream ? (hipStream_t)stream : d->stream;
  CertArgs a;
  a.hdr_data = d_header_data;
  a.hdr_off = d_header_offsets;
  a.ids = reinterpret_cast<const uint32_t*>(d_ids);
  a.origins = reinterpret_cast<const uint32_t*>(d_origins);
  a.hsigs = reinterpret_cast<const uint32_t*>(d_header_sigs);
  a.rounds = d_rounds;
  a.vpks = reinterpret_cast<const uint32_t*>(d_vote_pks);
  a.vsigs = reinterpret_cast<const uint32_t*>(d_vote_sigs);
  a.voff = d_vote_offsets;
  a.nc = (uint32_t)n;
  a.nv = (uint32_t)n_votes;
  a.hdr_blocks = 0;
  const KeySetP ks = keys_now(*d);  // pinned (the queue) or current; see coa_lat_verify_device
  a.keys = ks->ckeys.as<uint32_t>();
  a.kflags = ks->kflags.as<uint32_t>();
  a.ktabs = ks->ktabs.as<uint32_t>();
  a.nk = ks->nkeys;
  a.comb = d->comb;
  a.wcomb = wcomb_of(*d);
  a.kwtabs = (ks->kwide && !env_is("COA_KEY_WCOMB", "0")) ? ks->kwtabs.as<uint32_t>() : nullptr;
  a.kw20 = ks->kw20 ? 1u : 0u;
  a.status = d_status;
  a.key_order = key_order ? 1u : 0u;
  const int lanes = cert_lanes(n + n_votes);
  HIP_TRY(hipMemsetAsync(d_status, 0, n * 4, s));
  if (workspace || lanes == 64) {
    HIP_TRY(coa_launch_cert_verify(a, lanes, static_cast<uint32_t*>(workspace), s));
    return trail_keys(*d, ks, s);
  }
  std::lock_guard<std::mutex> l(d->mu);
  HIP_TRY(d->cscr.ensure(coa_cert_scratch_bytes(n + n_votes, a.key_order != 0)));
  HIP_TRY(coa_launch_cert_verify(a, lanes, d->cscr.as<uint32_t>(), s));
  HIP_TRY(hipStreamSynchronize(s));  // engine-owned workspace: drain before release
  return COA_OK;
}

}  // extern "C"
