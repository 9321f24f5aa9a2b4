// HIP launch backend of the aggregation queue (coa_queue.h), one per lane:
// device slots (four per opened GPU and lane by default:
// COA_QUEUE_SLOTS for the verify lane, COA_QUEUE_DIGEST_SLOTS for the digest
// lane), each with its own stream, event, page-locked staging and device
// buffers.
//
// Hardware queues.  HIP gives a process GPU_MAX_HW_QUEUES hardware queues
// per priority (4 by default, and a node cannot rely on exporting more
// before its first HIP call) and maps every stream onto them; streams that
// share a hardware queue run one after another.  With the engine's context
// streams, a host's own streams and eight slots on four queues, a 14 ms
// digest window would sit in front of a certificate window (round 3:
// queue_round_mix p99 7.2-7.7 ms and c4_stream 4,000/s p50 94 ms on a box
// with the default 4).  So a slot's stream is made to get a hardware queue
// of its own (COA_QUEUE_STREAMS, tools/hwq_probe.hip measures which kind
// does): "cumask" (the default) -- hipExtStreamCreateWithCUMask with every
// CU enabled: HIP never shares a CU-masked stream's queue, whatever
// GPU_MAX_HW_QUEUES says; "priority" -- the high-priority pool (its own 4
// queues) for the verify lane; "plain" -- shared queues (the round-3 form).  launch() packs the
// launch's parts (one per intake shard) straight into one pinned block --
// the parts are never merged first -- issues ONE host-to-device copy, the
// engine's device-resident entry points (asynchronous with an explicit
// workspace, no engine lock) and ONE device-to-host copy on the slot's
// stream, records an event and returns; complete() waits for the event and
// scatters the outputs back to the parts.  So while window N runs on slot A,
// window N + 1 is packed and enqueued on slot B, and the copies of one window
// overlap the kernels of the other.
//
// Per kind:
//   signatures    coa_ed25519_verify_strict_many_device (Signature::verify);
//                 windows of at most COA_LAT_MAX (2,048) signatures take the
//                 latency kernel instead (one workgroup per signature)
//   certificates  coa_certificate_verify_many_device (the fused
//                 Certificate::verify crypto); the certificates whose raw
//                 status words need the exact random-linear-combination check
//                 or carry a key outside the registered committee are left
//                 open by complete() (Window::c_defer) and decided by
//                 resolve() on the lane's resolver thread with
//                 coa_certificate_resolve_raw -- the exact path alone, not a
//                 second fused launch -- while the rest of the window is
//                 answered at once.  A window with certificates pins its
//                 device's key-cache generation from launch to completion
//   digests       coa_sha512_many_device (worker/src/processor.rs:38)
//   vote batches  coa_ed25519_verify_batch_groups in resolve() (host
//                 pointers; bare batches are rare next to whole certificates)
//
// Engine-failure recovery: a failed launch drains its stream (the error code
// kept), its slot is rebuilt (new stream and event, device buffers freed and
// regrown on demand) and freed; the queue then re-runs the window through
// retry() on the recovery context of another device (one per device, used
// only by retries).  COA_QUEUE_FAULT=<k> makes every k-th window's launch
// fail after its input copy is enqueued (fault injection for the recovery
// tests; never set in production).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "coa_committee.h"
#include "coa_latency.h"
#include "coa_queue.h"

#define COA_QUEUE_SLOTS_DEFAULT 4
// The digest lane's windows are one ~14 ms SHA-512 chain each on a few
// waves (L = 64 lanes per batch), so more of them in flight cost the GPU
// nothing and shorten the wait for a slot: at C4's 1,000 batches/s, 8 slots
// give p50 16.0 ms against 19.6 with 4 (profiles/r05_digest_slots_ab.jsonl)
#define COA_QUEUE_DIGEST_SLOTS_DEFAULT 8
#define COA_LAT_RES_WORDS 64  // result words of an inline latency or published certificate window

namespace {

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
inline int64_t ns_between(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
}

struct Grave {  // an outgrown staging buffer (see grow_pinned)
  void* p;
  bool pinned;
};

struct Slot {
  int dev = -1;
  int kind = COA_QUEUE_STREAM_PLAIN;  // how its stream is made
  int lane = 0;
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  void* hin = nullptr;   // pinned input block
  void* hout = nullptr;  // pinned output block
  void* din = nullptr;   // device input block
  void* dout = nullptr;  // device output block
  void* ws = nullptr;    // device workspace (verify + certificates)
  size_t cap_hin = 0, cap_hout = 0, cap_din = 0, cap_dout = 0, cap_ws = 0;
  std::vector<Grave> grave;  // outgrown staging, freed with the slot
  bool busy = false;
  bool launched = false;  // device work was enqueued (complete() must drain it)
  void* keys = nullptr;   // the key-cache generation the launch pinned (coa_keycache_pin)
  bool lat = false;       // the launch's signatures took the latency kernel (result words)
  // a window of at most COA_LAT_INLINE signatures and nothing else: records in
  // the kernel arguments, verdict words straight into lres (page-locked,
  // coherent), which complete() polls for ltag -- no copies, no event wait
  bool inl = false;
  uint32_t* lres = nullptr;  // COA_LAT_RES_WORDS words
  uint32_t ltag = 0;
  // a window of at most 64 certificates and nothing else, on the latency
  // kernel: its last block writes the status words into lres (no status
  // memset, no D2H copy, no event wait; inline arguments when the window
  // fits, coa_certificate_verify_publish); dctr is its device counter block
  bool cpub = false;
  uint32_t* dctr = nullptr;  // 65 device words, zero between launches
  // output offsets of the current launch
  size_t o_v = 0, o_c = 0, o_d = 0;
};

// A slot's staging grows geometrically (twice what a window needs) and an
// outgrown buffer is not freed on the launch path: hipFree / hipHostFree wait
// for the whole device, i.e. for every other slot's window in flight (round
// 4: a 3-batch digest window took 136 ms behind its lane's regrowths at
// 4,000 batches/s).  Outgrown buffers go to the slot's graveyard, freed with
// the slot; the geometric growth bounds them to the final size.
hipError_t grow_pinned(void*& p, size_t& cap, size_t want, std::vector<Grave>& grave) {
  if (want <= cap) return hipSuccess;
  if (p) grave.push_back({p, true});
  p = nullptr;
  cap = 0;
  want = 2 * want + 4096;
  hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
  if (e == hipSuccess) cap = want;
  return e;
}
hipError_t grow_dev(void*& p, size_t& cap, size_t want, std::vector<Grave>& grave) {
  if (want <= cap) return hipSuccess;
  if (p) grave.push_back({p, false});
  p = nullptr;
  cap = 0;
  want = 2 * want + 4096;
  hipError_t e = hipMalloc(&p, want);
  if (e == hipSuccess) cap = want;
  return e;
}
void bury(std::vector<Grave>& grave) {
  for (const Grave& g : grave) (void)(g.pinned ? hipHostFree(g.p) : hipFree(g.p));
  grave.clear();
}

// Process-wide pool of the slots' streams.  Every queue used to create its
// slots' streams and destroy them with the queue: a CU-masked stream is a
// hardware queue of its own, so a process that makes many queues (bench.py
// makes ~40) created and tore down ~500 hardware queues.  Under
// `rocprofv3 --kernel-trace` that ended in a SIGSEGV at address 0x34 inside
// hipExtStreamCreateWithCUMask (round 5, gpurun_out/fullprof.err: stack
// make_stream <- HipBackend::ready <- coa_queue_create <-
// latc_stream_certificates, late in the run; the same section alone
// profiled clean).  A healthy slot's stream now returns here when its queue
// is destroyed and the next queue takes it, so a process holds at most the
// streams of the queues alive at once, and a later queue also skips the
// first-dispatch cost of a new hardware queue (~25-75 ms for a CU-masked
// one).  A stream whose window failed is destroyed, never pooled.
struct PooledStream {
  int dev, kind, prio;
  hipStream_t s;
};
std::mutex g_pool_mu;
std::vector<PooledStream>& stream_pool() {
  static auto* pool = new std::vector<PooledStream>();  // never destroyed: streams outlive static teardown
  return *pool;
}
int slot_prio(const Slot& sl) { return sl.kind == COA_QUEUE_STREAM_PRIORITY && sl.lane == coa_q::LANE_VERIFY; }
hipStream_t pool_take(const Slot& sl) {
  std::lock_guard<std::mutex> l(g_pool_mu);
  auto& pool = stream_pool();
  for (size_t i = 0; i < pool.size(); i++)
    if (pool[i].dev == sl.dev && pool[i].kind == sl.kind && pool[i].prio == slot_prio(sl)) {
      const hipStream_t s = pool[i].s;
      pool[i] = pool.back();
      pool.pop_back();
      return s;
    }
  return nullptr;
}
// Hands a slot's stream to the pool (drained first); a stream that does not
// drain cleanly is destroyed instead.
void pool_give(Slot& sl) {
  if (!sl.s) return;
  if (hipStreamSynchronize(sl.s) == hipSuccess && hipStreamQuery(sl.s) == hipSuccess) {
    std::lock_guard<std::mutex> l(g_pool_mu);
    stream_pool().push_back({sl.dev, sl.kind, slot_prio(sl), sl.s});
  } else {
    (void)hipStreamDestroy(sl.s);
    (void)hipGetLastError();
  }
  sl.s = nullptr;
}

// New stream and event for a slot; its device buffers are freed (regrown by
// the next launch).  The pinned host blocks are kept.  A slot without a
// stream takes one from the pool when one of its kind is there; a slot being
// rebuilt after a failed window gets a fresh one.
int make_stream(Slot& sl) {
  if (hipSetDevice(sl.dev) != hipSuccess) return COA_EHIP;
  const bool rebuild = sl.s != nullptr;
  if (sl.s) {
    (void)hipStreamSynchronize(sl.s);
    (void)hipStreamDestroy(sl.s);
    sl.s = nullptr;
  }
  if (sl.ev) {
    (void)hipEventDestroy(sl.ev);
    sl.ev = nullptr;
  }
  for (void** p : {&sl.din, &sl.dout, &sl.ws, reinterpret_cast<void**>(&sl.dctr)})
    if (*p) {
      (void)hipFree(*p);
      *p = nullptr;
    }
  sl.cap_din = sl.cap_dout = sl.cap_ws = 0;
  bury(sl.grave);
  (void)hipGetLastError();  // a failed launch's error is not sticky for the new stream
  hipError_t e = hipSuccess;
  if (!rebuild) sl.s = pool_take(sl);
  if (sl.s) {
    // pooled
  } else if (sl.kind == COA_QUEUE_STREAM_CUMASK) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, sl.dev) != hipSuccess || cus <= 0)
      return COA_EHIP;
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int c = 0; c < cus; c++) mask[(size_t)c / 32] |= 1u << (c % 32);
    e = hipExtStreamCreateWithCUMask(&sl.s, (uint32_t)mask.size(), mask.data());
  } else if (sl.kind == COA_QUEUE_STREAM_PRIORITY) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return COA_EHIP;
    e = hipStreamCreateWithPriority(&sl.s, hipStreamNonBlocking, sl.lane == coa_q::LANE_VERIFY ? greatest : least);
  } else {
    e = hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking);
  }
  if (e != hipSuccess || hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) != hipSuccess) return COA_EHIP;
  return COA_OK;
}

// True when rocprofv3's tool library is loaded into this process (the
// environment rocprofv3 gives the program it runs).  The slots then use plain
// streams: CU-masked stream creation under its tracer is what faulted in
// round 5 (see stream_pool), and the kernels -- what a profile measures --
// are the same on either kind.
bool under_rocprofiler() { return getenv("ROCP_TOOL_LIBRARIES") || getenv("ROCPROFILER_LIBRARY_CTOR"); }

int stream_kind_env() {
  const char* e = getenv("COA_QUEUE_STREAMS");
  if (!e) return under_rocprofiler() ? COA_QUEUE_STREAM_PLAIN : COA_QUEUE_STREAM_CUMASK;
  const std::string v(e);
  if (v == "plain") return COA_QUEUE_STREAM_PLAIN;
  if (v == "priority") return COA_QUEUE_STREAM_PRIORITY;
  return COA_QUEUE_STREAM_CUMASK;
}

void free_slot(Slot& sl) {
  if (sl.dev < 0) return;
  (void)hipSetDevice(sl.dev);
  if (sl.s) (void)hipStreamSynchronize(sl.s);
  if (sl.hin) (void)hipHostFree(sl.hin);
  if (sl.hout) (void)hipHostFree(sl.hout);
  if (sl.din) (void)hipFree(sl.din);
  if (sl.dout) (void)hipFree(sl.dout);
  if (sl.ws) (void)hipFree(sl.ws);
  if (sl.lres) (void)hipHostFree(sl.lres);
  if (sl.dctr) (void)hipFree(sl.dctr);
  if (sl.ev) (void)hipEventDestroy(sl.ev);
  pool_give(sl);
  bury(sl.grave);
}

class HipBackend : public coa_q::Backend {
 public:
  explicit HipBackend(int lane) : lane_(lane) {}
  ~HipBackend() override {
    for (Slot& sl : slots_) free_slot(sl);
    for (Slot& sl : rescue_) free_slot(sl);
  }

  int slots() const override { return (int)slots_.size(); }
  int devices() const override { return std::max<int>(1, (int)devs_.size()); }
  // windows of this queue lane that had to enlarge a slot's staging or
  // workspace (the warm-up at creation not counted)
  uint64_t grows() const override { return grows_.load(); }
  void reset_grows() override { grows_.store(0); }

  // Everything a first window would otherwise pay for, done at queue
  // creation: the slots' streams, their page-locked and device staging, and
  // one small copy through each stream, which makes HIP create the stream's
  // hardware queue (a CU-masked stream's first dispatch took ~25-75 ms:
  // round-4 paced runs, one queue per rate, p99 20-75 ms from that alone).
  //
  // The verify lane is sized for the largest window the collector can close:
  // whole shards are taken until max_batch items are in, and a shard holds up
  // to max_batch items, so a window holds < 2 x max_batch items.  Certificate
  // items (a certificate and its votes: 9,920 B per committee-100 certificate
  // of 68 items) take <= 160 B each in the input block, signatures 128 B.
  // Sized for half of that (grow_* double it), staging never regrows on the
  // launch path (round 4's streamed C3 regrew 2-4 times per run, windows of
  // up to 107 K items, p99 wait 8-12 ms).
  void prepare(size_t max_batch) override {
    if (!ready()) return;
    // capped at 65,536 (a larger max_batch's windows regrow on demand): a
    // queue made with max_batch 2^20 would otherwise stage ~20 GB of HBM
    const size_t items = std::min<size_t>(std::max<size_t>(max_batch, 1024), 65536);
    const size_t pre_in = lane_ == coa_q::LANE_DIGEST ? (32u << 20) : items * 160 + (1u << 20);
    const size_t pre_out = lane_ == coa_q::LANE_DIGEST ? (256u << 10) : items * 4 + (64u << 10);
    // workspace for the widest window of each kind (each regrowth is a
    // hipMalloc on the launch path: the round mix showed 6-9 per queue, with
    // windows held 3-12 ms)
    const size_t pre_ws = lane_ == coa_q::LANE_DIGEST
                              ? 256
                              : std::max(coa_verify_workspace_bytes(items),
                                         coa_cert_scratch_bytes(items / 68 + 1 + items, keysort_)) + 256;
    for (Slot& sl : slots_) {
      if (lane_ == coa_q::LANE_VERIFY && hipSetDevice(sl.dev) == hipSuccess) {
        (void)lat_words(sl);
        (void)ctr_words(sl);
      }
      if (hipSetDevice(sl.dev) != hipSuccess || grow_pinned(sl.hin, sl.cap_hin, pre_in, sl.grave) != hipSuccess ||
          grow_pinned(sl.hout, sl.cap_hout, pre_out, sl.grave) != hipSuccess ||
          grow_dev(sl.din, sl.cap_din, pre_in, sl.grave) != hipSuccess ||
          grow_dev(sl.dout, sl.cap_dout, pre_out, sl.grave) != hipSuccess ||
          grow_dev(sl.ws, sl.cap_ws, pre_ws, sl.grave) != hipSuccess)
        continue;  // the first launch regrows and reports any failure
      (void)hipMemcpyAsync(sl.din, sl.hin, 4096, hipMemcpyHostToDevice, sl.s);
      (void)hipMemsetAsync(sl.dout, 0, 4096, sl.s);
      (void)hipStreamSynchronize(sl.s);
    }
    (void)hipGetLastError();
  }
  int stream_kind() const override { return kind_; }

  // The slot's page-locked result words for inline latency windows
  // (allocated once; null when the allocation failed: such windows then take
  // the staged path)
  static uint32_t* lat_words(Slot& sl) {
    if (!sl.lres && hipHostMalloc(reinterpret_cast<void**>(&sl.lres), COA_LAT_RES_WORDS * sizeof(uint32_t),
                                  hipHostMallocCoherent) != hipSuccess) {
      sl.lres = nullptr;
      (void)hipGetLastError();
    }
    return sl.lres;
  }
  // ... and its device counter block for published certificate windows
  // (zeroed once; the kernel re-zeroes it after each window)
  static uint32_t* ctr_words(Slot& sl) {
    if (!sl.dctr) {
      if (hipMalloc(reinterpret_cast<void**>(&sl.dctr), 65 * sizeof(uint32_t)) != hipSuccess ||
          hipMemset(sl.dctr, 0, 65 * sizeof(uint32_t)) != hipSuccess) {
        if (sl.dctr) (void)hipFree(sl.dctr);
        sl.dctr = nullptr;
        (void)hipGetLastError();
      }
    }
    return sl.dctr;
  }

  void launch(coa_q::Launch& L) override {
    if (!ready()) {
      L.rc = init_rc_;
      return;
    }
    Slot* sl;
    bool inject = false;
    {
      // the next free slot in turn (a busy slot is passed over, not waited for)
      std::unique_lock<std::mutex> l(m_);
      auto free_slot = [&]() -> long {
        for (size_t k = 0; k < slots_.size(); k++) {
          const size_t i = (next_ + k) % slots_.size();
          if (!slots_[i].busy) return (long)i;
        }
        return -1;
      };
      long k = free_slot();
      if (k < 0) {
        const auto t0 = std::chrono::steady_clock::now();
        cv_.wait(l, [&] { return (k = free_slot()) >= 0; });
        L.slot_wait_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                             .count();
      }
      next_ = (size_t)k + 1;
      slots_[k].busy = true;
      L.slot = (int)k;
      sl = &slots_[k];
      inject = fault_every_ && ++launches_ % fault_every_ == 0;
    }
    sl->launched = false;
    L.rc = enqueue(*sl, L, inject);
  }

  bool wait_free_slot() override {
    if (!ready()) return false;
    std::unique_lock<std::mutex> l(m_);
    auto any_free = [&] {
      for (const Slot& s : slots_)
        if (!s.busy) return true;
      return false;
    };
    if (any_free()) return false;
    cv_.wait(l, any_free);
    return true;
  }

  void complete(coa_q::Launch& L) override {
    if (L.slot < 0) return;  // never staged (no device)
    Slot& sl = slots_[L.slot];
    finish(sl, L);
    if (L.rc != COA_OK) (void)make_stream(sl);  // rebuilt before reuse
    std::lock_guard<std::mutex> l(m_);
    sl.busy = false;
    cv_.notify_all();
  }

  void retry(coa_q::Launch& L, int attempt) override {
    if (!ready() || devs_.empty()) {
      L.rc = init_rc_ != COA_OK ? init_rc_ : COA_ENODEVICE;
      return;
    }
    size_t pos = 0;
    if (L.slot >= 0)
      for (size_t i = 0; i < devs_.size(); i++)
        if (devs_[i] == slots_[L.slot].dev) pos = i;
    Slot& sl = rescue_[(pos + (size_t)attempt) % devs_.size()];
    if (!sl.s && make_stream(sl) != COA_OK) {
      L.rc = COA_EHIP;
      return;
    }
    sl.launched = false;
    L.rc = enqueue(sl, L, false);
    finish(sl, L);
    if (L.rc != COA_OK) (void)make_stream(sl);
  }

 private:
  bool ready() {
    std::lock_guard<std::mutex> l(m_);
    if (inited_) return init_rc_ == COA_OK;
    inited_ = true;
    int ids[64];
    const int n = coa_device_ids(ids, 64);
    if (n <= 0) {
      init_rc_ = n < 0 ? n : COA_ENODEVICE;
      return false;
    }
    const int nctx = std::min(n, 64);
    for (int i = 0; i < nctx; i++)
      if (std::find(devs_.begin(), devs_.end(), ids[i]) == devs_.end()) devs_.push_back(ids[i]);
    // device slots per GPU (not per engine context: eight contexts open on
    // one GPU made 32 slots per lane there, 64 CU-masked streams and so 64
    // hardware queues on one device, more than its scheduler maps at once --
    // the suspected cause of round 4's 84-149 ms window on a re-opened
    // 8-context engine): windows in flight at once (1..8; COA_QUEUE_SLOTS for
    // the verify lane, COA_QUEUE_DIGEST_SLOTS for the digest lane;
    // tools/queue_probe.c measures the choice)
    size_t per = lane_ == coa_q::LANE_DIGEST ? COA_QUEUE_DIGEST_SLOTS_DEFAULT : COA_QUEUE_SLOTS_DEFAULT;
    if (const char* e = getenv(lane_ == coa_q::LANE_DIGEST ? "COA_QUEUE_DIGEST_SLOTS" : "COA_QUEUE_SLOTS")) {
      const int v = atoi(e);
      if (v >= 1 && v <= 8) per = (size_t)v;
    }
    if (const char* e = getenv("COA_QUEUE_FAULT")) fault_every_ = strtoull(e, nullptr, 10);
    // COA_QUEUE_INLINE=0: small signature windows take the staged path too (A/B)
    if (const char* e = getenv("COA_QUEUE_INLINE")) inline_ok_ = e[0] != '0';
    // COA_QUEUE_KEYSORT=0|1: certificate windows of >= 16,384 jobs take their
    // jobs in committee-key order (coa_certificate_verify_many_device_order).
    // Default on: round 6's same-box A/B of the streamed C3 lines was within
    // noise either way (profiles/r06_keysort_ab.txt), and the fused kernel's
    // translation misses fall from ~50 % to ~1.5 % of requests in key order
    // (round 5); coa_committee.hip's note that queue windows do not sort
    // predates this switch
    if (const char* e = getenv("COA_QUEUE_KEYSORT")) keysort_ = e[0] != '0';
    kind_ = stream_kind_env();
    slots_.resize(per * devs_.size());
    // (page-locked staging is sized by prepare(): a reallocation on the
    // launch path is a hipHostFree/hipHostMalloc pair, milliseconds)
    for (size_t k = 0; k < slots_.size(); k++) {
      Slot& sl = slots_[k];
      sl.dev = devs_[k % devs_.size()];
      sl.kind = kind_;
      sl.lane = lane_;
      if (make_stream(sl) != COA_OK) {
        init_rc_ = COA_EHIP;
        return false;
      }
    }
    rescue_.resize(devs_.size());
    for (size_t i = 0; i < devs_.size(); i++) {
      rescue_[i].dev = devs_[i];
      rescue_[i].kind = kind_;
      rescue_[i].lane = lane_;
    }
    return true;
  }

  // Input block: verify msgs | pks | sigs, certificate arrays, digest data |
  // offsets (256-byte aligned sections), each section the parts' arrays one
  // after another (offsets rebased).  Output block: verdicts | status words |
  // 64-byte digests.
  int enqueue(Slot& sl, coa_q::Launch& L, bool inject) {
    if (hipSetDevice(sl.dev) != hipSuccess) return COA_EHIP;
    const auto t_pack = std::chrono::steady_clock::now();
    // a window of few signatures takes the latency kernel (one four-wave
    // workgroup per signature: ~0.1 ms however few, against ~0.8 ms for the
    // one-lane throughput kernels); its inputs are interleaved 128-byte
    // records and its results 32-bit words
    sl.lat = L.nv > 0 && L.nv <= coa_lat_max();
    size_t o = 0;
    auto take = [&](size_t bytes) {
      const size_t at = o;
      o = al256(o + bytes);
      return at;
    };
    const size_t i_vm = take(L.nv * (sl.lat ? 128 : 32)), i_vp = take(sl.lat ? 0 : L.nv * 32),
                 i_vs = take(sl.lat ? 0 : L.nv * 64);
    const size_t i_ch = take(L.hbytes + 16), i_cho = take((L.nc + 1) * 8), i_cid = take(L.nc * 32),
                 i_cor = take(L.nc * 32), i_chs = take(L.nc * 64), i_crd = take(L.nc * 8),
                 i_cvp = take(L.nvotes * 32), i_cvs = take(L.nvotes * 64), i_cvo = take((L.nc + 1) * 8);
    const size_t i_dd = take(L.dbytes + 16), i_do = take((L.nd + 1) * 8);
    const size_t in_bytes = o;
    o = 0;
    sl.o_v = take(sl.lat ? L.nv * 4 : L.nv);
    sl.o_c = take(L.nc * 4);
    sl.o_d = take(L.nd * 64);
    const size_t out_bytes = o;
    const size_t ws_v = L.nv ? coa_verify_workspace_bytes(L.nv) : 0;
    const size_t ws_c = L.nc ? coa_cert_scratch_bytes(L.nc + L.nvotes, keysort_) : 0;
    const size_t caps0 = sl.cap_hin + sl.cap_hout + sl.cap_din + sl.cap_dout + sl.cap_ws;
    if (grow_pinned(sl.hin, sl.cap_hin, in_bytes, sl.grave) != hipSuccess ||
        grow_pinned(sl.hout, sl.cap_hout, out_bytes, sl.grave) != hipSuccess ||
        grow_dev(sl.din, sl.cap_din, in_bytes, sl.grave) != hipSuccess ||
        grow_dev(sl.dout, sl.cap_dout, out_bytes, sl.grave) != hipSuccess ||
        grow_dev(sl.ws, sl.cap_ws, std::max(ws_v, ws_c) + 256, sl.grave) != hipSuccess)
      return COA_ENOMEM;
    if (sl.cap_hin + sl.cap_hout + sl.cap_din + sl.cap_dout + sl.cap_ws != caps0) grows_++;
    uint8_t* h = static_cast<uint8_t*>(sl.hin);
    // the bulk copies of a large window go to the runtime's copy threads (a
    // C3 round is ~68 MB: one thread's memcpy would be slower than PCIe)
    std::vector<CoaCopySeg> bulk;
    auto copy = [&bulk](void* dst, const void* src, size_t bytes) {
      if (bytes) bulk.push_back({dst, src, bytes});
    };
    size_t v = 0, c = 0, cv = 0, hb = 0, dn = 0, db = 0;
    uint64_t* cho = reinterpret_cast<uint64_t*>(h + i_cho);
    uint64_t* cvo = reinterpret_cast<uint64_t*>(h + i_cvo);
    uint64_t* dof = reinterpret_cast<uint64_t*>(h + i_do);
    cho[0] = cvo[0] = dof[0] = 0;
    for (const coa_q::Window* w : L.parts) {
      if (w->nv && sl.lat) {  // i_vm .. : [nv][msg | pk | R | s]
        for (size_t i = 0; i < w->nv; i++) {
          uint8_t* r = h + i_vm + (v + i) * 128;
          std::memcpy(r, w->v_msgs.data() + i * 32, 32);
          std::memcpy(r + 32, w->v_pks.data() + i * 32, 32);
          std::memcpy(r + 64, w->v_sigs.data() + i * 64, 64);
        }
        v += w->nv;
      } else if (w->nv) {
        copy(h + i_vm + v * 32, w->v_msgs.data(), w->nv * 32);
        copy(h + i_vp + v * 32, w->v_pks.data(), w->nv * 32);
        copy(h + i_vs + v * 64, w->v_sigs.data(), w->nv * 64);
        v += w->nv;
      }
      // certificates from their refs (the window's own bytes, or a borrowed
      // request's arrays): the small fixed fields here, the header input and
      // the votes (~9.7 KB of a C3 certificate's 9.9) as bulk segments
      for (size_t i = 0; i < w->nc; i++, c++) {
        const coa_q::Window::CertRef& r = w->c_refs[i];
        copy(h + i_ch + hb, r.hdr, r.hlen);
        hb += r.hlen;
        cho[c + 1] = hb;
        std::memcpy(h + i_cid + c * 32, r.id, 32);
        std::memcpy(h + i_cor + c * 32, r.origin, 32);
        std::memcpy(h + i_chs + c * 64, r.hsig, 64);
        std::memcpy(h + i_crd + c * 8, &r.round, 8);
        copy(h + i_cvp + cv * 32, r.vpks, r.nv * 32);
        copy(h + i_cvs + cv * 64, r.vsigs, r.nv * 64);
        cv += r.nv;
        cvo[c + 1] = cv;
      }
      if (w->nd) {
        copy(h + i_dd + db, w->d_data.data(), w->d_data.size());
        for (size_t i = 1; i <= w->nd; i++) dof[dn + i] = db + w->d_offs[i];
        dn += w->nd;
        db += w->d_data.size();
      }
    }
    size_t bulk_bytes = 0;
    for (const CoaCopySeg& g : bulk) bulk_bytes += g.bytes;
    if (bulk_bytes >= (1u << 20)) {
      coa_copy_segments(bulk.data(), bulk.size());
    } else {
      for (const CoaCopySeg& g : bulk) std::memcpy(g.dst, g.src, g.bytes);
    }
    const auto t_enq = std::chrono::steady_clock::now();
    L.stage_ns[COA_QSTAGE_PACK] += ns_between(t_pack, t_enq);
    if (L.nv + L.nc + L.nd == 0) return COA_OK;  // bare vote batches only: left to resolve()
    struct EnqClock {  // ENQUEUE stage: every return below
      coa_q::Launch& L;
      std::chrono::steady_clock::time_point t;
      ~EnqClock() { L.stage_ns[COA_QSTAGE_ENQUEUE] += ns_between(t, std::chrono::steady_clock::now()); }
    } enq_clock{L, t_enq};
    // the ENQUEUE stage's parts (Launch::enq_ns): each mark() charges the time
    // since the previous one to part k
    auto t_mark = t_enq;
    auto mark = [&](int k) {
      const auto t = std::chrono::steady_clock::now();
      L.enq_ns[k] += ns_between(t_mark, t);
      t_mark = t;
    };
    sl.cpub = false;
    sl.inl = inline_ok_ && sl.lat && L.nv <= COA_LAT_INLINE && L.nc == 0 && L.nd == 0 && lat_words(sl) != nullptr;
    if (sl.inl) {
      // a few signatures alone (Header::verify / Vote::verify at low load):
      // the packed records go in the kernel arguments and the verdict words
      // come back by the kernel's own stores, as coa_ed25519_verify_strict
      // does -- the staged path's two copies (and the event wait) were most
      // of such a window's time besides the kernel
      std::memset(sl.lres, 0, L.nv * sizeof(uint32_t));  // no tag matches 0
      sl.ltag = (sl.ltag + 1) & 0xffffffu;
      if (sl.ltag == 0) sl.ltag = 1;
      sl.launched = true;
      if (inject) return COA_EHIP;  // fault injection: nothing launched
      if (!sl.keys) sl.keys = coa_keycache_pin(sl.dev);
      coa_keycache_use(sl.keys);
      mark(coa_q::Launch::ENQ_PIN);
      const int rc = coa_lat_verify_inline(sl.dev, h + i_vm, L.nv, sl.lres, sl.ltag, sl.s);
      coa_keycache_use(nullptr);
      mark(coa_q::Launch::ENQ_LAUNCH);
      if (rc != COA_OK) return rc;
      const hipError_t er = hipEventRecord(sl.ev, sl.s);
      mark(coa_q::Launch::ENQ_EVENT);
      return er == hipSuccess ? COA_OK : COA_EHIP;
    }
    sl.cpub = inline_ok_ && L.nc > 0 && L.nc <= COA_LAT_RES_WORDS && L.nv == 0 && L.nd == 0 &&
              lat_words(sl) != nullptr && ctr_words(sl) != nullptr;
    if (sl.cpub) {
      // certificates alone, few (Certificate::verify at low load): see Slot::cpub
      if (inject) {
        sl.launched = true;
        return COA_EHIP;  // fault injection: nothing launched
      }
      std::memset(sl.lres, 0, L.nc * sizeof(uint32_t));
      sl.ltag = (sl.ltag + 1) & 0xffffffu;
      if (sl.ltag == 0) sl.ltag = 1;
      if (!sl.keys) sl.keys = coa_keycache_pin(sl.dev);
      coa_keycache_use(sl.keys);
      mark(coa_q::Launch::ENQ_PIN);
      const CoaCertOffsets off{i_ch, i_cho, i_cid, i_cor, i_chs, i_crd, i_cvp, i_cvs, i_cvo};
      const int rc = coa_certificate_verify_publish(sl.dev, h, static_cast<uint8_t*>(sl.din), in_bytes, &off, L.nc,
                                                    L.nvotes, sl.dctr, sl.lres, sl.ltag, sl.s);
      coa_keycache_use(nullptr);
      mark(coa_q::Launch::ENQ_LAUNCH);  // (its H2D copy, when the window does not fit the arguments, included)
      if (rc == COA_OK) {
        sl.launched = true;
        const hipError_t er = hipEventRecord(sl.ev, sl.s);
        mark(coa_q::Launch::ENQ_EVENT);
        return er == hipSuccess ? COA_OK : COA_EHIP;
      }
      if (rc != 1) {
        sl.launched = true;  // something may be enqueued: finish() drains the stream
        return rc;
      }
      sl.cpub = false;  // too many jobs for the latency kernel: the staged path below
    }
    uint8_t* d = static_cast<uint8_t*>(sl.din);
    uint8_t* dout = static_cast<uint8_t*>(sl.dout);
    if (hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, sl.s) != hipSuccess) return COA_EHIP;
    mark(coa_q::Launch::ENQ_H2D);
    sl.launched = true;
    if (inject) return COA_EHIP;  // fault injection: the copy is in flight, the kernels never run
    int rc = COA_OK;
    // both read the committee key cache: the launch pins the current
    // generation until complete() (a registration meanwhile builds the next
    // one beside it) and its launches read that one
    if ((sl.lat || L.nc) && !sl.keys) sl.keys = coa_keycache_pin(sl.dev);
    coa_keycache_use(sl.keys);
    mark(coa_q::Launch::ENQ_PIN);
    if (L.nv && sl.lat)
      rc = coa_lat_verify_device(sl.dev, d + i_vm, L.nv, reinterpret_cast<uint32_t*>(dout + sl.o_v), sl.s);
    else if (L.nv)
      rc = coa_ed25519_verify_strict_many_device(sl.dev, d + i_vm, 32, d + i_vp, d + i_vs, L.nv, dout + sl.o_v, sl.ws,
                                                 sl.s);
    if (rc == COA_OK && L.nc) {
      // key order for a large window (COA_QUEUE_KEYSORT): see
      // coa_certificate_verify_many_device_order
      rc = coa_certificate_verify_many_device_order(
          sl.dev, d + i_ch, reinterpret_cast<const uint64_t*>(d + i_cho), d + i_cid, d + i_cor, d + i_chs,
          reinterpret_cast<const uint64_t*>(d + i_crd), d + i_cvp, d + i_cvs,
          reinterpret_cast<const uint64_t*>(d + i_cvo), L.nc, L.nvotes, reinterpret_cast<uint32_t*>(dout + sl.o_c),
          sl.ws, sl.s, keysort_ ? 1 : 0);
    }
    if (rc == COA_OK && L.nd)
      rc = coa_sha512_many_device(sl.dev, d + i_dd, reinterpret_cast<const uint64_t*>(d + i_do), L.nd, dout + sl.o_d,
                                  sl.s);
    coa_keycache_use(nullptr);
    mark(coa_q::Launch::ENQ_LAUNCH);
    if (rc != COA_OK) return rc;
    if (hipMemcpyAsync(sl.hout, dout, out_bytes, hipMemcpyDeviceToHost, sl.s) != hipSuccess) return COA_EHIP;
    mark(coa_q::Launch::ENQ_D2H);
    if (hipEventRecord(sl.ev, sl.s) != hipSuccess) return COA_EHIP;
    mark(coa_q::Launch::ENQ_EVENT);
    return COA_OK;
  }

  // Waits for the slot's work (a failed enqueue drains its stream, keeping
  // the error), then scatters the outputs to the parts; what the kernels left
  // open (and every bare vote batch) is marked for resolve().
  void finish(Slot& sl, coa_q::Launch& L) {
    const auto t_wait = std::chrono::steady_clock::now();
    if (sl.launched) {
      (void)hipSetDevice(sl.dev);
      if (L.rc == COA_OK && (sl.inl || sl.cpub)) {
        L.rc = poll_words(sl, sl.inl ? L.nv : L.nc);
      } else if (L.rc == COA_OK) {
        if (hipEventSynchronize(sl.ev) != hipSuccess) L.rc = COA_EHIP;
      } else {
        (void)hipStreamSynchronize(sl.s);  // nothing may still read the staging when the slot is reused
      }
      sl.launched = false;
    }
    const auto t_scatter = std::chrono::steady_clock::now();
    L.stage_ns[COA_QSTAGE_DEVICE_WAIT] += ns_between(t_wait, t_scatter);
    if (L.rc == COA_OK) {
      const uint8_t* h = static_cast<const uint8_t*>(sl.hout);
      size_t v = 0, c = 0, dn = 0;
      for (coa_q::Window* w : L.parts) {
        if (w->nv && sl.lat) {
          const uint32_t* words = (sl.inl ? sl.lres : reinterpret_cast<const uint32_t*>(h + sl.o_v)) + v;
          for (size_t i = 0; i < w->nv; i++) w->v_out[i] = (uint8_t)(words[i] & 0xffu);
        } else if (w->nv) {
          std::memcpy(w->v_out.data(), h + sl.o_v + v, w->nv);
        }
        for (size_t i = 0; i < w->nd; i++) std::memcpy(&w->d_out[i * 32], h + sl.o_d + (dn + i) * 64, 32);
        if (w->nc && sl.cpub) {
          uint32_t st[COA_LAT_RES_WORDS];
          for (size_t i = 0; i < w->nc; i++) st[i] = sl.lres[c + i] & 0xffu;  // the tag off
          scatter_certs(*w, st);
        } else if (w->nc) {
          scatter_certs(*w, reinterpret_cast<const uint32_t*>(h + sl.o_c) + c);
        }
        w->g_defer = w->ng > 0;
        v += w->nv;
        c += w->nc;
        dn += w->nd;
      }
    }
    if (sl.keys) {
      coa_keycache_unpin(sl.keys);
      sl.keys = nullptr;
    }
    L.stage_ns[COA_QSTAGE_SCATTER] += ns_between(t_scatter, std::chrono::steady_clock::now());
  }

  // An inline latency window's n result words, polled for the slot's tag.
  // A kernel that ended without publishing (a fault) ends the wait through
  // the slot's event; a bound stops a hang.  On failure the stream is
  // drained before the slot is reused.
  static int poll_words(Slot& sl, size_t n) {
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < n; i++) {
      const volatile uint32_t* w = sl.lres + i;
      for (uint64_t spin = 0; (*w >> 8) != sl.ltag; spin++) {
        if ((spin & 1023) != 1023) continue;
        const hipError_t q = hipEventQuery(sl.ev);
        const bool stuck = std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10);
        if ((q != hipSuccess && q != hipErrorNotReady) || (q == hipSuccess && (*w >> 8) != sl.ltag) || stuck) {
          (void)hipStreamSynchronize(sl.s);
          return COA_EHIP;
        }
      }
    }
    return COA_OK;
  }

  // Raw certificate status words -> COA_CERT_* bits; the certificates the
  // fused kernel could not decide alone keep their raw words and are left
  // open for resolve().
  static void scatter_certs(coa_q::Window& w, const uint32_t* st) {
    w.c_raw.assign(st, st + w.nc);
    w.c_defer.clear();
    for (size_t c = 0; c < w.nc; c++) {
      // exactly the words coa_certificate_resolve_raw re-decides: a key
      // outside the committee, or inconclusive votes not already bad
      const bool open = (st[c] & COA_CST_UNCACHED) ||
                        ((st[c] & COA_CST_VOTES_INCONCLUSIVE) && !(st[c] & COA_CST_BAD_VOTES));
      if (open) w.c_defer.push_back((uint32_t)c);
      w.c_out[c] = (uint8_t)(st[c] & 7u);
    }
  }

 public:
  // The open certificates of every window in `ws` in one exact pass
  // (coa_certificate_resolve_raw: header signature by verify_strict and votes
  // by the RLC kernels for a key outside the committee, the RLC kernels alone
  // for inconclusive votes -- never the fused kernel again), and every bare
  // vote batch in one coa_ed25519_verify_batch_groups call.
  int resolve(const std::vector<coa_q::Window*>& ws) override {
    std::vector<uint8_t> ids, org, hs, vp, vs;
    std::vector<uint64_t> rd, vo{0};
    std::vector<uint32_t> raw;
    std::vector<uint8_t> gm, gp, gs;
    std::vector<uint64_t> go{0};
    for (const coa_q::Window* w : ws) {
      for (uint32_t c : w->c_defer) {
        const coa_q::Window::CertRef& r = w->c_refs[c];
        ids.insert(ids.end(), r.id, r.id + 32);
        org.insert(org.end(), r.origin, r.origin + 32);
        hs.insert(hs.end(), r.hsig, r.hsig + 64);
        rd.push_back(r.round);
        vp.insert(vp.end(), r.vpks, r.vpks + r.nv * 32);
        vs.insert(vs.end(), r.vsigs, r.vsigs + r.nv * 64);
        vo.push_back(vp.size() / 32);
        raw.push_back(w->c_raw[c]);
      }
      if (w->g_defer) {
        gm.insert(gm.end(), w->g_msgs.begin(), w->g_msgs.end());
        gp.insert(gp.end(), w->g_pks.begin(), w->g_pks.end());
        gs.insert(gs.end(), w->g_sigs.begin(), w->g_sigs.end());
        for (size_t g = 1; g <= w->ng; g++) go.push_back(go.back() + (w->g_offs[g] - w->g_offs[g - 1]));
      }
    }
    if (!raw.empty()) {
      std::vector<uint8_t> out(raw.size(), 7);
      const int rc = coa_certificate_resolve_raw(ids.data(), org.data(), hs.data(), rd.data(), vp.data(), vs.data(),
                                                 vo.data(), raw.size(), raw.data(), out.data());
      if (rc != COA_OK) return rc;
      size_t j = 0;
      for (coa_q::Window* w : ws)
        for (uint32_t c : w->c_defer) w->c_out[c] = out[j++];
    }
    if (go.size() > 1) {
      std::vector<uint8_t> out(go.size() - 1, 1);
      const int rc = coa_ed25519_verify_batch_groups(gm.data(), gp.data(), gs.data(), go.data(), go.size() - 1,
                                                     out.data(), 0);
      if (rc != COA_OK) return rc;
      size_t j = 0;
      for (coa_q::Window* w : ws)
        if (w->g_defer)
          for (size_t g = 0; g < w->ng; g++) w->g_out[g] = out[j++];
    }
    return COA_OK;
  }

 private:
  std::vector<Slot> slots_;
  std::vector<Slot> rescue_;  // one recovery context per device, used only by retry()
  std::vector<int> devs_;     // distinct device ids
  const int lane_;
  int kind_ = COA_QUEUE_STREAM_PLAIN;
  std::atomic<uint64_t> grows_{0};
  size_t next_ = 0;
  std::mutex m_;
  std::condition_variable cv_;
  bool inited_ = false;
  int init_rc_ = COA_OK;
  unsigned long long fault_every_ = 0, launches_ = 0;
  bool inline_ok_ = true;  // COA_QUEUE_INLINE
  bool keysort_ = true;     // COA_QUEUE_KEYSORT
};

}  // namespace

coa_q::Backend* coa_q::make_backend(int lane) { return new HipBackend(lane); }
