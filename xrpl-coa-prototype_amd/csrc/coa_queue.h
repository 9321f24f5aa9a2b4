// Internal interface between the aggregation queue (coa_queue.cpp: request
// intake, windows, callbacks, metrics, recovery; no HIP) and its launch
// backend (coa_queue_hip.cpp: pinned staging, HIP streams and events over the
// device-resident entry points; the sanitizer and CPU tests link a stub
// instead, tests/sanitize/queue_tsan.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "../../include/coa_verify.h"

namespace coa_q {

// One intake shard's requests, packed contiguously by kind (the arrays the
// engine's batched entry points take).  A launch takes the windows of every
// shard that had requests (its "parts") and the backend packs them straight
// into its pinned staging block -- the parts are never merged on the host.
// The backend fills each part's outputs.
struct Window {
  // header / vote signatures (coa_ed25519_verify_strict semantics)
  size_t nv = 0;
  std::vector<uint8_t> v_msgs, v_pks, v_sigs;  // nv x 32, 32, 64
  std::vector<uint8_t> v_out;                  // nv verdicts
  // bare vote batches (coa_ed25519_verify_batch_groups semantics)
  size_t ng = 0;
  std::vector<uint8_t> g_msgs, g_pks, g_sigs;
  std::vector<uint64_t> g_offs;  // ng + 1
  std::vector<uint8_t> g_out;    // ng verdicts
  // whole certificates (coa_certificate_verify_many semantics), one CertRef
  // each.  A copied request (coa_queue_submit_certificate) keeps its bytes in
  // c_own -- header input | id | origin | header signature | vote keys | vote
  // signatures -- and its ref holds offsets into c_own until bind(); a
  // borrowed one (coa_queue_submit_certificate_borrowed) points at the
  // caller's arrays, which stay valid until its callback.  After bind() (the
  // collector's take) every ref holds pointers, which the backend packs from
  // and the resolver reads.
  struct CertRef {
    const uint8_t *hdr, *id, *origin, *hsig, *vpks, *vsigs;
    uint64_t hlen, round, nv;
    bool owned;
  };
  size_t nc = 0;
  std::vector<CertRef> c_refs;
  std::vector<uint8_t> c_own;
  uint64_t c_votes = 0, c_hbytes = 0;  // totals over the window's certificates
  std::vector<uint8_t> c_out;          // nc status bytes (COA_CERT_* bits)
  // worker batch digests (coa_sha512_trunc32_many semantics)
  size_t nd = 0;
  std::vector<uint8_t> d_data;
  std::vector<uint64_t> d_offs;  // nd + 1
  std::vector<uint8_t> d_out;    // nd x 32
  // Left open by Backend::complete (or retry) for the lane's resolver
  // (Backend::resolve): certificates the fused kernel could not decide alone
  // (their raw status words kept) and, with g_defer, every bare vote batch.
  // Their requests are answered after the rest of the window.
  std::vector<uint32_t> c_raw;    // nc raw status words (COA_CST_*), or empty
  std::vector<uint32_t> c_defer;  // ascending certificate indices
  bool g_defer = false;
  int64_t intake_ns = 0;          // producers' time copying requests in (COA_QSTAGE_INTAKE)

  bool deferred() const { return !c_defer.empty() || (g_defer && ng); }
  bool is_deferred_cert(uint32_t c) const { return std::binary_search(c_defer.begin(), c_defer.end(), c); }
  size_t items() const { return nv + nd + nc + c_votes + g_offs.back(); }
  // Owned refs' offsets -> pointers into c_own (which no longer changes once
  // the collector has taken the window).
  void bind() {
    const uintptr_t base = reinterpret_cast<uintptr_t>(c_own.data());
    for (CertRef& r : c_refs)
      if (r.owned) {
        for (const uint8_t** f : {&r.hdr, &r.id, &r.origin, &r.hsig, &r.vpks, &r.vsigs})
          *f = reinterpret_cast<const uint8_t*>(base + reinterpret_cast<uintptr_t>(*f));
        r.owned = false;
      }
  }
  // Outputs sized and set to "failed" (verdict Err, all certificate bits,
  // zero digests) before a launch or a retry.
  void reset_outputs() {
    v_out.assign(nv, 1);
    g_out.assign(ng, 1);
    c_out.assign(nc, 7);
    d_out.assign(nd * 32, 0);
    c_raw.clear();
    c_defer.clear();
    g_defer = false;
  }
  // Capacity for the largest window the lane's collector closes (`items` =
  // twice max_batch: whole shards are taken until max_batch items are in),
  // reserved when the window is made: a producer then never grows (reallocates
  // and copies) a multi-MB vector while it holds the shard lock, which the
  // collector's take waits for (round 4's streamed C3: 60-310 us per take).
  // Only address space until written (the pages of a large allocation are
  // faulted in on first touch); bare vote batches (rare) grow on demand.
  bool reserved = false;  // reserve_for ran (capacity is kept across reset())
  void reserve_for(size_t items, bool digest_lane) {
    reserved = true;
    if (digest_lane) {
      d_data.reserve(items * (512u << 10));  // ~500 KB worker batches
      d_offs.reserve(items + 1);
      return;
    }
    v_msgs.reserve(items * 32), v_pks.reserve(items * 32), v_sigs.reserve(items * 64);
    // copied certificates: votes 96 B per item, a header input of up to ~4 KB
    // and 128 B more per certificate of >= 15 votes (C1's committee of 4 has
    // 3: those regrow)
    c_own.reserve(items * 96 + (items / 16 + 1) * 4224);
    c_refs.reserve(items / 16 + 1);
  }
  // Empty again for the next intake, keeping every vector's capacity (the
  // queue recycles answered windows, so a window fills without reallocating
  // under the intake lock).
  void reset() {
    nv = ng = nc = nd = 0;
    intake_ns = 0;
    g_defer = false;
    c_raw.clear();
    c_defer.clear();
    for (auto* v : {&v_msgs, &v_pks, &v_sigs, &v_out, &g_msgs, &g_pks, &g_sigs, &g_out, &c_own, &c_out, &d_data, &d_out})
      v->clear();
    for (auto* v : {&g_offs, &d_offs}) v->clear();
    c_refs.clear();
    c_votes = c_hbytes = 0;
    g_offs.push_back(0);
    d_offs.push_back(0);
  }
};

// The parts one launch takes, with their totals.
struct Launch {
  std::vector<Window*> parts;
  size_t nv = 0, ng = 0, nc = 0, nd = 0;
  size_t nvotes = 0;   // certificate votes
  size_t hbytes = 0;   // certificate header bytes
  size_t dbytes = 0;   // digest input bytes
  size_t gvotes = 0;   // bare-batch votes
  int rc = COA_OK;     // engine status (negative = failure), set by the backend
  int slot = -1;       // backend slot the launch ran on
  int attempts = 0;    // launches of this window (1 + retries)
  int64_t slot_wait_ns = 0;  // how long launch() waited for a free slot (set by the backend)
  // time per COA_QSTAGE_* stage; the backend adds PACK, ENQUEUE, DEVICE_WAIT
  // and SCATTER (retries included), the queue the others
  int64_t stage_ns[COA_QSTAGES] = {};
  // the ENQUEUE stage split by the backend's calls (diagnostics, printed with
  // COA_QUEUE_TRACE_SLOW_US): key-cache pin, host-to-device copy, kernel
  // launches, device-to-host copy, completion event
  enum { ENQ_PIN, ENQ_H2D, ENQ_LAUNCH, ENQ_D2H, ENQ_EVENT, ENQ_PARTS };
  int64_t enq_ns[ENQ_PARTS] = {};
  // COA_QUEUE_KIND_* bits of the kinds the launch holds
  uint32_t kinds() const {
    return (nv ? COA_QUEUE_KIND_SIGNATURES : 0u) | (ng ? COA_QUEUE_KIND_BATCHES : 0u) |
           (nc ? COA_QUEUE_KIND_CERTIFICATES : 0u) | (nd ? COA_QUEUE_KIND_DIGESTS : 0u);
  }
  void tally() {
    nv = ng = nc = nd = nvotes = hbytes = dbytes = gvotes = 0;
    for (const Window* w : parts) {
      nv += w->nv;
      ng += w->ng;
      nc += w->nc;
      nd += w->nd;
      nvotes += w->c_votes;
      hbytes += w->c_hbytes;
      dbytes += w->d_data.size();
      gvotes += w->g_offs.back();
    }
  }
  size_t items() const { return nv + nd + nc + nvotes + gvotes; }
  void reset_outputs() {
    for (Window* w : parts) w->reset_outputs();
    rc = COA_OK;
  }
};

class Backend {
 public:
  virtual ~Backend() {}
  // Copies the launch's inputs to a free slot and enqueues its device work;
  // blocks while every slot is still busy with an earlier launch (at most
  // `slots()` launches in flight).  Sets l.slot and, on a failure already
  // known at enqueue time, l.rc.
  virtual void launch(Launch& l) = 0;
  // Waits for the launch's work and fills its outputs (and l.rc); frees its
  // slot.  On a failure the slot's device work has drained and the slot has
  // been rebuilt (a new stream and event, its buffers freed and regrown on
  // demand -- in the same process, never an exec) before it is freed.
  virtual void complete(Launch& l) = 0;
  // Engine-failure recovery, called by the completion thread after a failed
  // launch (l.slot = the slot it failed on): re-runs the launch synchronously
  // on the recovery context of the device `attempt` places after the failed
  // one -- its own stream and buffers, used only here, so a retry never waits
  // for a slot that a later launch holds.  Sets l.rc.
  virtual void retry(Launch& l, int attempt) = 0;
  virtual int slots() const = 0;
  // Blocks while every slot is busy; true if it had to wait.  Reserves
  // nothing (launch() still picks the slot): the collector calls it before
  // it closes a window, so a backlog that builds up meanwhile joins that
  // window instead of queueing behind it.
  virtual bool wait_free_slot() { return false; }
  // Number of device contexts retries can go to (at least 1).
  virtual int devices() const = 0;
  // Decides what complete() / retry() left open in the windows `ws`
  // (Window::c_defer, g_defer), writing their c_out / g_out.  Called by the
  // lane's resolver thread -- concurrently with launch() and complete() of
  // later windows, never with itself.  Returns the engine status.
  virtual int resolve(const std::vector<Window*>& ws) {
    (void)ws;
    return COA_OK;
  }
  // Sets the slots up (streams, staging sized for windows of up to twice
  // max_batch items) before the first window: called once at queue creation,
  // so no request pays for it.
  virtual void prepare(size_t max_batch) { (void)max_batch; }
  // Staging reallocations so far (each a page-locked or device allocation).
  virtual uint64_t grows() const { return 0; }
  virtual void reset_grows() {}
  // How the slots' streams were made (COA_QUEUE_STREAM_*).
  virtual int stream_kind() const { return 0; }
};

// The queue's lanes: signature, vote-batch and certificate windows
// (latency-bound, ~0.1-1 ms on the device) and worker-batch digest windows
// (a 14 ms serial SHA-512 chain per batch) never share a window, a slot, a
// stream or a completion order.
enum LaneId { LANE_VERIFY = 0, LANE_DIGEST = 1, LANES = 2 };

// The HIP backend (coa_queue_hip.cpp), or a test stub, for one lane.
Backend* make_backend(int lane);

}  // namespace coa_q
