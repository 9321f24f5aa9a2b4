// HIP launch backend of the aggregation queue (coa_queue.h): two device
// slots per opened GPU context, each with its own non-blocking stream, event,
// page-locked staging and device buffers.  launch() packs a window into one
// pinned block, issues ONE host-to-device copy, the engine's device-resident
// entry points (asynchronous with an explicit workspace, no engine lock) and
// ONE device-to-host copy on the slot's stream, records an event and returns;
// complete() waits for the event.  So while window N runs on slot A, window
// N + 1 is packed and enqueued on slot B, and the copies of one window overlap
// the kernels of the other.
//
// Per kind:
//   signatures    coa_ed25519_verify_strict_many_device (Signature::verify)
//   certificates  coa_certificate_verify_many_device (the fused
//                 Certificate::verify crypto); the raw status words that need
//                 the exact random-linear-combination check or carry a key
//                 outside the registered committee are re-decided in
//                 complete() through coa_certificate_verify_many, as the
//                 host-pointer entry point does
//   digests       coa_sha512_many_device (worker/src/processor.rs:38)
//   vote batches  coa_ed25519_verify_batch_groups in complete() (host
//                 pointers; bare batches are rare next to whole certificates)
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "coa_committee.h"
#include "coa_queue.h"

#define COA_QUEUE_SLOTS_DEFAULT 2

namespace {

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Slot {
  int dev = -1;
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  void* hin = nullptr;   // pinned input block
  void* hout = nullptr;  // pinned output block
  void* din = nullptr;   // device input block
  void* dout = nullptr;  // device output block
  void* ws = nullptr;    // device workspace (verify + certificates)
  size_t cap_hin = 0, cap_hout = 0, cap_din = 0, cap_dout = 0, cap_ws = 0;
  bool busy = false;
  bool launched = false;  // device work was enqueued (else complete() skips the wait)
  // output offsets of the current window
  size_t o_v = 0, o_c = 0, o_d = 0;
};

hipError_t grow_pinned(void*& p, size_t& cap, size_t want) {
  if (want <= cap) return hipSuccess;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  cap = 0;
  want = want + want / 4 + 4096;
  hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
  if (e == hipSuccess) cap = want;
  return e;
}
hipError_t grow_dev(void*& p, size_t& cap, size_t want) {
  if (want <= cap) return hipSuccess;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  want = want + want / 4 + 4096;
  hipError_t e = hipMalloc(&p, want);
  if (e == hipSuccess) cap = want;
  return e;
}

class HipBackend : public coa_q::Backend {
 public:
  ~HipBackend() override {
    for (Slot& sl : slots_) {
      if (sl.dev < 0) continue;
      (void)hipSetDevice(sl.dev);
      if (sl.s) (void)hipStreamSynchronize(sl.s);
      if (sl.hin) (void)hipHostFree(sl.hin);
      if (sl.hout) (void)hipHostFree(sl.hout);
      if (sl.din) (void)hipFree(sl.din);
      if (sl.dout) (void)hipFree(sl.dout);
      if (sl.ws) (void)hipFree(sl.ws);
      if (sl.ev) (void)hipEventDestroy(sl.ev);
      if (sl.s) (void)hipStreamDestroy(sl.s);
    }
  }

  int slots() const override { return (int)slots_.size(); }

  void launch(coa_q::Window& w) override {
    w.v_out.assign(w.nv, 1);
    w.g_out.assign(w.ng, 1);
    w.c_out.assign(w.nc, 7);
    w.d_out.assign(w.nd * 32, 0);
    if (!ready()) {
      w.rc = init_rc_;
      return;
    }
    Slot* sl;
    {
      std::unique_lock<std::mutex> l(m_);
      const size_t k = next_++ % slots_.size();
      cv_.wait(l, [&] { return !slots_[k].busy; });
      slots_[k].busy = true;
      w.slot = (int)k;
      sl = &slots_[k];
    }
    sl->launched = false;
    w.rc = enqueue(*sl, w);
  }

  void complete(coa_q::Window& w) override {
    if (w.slot < 0) return;  // never staged (no device)
    Slot& sl = slots_[w.slot];
    if (w.rc == COA_OK && sl.launched) {
      const hipError_t e = hipEventSynchronize(sl.ev);
      if (e != hipSuccess) w.rc = COA_EHIP;
    }
    if (w.rc == COA_OK) {
      const uint8_t* h = static_cast<const uint8_t*>(sl.hout);
      if (w.nv) std::memcpy(w.v_out.data(), h + sl.o_v, w.nv);
      if (w.nd) {
        for (size_t i = 0; i < w.nd; i++) std::memcpy(&w.d_out[i * 32], h + sl.o_d + i * 64, 32);
      }
      if (w.nc) w.rc = resolve_certs(w, reinterpret_cast<const uint32_t*>(h + sl.o_c));
      if (w.rc == COA_OK && w.ng)
        w.rc = coa_ed25519_verify_batch_groups(w.g_msgs.data(), w.g_pks.data(), w.g_sigs.data(), w.g_offs.data(),
                                               w.ng, w.g_out.data(), 0);
    }
    std::lock_guard<std::mutex> l(m_);
    sl.busy = false;
    cv_.notify_all();
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
    // device slots per GPU: windows in flight at once (COA_QUEUE_SLOTS,
    // 1..8; tools/queue_probe.c measures the choice)
    size_t per = COA_QUEUE_SLOTS_DEFAULT;
    if (const char* e = getenv("COA_QUEUE_SLOTS")) {
      const int v = atoi(e);
      if (v >= 1 && v <= 8) per = (size_t)v;
    }
    slots_.resize(per * (size_t)std::min(n, 64));
    for (size_t k = 0; k < slots_.size(); k++) {
      Slot& sl = slots_[k];
      sl.dev = ids[k % (size_t)std::min(n, 64)];
      if (hipSetDevice(sl.dev) != hipSuccess || hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) != hipSuccess) {
        init_rc_ = COA_EHIP;
        return false;
      }
    }
    return true;
  }

  // Input block: verify msgs | pks | sigs, certificate arrays, digest data |
  // offsets (256-byte aligned sections).  Output block: verdicts | status
  // words | 64-byte digests.
  int enqueue(Slot& sl, coa_q::Window& w) {
    if (hipSetDevice(sl.dev) != hipSuccess) return COA_EHIP;
    const size_t nvotes = w.nc ? w.c_voff.back() : 0;
    size_t o = 0;
    auto take = [&](size_t bytes) {
      const size_t at = o;
      o = al256(o + bytes);
      return at;
    };
    const size_t i_vm = take(w.nv * 32), i_vp = take(w.nv * 32), i_vs = take(w.nv * 64);
    const size_t i_ch = take(w.c_hdata.size() + 16), i_cho = take((w.nc + 1) * 8), i_cid = take(w.nc * 32),
                 i_cor = take(w.nc * 32), i_chs = take(w.nc * 64), i_crd = take(w.nc * 8),
                 i_cvp = take(nvotes * 32), i_cvs = take(nvotes * 64), i_cvo = take((w.nc + 1) * 8);
    const size_t i_dd = take(w.d_data.size() + 16), i_do = take((w.nd + 1) * 8);
    const size_t in_bytes = o;
    o = 0;
    sl.o_v = take(w.nv);
    sl.o_c = take(w.nc * 4);
    sl.o_d = take(w.nd * 64);
    const size_t out_bytes = o;
    const size_t ws_v = w.nv ? coa_verify_workspace_bytes(w.nv) : 0;
    const size_t ws_c = w.nc ? coa_certificate_workspace_bytes(w.nc, nvotes) : 0;
    if (grow_pinned(sl.hin, sl.cap_hin, in_bytes) != hipSuccess ||
        grow_pinned(sl.hout, sl.cap_hout, out_bytes) != hipSuccess ||
        grow_dev(sl.din, sl.cap_din, in_bytes) != hipSuccess || grow_dev(sl.dout, sl.cap_dout, out_bytes) != hipSuccess ||
        grow_dev(sl.ws, sl.cap_ws, std::max(ws_v, ws_c) + 256) != hipSuccess)
      return COA_ENOMEM;
    uint8_t* h = static_cast<uint8_t*>(sl.hin);
    auto put = [&](size_t at, const void* src, size_t bytes) {
      if (bytes) std::memcpy(h + at, src, bytes);
    };
    put(i_vm, w.v_msgs.data(), w.v_msgs.size());
    put(i_vp, w.v_pks.data(), w.v_pks.size());
    put(i_vs, w.v_sigs.data(), w.v_sigs.size());
    if (w.nc) {
      put(i_ch, w.c_hdata.data(), w.c_hdata.size());
      put(i_cho, w.c_hoff.data(), (w.nc + 1) * 8);
      put(i_cid, w.c_ids.data(), w.nc * 32);
      put(i_cor, w.c_origins.data(), w.nc * 32);
      put(i_chs, w.c_hsigs.data(), w.nc * 64);
      put(i_crd, w.c_rounds.data(), w.nc * 8);
      put(i_cvp, w.c_pks.data(), nvotes * 32);
      put(i_cvs, w.c_sigs.data(), nvotes * 64);
      put(i_cvo, w.c_voff.data(), (w.nc + 1) * 8);
    }
    if (w.nd) {
      put(i_dd, w.d_data.data(), w.d_data.size());
      put(i_do, w.d_offs.data(), (w.nd + 1) * 8);
    }
    if (w.nv + w.nc + w.nd == 0) return COA_OK;  // bare vote batches only: done in complete()
    uint8_t* d = static_cast<uint8_t*>(sl.din);
    uint8_t* dout = static_cast<uint8_t*>(sl.dout);
    if (hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, sl.s) != hipSuccess) return COA_EHIP;
    sl.launched = true;
    int rc = COA_OK;
    if (w.nv)
      rc = coa_ed25519_verify_strict_many_device(sl.dev, d + i_vm, 32, d + i_vp, d + i_vs, w.nv, dout + sl.o_v, sl.ws,
                                                 sl.s);
    if (rc == COA_OK && w.nc)
      rc = coa_certificate_verify_many_device(
          sl.dev, d + i_ch, reinterpret_cast<const uint64_t*>(d + i_cho), d + i_cid, d + i_cor, d + i_chs,
          reinterpret_cast<const uint64_t*>(d + i_crd), d + i_cvp, d + i_cvs,
          reinterpret_cast<const uint64_t*>(d + i_cvo), w.nc, nvotes, reinterpret_cast<uint32_t*>(dout + sl.o_c),
          sl.ws, sl.s);
    if (rc == COA_OK && w.nd)
      rc = coa_sha512_many_device(sl.dev, d + i_dd, reinterpret_cast<const uint64_t*>(d + i_do), w.nd, dout + sl.o_d,
                                  sl.s);
    if (rc != COA_OK) return rc;
    if (hipMemcpyAsync(sl.hout, dout, out_bytes, hipMemcpyDeviceToHost, sl.s) != hipSuccess) return COA_EHIP;
    if (hipEventRecord(sl.ev, sl.s) != hipSuccess) return COA_EHIP;
    return COA_OK;
  }

  // Raw certificate status words -> COA_CERT_* bits; certificates the fused
  // kernel could not decide alone are re-run through the host-pointer entry
  // point, which decides them exactly (as coa_certificate_verify_many does).
  static int resolve_certs(coa_q::Window& w, const uint32_t* st) {
    std::vector<size_t> redo;
    for (size_t c = 0; c < w.nc; c++) {
      if (st[c] & (COA_CST_VOTES_INCONCLUSIVE | COA_CST_UNCACHED)) redo.push_back(c);
      w.c_out[c] = (uint8_t)(st[c] & 7u);
    }
    if (redo.empty()) return COA_OK;
    std::vector<uint8_t> hd, ids, org, hs, vp, vs, out(redo.size(), 7);
    std::vector<uint64_t> ho{0}, rd, vo{0};
    for (size_t c : redo) {
      hd.insert(hd.end(), w.c_hdata.begin() + (long)w.c_hoff[c], w.c_hdata.begin() + (long)w.c_hoff[c + 1]);
      ho.push_back(hd.size());
      ids.insert(ids.end(), w.c_ids.begin() + (long)c * 32, w.c_ids.begin() + (long)c * 32 + 32);
      org.insert(org.end(), w.c_origins.begin() + (long)c * 32, w.c_origins.begin() + (long)c * 32 + 32);
      hs.insert(hs.end(), w.c_hsigs.begin() + (long)c * 64, w.c_hsigs.begin() + (long)c * 64 + 64);
      rd.push_back(w.c_rounds[c]);
      vp.insert(vp.end(), w.c_pks.begin() + (long)w.c_voff[c] * 32, w.c_pks.begin() + (long)w.c_voff[c + 1] * 32);
      vs.insert(vs.end(), w.c_sigs.begin() + (long)w.c_voff[c] * 64, w.c_sigs.begin() + (long)w.c_voff[c + 1] * 64);
      vo.push_back(vp.size() / 32);
    }
    hd.push_back(0);
    const int rc = coa_certificate_verify_many(hd.data(), ho.data(), ids.data(), org.data(), hs.data(), rd.data(),
                                               vp.data(), vs.data(), vo.data(), redo.size(), 0, out.data());
    if (rc != COA_OK) return rc;
    for (size_t j = 0; j < redo.size(); j++) w.c_out[redo[j]] = out[j];
    return COA_OK;
  }

  std::vector<Slot> slots_;
  size_t next_ = 0;
  std::mutex m_;
  std::condition_variable cv_;
  bool inited_ = false;
  int init_rc_ = COA_OK;
};

}  // namespace

coa_q::Backend* coa_q::make_backend() { return new HipBackend(); }
