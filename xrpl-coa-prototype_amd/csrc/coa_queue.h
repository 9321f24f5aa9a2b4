// Internal interface between the aggregation queue (coa_queue.cpp: request
// intake, windows, callbacks, metrics; no HIP) and its launch backend
// (coa_queue_hip.cpp: pinned staging, HIP streams and events over the
// device-resident entry points; a test build links a stub instead,
// tests/sanitize/queue_tsan.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/coa_verify.h"

namespace coa_q {

// One launch window: every request the collector took in one go, packed
// contiguously by kind.  The backend fills the outputs and `rc`.
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
  // whole certificates (coa_certificate_verify_many semantics)
  size_t nc = 0;
  std::vector<uint8_t> c_hdata, c_ids, c_origins, c_hsigs, c_pks, c_sigs;
  std::vector<uint64_t> c_hoff, c_rounds, c_voff;  // nc + 1, nc, nc + 1
  std::vector<uint8_t> c_out;                      // nc status bytes (COA_CERT_* bits)
  // worker batch digests (coa_sha512_trunc32_many semantics)
  size_t nd = 0;
  std::vector<uint8_t> d_data;
  std::vector<uint64_t> d_offs;  // nd + 1
  std::vector<uint8_t> d_out;    // nd x 32
  int rc = COA_OK;               // engine status of the window (negative = failure)
  int slot = -1;                 // backend slot the window ran on

  // Empty again for the next window, keeping every vector's capacity (the
  // queue recycles answered windows, so a window fills without reallocating
  // under the intake lock).
  void reset() {
    nv = ng = nc = nd = 0;
    for (auto* v : {&v_msgs, &v_pks, &v_sigs, &v_out, &g_msgs, &g_pks, &g_sigs, &g_out, &c_hdata, &c_ids, &c_origins,
                    &c_hsigs, &c_pks, &c_sigs, &c_out, &d_data, &d_out})
      v->clear();
    for (auto* v : {&g_offs, &c_hoff, &c_rounds, &c_voff, &d_offs}) v->clear();
    g_offs.push_back(0);
    c_hoff.push_back(0);
    c_voff.push_back(0);
    d_offs.push_back(0);
    rc = COA_OK;
    slot = -1;
  }
};

class Backend {
 public:
  virtual ~Backend() {}
  // Copies the window's inputs to a free slot and enqueues its device work;
  // blocks while every slot is still busy with an earlier window (the
  // double buffering: at most `slots()` windows in flight).
  virtual void launch(Window& w) = 0;
  // Waits for the window's work and fills its outputs; frees its slot.
  virtual void complete(Window& w) = 0;
  virtual int slots() const = 0;
};

// The HIP backend (coa_queue_hip.cpp), or a test stub.
Backend* make_backend();

}  // namespace coa_q
