// Internal launch wrapper of the single-signature latency kernel
// (coa_latency.hip): crypto::Signature::verify (crypto/src/lib.rs:200-204)
// for the few-at-a-time callers -- Header::verify and Vote::verify verify one
// message at a time (primary/src/messages.rs:64-66,139-141).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Signatures of a call passed inline in the kernel arguments (no H2D copy).
#define COA_LAT_INLINE 16

struct LatArgs {
  const uint32_t* in;      // [n][32] dwords: msg (8) | pk (8) | R (8) | s (8), items >= n_inline
  uint32_t n;
  uint32_t n_inline;       // items [0, n_inline) are in inl
  uint32_t inl[COA_LAT_INLINE][32];
  uint32_t* res;           // [n] result words in page-locked host memory: (tag << 8) | verdict
  uint32_t tag;            // nonzero, per call: the host polls res for it
  const uint32_t* keys;    // registered committee keys (sorted), or null
  const uint32_t* kflags;  // [nk]
  const uint32_t* ktabs;   // [nk] radix-256 combs of -A (coa_committee.h)
  uint32_t nk;
  const uint32_t* comb;    // radix-256 comb of B (coa_halved.h)
  // verify_batch prefilter for items [0, batch_n): a verdict of 0 also
  // certifies [l]A == O (the registered key's flag, or [l](-A) computed
  // in-kernel for an unregistered one), so a group whose votes all give 0
  // passes dalek's batch equation for every z (coa_committee.hip,
  // "verify_batch exactness"); items [batch_n, n) are plain verify_strict
  // (one launch can carry a certificate's votes and its header signature)
  uint32_t batch_n;
  // Certificate::digest inputs (id || round LE || origin, 72 bytes = 18
  // dwords each), or null.  With them, a prefilter item's record carries the
  // certificate's index in its first message dword, and its message is
  // SHA-512(cd_in[index])[..32], hashed in the kernel (the exact certificate
  // path no longer needs a digest launch and a host round trip first)
  const uint32_t* cd_in;
};

// One 256-thread workgroup (four waves) per signature.
hipError_t coa_launch_verify_lat(const LatArgs& a, hipStream_t s);

// The latency kernel over device-resident inputs, enqueued on `stream`
// (coa_runtime.cpp; the aggregation queue's small signature windows):
// d_in [n][128 B] = msg | pk | R | s, d_res [n] words (1 << 8) | verdict.
// Reads device `device`'s committee key cache: the generation the calling
// thread pinned (coa_keycache_use, held until the kernel has run), else the
// current one.  Returns COA_OK or a negative COA_E*.
extern "C" int coa_lat_verify_device(int device, const uint8_t* d_in, size_t n, uint32_t* d_res, void* stream);
// The same for n <= COA_LAT_INLINE records in host memory, passed in the
// kernel arguments (no host-to-device copy), the result words
// (tag << 8) | verdict written straight into `res` (page-locked host memory
// the caller polls for `tag`, nonzero; no device-to-host copy): the queue's
// windows of a few signatures (coa_queue_hip.cpp).
extern "C" int coa_lat_verify_inline(int device, const uint8_t* h_records, size_t n, uint32_t* res, uint32_t tag,
                                     void* stream);
// Calls of at most this many signatures (32-byte messages) take the latency
// kernel (COA_LAT_MAX, default 2048).
extern "C" size_t coa_lat_max(void);
