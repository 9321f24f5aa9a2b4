// Internal launch wrappers for the committee key cache (f2) and the fused
// Certificate::verify kernel (f3) -- coa_committee.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// per-key comb of -A: 32 byte positions x 128 multiples x 24 dwords (384 KiB)
#define COA_KEY_TAB_ENTRIES (32 * 128)
#define COA_KEY_TAB_DWORDS (COA_KEY_TAB_ENTRIES * 24)

// per-key wide comb of -A (coa_smul.h wc_*): 16 positions x 2^15 multiples,
// entry (j, m-1) = m * 2^(16 j) * (-A), exact integer multiples (torsion
// kept), 24 dwords each: 48 MiB per key, built at registration when the
// committee fits the COA_KEY_WCOMB_MB budget
#define COA_KWCOMB_W 16
#define COA_KWCOMB_POS 16
#define COA_KWCOMB_ENTRIES ((uint64_t)COA_KWCOMB_POS << (COA_KWCOMB_W - 1))
#define COA_KWCOMB_DWORDS (COA_KWCOMB_ENTRIES * COA_KWC_STRIDE)
// the widest per-key comb: 13 positions x 2^19 multiples, entry (j, m-1) =
// m * 2^(20 j) * (-A), exact integer multiples: 654 MB per key (B's wide
// comb layout at W = 20), 13 additions for [k](-A) instead of 16;
// built when the committee fits the COA_KEY_WCOMB20_MB budget (shared by the
// contexts open on a device), else the 48 MiB combs above
#define COA_KWCOMB20_W 20
#define COA_KWCOMB20_POS 13
#define COA_KWCOMB20_ENTRIES ((uint64_t)COA_KWCOMB20_POS << (COA_KWCOMB20_W - 1))
#define COA_KWCOMB20_DWORDS (COA_KWCOMB20_ENTRIES * COA_KWC_STRIDE)

// Dwords per entry of the keys' wide combs (24: packed; a 128-byte-line
// layout, 32, measured no faster on the C3 round and takes a third more of
// the 65 GB per committee-100 generation)
#ifndef COA_KWC_STRIDE
#define COA_KWC_STRIDE 24
#endif

// key flag bits (k_key_flags)
#define COA_KEY_DECOMPRESSES 1u   // CompressedEdwardsY::decompress succeeds
#define COA_KEY_SMALL_ORDER 2u    // [8]A == O  (verify_strict rejects)
#define COA_KEY_TORSION_FREE 4u   // [l]A == O  (batch fast path is exact)

// Internal status bits of k_cert_verify (low three are the public
// COA_CERT_BAD_* bits of include/coa_verify.h).
#define COA_CST_BAD_HEADER_ID 1u
#define COA_CST_BAD_HEADER_SIG 2u
#define COA_CST_BAD_VOTES 4u
#define COA_CST_VOTES_INCONCLUSIVE 8u  // some vote failed its own equation, or a key has torsion
#define COA_CST_UNCACHED 16u           // author or a voter is not in the registered committee

struct CertArgs {
  const uint8_t* hdr_data;      // Header::digest inputs, concatenated
  const uint64_t* hdr_off;      // [nc + 1]
  const uint32_t* ids;          // [nc][8]   header.id
  const uint32_t* origins;      // [nc][8]   header.author (Certificate::origin)
  const uint32_t* hsigs;        // [nc][16]  header.signature R || s
  const uint64_t* rounds;       // [nc]
  const uint32_t* vpks;         // [nv][8]   voter public keys
  const uint32_t* vsigs;        // [nv][16]  vote signatures
  const uint64_t* voff;         // [nc + 1]  certificate c owns votes [voff[c], voff[c+1])
  uint32_t nc, nv;
  uint32_t hdr_blocks;          // set by the launcher
  const uint32_t* keys;         // [nk][8] registered keys, sorted as dword tuples
  const uint32_t* kflags;       // [nk]
  const uint32_t* ktabs;        // [nk][COA_KEY_TAB_DWORDS] comb of -A per key
  const uint32_t* kwtabs;       // [nk][COA_KWCOMB_DWORDS] wide comb of -A per key, or null
  uint32_t kw20;                // 1: kwtabs is [nk][COA_KWCOMB20_DWORDS] (radix 2^20)
  uint32_t nk;
  const uint32_t* comb;         // B comb (coa_halved.h)
  const uint32_t* wcomb;        // wide B comb (coa_smul.h) or null
  uint32_t* status;             // [nc], zeroed by the caller
  // throughput variant: [nc][8] Certificate::digest of each certificate,
  // written by a prologue kernel (set by the launcher; null = per vote)
  const uint32_t* cdig = nullptr;
  // latency variant only (optional): the last block publishes (tag << 8) |
  // status into host_res[c] (page-locked) and re-zeroes status and done_ctr
  uint32_t* host_res = nullptr;
  uint32_t* done_ctr = nullptr;  // device word, 0 between calls
  uint32_t tag = 0;
  uint32_t total_blocks = 0;     // set by the launcher
  // throughput variant: the jobs in key order (set by the launcher, null =
  // in order; see k_cert_verify)
  const uint32_t* perm = nullptr;
  // 1: the caller asks for key order (the launcher sorts when the call is
  // large enough and COA_CERT_KEYSORT is not 0)
  uint32_t key_order = 0;
};

// A small certificate passed inline in the kernel arguments of the latency
// kernel (no host-to-device copy on the one-certificate path): the arrays of
// CertArgs sit at the given byte offsets of buf (16-byte aligned; the header
// bytes are followed by 16 bytes of slack for the aligned-dword reads).
// CertArgs' pointers of those arrays are ignored; status, done_ctr and the
// key-cache pointers are used as given.
#define COA_CERT_INLINE_BYTES 2816
struct CertInl {
  CertArgs a;
  uint32_t off_hdr, off_hoff, off_ids, off_origins, off_hsigs, off_rounds, off_voff, off_vpks, off_vsigs;
  alignas(16) uint8_t buf[COA_CERT_INLINE_BYTES];
};
hipError_t coa_launch_cert_verify_inl(const CertInl& ci, hipStream_t s);

// Committee key-cache generations of HIP device `device` (coa_runtime.cpp).
// coa_committee_register builds a new generation of the key tables while
// every call and queue window keeps reading the one it started with, swaps
// it in, and frees the old one once nothing holds it -- so registration
// never waits for a window and never holds one back.  The aggregation queue
// pins the current generation from a window's launch to its completion (the
// kernels read the tables asynchronously) and has its launches read that
// pinned generation (coa_keycache_use on the launching thread).
extern "C" void* coa_keycache_pin(int device);  // opaque handle (null: device not open)
extern "C" void coa_keycache_unpin(void* pin);  // any thread; null is a no-op
extern "C" void coa_keycache_use(void* pin);    // this thread's launches read `pin` (null: the current one)

// The exact decision of certificates the fused kernel left open (raw status
// words with COA_CST_UNCACHED or COA_CST_VOTES_INCONCLUSIVE; the others pass
// through): host arrays as coa_certificate_verify_many takes them, minus the
// header bytes.  `raw` is updated in place; status_out gets the COA_CERT_*
// bits.  The aggregation queue's resolver calls it off the completion thread
// (coa_queue.cpp), so an open certificate never holds its window back.
extern "C" int coa_certificate_resolve_raw(const uint8_t* ids, const uint8_t* origins, const uint8_t* header_sigs,
                                           const uint64_t* rounds, const uint8_t* vote_pks, const uint8_t* vote_sigs,
                                           const uint64_t* vote_offsets, size_t n, uint32_t* raw,
                                           uint8_t* status_out);

// The aggregation queue's certificate windows of at most 64 certificates
// whose jobs take the latency kernel (coa_queue_hip.cpp): the window's arrays
// packed in page-locked h_base at the byte offsets `off` (header offsets
// relative to off->hdr, vote offsets window-relative), device copy d_base of
// in_bytes.  Inline in the kernel arguments when they fit
// COA_CERT_INLINE_BYTES (no copy), else one H2D copy into d_base; either way
// the kernel's last block writes (tag << 8) | status for each certificate
// into host_res (page-locked, polled by the caller) and re-zeroes d_ctr[0..64]
// (a device block of 65 words, zero before the first call).  Returns 1 when
// the window is not of that size (nothing enqueued), else COA_OK or a
// negative COA_E*.
struct CoaCertOffsets {
  uint64_t hdr, hoff, ids, origins, hsigs, rounds, vpks, vsigs, voff;
};
extern "C" int coa_certificate_verify_publish(int device, const uint8_t* h_base, uint8_t* d_base, size_t in_bytes,
                                              const CoaCertOffsets* off, size_t n, size_t n_votes, uint32_t* d_ctr,
                                              uint32_t* host_res, uint32_t tag, void* stream);

// Host copies spread over the runtime's copy threads (COA_PACK_THREADS):
// the aggregation queue packs large windows into page-locked staging with
// it.  Returns when every segment is copied.
struct CoaCopySeg {
  void* dst;
  const void* src;
  size_t bytes;
};
extern "C" void coa_copy_segments(const CoaCopySeg* segs, size_t n);

hipError_t coa_launch_key_flags(const uint32_t* keys, uint32_t nk, uint32_t* flags, hipStream_t s);
hipError_t coa_launch_key_tables(const uint32_t* keys, uint32_t nk, uint32_t* tabs, hipStream_t s);
// wide combs from the radix-256 key combs (tabs already built)
hipError_t coa_launch_key_wcombs(const uint32_t* tabs, uint32_t nk, uint32_t* wtabs, hipStream_t s);
hipError_t coa_launch_key_wcombs20(const uint32_t* tabs, uint32_t nk, uint32_t* wtabs, hipStream_t s);
// lanes_per_sig: 64 (latency: two waves per signature, comb terms split over
// a wave's lanes and summed by a butterfly) or 1 (throughput: K signatures
// per lane, K from the job count).
// pscr: device scratch of coa_cert_scratch_bytes(nc + nv, a.key_order)
// bytes (throughput variant only; may be null for lanes_per_sig == 64).
size_t coa_cert_scratch_bytes(uint64_t jobs, bool key_order);

// coa_certificate_verify_many_device with the job order chosen by the caller:
// key_order 1 (the public device-resident round) sorts a call of >= 16,384
// jobs by committee key, 0 keeps certificate order (the aggregation queue's
// windows: concurrent windows lost more to the sort's launches than the order
// gained, profiles/r05_cert_keysort_ab.txt).  The workspace must hold
// coa_cert_scratch_bytes(n + n_votes, key_order) bytes.
extern "C" int coa_certificate_verify_many_device_order(
    int device, const uint8_t* d_header_data, const uint64_t* d_header_offsets, const uint8_t* d_ids,
    const uint8_t* d_origins, const uint8_t* d_header_sigs, const uint64_t* d_rounds, const uint8_t* d_vote_pks,
    const uint8_t* d_vote_sigs, const uint64_t* d_vote_offsets, size_t n, size_t n_votes, uint32_t* d_status,
    void* workspace, void* stream, int key_order);
hipError_t coa_launch_cert_verify(CertArgs a, int lanes_per_sig, uint32_t* pscr, hipStream_t s);

// Row-parallel field arithmetic (coa_fe_wave.h) against coa_fe.h, one wave per
// input x_i (32 LE bytes, any value < 2^256): out[i] bit0 pow_p58, bit1
// invert, bit2 x_i * x_{i+1}, bit3 decompression of x_i as an encoding
// (verdict and coordinates), bit4 x_i + x_{i+1}, bit5 x_i - x_{i+1} differ.
hipError_t coa_launch_fe_rows_check(const uint8_t* in, uint32_t n, uint32_t* out, hipStream_t s);
