// Committee key cache helpers shared by the certificate kernels
// (coa_committee.hip) and the single-signature latency kernel
// (coa_latency.hip): word/byte access to 8-dword scalars, wave-uniform loads,
// the binary search of a key among the registered (sorted) keys, and field
// element exchange between lanes.
#pragma once
#include "coa_fe.h"
#include "coa_sha512.h"

namespace coa_kc {

COA_DEV uint32_t word_sel(const uint32_t* x, int i) {
  // masks, not selects: a select chain over a register array is turned back
  // into dynamic indexing, i.e. a scratch round trip
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) w |= x[k] & (0u - (uint32_t)(i == k));
  return w;
}

COA_DEV uint32_t byte_of(const uint32_t* x, int j) { return (word_sel(x, j >> 2) >> (8 * (j & 3))) & 0xffu; }

COA_DEV void load8(uint32_t* d, const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
  d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

// wave-uniform copies (SGPRs) of values every lane loaded alike
COA_DEV void load8u(uint32_t* d, const uint32_t* p) {
  load8(d, p);
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = coa_sha::uni(d[i]);
}
COA_DEV uint64_t uni64(uint64_t v) {
  return ((uint64_t)coa_sha::uni((uint32_t)(v >> 32)) << 32) | coa_sha::uni((uint32_t)v);
}

// Lexicographic compare of two 8-dword tuples (the registration sort order).
COA_DEV int cmp8(const uint32_t* a, const uint32_t* b) {
  int r = 0;
#pragma unroll
  for (int i = 7; i >= 0; i--) r = a[i] != b[i] ? (a[i] < b[i] ? -1 : 1) : r;
  return r;
}

COA_DEV int key_lookup(const uint32_t* __restrict__ keys, uint32_t nk, const uint32_t* pk) {
  int lo = 0, hi = (int)nk - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    uint32_t k[8];
    load8(k, keys + (uint64_t)mid * 8);
    const int c = cmp8(k, pk);
    if (c == 0) return mid;
    if (c < 0) lo = mid + 1;
    else hi = mid - 1;
  }
  return -1;
}

COA_DEV int key_lookup_u(const uint32_t* __restrict__ keys, uint32_t nk, const uint32_t* pk) {
  int lo = 0, hi = (int)nk - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    uint32_t k[8];
    load8u(k, keys + (uint64_t)mid * 8);
    const int c = cmp8(k, pk);
    if (c == 0) return mid;
    if (c < 0) lo = mid + 1;
    else hi = mid - 1;
  }
  return -1;
}

template <int L>
COA_DEV void shfl_fe(fe& r, const fe& a, int off) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)__shfl_xor((int)a.v[i], off, 64);
}

}  // namespace coa_kc
