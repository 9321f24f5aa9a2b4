// Shared scalar-multiplication helpers: the radix-256 fixed-base B table
// (LDS), signed-digit recoding read MSB-first from registers, and the
// fixed-base multiplication used for signing and table building.
#pragma once
#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_halved.h"

// ---------------------------------------------------------------------------
// Fixed-base table: entry j (0..127) = (j+1)·B as affine Niels
// (y+x, y-x, 2d·x·y), 24 dwords each, 12 KiB total.  Verification kernels
// copy it into LDS once per workgroup.
// ---------------------------------------------------------------------------
#define BTAB_ENTRIES 128
#define BTAB_DWORDS (BTAB_ENTRIES * 24)

COA_DEV void lds_load_btable(uint32_t* lds, const uint32_t* __restrict__ tab) {
  for (int i = threadIdx.x; i < BTAB_DWORDS / 4; i += blockDim.x)
    reinterpret_cast<uint4*>(lds)[i] = reinterpret_cast<const uint4*>(tab)[i];
  __syncthreads();
}

// Signed radix-256 digit e in [-128, 127] -> ±|e|·B (identity for 0).
COA_DEV void btab_select(ge_niels& q, const uint32_t* lds, int e) {
  const int m = e < 0 ? -e : e;
  const int idx = m == 0 ? 0 : m - 1;
  const uint4* src = reinterpret_cast<const uint4*>(lds + idx * 24);
  uint32_t w[24];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint4 v = src[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    q.yplusx.v[i] = w[i];
    q.yminusx.v[i] = w[8 + i];
    q.xy2d.v[i] = w[16 + i];
  }
  if (m == 0) ge_niels_identity(q);
  ge_niels_cneg(q, e < 0);
}

// ----------------------------------------------------------- scalar digits
// Signed radix-16 digits of k (< 2^253) are the nibbles of k + 0x88..8 minus 8;
// signed radix-256 digits of s (< 2^253) are the bytes of s + 0x8080..80
// minus 128.  Both sums stay < 2^256, so the recoding is exact and can be read
// most-significant digit first straight from registers.
COA_DEV void add_const_word(uint32_t* x, uint32_t c) {
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = addc32(x[i], c, cy, cy);
}
COA_DEV uint32_t take_top_bits(uint32_t* x, int nb) {
  const uint32_t top = x[7] >> (32 - nb);
#pragma unroll
  for (int i = 7; i > 0; i--) x[i] = (x[i] << nb) | (x[i - 1] >> (32 - nb));
  x[0] <<= nb;
  return top;
}

// [x]B for x < l with the radix-256 B table.
COA_DEV void fixed_base_mul(ge_p2& out, const uint32_t* x, const uint32_t* btab) {
  uint32_t sp[8];
#pragma unroll
  for (int i = 0; i < 8; i++) sp[i] = x[i];
  add_const_word(sp, 0x80808080u);
  ge_p3 acc3;
  ge_p2 acc2;
  ge_p1p1 t;
  ge_p3_identity(acc3);
#pragma unroll 1
  for (int j = 31; j >= 0; j--) {
    if (j != 31) {
#pragma unroll 1
      for (int dd = 0; dd < 7; dd++) {
        ge_p2_dbl(t, acc2);
        ge_p1p1_to_p2(acc2, t);
      }
      ge_p2_dbl(t, acc2);
      ge_p1p1_to_p3(acc3, t);
    }
    const int e = (int)take_top_bits(sp, 8) - 128;
    ge_niels qb;
    btab_select(qb, btab, e);
    ge_madd(t, acc3, qb);
    ge_p1p1_to_p2(acc2, t);
  }
  out = acc2;
}

// ---------------------------------------------------------------------------
// Comb tables: 32 byte positions x 128 multiples, entry (j, v) =
// (v+1)*256^j*P as affine Niels (24 dwords).  The B comb is built at
// coa_init (k_build_comb); committee keys get one comb of -A each
// (coa_committee.hip).  Digits are the signed radix-256 recoding below.
// ---------------------------------------------------------------------------
// Comb entry (j, |e|): signed radix-256 digit e of byte position j -> ±|e|*256^j*B.
COA_DEV void comb_select(ge_niels& q, const uint32_t* __restrict__ comb, int j, int e) {
  const int m = e < 0 ? -e : e;
  const int idx = m == 0 ? 0 : m - 1;
  const uint4* src = reinterpret_cast<const uint4*>(comb + ((uint64_t)j * 128 + idx) * 24);
  uint32_t w[24];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint4 v = src[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    q.yplusx.v[i] = w[i];
    q.yminusx.v[i] = w[8 + i];
    q.xy2d.v[i] = w[16 + i];
  }
  if (m == 0) ge_niels_identity(q);
  ge_niels_cneg(q, e < 0);
}

// ---------------------------------------------------------------------------
// Wide B comb, HBM resident: COA_WCOMB_POS positions x 2^(W-1) magnitudes,
// entry (j, m-1) = m * 2^(W j) * B as canonical affine Niels (24 dwords).
// A scalar x < 2^253 is recoded as the W-bit digits of
// x + sum_j 2^(W j + W - 1) minus 2^(W-1), so [x]B is COA_WCOMB_POS mixed
// additions instead of the 32 of the radix-256 comb above.  W = 24: 11
// positions, 92 M entries, 8.9 GB of the 288 GB HBM (round 3; W = 20, 13
// positions and 654 MB before: C3 +3 %, C1 +3.5 %, C2 +1 % same box).
// ---------------------------------------------------------------------------

// Generic wide comb of a point P: POS positions x 2^(W-1) magnitudes,
// entry (j, m-1) = m * 2^(W j) * P as affine Niels (24 dwords).  A scalar
// x < 2^253 is recoded as the W-bit digits of x + sum_j 2^(W j + W - 1)
// minus 2^(W-1); the offsets are single distinct bits, so the constant is a
// bit pattern.
template <int W, int POS>
COA_DEV void wc_recode(uint32_t* r, const uint32_t* x) {
  static_assert(W * POS >= 255 && W * POS <= 288, "wide comb recoding");
  uint32_t c[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < POS; j++) {
    const int b = W * j + W - 1;
    c[b >> 5] |= 1u << (b & 31);
  }
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = addc32(x[i], c[i], cy, cy);
  r[8] = c[8] + cy;
}
// Low W bits of r as a signed digit, then r >>= W.
template <int W>
COA_DEV int wc_take_digit(uint32_t* r) {
  const int d = (int)(r[0] & ((1u << W) - 1)) - (1 << (W - 1));
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = __builtin_amdgcn_alignbit(r[i + 1], r[i], W);
  r[8] >>= W;
  return d;
}
// Raw 24 words of entry (j, |d|) (entry (j, 0) for d == 0; ignored then);
// entries STRIDE dwords apart.
template <int W, int STRIDE>
COA_DEV void wc_load(uint32_t* w, const uint32_t* __restrict__ tab, int j, int d) {
  const uint32_t m = (uint32_t)(d < 0 ? -d : d);
  const uint64_t idx = (uint64_t)j * (1u << (W - 1)) + (m ? m - 1 : 0);
  const uint4* src = reinterpret_cast<const uint4*>(tab + idx * STRIDE);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint4 v = src[i];
    w[4 * i] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}
COA_DEV void wcomb_apply(ge_niels& q, const uint32_t* w, int d) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    q.yplusx.v[i] = w[i];
    q.yminusx.v[i] = w[8 + i];
    q.xy2d.v[i] = w[16 + i];
  }
  if (d == 0) ge_niels_identity(q);
  ge_niels_cneg(q, d < 0);
}
// acc += [x]P from P's wide comb (x < 2^253; a larger x gives some point,
// never an out-of-range entry).  Entry j+1 is loaded while addition j runs.
template <int W, int POS, int STRIDE, bool IL = false>
COA_DEV void wc_accumulate(ge_p3& acc, const uint32_t* x, const uint32_t* __restrict__ tab) {
  uint32_t r[9], cur[24], nxt[24];
  wc_recode<W, POS>(r, x);
  int d = wc_take_digit<W>(r);
  wc_load<W, STRIDE>(cur, tab, 0, d);
  ge_p1p1 t;
#pragma unroll 1
  for (int j = 0; j < POS; j++) {
    const int jn = j + 1 < POS ? j + 1 : j;
    const int dn = wc_take_digit<W>(r);
    wc_load<W, STRIDE>(nxt, tab, jn, dn);
    ge_niels q;
    wcomb_apply(q, cur, d);
    if constexpr (IL) {  // interleaved products (coa_ge.h *_il)
      ge_madd_il(t, acc, q);
      ge_p1p1_to_p3_il(acc, t);
    } else {
      ge_madd(t, acc, q);
      ge_p1p1_to_p3(acc, t);
    }
    d = dn;
#pragma unroll
    for (int i = 0; i < 24; i++) cur[i] = nxt[i];
  }
}

// The wide comb of B (COA_WCOMB_*, coa_halved.h).
COA_DEV void wcomb_load(uint32_t* w, const uint32_t* __restrict__ tab, int j, int d) {
  wc_load<COA_WCOMB_W, COA_WC_STRIDE>(w, tab, j, d);
}
template <bool IL = false>
COA_DEV void wcomb_accumulate(ge_p3& acc, const uint32_t* x, const uint32_t* __restrict__ tab) {
  wc_accumulate<COA_WCOMB_W, COA_WCOMB_POS, COA_WC_STRIDE, IL>(acc, x, tab);
}

COA_DEV uint32_t take_low_byte(uint32_t* x) {
  const uint32_t lo = x[0] & 0xffu;
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = __builtin_amdgcn_alignbit(x[i + 1], x[i], 8);
  x[7] >>= 8;
  return lo;
}

