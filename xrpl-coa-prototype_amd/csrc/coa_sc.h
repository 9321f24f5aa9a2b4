// Scalars mod l = 2^252 + 27742317777372353535851937790883648493 (one per lane).
//
// Replaces curve25519-dalek 3.x `Scalar` for the verification path:
//   * Scalar::from_canonical_bytes  (ed25519-dalek 1.0.1 `check_scalar`)
//   * Scalar::from_hash             (k = H(R||A||M) mod l)
//   * Scalar mul / add              (verify_batch weights, signing)
// Representation: 8 x 32-bit little-endian limbs, canonical (< l) unless a
// function says otherwise.  Reduction of 512-bit values is Barrett
// (HAC 14.42, base 2^32, k = 8) with mu = floor(2^512 / l).
#pragma once
#include "coa_fe.h"

struct sc {
  uint32_t v[8];
};

COA_DEV void sc_const_l(uint32_t* l) {
  const uint32_t c[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                         0x00000000u, 0x00000000u, 0x00000000u, 0x10000000u};
#pragma unroll
  for (int i = 0; i < 8; i++) l[i] = c[i];
}

// s < l  (ed25519-dalek 1.0.1 check_scalar / Scalar::from_canonical_bytes;
// the ed25519 1.x top-3-bit test on byte 31 is implied).
COA_DEV bool sc_is_canonical(const uint32_t* s) {
  uint32_t l[8];
  sc_const_l(l);
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)subb32(s[i], l[i], b, b);
  return b != 0;  // s - l borrowed  <=>  s < l
}

// r = x mod l for a 512-bit x (16 limbs).   Scalar::from_bytes_mod_order_wide
COA_DEV void sc_reduce512(sc& r, const uint32_t* x) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  uint32_t l[8];
  sc_const_l(l);
  // q3 = floor(floor(x / 2^224) * mu / 2^288); only columns >= 8 matter, the
  // lower ones contribute at most a carry that Barrett's bound absorbs, but
  // we compute them for exactness of the carry chain.
  const uint32_t* q1 = x + 7;  // 9 limbs
  uint32_t q3[9];
  {
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
      for (int i = 0; i < 9; i++) {
        const int j = k - i;
        if (j < 0 || j > 8) continue;
        mac(acc, c2, q1[i], mu[j]);
      }
      if (k >= 9) q3[k - 9] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)c2 << 32);
      c2 = 0;
    }
    q3[8] = (uint32_t)acc;
  }
  // r2 = q3 * l mod 2^288 (9 limbs)
  uint32_t r2[9];
  {
    uint64_t acc = 0;
    uint32_t c2 = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
#pragma unroll
      for (int i = 0; i < 9; i++) {
        const int j = k - i;
        if (j < 0 || j > 7) continue;
        mac(acc, c2, q3[i], l[j]);
      }
      r2[k] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)c2 << 32);
      c2 = 0;
    }
  }
  // t = x mod 2^288 - r2 (mod 2^288); t < 3l
  uint32_t t[9];
  uint32_t b = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = subb32(x[i], r2[i], b, b);
  // subtract l at most twice
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    uint32_t u[9];
    uint32_t bb = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = subb32(t[i], l[i], bb, bb);
    u[8] = subb32(t[8], 0, bb, bb);
    const bool ge = bb == 0;
#pragma unroll
    for (int i = 0; i < 9; i++) t[i] = ge ? u[i] : t[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
}

// r = a * b + c mod l (a, b, c < 2^256).
COA_DEV void sc_muladd(sc& r, const uint32_t* a, const uint32_t* b, const uint32_t* c) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      mac(acc, c2, a[i], b[j]);
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    c2 = 0;
  }
  t[15] = (uint32_t)acc;
  uint32_t cy = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = addc32(t[i], c[i], cy, cy);
#pragma unroll
  for (int i = 8; i < 16; i++) t[i] = addc32(t[i], 0, cy, cy);
  sc_reduce512(r, t);
}

COA_DEV void sc_mul(sc& r, const uint32_t* a, const uint32_t* b) {
  const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  sc_muladd(r, a, b, z);
}

// r = a + b mod l for canonical a, b.
COA_DEV void sc_add(sc& r, const uint32_t* a, const uint32_t* b) {
  uint32_t l[8];
  sc_const_l(l);
  uint32_t t[8], u[8];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = addc32(a[i], b[i], c, c);
  uint32_t bb = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) u[i] = subb32(t[i], l[i], bb, bb);
  const bool ge = (c != 0) || (bb == 0);
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = ge ? u[i] : t[i];
}

// r = -a mod l for canonical a.
COA_DEV void sc_neg(sc& r, const uint32_t* a) {
  uint32_t l[8];
  sc_const_l(l);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a[i];
  uint32_t bb = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb32(l[i], a[i], bb, bb);
  if (o == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
  }
}
