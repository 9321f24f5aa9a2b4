// GF(2^255 - 19) arithmetic for gfx950 (CDNA4) -- one field element per lane.
//
// Representation: 8 x 32-bit little-endian limbs holding a value in [0, 2^256)
// that is congruent to the element mod p ("weakly reduced").  Canonical form
// (< p) is produced only where the reference compares encodings
// (curve25519-dalek FieldElement::ct_eq / is_negative / to_bytes), by
// fe_canon().
//
// Why radix 2^32: the measured gfx950 issue costs (tools/ubench_valu.hip,
// profiles/r01_ubench_valu.txt) put v_mad_u64_u32 -- a full 32x32->64 product
// plus a 64-bit addend -- at the same rate as a lone v_mul_lo_u32, so 64 of
// them per schoolbook product beat the 100 of a 10 x 25.5-bit layout.  The
// column (comba) accumulation keeps a 96-bit accumulator (64-bit pair + carry
// word) and takes the mad's own carry-out, so each partial product costs one
// v_mad_u64_u32 + one v_addc_co_u32 (tools/ubench_fe.hip: 214 VALU
// instructions per multiply, 176 per squaring; profiles/r01_ubench_fe*.txt).
//
// Reduction uses 2^256 == 38 (mod p).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define COA_DEV __device__ __forceinline__

struct fe {
  uint32_t v[8];
};

// ---------------------------------------------------------------- helpers
COA_DEV uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
  unsigned int c;
  uint32_t r = __builtin_addc(a, b, cin, &c);
  cout = c;
  return r;
}
COA_DEV uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t& bout) {
  unsigned int c;
  uint32_t r = __builtin_subc(a, b, bin, &c);
  bout = c;
  return r;
}

// (acc:64, c2:32) += a * b.  v_mad_u64_u32 writes its carry-out to an SGPR
// pair (one bit per lane), which v_addc_co_u32 folds into the third word.
COA_DEV void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t sc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(sc), "+v"(c2)
      : "v"(a), "v"(b));
}

// First product of a column: the carry word starts from the mad's carry-out
// instead of a separately zeroed register.
COA_DEV void mac0(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t sc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32 %2, %1, 0, 0, %1"
      : "+v"(acc), "=&s"(sc), "=v"(c2)
      : "v"(a), "v"(b));
}

COA_DEV void fe_set(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = 0;
}

// ------------------------------------------------------- add / sub / neg
// r = a + b (mod p), result < 2^256.
COA_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(a.v[i], b.v[i], c, c);
  // 2^256 == 38: fold the carry; a second carry can only occur when the sum
  // wrapped to a value < 38, so the last fold cannot carry.
  uint32_t c2 = 0;
  r.v[0] = addc32(r.v[0], c * 38u, 0, c2);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc32(r.v[i], 0, c2, c2);
  r.v[0] += c2 * 38u;
}

// r = a - b (mod p), result < 2^256.
COA_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb32(a.v[i], b.v[i], bw, bw);
  // a - b + 2^256 was computed: subtract 2^256 == 38.
  uint32_t b2 = 0;
  r.v[0] = subb32(r.v[0], bw * 38u, 0, b2);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = subb32(r.v[i], 0, b2, b2);
  r.v[0] -= b2 * 38u;
}

COA_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

// ------------------------------------------------------------- reduction
// r = t[0..15] (512-bit) mod p, result < 2^256.
COA_DEV void fe_reduce512(fe& r, const uint32_t* t) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c = (uint64_t)t[8 + i] * 38u + (c >> 32) + t[i];
    r.v[i] = (uint32_t)c;
  }
  uint32_t hi = (uint32_t)(c >> 32) * 38u;  // < 39 * 38
  uint32_t cc = 0;
  r.v[0] = addc32(r.v[0], hi, 0, cc);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc32(r.v[i], 0, cc, cc);
  r.v[0] += cc * 38u;
}

// ------------------------------------------------------------ multiply
COA_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j < 0 || j > 7) continue;
      if (first) mac0(acc, c2, a.v[i], b.v[j]);
      else mac(acc, c2, a.v[i], b.v[j]);
      first = false;
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

// Squaring: the 28 cross products by comba, doubled with one carry chain,
// then the 8 squares added with a second chain (44 mads vs 72 for fe_mul).
COA_DEV void fe_sq(fe& r, const fe& a) {
  uint32_t t[16];
  t[0] = 0;
  uint64_t acc = 0;
  uint32_t c2 = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j <= i || j > 7) continue;
      if (first) mac0(acc, c2, a.v[i], a.v[j]);
      else mac(acc, c2, a.v[i], a.v[j]);
      first = false;
    }
    t[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
  }
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = addc32(t[i], t[i], c, c);
  uint32_t d[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t p = (uint64_t)a.v[i] * a.v[i];
    d[2 * i] = (uint32_t)p;
    d[2 * i + 1] = (uint32_t)(p >> 32);
  }
  c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = addc32(t[i], d[i], c, c);
  fe_reduce512(r, t);
}

COA_DEV void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
  for (int i = 1; i < n; i++) fe_sq(r, r);
}

// r = a * c for a small constant c < 2^26.
COA_DEV void fe_mul_small(fe& r, const fe& a, uint32_t c) {
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc = (uint64_t)a.v[i] * c + (acc >> 32);
    r.v[i] = (uint32_t)acc;
  }
  uint32_t hi = (uint32_t)(acc >> 32) * 38u;
  uint32_t cc = 0;
  r.v[0] = addc32(r.v[0], hi, 0, cc);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc32(r.v[i], 0, cc, cc);
  r.v[0] += cc * 38u;
}

// ------------------------------------------------------------ canonical
// Fully reduce to [0, p).
COA_DEV void fe_canon(fe& r, const fe& a) {
  fe t = a;
  // two folds of bit 255 (2^255 == 19) bring the value below 2^255
#pragma unroll
  for (int rep = 0; rep < 2; rep++) {
    uint32_t q = t.v[7] >> 31;
    t.v[7] &= 0x7fffffffu;
    uint32_t c = 0;
    t.v[0] = addc32(t.v[0], q * 19u, 0, c);
#pragma unroll
    for (int i = 1; i < 8; i++) t.v[i] = addc32(t.v[i], 0, c, c);
  }
  // t in [0, 2^255): t >= p  <=>  t + 19 >= 2^255
  fe u;
  uint32_t c = 0;
  u.v[0] = addc32(t.v[0], 19u, 0, c);
#pragma unroll
  for (int i = 1; i < 8; i++) u.v[i] = addc32(t.v[i], 0, c, c);
  const bool ge = (u.v[7] >> 31) != 0;
  u.v[7] &= 0x7fffffffu;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = ge ? u.v[i] : t.v[i];
}

COA_DEV bool fe_iszero(const fe& a) {
  fe c;
  fe_canon(c, a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= c.v[i];
  return o == 0;
}

// curve25519-dalek FieldElement::is_negative: low bit of the canonical encoding.
COA_DEV uint32_t fe_isneg(const fe& a) {
  fe c;
  fe_canon(c, a);
  return c.v[0] & 1u;
}

COA_DEV bool fe_eq(const fe& a, const fe& b) {
  fe d;
  fe_sub(d, a, b);
  return fe_iszero(d);
}

COA_DEV void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : r.v[i];
}

COA_DEV void fe_cneg(fe& r, bool c) {
  fe n;
  fe_neg(n, r);
  fe_cmov(r, n, c);
}

// ---------------------------------------------------------------- bytes
// curve25519-dalek FieldElement51::from_bytes: 255 bits, bit 255 ignored,
// values in [p, 2^255) kept (they are congruent to y - p).
COA_DEV void fe_from_words(fe& r, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = w[i];
  r.v[7] &= 0x7fffffffu;
}

COA_DEV void fe_to_words(uint32_t* w, const fe& a) {
  fe c;
  fe_canon(c, a);
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = c.v[i];
}

// ---------------------------------------------------------------- powers
// z^(2^252 - 3) = z^((p-5)/8)   (curve25519-dalek FieldElement::pow_p58)
// Also returns z^11 and z^(2^250-1) for the inversion chain.
COA_DEV void fe_pow_chain(fe& z_250_0, fe& z11, const fe& z) {
  fe z2, t, z9, z_5_0, z_10_0, z_20_0, z_40_0, z_50_0, z_100_0;
  fe_sq(z2, z);              // z^2
  fe_sqn(t, z2, 2);          // z^8
  fe_mul(z9, t, z);          // z^9
  fe_mul(z11, z9, z2);       // z^11
  fe_sq(t, z11);             // z^22
  fe_mul(z_5_0, t, z9);      // z^(2^5-1)
  fe_sqn(t, z_5_0, 5);
  fe_mul(z_10_0, t, z_5_0);  // 2^10-1
  fe_sqn(t, z_10_0, 10);
  fe_mul(z_20_0, t, z_10_0);  // 2^20-1
  fe_sqn(t, z_20_0, 20);
  fe_mul(z_40_0, t, z_20_0);  // 2^40-1
  fe_sqn(t, z_40_0, 10);
  fe_mul(z_50_0, t, z_10_0);  // 2^50-1
  fe_sqn(t, z_50_0, 50);
  fe_mul(z_100_0, t, z_50_0);  // 2^100-1
  fe_sqn(t, z_100_0, 100);
  fe_mul(t, t, z_100_0);  // 2^200-1
  fe_sqn(t, t, 50);
  fe_mul(z_250_0, t, z_50_0);  // 2^250-1
}

COA_DEV void fe_pow_p58(fe& r, const fe& z) {
  fe z_250_0, z11, t;
  fe_pow_chain(z_250_0, z11, z);
  fe_sqn(t, z_250_0, 2);  // 2^252-4
  fe_mul(r, t, z);        // 2^252-3
}

COA_DEV void fe_invert(fe& r, const fe& z) {
  fe z_250_0, z11, t;
  fe_pow_chain(z_250_0, z11, z);
  fe_sqn(t, z_250_0, 5);  // 2^255-32
  fe_mul(r, t, z11);      // 2^255-21 = p-2
}

// ------------------------------------------------------------- constants
COA_DEV void fe_const_d(fe& r) {
  const uint32_t c[8] = {0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du,
                         0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu};
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
}
COA_DEV void fe_const_d2(fe& r) {
  const uint32_t c[8] = {0x26b2f159u, 0xebd69b94u, 0x8283b156u, 0x00e0149au,
                         0xeef3d130u, 0x198e80f2u, 0x56dffce7u, 0x2406d9dcu};
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
}
COA_DEV void fe_const_sqrtm1(fe& r) {
  const uint32_t c[8] = {0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u,
                         0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u};
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
}
