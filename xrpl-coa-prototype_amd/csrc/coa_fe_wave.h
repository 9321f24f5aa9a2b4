// Row-parallel GF(2^255 - 19) arithmetic for latency-bound chains on gfx950.
//
// A lone wave issues one VALU instruction every ~5 cycles, so a field
// squaring done by one lane (176 instructions, coa_fe.h) costs ~900 cycles
// and the ~254 squarings of a decompression or inversion chain take ~90 us.
// Here ONE field element is spread over a 16-lane DPP row: lane c of the row
// holds limb c (32-bit, c < 8; lanes 8..15 hold 0), so a product is
//   8 row broadcasts of b's limbs (DPP row_newbcast),
//   7 row shifts of a (DPP row_shr, zero fill),
//   8 multiply-accumulates per lane (lane c sums column c = sum_k a_{c-k} b_k),
//   the spread of each column's upper words to the next lanes (row_shr:1 /
//   :2), the fold of limbs 8..15 by 2^256 = 38 (mod p) (row_shl:8), and two
//   carry passes with limb 7's carry wrapped into limb 0 (a uniform branch
//   to a rippling loop only while a carry is left),
// about 60 instructions on the chain instead of 176-214.  The four rows of a
// wave are independent: each row computes its own product (the Horner step of
// k_msm_final runs four different products at once), or all four compute the
// same one (decompression in the certificate latency kernel).
//
// Values are < 2^256 in 8 limbs, not canonical; fw::to_fe returns them in
// the ordinary (replicated per lane) representation of coa_fe.h, where
// fe_canon finishes.  All 16 lanes of a row must execute these functions
// together (DPP reads the row's other lanes); rows are independent, and a
// whole row may sit out (k_msm_prep's last rows).  Checked against coa_fe.h by
// coa_fe_rows_check_device (tests/test_gpu_fe_rows.py).
#pragma once
#include "coa_fe.h"

namespace fw {

COA_DEV uint32_t row_lane() { return __lane_id() & 15u; }

template <int K>
COA_DEV uint32_t shr(uint32_t x) {  // lane c of the row gets lane c-K, 0 below the row
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x110 + K, 0xf, 0xf, true);
}
template <int K>
COA_DEV uint32_t shl(uint32_t x) {  // lane c gets lane c+K, 0 past the row
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x100 + K, 0xf, 0xf, true);
}
template <int K>
COA_DEV uint32_t bcast(uint32_t x) {  // every lane of the row gets the row's lane K
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + K, 0xf, 0xf, false);
}

// One carry pass over the row's 8 limbs of per-lane 64-bit values: lane c
// keeps its low word plus lane c-1's high word; limb 7's high word re-enters
// limb 0 times 38 (2^256 = 38 mod p).  Lanes 8..15 stay 0.  (Selects, not
// branches: lane-dependent ternaries on 64-bit values would become exec-mask
// branches.)
COA_DEV uint32_t wrap_step(uint64_t& m, uint32_t r) {
  const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
  const uint32_t h7 = bcast<7>(hi);
  const uint32_t sh = shr<1>(hi);
  uint32_t add = r == 0 ? __umul24(h7, 38u) : sh;  // h7 < 2^9: the full-rate 24-bit multiply
  add = r < 8 ? add : 0u;
  m = (uint64_t)lo + add;
  return r < 8 ? hi : 0u;
}
// Per-lane values m_c < 2^40 on lanes 0..7 (0 above) -> 32-bit limbs of a
// congruent value < 2^256.  One pass leaves every lane below 2^32 + 2^14
// (the carry from the lane below, or 38 times limb 7's), so a lane still has
// a high word only when its low word was within 2^14 of 2^32: the uniform
// branch to the rippling passes is almost never taken.  It is marked so
// (__builtin_expect): as a plain loop the common path took three branches
// per product, which made a lone wave's row squaring 352 cycles instead of
// 293 (tools/ubench_rows2.hip).
COA_DEV uint32_t normalize(uint64_t m) {
  const uint32_t r = row_lane();
  wrap_step(m, r);
  if (__builtin_expect(__any((uint32_t)(m >> 32) != 0u), 0)) {
#pragma unroll 1
    do wrap_step(m, r);
    while (__any((uint32_t)(m >> 32) != 0u));
  }
  return (uint32_t)m;
}
// 4p and 8p in unnormalised limbs (limb 0: 4p_0 = 2^33 - 76, limbs 1..7:
// 2^33 - 2; doubled for 8p; 0 on lanes 8..15): added before a subtraction so
// no lane goes negative
COA_DEV uint64_t four_p() {
  const uint32_t r = row_lane();
  return r == 0 ? 0x1ffffffb4ull : (r < 8 ? 0x1fffffffeull : 0ull);
}

// Per-lane constants of the asm forms below (loop-invariant, kept in
// registers by the compiler).
COA_DEV uint32_t lanes_lo8() { return row_lane() < 8 ? 0xffffffffu : 0u; }
COA_DEV uint32_t k38_lane0() { return row_lane() == 0 ? 38u : 0u; }

// wrap_step as one asm statement whose adds read their shifted and broadcast
// operands through DPP themselves (VOP2 DPP), instead of separate DPP moves,
// lane-index compares and selects: lanes 0..7 get lo + hi_{c-1} (lane 0:
// lo + 38 * hi_7) and the carry in hi; bank_mask 0x3 leaves lanes 8..15
// (which must hold 0) unwritten.  The leading s_nop covers the DPP read of
// `hi`, which the compiler's hazard check cannot see inside the statement.
COA_DEV void wrap_dpp(uint32_t& lo, uint32_t& hi) {
  uint32_t t;
  asm("s_nop 1\n\t"
      "v_mul_u32_u24_dpp %[t], %[hi], %[k] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_add_co_u32_dpp %[lo], vcc, %[hi], %[lo] row_shr:1 row_mask:0xf bank_mask:0x3 bound_ctrl:1\n\t"
      "v_addc_co_u32_dpp %[hi], vcc, %[z], %[z], vcc quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x3\n\t"
      "v_add_co_u32_e32 %[lo], vcc, %[t], %[lo]\n\t"
      "v_addc_co_u32_e32 %[hi], vcc, 0, %[hi], vcc"
      : [lo] "+v"(lo), [hi] "+v"(hi), [t] "=&v"(t)
      : [k] "v"(k38_lane0()), [z] "v"(0u)
      : "vcc");
}
// normalize with the first pass as wrap_dpp (lanes 8..15 of m must be 0).
COA_DEV uint32_t normalize_dpp(uint64_t m) {
  uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
  wrap_dpp(lo, hi);
  if (__builtin_expect(__any(hi != 0u), 0)) {
    const uint32_t r = row_lane();
    uint64_t v = ((uint64_t)hi << 32) | lo;
#pragma unroll 1
    do wrap_step(v, r);
    while (__any((uint32_t)(v >> 32) != 0u));
    lo = (uint32_t)v;
  }
  return lo;
}

// a + b and a - b mod p (not canonical).  The difference adds 4p in
// unnormalised limbs (limb 0: 2^33 - 76, limbs 1..7: 2^33 - 2), so no lane
// goes negative.
COA_DEV uint32_t add(uint32_t a, uint32_t b) { return normalize_dpp((uint64_t)a + b); }
COA_DEV uint32_t sub(uint32_t a, uint32_t b) { return normalize_dpp((uint64_t)a + four_p() - b); }

// a * b mod p (not canonical), one product per 16-lane row.  Round 3: the
// round-2 steps with fewer instructions on the chain: the column sums
// start from the first product (no zeroed accumulator, the first carry word
// from the second product's carry), the spread of each column's upper words
// is two VOP2 adds that read them through DPP, lanes 8..15 are cleared by a
// mask instead of a lane compare and selects, and the wrap pass is wrap_dpp.
// tools/ubench_rows3.hip (one wave, dependent squarings): 283-290 -> 259-265
// cycles per squaring against the round-2 form; forms with the whole tail in
// one statement (272) or the operand moves interleaved with the
// multiply-accumulates (265-272) measured slower and are kept there only.
COA_DEV uint32_t mul(uint32_t a, uint32_t b) {
  uint32_t bk[8], ak[8];
  bk[0] = bcast<0>(b);
  bk[1] = bcast<1>(b);
  bk[2] = bcast<2>(b);
  bk[3] = bcast<3>(b);
  bk[4] = bcast<4>(b);
  bk[5] = bcast<5>(b);
  bk[6] = bcast<6>(b);
  bk[7] = bcast<7>(b);
  ak[0] = a;
  ak[1] = shr<1>(a);
  ak[2] = shr<2>(a);
  ak[3] = shr<3>(a);
  ak[4] = shr<4>(a);
  ak[5] = shr<5>(a);
  ak[6] = shr<6>(a);
  ak[7] = shr<7>(a);
  uint64_t acc;
  uint32_t c2;
  asm("v_mad_u64_u32 %0, vcc, %2, %10, 0\n\t"
      "v_mad_u64_u32 %0, vcc, %3, %11, %0\n\t"
      "v_addc_co_u32_e64 %1, vcc, 0, 0, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %12, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %5, %13, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %6, %14, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %7, %15, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %8, %16, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %9, %17, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "=&v"(acc), "=&v"(c2)
      : "v"(ak[0]), "v"(ak[1]), "v"(ak[2]), "v"(ak[3]), "v"(ak[4]), "v"(ak[5]), "v"(ak[6]), "v"(ak[7]), "v"(bk[0]),
        "v"(bk[1]), "v"(bk[2]), "v"(bk[3]), "v"(bk[4]), "v"(bk[5]), "v"(bk[6]), "v"(bk[7])
      : "vcc");
  // n_c = w0_c + w1_{c-1} + c2_{c-2} (< 2^34) as nlo + 2^32 nhi; ml/mh = n on
  // lanes 0..7 (0 above); ul/uh = n_{c+8} (0 past the row)
  uint32_t nlo, nhi, ml, mh, ul, uh;
  asm("s_nop 1\n\t"
      "v_add_co_u32_dpp %[nlo], vcc, %[w1], %[w0] row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_addc_co_u32_e64 %[nhi], vcc, 0, 0, vcc\n\t"
      "v_add_co_u32_dpp %[nlo], vcc, %[c2], %[nlo] row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_addc_co_u32_e32 %[nhi], vcc, 0, %[nhi], vcc\n\t"
      "v_and_b32_e32 %[ml], %[nlo], %[m8]\n\t"
      "v_and_b32_e32 %[mh], %[nhi], %[m8]\n\t"
      "v_mov_b32_dpp %[ul], %[nlo] row_shl:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      "v_mov_b32_dpp %[uh], %[nhi] row_shl:8 row_mask:0xf bank_mask:0xf bound_ctrl:1"
      : [nlo] "=&v"(nlo), [nhi] "=&v"(nhi), [ml] "=&v"(ml), [mh] "=&v"(mh), [ul] "=&v"(ul), [uh] "=&v"(uh)
      : [w0] "v"((uint32_t)acc), [w1] "v"((uint32_t)(acc >> 32)), [c2] "v"(c2), [m8] "v"(lanes_lo8())
      : "vcc");
  // fold n_{c+8} by 2^256 = 38 (mod p): < 2^40 on lanes 0..7, 0 above
  uint64_t m = (uint64_t)ul * 38u + (((uint64_t)mh << 32) | ml);
  m += (uint64_t)__umul24(uh, 38u) << 32;  // uh <= 3
  return normalize_dpp(m);
}
COA_DEV uint32_t sq(uint32_t a) { return mul(a, a); }
// a^(2^N): four squarings per loop trip (one loop branch per four: 293 ->
// ~278 cycles per squaring, tools/ubench_rows2.hip)
template <int N>
COA_DEV uint32_t sqn(uint32_t a) {
#pragma unroll 1
  for (int i = 0; i < N / 4; i++) {
    a = mul(a, a);
    a = mul(a, a);
    a = mul(a, a);
    a = mul(a, a);
  }
#pragma unroll
  for (int i = 0; i < N % 4; i++) a = mul(a, a);
  return a;
}

COA_DEV uint32_t from_fe(const fe& a) {  // this lane's limb of its own copy of a
  const uint32_t r = row_lane();
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x = r == (uint32_t)i ? a.v[i] : x;
  return x;
}
COA_DEV void to_fe(fe& r, uint32_t x) {  // every lane of the row gets the row's value
  r.v[0] = bcast<0>(x);
  r.v[1] = bcast<1>(x);
  r.v[2] = bcast<2>(x);
  r.v[3] = bcast<3>(x);
  r.v[4] = bcast<4>(x);
  r.v[5] = bcast<5>(x);
  r.v[6] = bcast<6>(x);
  r.v[7] = bcast<7>(x);
}

// z^(2^252 - 3) (FieldElement::pow_p58) and z^(p - 2), the chains of
// coa_fe.h fe_pow_chain on rows.
COA_DEV uint32_t pow_chain(uint32_t& z11, uint32_t z) {
  const uint32_t z2 = sq(z);
  const uint32_t z9 = mul(sqn<2>(z2), z);
  z11 = mul(z9, z2);
  const uint32_t z_5_0 = mul(sq(z11), z9);
  const uint32_t z_10_0 = mul(sqn<5>(z_5_0), z_5_0);
  const uint32_t z_20_0 = mul(sqn<10>(z_10_0), z_10_0);
  const uint32_t z_40_0 = mul(sqn<20>(z_20_0), z_20_0);
  const uint32_t z_50_0 = mul(sqn<10>(z_40_0), z_10_0);
  const uint32_t z_100_0 = mul(sqn<50>(z_50_0), z_50_0);
  const uint32_t z_200_0 = mul(sqn<100>(z_100_0), z_100_0);
  return mul(sqn<50>(z_200_0), z_50_0);  // 2^250 - 1
}
COA_DEV uint32_t pow_p58(uint32_t z) {
  uint32_t z11;
  const uint32_t t = pow_chain(z11, z);
  return mul(sqn<2>(t), z);
}
COA_DEV uint32_t invert(uint32_t z) {
  uint32_t z11;
  const uint32_t t = pow_chain(z11, z);
  return mul(sqn<5>(t), z11);
}

}  // namespace fw

// fe_pow_p58 / fe_invert with the chain on rows (replicated fe in and out).
COA_DEV void fe_pow_p58_rows(fe& r, const fe& z) { fw::to_fe(r, fw::pow_p58(fw::from_fe(z))); }
COA_DEV void fe_invert_rows(fe& r, const fe& z) { fw::to_fe(r, fw::invert(fw::from_fe(z))); }
