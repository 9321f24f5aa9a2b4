// decompress(R) == P for the latency kernels (k_verify_lat's and
// k_cert_verify_lat's registered-key path), with R's decompression fused
// into the compare.
//
// dalek's verify_strict ends with `R == signature_R` after
// CompressedEdwardsY::decompress (curve25519-dalek 3.x edwards.rs,
// FieldElement::sqrt_ratio_i): y from the encoding, u = y^2 - 1,
// v = d y^2 + 1, r = u v^3 (u v^7)^((p-5)/8), check = v r^2 compared with u,
// -u and -u i, then r (times i) made non-negative and negated by the sign bit.
// Its ~254 dependent squarings are the critical chain of these kernels, so
// everything else moves off it:
//   * the wave that owns P prepares, while the chain runs, Z_P, Z_P i, the
//     canonical +-X_P, whether u == 0, and the y half of the compare,
//     y_R Z_P == Y_P (rcmp::prepare);
//   * after the chain two row products finish everything, the four rows of
//     the wave each taking one (coa_ge_rows.h): first t^2 and r = u v^3 t,
//     then w = u v^7 t^2 (check = v r^2 = u w, so check == u, -u, -u i
//     become u == 0 or w == 1, -1, -i) beside r Z_P, r i Z_P and r i.
// The verdict bits are dalek's exactly: decompress(R) is Some iff
// check == +-u, and x_R = sigma r' with r' = r or r i and
// sigma = (-1)^(isneg(r') + sign bit), so X_P == x_R Z_P iff
// r' Z_P == sigma X_P (canonical compare).
//
// Also here: the registered-key comb sums of those kernels on the rows
// (comb_sum_rows), and prepare_rows, P's half of the compare for a P in row
// form.
#pragma once
#include "coa_ge_rows.h"
#include "coa_keycache.h"
#include "coa_smul.h"

namespace rcmp {

// LDS hand-off from the wave that owns P to the wave that decompresses R
struct Shared {
  uint32_t zp[8], zi[8], xc[8], nxc[8];
  uint32_t y_eq, u_zero, bits, ready;
};

// canonical p - 1 and -i (= p - sqrt(-1))
COA_DEV bool eq_m1(const fe& c) {
  bool e = c.v[0] == 0xffffffecu && c.v[7] == 0x7fffffffu;
#pragma unroll
  for (int k = 1; k < 7; k++) e = e && c.v[k] == 0xffffffffu;
  return e;
}
COA_DEV bool eq_mi(const fe& c) {
  const uint32_t m[8] = {0xb5f15f3du, 0x3b11e4d8u, 0x52d01b87u, 0xd0bce7f9u,
                         0xc2042858u, 0xd4b2ff66u, 0xb03e20f4u, 0x547cdb7fu};
  bool e = true;
#pragma unroll
  for (int k = 0; k < 8; k++) e = e && c.v[k] == m[k];
  return e;
}
COA_DEV bool eq_one(const fe& c) {
  bool e = c.v[0] == 1u;
#pragma unroll
  for (int k = 1; k < 8; k++) e = e && c.v[k] == 0u;
  return e;
}
COA_DEV bool eq_fe(const fe& a, const fe& b) {
  bool e = true;
#pragma unroll
  for (int k = 0; k < 8; k++) e = e && a.v[k] == b.v[k];
  return e;
}

// (the wave that owns P; `write` on one lane) the compare's half that needs
// only P and R's encoding rw; bits travel to the deciding wave unchanged.
// Sets ready last (release).
COA_DEV void prepare(Shared& s, const ge_p2& P, const uint32_t* rw, uint32_t bits, bool write) {
  fe y, yc, yz, i, zi, xc, nx, nxc;
  fe_from_words(y, rw);
  fe_mul(yz, y, P.Z);
  const bool y_eq = fe_eq(yz, P.Y);
  fe_canon(yc, y);
  const bool u_zero = eq_one(yc) || eq_m1(yc);  // u = y^2 - 1 == 0
  fe_const_sqrtm1(i);
  fe_mul(zi, P.Z, i);
  fe_canon(xc, P.X);
  fe_neg(nx, P.X);
  fe_canon(nxc, nx);
  if (!write) return;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    s.zp[k] = P.Z.v[k];
    s.zi[k] = zi.v[k];
    s.xc[k] = xc.v[k];
    s.nxc[k] = nxc.v[k];
  }
  s.y_eq = y_eq;
  s.u_zero = u_zero;
  s.bits = bits;
  __hip_atomic_store(&s.ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// no P to compare with (the key is not registered): only the bits
COA_DEV void skip(Shared& s, uint32_t bits, bool write) {
  if (!write) return;
  s.bits = bits;
  __hip_atomic_store(&s.ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// row k's element as a wave-uniform fe (lane 16k + j holds limb j)
COA_DEV void row_fe(fe& r, uint32_t x, int k) {
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = __builtin_amdgcn_readlane(x, 16 * k + j);
}

// P's half for a P in row form (every row holding it): one row product step
// gives X^2, Y^2 (verify_strict's small-order test of R, taken on P: an
// accepting verdict needs R == P), y_R Z and Z i.  small_bit is OR-ed into
// bits when P has small order.
COA_DEV void prepare_rows(Shared& s, const rp::P1& P, const uint32_t* rw, uint32_t bits, uint32_t small_bit,
                          bool write) {
  fe y, i;
  fe_from_words(y, rw);
  fe_const_sqrtm1(i);
  uint32_t xx, yy, zy, zi;
  rp::rows4(fw::mul(rp::pick(P.X, P.Y, P.Z, P.Z), rp::pick(P.X, P.Y, fw::from_fe(y), fw::from_fe(i))), xx, yy, zy,
            zi);
  fe X, Y, Z, XX, YY, ZY, ZI;
  row_fe(X, P.X, 0);
  row_fe(Y, P.Y, 0);
  row_fe(Z, P.Z, 0);
  row_fe(XX, xx, 0);
  row_fe(YY, yy, 0);
  row_fe(ZY, zy, 0);
  row_fe(ZI, zi, 0);
  fe xc, yc, sc, nx, nxc, zyc, ycan;
  fe_canon(xc, X);
  fe_canon(yc, Y);
  fe_add(sc, XX, YY);
  fe_canon(sc, sc);
  // is_small_order as in coa_ge.h: X = 0, Y = 0 or X^2 + Y^2 = 0
  const bool small = eq_fe(xc, fe{}) || eq_fe(yc, fe{}) || eq_fe(sc, fe{});
  fe_canon(zyc, ZY);
  const bool y_eq = eq_fe(zyc, yc);
  fe_canon(ycan, y);
  const bool u_zero = eq_one(ycan) || eq_m1(ycan);
  fe_neg(nx, X);
  fe_canon(nxc, nx);
  if (small) bits |= small_bit;
  if (!write) return;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    s.zp[k] = Z.v[k];
    s.zi[k] = ZI.v[k];
    s.xc[k] = xc.v[k];
    s.nxc[k] = nxc.v[k];
  }
  s.y_eq = y_eq;
  s.u_zero = u_zero;
  s.bits = bits;
  __hip_atomic_store(&s.ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// lane k's extended point in row form
COA_DEV void lane_point(rp::P1& r, const ge_p3& p, int k) {
  fe x, y, z, t;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.v[i] = __builtin_amdgcn_readlane(p.X.v[i], k);
    y.v[i] = __builtin_amdgcn_readlane(p.Y.v[i], k);
    z.v[i] = __builtin_amdgcn_readlane(p.Z.v[i], k);
    t.v[i] = __builtin_amdgcn_readlane(p.T.v[i], k);
  }
  r.X = fw::from_fe(x);
  r.Y = fw::from_fe(y);
  r.Z = fw::from_fe(z);
  r.T = fw::from_fe(t);
}

// (one whole wave) sum_j tab[j][byte j of dg] over the 32 signed radix-256
// digits of dg (the comb layout of coa_smul.h), in row form: one term per
// lane (lanes 32..63 repeat 0..31), two xor-butterfly levels on single lanes
// (each a whole one-lane point addition, ~9 products) leave 8 partial sums
// on lanes 0..7, which are then added on the rows (three row products each).
// The three one-lane levels this replaces cost ~22k cycles on a lone wave.
COA_DEV void comb_sum_rows(rp::P1& out, uint32_t* dg, const uint32_t* tab, uint32_t lane) {
  add_const_word(dg, 0x80808080u);
  const int j = lane & 31;
  const int e = (int)coa_kc::byte_of(dg, j) - 128;
  ge_niels q;
  comb_select(q, tab, j, e);
  ge_p1p1 t;
  ge_p3 P;
  ge_p3_identity(P);
  ge_madd(t, P, q);
  ge_p1p1_to_p3(P, t);
#pragma unroll 1
  for (int off = 16; off >= 8; off >>= 1) {
    ge_p3 O;
    coa_kc::shfl_fe<64>(O.X, P.X, off);
    coa_kc::shfl_fe<64>(O.Y, P.Y, off);
    coa_kc::shfl_fe<64>(O.Z, P.Z, off);
    coa_kc::shfl_fe<64>(O.T, P.T, off);
    ge_cached oc;
    ge_p3_to_cached(oc, O);
    ge_add(t, P, oc);
    ge_p1p1_to_p3(P, t);
  }
  rp::P1 acc, pk;
  rp::Ca c;
  rp::L1 l;
  lane_point(acc, P, 0);
#pragma unroll
  for (int k = 1; k < 8; k++) {
    lane_point(pk, P, k);
    rp::to_cached(c, pk);
    rp::add(l, acc, c);
    rp::to_p3(acc, l);
  }
  out = acc;
}

// a + b in row form
COA_DEV void add_rows(rp::P1& r, const rp::P1& a, const rp::P1& b) {
  rp::Ca c;
  rp::L1 l;
  rp::to_cached(c, b);
  rp::add(l, a, c);
  rp::to_p3(r, l);
}

// (all 64 lanes of the deciding wave) R's decompression and the compare with
// the P that s describes, once prepare() or skip() has run.  Returns bit 0:
// decompress(R) is Some; bit 1: decompress(R) == P.  `bits` gets s.bits.
// chain_done() runs between the power chain and the wait (trace marks).
template <class ChainDone>
COA_DEV uint32_t decompress_eq(const Shared& s, const uint32_t* rw, uint32_t& bits, ChainDone chain_done) {
  const uint32_t row = __lane_id() >> 4;
  fe y, d, one, i;
  fe_from_words(y, rw);
  fe_const_d(d);
  fe_set(one, 1);
  fe_const_sqrtm1(i);
  const uint32_t fy = fw::from_fe(y), fd = fw::from_fe(d), f1 = fw::from_fe(one), fi = fw::from_fe(i);
  const uint32_t yy = fw::sq(fy);
  const uint32_t fu = fw::sub(yy, f1);
  const uint32_t fv = fw::add(fw::mul(yy, fd), f1);
  const uint32_t v3 = fw::mul(fw::sq(fv), fv);
  const uint32_t q = fw::mul(row == 0 ? v3 : fu, v3);  // row 0: v^6, rows 1..3: u v^3
  const uint32_t uv7 = fw::mul(fu, fw::mul(q, fv));     // row 0: u v^7
  uint32_t t, t1, t2, t3;
  rp::rows4(fw::pow_p58(uv7), t, t1, t2, t3);           // row 0's power on every row
  const uint32_t a = fw::mul(row == 0 ? t : q, t);      // row 0: t^2, rows 1..3: r = u v^3 t
  chain_done();
#pragma unroll 1
  while (__hip_atomic_load(&s.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u)
    __builtin_amdgcn_s_sleep(1);
  bits = s.bits;
  fe zp, zi;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    zp.v[k] = s.zp[k];
    zi.v[k] = s.zi[k];
  }
  // row 0: w = u v^7 t^2, row 1: r Z_P, row 2: r Z_P i, row 3: r i
  const uint32_t b = fw::mul(a, rp::pick(uv7, fw::from_fe(zp), fw::from_fe(zi), fi));
  fe w, rz, rzi, r, ri;
  row_fe(w, b, 0);
  row_fe(rz, b, 1);
  row_fe(rzi, b, 2);
  row_fe(ri, b, 3);
  row_fe(r, a, 1);
  fe wc;
  fe_canon(wc, w);
  const bool uz = s.u_zero != 0;
  const bool correct = uz || eq_one(wc), flipped = uz || eq_m1(wc), flipped_i = uz || eq_mi(wc);
  const bool flip = flipped || flipped_i;
  fe rs, xzc;
  fe_canon(rs, flip ? ri : r);
  fe_canon(xzc, flip ? rzi : rz);
  const bool neg = ((rs.v[0] & 1u) != 0) != ((rw[7] >> 31) != 0);
  fe xp;
#pragma unroll
  for (int k = 0; k < 8; k++) xp.v[k] = neg ? s.nxc[k] : s.xc[k];
  const bool eq = s.y_eq != 0 && eq_fe(xzc, xp);
  return (correct || flipped ? 1u : 0u) | (eq ? 2u : 0u);
}
COA_DEV uint32_t decompress_eq(const Shared& s, const uint32_t* rw, uint32_t& bits) {
  return decompress_eq(s, rw, bits, [] {});
}

}  // namespace rcmp
