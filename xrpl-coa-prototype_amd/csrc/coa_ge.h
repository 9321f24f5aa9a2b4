// Edwards25519 group operations for gfx950, one point per lane.
//
// Replaces curve25519-dalek 3.x `EdwardsPoint` on the verification path:
//   CompressedEdwardsY::decompress, EdwardsPoint::{is_small_order,
//   is_identity, ct_eq, double, add}, and the multiplications used by
//   vartime_double_scalar_mul_basepoint / the batch multiscalar sum.
// Coordinates (x = X/Z, y = Y/Z, xy = T/Z on -x^2 + y^2 = 1 + d x^2 y^2):
//   ge_p2     (X:Y:Z)            projective
//   ge_p3     (X:Y:Z:T)          extended
//   ge_p1p1   ((X:Z),(Y:T))      completed, output of dbl/add
//   ge_cached (Y+X, Y-X, Z, 2dT) addend form of an extended point
//   ge_niels  (y+x, y-x, 2dxy)   addend form of an affine point (Z = 1)
// The a = -1, d non-square addition law is complete, so every formula here
// is exact for all curve points, torsion included -- verdicts on adversarial
// small-order / mixed-order inputs depend only on group equality, exactly as
// in dalek.
#pragma once
#include "coa_fe.h"
#include "coa_fe_wave.h"

struct ge_p2 {
  fe X, Y, Z;
};
struct ge_p3 {
  fe X, Y, Z, T;
};
struct ge_p1p1 {
  fe X, Y, Z, T;
};
struct ge_cached {
  fe YplusX, YminusX, Z, T2d;
};
struct ge_niels {
  fe yplusx, yminusx, xy2d;
};

COA_DEV void ge_p3_identity(ge_p3& r) {
  fe_set(r.X, 0);
  fe_set(r.Y, 1);
  fe_set(r.Z, 1);
  fe_set(r.T, 0);
}
COA_DEV void ge_p2_identity(ge_p2& r) {
  fe_set(r.X, 0);
  fe_set(r.Y, 1);
  fe_set(r.Z, 1);
}
COA_DEV void ge_cached_identity(ge_cached& r) {
  fe_set(r.YplusX, 1);
  fe_set(r.YminusX, 1);
  fe_set(r.Z, 1);
  fe_set(r.T2d, 0);
}
COA_DEV void ge_niels_identity(ge_niels& r) {
  fe_set(r.yplusx, 1);
  fe_set(r.yminusx, 1);
  fe_set(r.xy2d, 0);
}

COA_DEV void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}
COA_DEV void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}
COA_DEV void ge_p3_to_p2(ge_p2& r, const ge_p3& p) {
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}
COA_DEV void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe d2;
  fe_const_d2(d2);
  fe_add(r.YplusX, p.Y, p.X);
  fe_sub(r.YminusX, p.Y, p.X);
  r.Z = p.Z;
  fe_mul(r.T2d, p.T, d2);
}

// 2P:  x3 = 2XY / (Y^2 - X^2),  y3 = (Y^2 + X^2) / (2Z^2 - Y^2 + X^2)
COA_DEV void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe xx, yy, b, a;
  fe_sq(xx, p.X);
  fe_sq(yy, p.Y);
  fe_sq(b, p.Z);
  fe_add(b, b, b);
  fe_add(a, p.X, p.Y);
  fe_sq(a, a);
  fe_add(r.Y, yy, xx);
  fe_sub(r.Z, yy, xx);
  fe_sub(r.X, a, r.Y);
  fe_sub(r.T, b, r.Z);
}
COA_DEV void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  ge_p3_to_p2(q, p);
  ge_p2_dbl(r, q);
}

// P + Q and P - Q with Q in cached form (add-2008-hwcd-3, k = 2d).
COA_DEV void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, zz;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
  fe_mul(b, r.X, q.YplusX);
  fe_mul(a, r.Y, q.YminusX);
  fe_mul(c, q.T2d, p.T);
  fe_mul(zz, p.Z, q.Z);
  fe_add(zz, zz, zz);
  fe_sub(r.X, b, a);
  fe_add(r.Y, b, a);
  fe_add(r.Z, zz, c);
  fe_sub(r.T, zz, c);
}
COA_DEV void ge_sub(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, zz;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
  fe_mul(b, r.X, q.YminusX);
  fe_mul(a, r.Y, q.YplusX);
  fe_mul(c, q.T2d, p.T);
  fe_mul(zz, p.Z, q.Z);
  fe_add(zz, zz, zz);
  fe_sub(r.X, b, a);
  fe_add(r.Y, b, a);
  fe_sub(r.Z, zz, c);
  fe_add(r.T, zz, c);
}
// Mixed addition with an affine Niels point (Z2 = 1).
COA_DEV void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe a, b, c, zz;
  fe_add(r.X, p.Y, p.X);
  fe_sub(r.Y, p.Y, p.X);
  fe_mul(b, r.X, q.yplusx);
  fe_mul(a, r.Y, q.yminusx);
  fe_mul(c, q.xy2d, p.T);
  fe_add(zz, p.Z, p.Z);
  fe_sub(r.X, b, a);
  fe_add(r.Y, b, a);
  fe_add(r.Z, zz, c);
  fe_sub(r.T, zz, c);
}

// The same formulas with their independent products interleaved column by
// column (fe_mul_n / fe_sq_n): for a wave alone on its SIMD, where the
// per-column dependency chains are exposed.  More live registers than the
// plain forms (up to four 16-word column buffers).
COA_DEV void ge_p1p1_to_p2_il(ge_p2& r, const ge_p1p1& p) {
  const fe a[3] = {p.X, p.Y, p.Z}, b[3] = {p.T, p.Z, p.T};
  fe o[3];
  fe_mul_n<3>(o, a, b);
  r.X = o[0];
  r.Y = o[1];
  r.Z = o[2];
}
COA_DEV void ge_p1p1_to_p3_il(ge_p3& r, const ge_p1p1& p) {
  const fe a[4] = {p.X, p.Y, p.Z, p.X}, b[4] = {p.T, p.Z, p.T, p.Y};
  fe o[4];
  fe_mul_n<4>(o, a, b);
  r.X = o[0];
  r.Y = o[1];
  r.Z = o[2];
  r.T = o[3];
}
COA_DEV void ge_p2_dbl_il(ge_p1p1& r, const ge_p2& p) {
  fe s[4];
  s[0] = p.X;
  s[1] = p.Y;
  s[2] = p.Z;
  fe_add(s[3], p.X, p.Y);
  fe o[4];
  fe_sq_n<4>(o, s);
  fe_add(o[2], o[2], o[2]);
  fe_addsub(r.Y, r.Z, o[1], o[0]);
  fe_sub(r.X, o[3], r.Y);
  fe_sub(r.T, o[2], r.Z);
}
COA_DEV void ge_add_il(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a[4], o[4];
  fe_addsub(a[0], a[1], p.Y, p.X);
  a[2] = q.T2d;
  a[3] = p.Z;
  const fe b[4] = {q.YplusX, q.YminusX, p.T, q.Z};
  fe_mul_n<4>(o, a, b);
  fe_add(o[3], o[3], o[3]);
  fe_addsub(r.Y, r.X, o[0], o[1]);
  fe_addsub(r.Z, r.T, o[3], o[2]);
}

COA_DEV void ge_madd_il(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe a[3], o[3], zz;
  fe_addsub(a[0], a[1], p.Y, p.X);
  a[2] = q.xy2d;
  const fe b[3] = {q.yplusx, q.yminusx, p.T};
  fe_mul_n<3>(o, a, b);
  fe_add(zz, p.Z, p.Z);
  fe_addsub(r.Y, r.X, o[0], o[1]);
  fe_addsub(r.Z, r.T, zz, o[2]);
}

// Conditionally negate an addend: -(x, y) = (-x, y) swaps Y+X / Y-X and
// negates the T term.
COA_DEV void ge_cached_cneg(ge_cached& q, bool neg) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t a = q.YplusX.v[i], b = q.YminusX.v[i];
    q.YplusX.v[i] = neg ? b : a;
    q.YminusX.v[i] = neg ? a : b;
  }
  fe_cneg(q.T2d, neg);
}
COA_DEV void ge_niels_cneg(ge_niels& q, bool neg) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t a = q.yplusx.v[i], b = q.yminusx.v[i];
    q.yplusx.v[i] = neg ? b : a;
    q.yminusx.v[i] = neg ? a : b;
  }
  fe_cneg(q.xy2d, neg);
}

// curve25519-dalek FieldElement::sqrt_ratio_i(u, v): (was_nonzero_square, r)
// with r the non-negative root of u/v (or of i*u/v when u/v is a non-square).
// Rows = true: every product on 16-lane DPP rows (coa_fe_wave.h); all lanes
// of a row must then take part.
template <bool Rows = false>
COA_DEV bool fe_sqrt_ratio_i(fe& r, const fe& u, const fe& v) {
  fe check, nu, nui, i, ri;
  fe_const_sqrtm1(i);
  fe_neg(nu, u);
  if constexpr (Rows) {  // every product on the rows; back to lanes for the tests
    const uint32_t fu = fw::from_fe(u), fv = fw::from_fe(v), fi = fw::from_fe(i);
    const uint32_t v3 = fw::mul(fw::sq(fv), fv);
    const uint32_t v7 = fw::mul(fw::sq(v3), fv);
    const uint32_t t = fw::pow_p58(fw::mul(fu, v7));
    const uint32_t rr = fw::mul(fw::mul(fu, v3), t);
    fw::to_fe(r, rr);
    fw::to_fe(check, fw::mul(fw::sq(rr), fv));
    fw::to_fe(ri, fw::mul(rr, fi));
    fw::to_fe(nui, fw::mul(fw::from_fe(nu), fi));
  } else {
    fe v3, v7, t;
    fe_sq(v3, v);
    fe_mul(v3, v3, v);  // v^3
    fe_sq(v7, v3);
    fe_mul(v7, v7, v);  // v^7
    fe_mul(t, u, v7);
    fe_pow_p58(t, t);   // (u v^7)^((p-5)/8)
    fe_mul(r, u, v3);
    fe_mul(r, r, t);    // u v^3 (u v^7)^((p-5)/8)
    fe_sq(check, r);
    fe_mul(check, check, v);
    fe_mul(nui, nu, i);
    fe_mul(ri, r, i);
  }
  const bool correct = fe_eq(check, u);
  const bool flipped = fe_eq(check, nu);
  const bool flipped_i = fe_eq(check, nui);
  fe_cmov(r, ri, flipped || flipped_i);
  fe_cneg(r, fe_isneg(r) != 0);
  return correct || flipped;
}

// curve25519-dalek 3.x CompressedEdwardsY::decompress on the 8 little-endian
// dwords of the encoding.  Accepts y in [p, 2^255) (means y - p) and
// "negative zero" (x = 0 with the sign bit set), exactly as dalek does.
template <bool Rows = false>
COA_DEV bool ge_decompress(ge_p3& r, const uint32_t* w) {
  fe y, yy, u, v, x, one, d;
  fe_from_words(y, w);
  fe_set(one, 1);
  fe_const_d(d);
  fe_sq(yy, y);
  fe_sub(u, yy, one);   // u = y^2 - 1
  fe_mul(v, yy, d);
  fe_add(v, v, one);    // v = d y^2 + 1
  const bool ok = fe_sqrt_ratio_i<Rows>(x, u, v);
  fe_cneg(x, (w[7] >> 31) != 0);
  r.X = x;
  r.Y = y;
  fe_set(r.Z, 1);
  fe_mul(r.T, x, y);
  return ok;
}

// EdwardsPoint::is_identity: projective compare with (0 : 1 : 1).
COA_DEV bool ge_p2_is_identity(const ge_p2& p) {
  return fe_iszero(p.X) && fe_eq(p.Y, p.Z);
}

// EdwardsPoint::is_small_order ([8]P == identity), as a coordinate test.
// The eight points of E[8] are exactly those with X = 0 (orders 1 and 2),
// Y = 0 (order 4: x^2 = -1) or X^2 + Y^2 = 0 (order 8: y^2 = -x^2 on
// -x^2 + y^2 = 1 + d x^2 y^2 gives d x^4 - 2 x^2 - 1 = 0, whose four points
// are the order-8 ones).  Homogeneous, so valid for any Z != 0.  Two
// squarings instead of three doublings (~21 field operations); checked
// against [8]P == O on every torsion point and on random and mixed-order
// points with the oracle, and by the small-order golden classes.
COA_DEV bool ge_is_small_order(const ge_p3& p) {
  fe xx, yy, s;
  fe_sq(xx, p.X);
  fe_sq(yy, p.Y);
  fe_add(s, xx, yy);
  return fe_iszero(p.X) || fe_iszero(p.Y) || fe_iszero(s);
}

// EdwardsPoint::ct_eq between a projective P and an extended Q.
COA_DEV bool ge_p2_eq_p3(const ge_p2& p, const ge_p3& q) {
  fe a, b;
  fe_mul(a, p.X, q.Z);
  fe_mul(b, q.X, p.Z);
  if (!fe_eq(a, b)) return false;
  fe_mul(a, p.Y, q.Z);
  fe_mul(b, q.Y, p.Z);
  return fe_eq(a, b);
}

// Compression (signing / table building only).
COA_DEV void ge_p2_compress(uint32_t* out, const ge_p2& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_to_words(out, y);
  out[7] |= fe_isneg(x) << 31;
}

// Base point B (RFC 8032 5.1) in extended coordinates.
COA_DEV void ge_basepoint(ge_p3& r) {
  const uint32_t bx[8] = {0x8f25d51au, 0xc9562d60u, 0x9525a7b2u, 0x692cc760u,
                          0xfdd6dc5cu, 0xc0a4e231u, 0xcd6e53feu, 0x216936d3u};
  const uint32_t by[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.X.v[i] = bx[i];
    r.Y.v[i] = by[i];
  }
  fe_set(r.Z, 1);
  fe_mul(r.T, r.X, r.Y);
}
