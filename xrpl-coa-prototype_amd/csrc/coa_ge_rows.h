// Row-form curve arithmetic on gfx950 (coa_fe_wave.h): every coordinate of a
// point is one uint32 per lane, each 16-lane DPP row holding the whole element
// (limb c on lane c of the row, lanes 8..15 zero), and the four rows of the
// wave hold the same point.  A step's four products run on the four rows at
// once, row r on operand pair r (a per-lane select), and every row then reads
// all four results back (three lane-swap instructions, rows4).  Additions and
// subtractions stay on the rows.  Used by the latency-bound chains: the
// Pippenger Horner pass (k_msm_final) and the single-signature kernel
// (k_verify_lat).  All 64 lanes of the wave must execute these together.
#pragma once
#include "coa_fe_wave.h"
#include "coa_ge.h"

namespace rp {
struct P2 {
  uint32_t X, Y, Z;
};
struct P1 {
  uint32_t X, Y, Z, T;
};
struct Ca {
  uint32_t ypx, ymx, Z, t2d;
};
struct L1 {  // completed point (p1p1), unnormalised 64-bit lane values
  uint64_t X, Y, Z, T;
};
COA_DEV uint32_t pick(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t r = __lane_id() >> 4;
  return r == 0 ? a : (r == 1 ? b : (r == 2 ? c : d));
}
// Row r's value to every row, for all four rows at once: v_permlane32_swap
// of q with itself gives (r0 r1 r0 r1) and (r2 r3 r2 r3); v_permlane16_swap of
// each with itself splits it into two broadcasts (tools/probe_permlane.hip
// checked the lane mapping on gfx950).  Three VALU instructions, no LDS.
COA_DEV void rows4(uint32_t q, uint32_t& r0, uint32_t& r1, uint32_t& r2, uint32_t& r3) {
  const auto h = __builtin_amdgcn_permlane32_swap(q, q, false, false);
  const auto lo = __builtin_amdgcn_permlane16_swap(h[0], h[0], false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(h[1], h[1], false, false);
  r0 = lo[0];
  r1 = lo[1];
  r2 = hi[0];
  r3 = hi[1];
}
// Sums and differences between the products stay unnormalised (64-bit lane
// values, < 2^36): a product normalises only the two operands it picks
// (fw::normalize_dpp), so a level costs two normalisations instead of one
// per addition.
COA_DEV uint64_t pick64(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  const uint32_t r = __lane_id() >> 4;
  return r == 0 ? a : (r == 1 ? b : (r == 2 ? c : d));
}
COA_DEV uint32_t nm(uint64_t v) { return fw::normalize_dpp(v); }
// 2P (p1p1, lazy) from projective P: ge_p2_dbl with its four squarings on
// the rows
COA_DEV void dbl(L1& r, const P2& p) {
  const uint32_t x = nm(pick64(p.X, p.Y, p.Z, (uint64_t)p.X + p.Y));
  uint32_t xx, yy, zz, aa;
  rows4(fw::mul(x, x), xx, yy, zz, aa);
  const uint64_t p4 = fw::four_p();
  r.Y = (uint64_t)yy + xx;                   // yy + xx
  r.Z = (uint64_t)yy + p4 - xx;              // yy - xx
  r.X = (uint64_t)aa + 2 * p4 - xx - yy;     // aa - Y
  r.T = 2 * (uint64_t)zz + xx + p4 - yy;     // 2 zz - Z
}
COA_DEV void to_p2(P2& r, const L1& p) {
  uint32_t unused;
  rows4(fw::mul(nm(pick64(p.X, p.Y, p.Z, p.Z)), nm(pick64(p.T, p.Z, p.T, p.T))), r.X, r.Y, r.Z, unused);
}
COA_DEV void to_p3(P1& r, const L1& p) {
  rows4(fw::mul(nm(pick64(p.X, p.Y, p.Z, p.X)), nm(pick64(p.T, p.Z, p.T, p.Y))), r.X, r.Y, r.Z, r.T);
}
// p (extended) + q (cached) -> p1p1 (lazy), as ge_add
COA_DEV void add(L1& r, const P1& p, const Ca& c) {
  const uint64_t p4 = fw::four_p();
  const uint32_t x = nm(pick64((uint64_t)p.Y + p.X, (uint64_t)p.Y + p4 - p.X, c.t2d, p.Z));
  uint32_t b, a, cc, zz;
  rows4(fw::mul(x, pick(c.ypx, c.ymx, p.T, c.Z)), b, a, cc, zz);
  r.X = (uint64_t)b + p4 - a;
  r.Y = (uint64_t)b + a;
  r.Z = 2 * (uint64_t)zz + cc;
  r.T = 2 * (uint64_t)zz + p4 - cc;
}
COA_DEV uint32_t ld(const uint32_t* base) {  // this lane's limb (0 on lanes 8..15 of the row)
  const uint32_t c = __lane_id() & 15u;
  return c < 8 ? base[c] : 0u;
}

// extended (p1p1 completed) -> cached (Y+X, Y-X, Z, 2dT) of the P1 given as
// extended coordinates (X, Y, Z, T)
COA_DEV void to_cached(Ca& c, const P1& p) {
  fe d2;
  fe_const_d2(d2);
  c.ypx = fw::add(p.Y, p.X);
  c.ymx = fw::sub(p.Y, p.X);
  c.Z = p.Z;
  c.t2d = fw::mul(p.T, fw::from_fe(d2));
}
// identity in extended coordinates (0 : 1 : 1 : 0)
COA_DEV void identity(P1& p) {
  const uint32_t one = (__lane_id() & 15u) == 0 ? 1u : 0u;
  p.X = 0;
  p.Y = one;
  p.Z = one;
  p.T = 0;
}
// -p in extended coordinates
COA_DEV void neg(P1& r, const P1& p) {
  r.X = fw::sub(0u, p.X);
  r.Y = p.Y;
  r.Z = p.Z;
  r.T = fw::sub(0u, p.T);
}
// row form of a replicated extended point, and back
COA_DEV void from_p3(P1& r, const ge_p3& p) {
  r.X = fw::from_fe(p.X);
  r.Y = fw::from_fe(p.Y);
  r.Z = fw::from_fe(p.Z);
  r.T = fw::from_fe(p.T);
}
COA_DEV void to_ge_p3(ge_p3& r, const P1& p) {
  fw::to_fe(r.X, p.X);
  fw::to_fe(r.Y, p.Y);
  fw::to_fe(r.Z, p.Z);
  fw::to_fe(r.T, p.T);
}
}  // namespace rp
