// Halved-scalar per-signature verification (crypto::Signature::verify ==
// ed25519-dalek 1.0.1 verify_strict, crypto/src/lib.rs:200-204) for gfx950.
//
// dalek checks P := [s]B - [k]A - R == O.  We check instead
//     Q := [e]B - [c]A - [d]R == O,   e = d*s mod l,
// where (c, d) is a short vector of the lattice {(c, d) : c == d*k (mod 8l)}
// with d odd (k_halve: a half-gcd on (8l, k) by the extended Euclidean
// algorithm with f64 quotient estimates).  Because A and R lie in
// a group of order 8l, [c]A == [d*k]A and [d*s mod l]B == [d*s]B exactly, so
// Q == [d]P for EVERY input, torsion components included; d odd and
// 0 < |d| < l make [d]P == O equivalent to P == O.  The verdict is therefore
// dalek's bit for bit, while c and d have ~128 bits instead of 253: the joint
// Horner pass needs ~33 signed radix-16 digits (132 doublings) instead of 64,
// and [e]B uses a doubling-free comb (32 byte positions x 128 multiples).
// When no short odd vector exists (adversarially ground k), k_halve falls
// back to (c, d) = (k, 1) -- the full-length check -- so correctness never
// depends on the reduction succeeding.
//
// Kernels:
//   k_build_comb     comb table: entry (j, v) = (v+1)*256^j*B, affine Niels
//   k_halve          (k, s) -> (c, |d|, e, H, sign d)
//   k_verify_halved  decompression + small-order checks + Q == O
#include "coa_halved.h"

#include <atomic>
#include <cstdlib>
#include "coa_kernels.h"

#include "coa_fe.h"
#include "coa_ge.h"
#include "coa_halve.h"
#include "coa_sc.h"
#include "coa_sha512.h"
#include "coa_smul.h"

namespace {
using namespace coa_halve;

// per-lane tables j*P, j = 1..8, for two bases; lane-major, 2 KiB per lane
COA_DEV void tab2_store(uint32_t* scr, uint32_t lane, int tab, int entry, const ge_cached& q) {
  const fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int h = 0; h < 2; h++)
      reinterpret_cast<uint4*>(scr)[((uint64_t)lane * 16 + tab * 8 + entry) * 8 + c * 2 + h] =
          make_uint4(f[c]->v[4 * h], f[c]->v[4 * h + 1], f[c]->v[4 * h + 2], f[c]->v[4 * h + 3]);
}

COA_DEV void tab2_select(ge_cached& q, const uint32_t* scr, uint32_t lane, int tab, int d) {
  const int m = d < 0 ? -d : d;
  const int entry = m == 0 ? 0 : m - 1;
  fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint4 v = reinterpret_cast<const uint4*>(scr)[((uint64_t)lane * 16 + tab * 8 + entry) * 8 + c * 2 + h];
      f[c]->v[4 * h] = v.x;
      f[c]->v[4 * h + 1] = v.y;
      f[c]->v[4 * h + 2] = v.z;
      f[c]->v[4 * h + 3] = v.w;
    }
  if (m == 0) ge_cached_identity(q);
  ge_cached_cneg(q, d < 0);
}

// tab2_select in two halves: the raw entry load (issued early, so a lone
// wave's doublings cover its latency) and the sign/zero fix-up at the use.
COA_DEV void tab2_load(ge_cached& q, const uint32_t* scr, uint32_t lane, int tab, int d) {
  const int m = d < 0 ? -d : d;
  const int entry = m == 0 ? 0 : m - 1;
  fe* f[4] = {&q.YplusX, &q.YminusX, &q.Z, &q.T2d};
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint4 v = reinterpret_cast<const uint4*>(scr)[((uint64_t)lane * 16 + tab * 8 + entry) * 8 + c * 2 + h];
      f[c]->v[4 * h] = v.x;
      f[c]->v[4 * h + 1] = v.y;
      f[c]->v[4 * h + 2] = v.z;
      f[c]->v[4 * h + 3] = v.w;
    }
}
COA_DEV void tab2_fix(ge_cached& q, int d) {
  if (d == 0) ge_cached_identity(q);
  ge_cached_cneg(q, d < 0);
}

COA_DEV void tab2_build(uint32_t* scr, uint32_t lane, int tab, const ge_p3& P) {
  ge_cached c1;
  ge_p3_to_cached(c1, P);
  tab2_store(scr, lane, tab, 0, c1);
  ge_p3 cur = P;
#pragma unroll 1
  for (int j = 1; j < 8; j++) {
    ge_p1p1 t;
    ge_add(t, cur, c1);
    ge_p1p1_to_p3(cur, t);
    ge_cached cj;
    ge_p3_to_cached(cj, cur);
    tab2_store(scr, lane, tab, j, cj);
  }
}

COA_DEV int wave_max(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  return v;
}

}  // namespace

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_build_comb(uint32_t* __restrict__ comb, const uint32_t* __restrict__ btab_g) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[BTAB_DWORDS];
  lds_load_btable(btab, btab_g);
  const int id = blockIdx.x * blockDim.x + threadIdx.x;  // 0 .. 4095
  const int j = id >> 7, v = id & 127;
  uint32_t wide[16];
#pragma unroll
  for (int i = 0; i < 16; i++) wide[i] = 0;
  // (v + 1) << (8 j) as a 512-bit value, reduced mod l
  const int bitpos = 8 * j;
  const uint64_t m = (uint64_t)(v + 1) << (bitpos & 31);
  for (int i = 0; i < 16; i++) {
    if (i == (bitpos >> 5)) wide[i] = (uint32_t)m;
    if (i == (bitpos >> 5) + 1) wide[i] = (uint32_t)(m >> 32);
  }
  sc x;
  sc_reduce512(x, wide);
  ge_p2 P;
  fixed_base_mul(P, x.v, btab);
  fe zi, xx, yy, xy, d2, n0, n1, n2;
  fe_invert(zi, P.Z);
  fe_mul(xx, P.X, zi);
  fe_mul(yy, P.Y, zi);
  fe_mul(xy, xx, yy);
  fe_const_d2(d2);
  fe_add(n0, yy, xx);
  fe_sub(n1, yy, xx);
  fe_mul(n2, xy, d2);
  fe_canon(n0, n0);
  fe_canon(n1, n1);
  fe_canon(n2, n2);
  uint32_t* e = comb + (uint64_t)id * 24;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    e[i] = n0.v[i];
    e[8 + i] = n1.v[i];
    e[16 + i] = n2.v[i];
  }
}

// Wide comb entry id = j * 2^(W-1) + (m - 1): m * 2^(W j) * B by the
// doubling-free radix-256 comb (32 mixed additions), made affine.
__global__ void __launch_bounds__(256) k_build_wcomb(uint32_t* __restrict__ wcomb, const uint32_t* __restrict__ comb) {
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= COA_WCOMB_ENTRIES) return;
  const int j = (int)(id / COA_WCOMB_MAG);
  const uint32_t m = (uint32_t)(id % COA_WCOMB_MAG) + 1;
  uint32_t wide[16];
#pragma unroll
  for (int i = 0; i < 16; i++) wide[i] = 0;
  const int bitpos = COA_WCOMB_W * j;
  const uint64_t mm = (uint64_t)m << (bitpos & 31);
  for (int i = 0; i < 16; i++) {
    if (i == (bitpos >> 5)) wide[i] = (uint32_t)mm;
    if (i == (bitpos >> 5) + 1) wide[i] = (uint32_t)(mm >> 32);
  }
  sc x;
  sc_reduce512(x, wide);
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = x.v[i];
  add_const_word(e, 0x80808080u);
  ge_p3 acc3;
  ge_p1p1 t;
  ge_p3_identity(acc3);
#pragma unroll 1
  for (int k = 0; k < 32; k++) {
    const int ek = (int)take_low_byte(e) - 128;
    ge_niels qb;
    comb_select(qb, comb, k, ek);
    ge_madd(t, acc3, qb);
    ge_p1p1_to_p3(acc3, t);
  }
  fe zi, xx, yy, xy, d2, n0, n1, n2;
  fe_invert(zi, acc3.Z);
  fe_mul(xx, acc3.X, zi);
  fe_mul(yy, acc3.Y, zi);
  fe_mul(xy, xx, yy);
  fe_const_d2(d2);
  fe_add(n0, yy, xx);
  fe_sub(n1, yy, xx);
  fe_mul(n2, xy, d2);
  fe_canon(n0, n0);
  fe_canon(n1, n1);
  fe_canon(n2, n2);
  uint4* o = reinterpret_cast<uint4*>(wcomb + id * COA_WC_STRIDE);
  o[0] = make_uint4(n0.v[0], n0.v[1], n0.v[2], n0.v[3]);
  o[1] = make_uint4(n0.v[4], n0.v[5], n0.v[6], n0.v[7]);
  o[2] = make_uint4(n1.v[0], n1.v[1], n1.v[2], n1.v[3]);
  o[3] = make_uint4(n1.v[4], n1.v[5], n1.v[6], n1.v[7]);
  o[4] = make_uint4(n2.v[0], n2.v[1], n2.v[2], n2.v[3]);
  o[5] = make_uint4(n2.v[4], n2.v[5], n2.v[6], n2.v[7]);
}

namespace {
COA_DEV void niels_to_p3(ge_p3& r, const ge_niels& q) {  // affine Niels -> extended (Z = 1)
  fe two_y, two_x, half;
  fe_add(two_y, q.yplusx, q.yminusx);
  fe_sub(two_x, q.yplusx, q.yminusx);
  // 1/2 mod p = (p + 1) / 2
  fe_set(half, 0);
  half.v[0] = 0xfffffff7u;
  for (int i = 1; i < 7; i++) half.v[i] = 0xffffffffu;
  half.v[7] = 0x3fffffffu;
  fe_mul(r.X, two_x, half);
  fe_mul(r.Y, two_y, half);
  fe_set(r.Z, 1);
  fe_mul(r.T, r.X, r.Y);
}
COA_DEV bool niels_eq_p3(const ge_niels& q, const ge_p3& p) {  // same point (p projective)?
  ge_p3 a;
  niels_to_p3(a, q);
  ge_p2 a2;
  ge_p3_to_p2(a2, a);
  return ge_p2_eq_p3(a2, p);
}
}  // namespace

// Whole-table consistency of the wide comb, independent of how it was built:
// entry(j, m) == entry(j, m-1) + entry(j, 1) for m >= 2, entry(j, 1) ==
// [2^W] entry(j-1, 1) for j >= 1, entry(0, 1) == B, and every entry's
// xy2d == 2d x y.  By induction every entry is m * 2^(W j) * B.  Each
// thread checks one entry and counts failures into *bad.
__global__ void __launch_bounds__(256) k_check_wcomb(const uint32_t* __restrict__ wcomb, uint32_t* __restrict__ bad) {
  const uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= COA_WCOMB_ENTRIES) return;
  const int j = (int)(id / COA_WCOMB_MAG);
  const uint32_t m = (uint32_t)(id % COA_WCOMB_MAG) + 1;
  uint32_t w[24];
  ge_niels q;
  wcomb_load(w, wcomb, j, (int)m);
  wcomb_apply(q, w, 1);
  bool ok = true;
  {  // internal consistency: xy2d == 2d x y, coordinates canonical
    ge_p3 a;
    niels_to_p3(a, q);
    fe d2, want, c;
    fe_const_d2(d2);
    fe_mul(want, a.T, d2);
    fe_canon(want, want);
    ok = ok && fe_eq(want, q.xy2d);
    // stored encodings are canonical (< p), word for word
    const fe* co[3] = {&q.yplusx, &q.yminusx, &q.xy2d};
    for (int k = 0; k < 3; k++) {
      fe_canon(c, *co[k]);
      for (int i = 0; i < 8; i++) ok = ok && c.v[i] == co[k]->v[i];
    }
  }
  ge_p3 expect;
  ge_p1p1 t;
  if (m >= 2) {
    ge_niels prev, one;
    wcomb_load(w, wcomb, j, (int)m - 1);
    wcomb_apply(prev, w, 1);
    wcomb_load(w, wcomb, j, 1);
    wcomb_apply(one, w, 1);
    ge_p3 pp;
    niels_to_p3(pp, prev);
    ge_madd(t, pp, one);
    ge_p1p1_to_p3(expect, t);
  } else if (j >= 1) {
    ge_niels base;
    wcomb_load(w, wcomb, j - 1, 1);
    wcomb_apply(base, w, 1);
    ge_p3 pp;
    niels_to_p3(pp, base);
    ge_p2 a2;
    ge_p3_to_p2(a2, pp);
    for (int k = 0; k < COA_WCOMB_W; k++) {
      ge_p2_dbl(t, a2);
      ge_p1p1_to_p2(a2, t);
    }
    ge_p1p1_to_p3(expect, t);
  } else {
    ge_basepoint(expect);
  }
  ok = ok && niels_eq_p3(q, expect);
  if (!ok) atomicAdd(bad, 1u);
}

// (k, s) -> record {c'[8], d'[8], e[8], meta, pad[7]}: c' = c + 0x88..8,
// d' = |d| + 0x88..8 (signed radix-16 recodings), meta = H | (d < 0) << 31.
namespace {
// One signature's halving record from k and s in registers; e = d*s (mod l,
// negated with d) is also returned for the [e]B term.
COA_DEV void halve_rec(uint32_t* k, const uint32_t* s, uint32_t i, uint32_t* __restrict__ rec, uint32_t* e_out) {
  uint32_t c[8], d[8];
  int cost;
  bool neg;
  halve(c, d, cost, neg, k);
  sc e;
  sc_mul(e, d, s);  // s may be non-canonical here; the verify kernel rejects those lanes
  if (neg) {
    sc en;
    sc_neg(en, e.v);
    e = en;
  }
  const int H = (cost + 2 + 3) / 4;  // c, d < 2^(4H - 2)
  // signed radix-16 recoding offset over all 64 nibbles: nibble p of
  // c + 0x88..8 minus 8 is digit p, and every digit at p >= H is 0
  add_const_word(c, 0x88888888u);
  add_const_word(d, 0x88888888u);
  uint4* o = reinterpret_cast<uint4*>(rec + (uint64_t)i * 32);
  o[0] = make_uint4(c[0], c[1], c[2], c[3]);
  o[1] = make_uint4(c[4], c[5], c[6], c[7]);
  o[2] = make_uint4(d[0], d[1], d[2], d[3]);
  o[3] = make_uint4(d[4], d[5], d[6], d[7]);
  o[4] = make_uint4(e.v[0], e.v[1], e.v[2], e.v[3]);
  o[5] = make_uint4(e.v[4], e.v[5], e.v[6], e.v[7]);
  o[6] = make_uint4((uint32_t)H | (neg ? 0x80000000u : 0u), 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 8; j++) e_out[j] = e.v[j];
}

// k_halve's per-signature body: k from kbuf.
COA_DEV void halve_one(const uint32_t* __restrict__ kbuf, const uint8_t* __restrict__ sigs, uint32_t i,
                       uint32_t* __restrict__ rec) {
  uint32_t k[8], s[8], e[8];
  const uint4* kq = reinterpret_cast<const uint4*>(kbuf + (uint64_t)i * 8);
  const uint4* sq = reinterpret_cast<const uint4*>(sigs + (uint64_t)i * 64 + 32);
  uint4 v0 = kq[0], v1 = kq[1];
  k[0] = v0.x; k[1] = v0.y; k[2] = v0.z; k[3] = v0.w;
  k[4] = v1.x; k[5] = v1.y; k[6] = v1.z; k[7] = v1.w;
  v0 = sq[0];
  v1 = sq[1];
  s[0] = v0.x; s[1] = v0.y; s[2] = v0.z; s[3] = v0.w;
  s[4] = v1.x; s[5] = v1.y; s[6] = v1.z; s[7] = v1.w;
  halve_rec(k, s, i, rec, e);
}

COA_DEV void load8_u4(uint32_t* dst, const void* src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  const uint4 a = q[0], b = q[1];
  dst[0] = a.x; dst[1] = a.y; dst[2] = a.z; dst[3] = a.w;
  dst[4] = b.x; dst[5] = b.y; dst[6] = b.z; dst[7] = b.w;
}

// The checks that do not need k (the "pre" roles of k_pre_halve), for one of
// the item's two points: which = 0 takes A (and s < l), which = 1 takes R.
// The point decompresses (dalek rules) and is not small order; then its
// table j*(-P), j = 1..8, goes to table `which` of slab i.  Returns ok.
COA_DEV bool pre_one(const uint8_t* __restrict__ pks, const uint8_t* __restrict__ sigs, uint32_t i, uint32_t which,
                     uint32_t* __restrict__ scr) {
  uint32_t w[8], sw[8];
  load8_u4(w, which ? sigs + (uint64_t)i * 64 : pks + (uint64_t)i * 32);
  load8_u4(sw, sigs + (uint64_t)i * 64 + 32);
  const bool s_ok = which || sc_is_canonical(sw);
  ge_p3 Q;
  const bool dec = ge_decompress(Q, w);
  const bool small = ge_is_small_order(Q);
  const bool ok = s_ok && dec && !small;
  fe_neg(Q.X, Q.X);
  fe_neg(Q.T, Q.T);
  // a table may be built for an item whose other point then fails: that
  // role's flag byte keeps k_verify_main from reading it
  if (ok) tab2_build(scr, i, (int)which, Q);
  return ok;
}
}  // namespace

__global__ void __launch_bounds__(256) k_halve(const uint32_t* __restrict__ kbuf, const uint8_t* __restrict__ sigs,
                                               uint32_t n, uint32_t* __restrict__ rec) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) halve_one(kbuf, sigs, i, rec);
}

// Split verification, phase 1 (one launch, three roles): blocks below
// pre_blocks run pre_one on A for item blockIdx*256 + t, the next pre_blocks
// on R; the others, for item (blockIdx - 2 pre_blocks)*256 + t, take k (from
// kbuf, or hashed here as SHA-512(R || A || M) mod l when msgs is set), the
// halving record, and optionally [e]B from the comb, stored in cached form in
// ebp (32 dwords per item).  No role needs another's output, and at <= 168
// VGPRs three waves share each SIMD: the two decompression waves issue into
// each other's gaps (a lone wave issues a VALU instruction at most every ~4
// cycles), and the latency-bound halving (f64 quotient chains) and the hash
// fill what is left.  flags[2i + which] is the A / R role's pre-check.
template <int WAVES>
__global__ void __launch_bounds__(256, WAVES) k_pre_halve(const uint8_t* __restrict__ pks,
                                                      const uint8_t* __restrict__ sigs,
                                                      const uint8_t* __restrict__ msgs, uint32_t msg_len,
                                                      int msgs_aligned, const uint32_t* __restrict__ kbuf,
                                                      uint32_t n, uint32_t* __restrict__ rec,
                                                      uint8_t* __restrict__ flags, uint32_t* __restrict__ scr,
                                                      uint32_t* __restrict__ ebp, const uint32_t* __restrict__ comb,
                                                      const uint32_t* __restrict__ wcomb, uint32_t pre_blocks,
                                                      int prio) {
  if (blockIdx.x < 2 * pre_blocks) {
    if (prio & 2) return;  // diagnostic (COA_PRE_DIAG): time the hash role alone
    const uint32_t which = blockIdx.x >= pre_blocks ? 1u : 0u;
    const uint32_t i = (blockIdx.x - which * pre_blocks) * blockDim.x + threadIdx.x;
    if (i < n) flags[2 * i + which] = pre_one(pks, sigs, i, which, scr) ? 1 : 0;
    return;
  }
  const uint32_t i = (blockIdx.x - 2 * pre_blocks) * blockDim.x + threadIdx.x;
  if (i >= n || (prio & 4)) return;  // diagnostic: time the decompression roles alone
  // The hash and the halving are dependency chains (f64 quotient estimates)
  // that need few issue slots but need them promptly; the decompression waves
  // beside them issue every cycle they can.  VALU issue goes to the higher
  // priority first (then the older wave), so at equal priority this role
  // would only run in the decompressions' leftover slots.
  if (prio & 1) __builtin_amdgcn_s_setprio(3);
  uint32_t k[8], sw[8], e[8];
  if (msgs) {
    coa_sha::Segs sg;
    sg.p[0] = sigs + (uint64_t)i * 64;
    sg.len[0] = 32;
    sg.p[1] = pks + (uint64_t)i * 32;
    sg.len[1] = 32;
    sg.p[2] = msgs + (uint64_t)i * msg_len;
    sg.len[2] = msg_len;
    uint64_t st[8];
    coa_sha::hash_segs(st, sg, msgs_aligned != 0);
    uint32_t h[16];
    coa_sha::state_to_le_words(h, st);
    sc kk;
    sc_reduce512(kk, h);
#pragma unroll
    for (int j = 0; j < 8; j++) k[j] = kk.v[j];
  } else {
    load8_u4(k, kbuf + (uint64_t)i * 8);
  }
  load8_u4(sw, sigs + (uint64_t)i * 64 + 32);
  halve_rec(k, sw, i, rec, e);
  if (!ebp) return;  // [e]B left to k_verify_main
  // the 13 comb additions are issue-bound, not a latency chain: back to the
  // default priority, so the decompression waves keep first call on issue
  // (COA_PRE_PRIO=3 keeps the raised priority through them, A/B)
  if ((prio & 9) == 1) __builtin_amdgcn_s_setprio(0);
  ge_p3 P;
  ge_p3_identity(P);
  if (wcomb) {
    wcomb_accumulate(P, e, wcomb);
  } else {
    ge_p1p1 t;
    add_const_word(e, 0x80808080u);
#pragma unroll 1
    for (int j = 0; j < 32; j++) {
      const int ej = (int)take_low_byte(e) - 128;
      ge_niels qb;
      comb_select(qb, comb, j, ej);
      ge_madd(t, P, qb);
      ge_p1p1_to_p3(P, t);
    }
  }
  ge_cached c;
  ge_p3_to_cached(c, P);
  const fe* f[4] = {&c.YplusX, &c.YminusX, &c.Z, &c.T2d};
  uint4* o = reinterpret_cast<uint4*>(ebp + (uint64_t)i * 32);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    o[2 * q] = make_uint4(f[q]->v[0], f[q]->v[1], f[q]->v[2], f[q]->v[3]);
    o[2 * q + 1] = make_uint4(f[q]->v[4], f[q]->v[5], f[q]->v[6], f[q]->v[7]);
  }
}

// Split verification, phase 2: one lane per item (n <= grid), Q = [c](-A) +
// [|d|](-sign(d) R) from the slab tables (for d < 0 the R digits are negated
// instead of the table), plus the [e]B point of phase 1.
// IL: for calls of at most one wave per SIMD, where a lone wave waits on its
// own dependency chains and memory: the point formulas with their independent
// products interleaved (coa_ge.h *_il), and both table entries of a digit
// loaded before its four doublings (launch bound of one wave per SIMD, up to
// 512 VGPRs); larger calls keep the plain formulas (156 VGPRs, three waves
// per SIMD).
#ifdef COA_MAIN_TRACE  // per-wave phase stamps of k_verify_main<1, true> (tools/main_trace.py)
__device__ unsigned long long g_main_trace[4096][4];
#define MAIN_MARK(k)                                                                       \
  if (IL && (threadIdx.x & 63) == 0 && (blockIdx.x * blockDim.x + threadIdx.x) / 64 < 4096) \
    g_main_trace[(blockIdx.x * blockDim.x + threadIdx.x) / 64][k] = clock64();
extern "C" int coa_main_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_main_trace), sizeof(g_main_trace)) == hipSuccess ? 0 : -1;
}
#else
#define MAIN_MARK(k)
#endif
template <int WAVES, bool IL>
__global__ void __launch_bounds__(256, WAVES) k_verify_main(const uint32_t* __restrict__ rec,
                                                        const uint8_t* __restrict__ flags, uint32_t n,
                                                        uint8_t* __restrict__ verdicts,
                                                        const uint32_t* __restrict__ scr,
                                                        const uint32_t* __restrict__ ebp,
                                                        const uint32_t* __restrict__ comb,
                                                        const uint32_t* __restrict__ wcomb) {
  MAIN_MARK(0)
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  const uint32_t ii = live ? i : 0u;  // every load below is in bounds, so none waits on a branch
  const uint32_t* myrec = rec + (uint64_t)ii * 32;
  // IL (a lone wave per SIMD): the flags, the record's meta and digit words
  // and the [e]B point of phase 1 are loaded together, one memory round trip
  // before the digit loop instead of one per dependent load (and the [e]B
  // point's after it)
  const uint16_t fl = reinterpret_cast<const uint16_t*>(flags)[ii];
  const uint32_t meta0 = myrec[24];
  uint32_t cw[8], dw[8];  // IL: the digit words in registers, not reloaded per digit
  uint32_t ebw[32];       // IL: the [e]B cached point of phase 1
  if constexpr (IL) {
    load8_u4(cw, myrec);
    load8_u4(dw, myrec + 8);
    if (ebp) {
#pragma unroll
      for (int q = 0; q < 4; q++) load8_u4(ebw + 8 * q, ebp + (uint64_t)ii * 32 + 8 * q);
    }
  }
  const bool ok = live && fl == 0x0101u;
  const uint32_t meta = live ? meta0 : 0u;
  const int H = wave_max(ok ? (int)(meta & 0xffu) : 0);
  MAIN_MARK(1)
  const bool dneg = (meta >> 31) != 0;
  uint8_t verdict = 1;
  if (ok) {
    ge_p3 acc3;
    ge_p2 acc2;
    ge_p1p1 t;
    ge_p3_identity(acc3);
#pragma unroll 1
    for (int pos = H - 1; pos >= 0; pos--) {
      const int sh = 4 * (pos & 7);
      const uint32_t wc = IL ? cw[pos >> 3] : myrec[pos >> 3];
      const uint32_t wd = IL ? dw[pos >> 3] : myrec[8 + (pos >> 3)];
      const int dc = (int)((wc >> sh) & 15u) - 8;
      const int dd = (int)((wd >> sh) & 15u) - 8;
      const int dr = dneg ? -dd : dd;
      ge_cached qa, qr;
      if constexpr (IL) {  // both entries in flight during the four doublings
        tab2_load(qa, scr, i, 0, dc);
        tab2_load(qr, scr, i, 1, dr);
      }
      if (pos != H - 1) {
#pragma unroll 1
        for (int k = 0; k < 3; k++) {
          if constexpr (IL) {
            ge_p2_dbl_il(t, acc2);
            ge_p1p1_to_p2_il(acc2, t);
          } else {
            ge_p2_dbl(t, acc2);
            ge_p1p1_to_p2(acc2, t);
          }
        }
        if constexpr (IL) {
          ge_p2_dbl_il(t, acc2);
          ge_p1p1_to_p3_il(acc3, t);
        } else {
          ge_p2_dbl(t, acc2);
          ge_p1p1_to_p3(acc3, t);
        }
      }
      if constexpr (IL) {
        tab2_fix(qa, dc);
        ge_add_il(t, acc3, qa);
        ge_p1p1_to_p3_il(acc3, t);
        tab2_fix(qr, dr);
        ge_add_il(t, acc3, qr);
        if (pos != 0) ge_p1p1_to_p2_il(acc2, t);
      } else {
        tab2_select(qa, scr, i, 0, dc);
        ge_add(t, acc3, qa);
        ge_p1p1_to_p3(acc3, t);
        tab2_select(qr, scr, i, 1, dr);
        ge_add(t, acc3, qr);
        if (pos != 0) ge_p1p1_to_p2(acc2, t);
      }
    }
    MAIN_MARK(2)
    if constexpr (IL)
      ge_p1p1_to_p3_il(acc3, t);
    else
      ge_p1p1_to_p3(acc3, t);
    if (!ebp) {  // [e]B here, from the combs
      uint32_t e[8];
#pragma unroll
      for (int j = 0; j < 8; j++) e[j] = myrec[16 + j];
      if (wcomb) {
        wcomb_accumulate<IL>(acc3, e, wcomb);
      } else {
        add_const_word(e, 0x80808080u);
#pragma unroll 1
        for (int j = 0; j < 32; j++) {
          const int ej = (int)take_low_byte(e) - 128;
          ge_niels qb;
          comb_select(qb, comb, j, ej);
          ge_madd(t, acc3, qb);
          ge_p1p1_to_p3(acc3, t);
        }
      }
    } else {
    // + [e]B, computed by the halving role
    ge_cached eb;
    fe* f[4] = {&eb.YplusX, &eb.YminusX, &eb.Z, &eb.T2d};
    if constexpr (IL) {
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int k = 0; k < 8; k++) f[q]->v[k] = ebw[8 * q + k];
    } else {
    const uint4* src = reinterpret_cast<const uint4*>(ebp + (uint64_t)i * 32);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint4 v0 = src[2 * q], v1 = src[2 * q + 1];
      f[q]->v[0] = v0.x; f[q]->v[1] = v0.y; f[q]->v[2] = v0.z; f[q]->v[3] = v0.w;
      f[q]->v[4] = v1.x; f[q]->v[5] = v1.y; f[q]->v[6] = v1.z; f[q]->v[7] = v1.w;
    }
    }
    ge_add(t, acc3, eb);
    ge_p1p1_to_p3(acc3, t);
    }
    ge_p2 q2;
    ge_p3_to_p2(q2, acc3);
    verdict = ge_p2_is_identity(q2) ? 0 : 1;
  }
  if (live) verdicts[i] = verdict;
  MAIN_MARK(3)
}

// Split verification, phase 2 with an item's two chains in two waves: a
// workgroup of 128 lanes takes 64 items; wave 0 runs [c](-A) over the c
// digits, wave 1 [|d|](-sign(d) R) over the d digits, each with its own
// doublings (twice k_verify_main's doublings per item) so that a call of one
// wave per SIMD of items runs two waves per SIMD (or, below that size, its
// waves on twice the SIMDs).  Wave 0 hands its point to wave 1 through LDS;
// wave 1 adds it and the [e]B point of phase 1 and checks for the identity.
__global__ void __launch_bounds__(128, 2) k_verify_main2(const uint32_t* __restrict__ rec,
                                                         const uint8_t* __restrict__ flags, uint32_t n,
                                                         uint8_t* __restrict__ verdicts,
                                                         const uint32_t* __restrict__ scr,
                                                         const uint32_t* __restrict__ ebp) {
  __shared__ uint32_t qa_lds[32][64];  // wave 0's point, cached form, [dword][lane]
  const uint32_t lane = threadIdx.x & 63u;
  const int role = (int)(threadIdx.x >> 6);  // wave-uniform
  const uint32_t i = blockIdx.x * 64u + lane;
  const bool live = i < n;
  const uint32_t ii = live ? i : 0u;
  const uint32_t* myrec = rec + (uint64_t)ii * 32;
  const uint16_t fl = reinterpret_cast<const uint16_t*>(flags)[ii];
  const uint32_t meta0 = myrec[24];
  uint32_t w[8], ebw[32];
  load8_u4(w, myrec + 8 * role);
  if (role == 1) {
#pragma unroll
    for (int q = 0; q < 4; q++) load8_u4(ebw + 8 * q, ebp + (uint64_t)ii * 32 + 8 * q);
  }
  const bool ok = live && fl == 0x0101u;
  const uint32_t meta = live ? meta0 : 0u;
  const int H = wave_max(ok ? (int)(meta & 0xffu) : 0);
  const bool neg = role == 1 && (meta >> 31) != 0;
  ge_p3 acc3;
  ge_p1p1 t;
  ge_p3_identity(acc3);
  if (ok) {
    ge_p2 acc2;
#pragma unroll 1
    for (int pos = H - 1; pos >= 0; pos--) {
      const int dd = (int)((w[pos >> 3] >> (4 * (pos & 7))) & 15u) - 8;
      const int dr = neg ? -dd : dd;
      ge_cached q;
      tab2_load(q, scr, i, role, dr);
      if (pos != H - 1) {
#pragma unroll 1
        for (int k = 0; k < 3; k++) {
          ge_p2_dbl_il(t, acc2);
          ge_p1p1_to_p2_il(acc2, t);
        }
        ge_p2_dbl_il(t, acc2);
        ge_p1p1_to_p3_il(acc3, t);
      }
      tab2_fix(q, dr);
      ge_add_il(t, acc3, q);
      if (pos != 0) ge_p1p1_to_p2_il(acc2, t);
    }
    ge_p1p1_to_p3_il(acc3, t);
    if (role == 0) {
      ge_cached c;
      ge_p3_to_cached(c, acc3);
      const fe* f[4] = {&c.YplusX, &c.YminusX, &c.Z, &c.T2d};
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int k = 0; k < 8; k++) qa_lds[8 * q + k][lane] = f[q]->v[k];
    }
  }
  __syncthreads();
  if (role == 0) return;
  uint8_t verdict = 1;
  if (ok) {
    ge_cached qa, eb;
    fe* fa[4] = {&qa.YplusX, &qa.YminusX, &qa.Z, &qa.T2d};
    fe* fb[4] = {&eb.YplusX, &eb.YminusX, &eb.Z, &eb.T2d};
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
      for (int k = 0; k < 8; k++) {
        fa[q]->v[k] = qa_lds[8 * q + k][lane];
        fb[q]->v[k] = ebw[8 * q + k];
      }
    ge_add_il(t, acc3, qa);
    ge_p1p1_to_p3_il(acc3, t);
    ge_add_il(t, acc3, eb);
    ge_p1p1_to_p3_il(acc3, t);
    ge_p2 q2;
    ge_p3_to_p2(q2, acc3);
    verdict = ge_p2_is_identity(q2) ? 0 : 1;
  }
  if (live) verdicts[i] = verdict;
}

template <int WAVES>
__global__ void __launch_bounds__(256, WAVES) k_verify_halved(const uint8_t* __restrict__ pks,
                                                          const uint8_t* __restrict__ sigs,
                                                          const uint32_t* __restrict__ rec, uint32_t n,
                                                          uint8_t* __restrict__ verdicts, uint32_t* __restrict__ scr,
                                                          const uint32_t* __restrict__ comb,
                                                          const uint32_t* __restrict__ wcomb) {
  const uint32_t lanes = gridDim.x * blockDim.x;
  const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
  // grid-stride with a wave-uniform trip count (wave_max below needs all lanes)
  const uint32_t wave0 = lane & ~63u;
  for (uint32_t base = wave0; base < n; base += lanes) {
    const uint32_t i = base + (lane & 63);
    const bool live = i < n;
    uint32_t aw[8], rw[8], sw[8];
    uint32_t meta = 0;
    const uint32_t* myrec = rec + (uint64_t)(live ? i : 0) * 32;
    if (live) {
      const uint4* p = reinterpret_cast<const uint4*>(pks + (uint64_t)i * 32);
      const uint4* g = reinterpret_cast<const uint4*>(sigs + (uint64_t)i * 64);
      const uint4* r = reinterpret_cast<const uint4*>(rec + (uint64_t)i * 32);
      uint4 v;
#define LD8(dst, src, o)                                                   \
  v = src[o];                                                              \
  dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;                  \
  v = src[o + 1];                                                          \
  dst[4] = v.x; dst[5] = v.y; dst[6] = v.z; dst[7] = v.w;
      LD8(aw, p, 0);
      LD8(rw, g, 0);
      LD8(sw, g, 2);
#undef LD8
      meta = r[6].x;
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++) aw[j] = rw[j] = sw[j] = 0;
    }
    // 1. s < l; 2./3. decompress A and R (dalek rules); 4. neither small order
    bool ok = live && sc_is_canonical(sw);
    ge_p3 A, R;
#pragma unroll 1
    for (int which = 0; which < 2; which++) {
      uint32_t w[8];
#pragma unroll
      for (int j = 0; j < 8; j++) w[j] = which ? rw[j] : aw[j];
      ge_p3 P;
      const bool dec = ge_decompress(P, w);
      const bool small = ge_is_small_order(P);
      ok = ok && dec && !small;
      if (which == 0) A = P;
      else R = P;
    }
    const int H = wave_max(ok ? (int)(meta & 0xffu) : 0);
    const bool dneg = (meta >> 31) != 0;
    uint8_t verdict = 1;
    if (ok) {
      // Q = [c](-A) + [|d|](-sign(d) R) + [e]B
      ge_p3 PA = A, PR = R;
      fe_neg(PA.X, A.X);
      fe_neg(PA.T, A.T);
      if (!dneg) {
        fe_neg(PR.X, R.X);
        fe_neg(PR.T, R.T);
      }
      tab2_build(scr, lane, 0, PA);
      tab2_build(scr, lane, 1, PR);
      ge_p3 acc3;
      ge_p2 acc2;
      ge_p1p1 t;
      ge_p3_identity(acc3);
#pragma unroll 1
      for (int pos = H - 1; pos >= 0; pos--) {
        const int sh = 4 * (pos & 7);
        const int dc = (int)((myrec[pos >> 3] >> sh) & 15u) - 8;
        const int dd = (int)((myrec[8 + (pos >> 3)] >> sh) & 15u) - 8;
        if (pos != H - 1) {
#pragma unroll 1
          for (int k = 0; k < 3; k++) {
            ge_p2_dbl(t, acc2);
            ge_p1p1_to_p2(acc2, t);
          }
          ge_p2_dbl(t, acc2);
          ge_p1p1_to_p3(acc3, t);
        }
        ge_cached q;
        tab2_select(q, scr, lane, 0, dc);
        ge_add(t, acc3, q);
        ge_p1p1_to_p3(acc3, t);
        tab2_select(q, scr, lane, 1, dd);
        ge_add(t, acc3, q);
        if (pos != 0) ge_p1p1_to_p2(acc2, t);
      }
      ge_p1p1_to_p3(acc3, t);
      uint32_t e[8];
#pragma unroll
      for (int j = 0; j < 8; j++) e[j] = myrec[16 + j];
      if (wcomb) {
        // [e]B from the wide HBM comb: 13 mixed additions
        wcomb_accumulate(acc3, e, wcomb);
      } else {
        // [e]B by the doubling-free radix-256 comb
        add_const_word(e, 0x80808080u);
#pragma unroll 1
        for (int j = 0; j < 32; j++) {
          const int ej = (int)take_low_byte(e) - 128;
          ge_niels qb;
          comb_select(qb, comb, j, ej);
          ge_madd(t, acc3, qb);
          ge_p1p1_to_p3(acc3, t);
        }
      }
      ge_p2 q2;
      ge_p3_to_p2(q2, acc3);
      verdict = ge_p2_is_identity(q2) ? 0 : 1;
    }
    if (live) verdicts[i] = verdict;
  }
}

// ---------------------------------------------------------------------------
hipError_t coa_launch_build_comb(uint32_t* comb, const uint32_t* btab, hipStream_t s) {
  hipLaunchKernelGGL(k_build_comb, dim3(COA_COMB_ENTRIES / 256), dim3(256), 0, s, comb, btab);
  return hipGetLastError();
}

hipError_t coa_launch_halve(const uint32_t* kbuf, const uint8_t* sigs, uint32_t n, uint32_t* rec, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_halve, dim3((uint32_t)blocks), dim3(256), 0, s, kbuf, sigs, n, rec);
  return hipGetLastError();
}

hipError_t coa_launch_build_wcomb(uint32_t* wcomb, const uint32_t* comb, hipStream_t s) {
  hipLaunchKernelGGL(k_build_wcomb, dim3((uint32_t)((COA_WCOMB_ENTRIES + 255) / 256)), dim3(256), 0, s, wcomb, comb);
  return hipGetLastError();
}
hipError_t coa_launch_check_wcomb(const uint32_t* wcomb, uint32_t* bad, hipStream_t s) {
  hipLaunchKernelGGL(k_check_wcomb, dim3((uint32_t)((COA_WCOMB_ENTRIES + 255) / 256)), dim3(256), 0, s, wcomb, bad);
  return hipGetLastError();
}

// Items that fill every SIMD of the current device with one wave (CUs x 4
// SIMDs x 64 lanes), read once per device.
static uint32_t one_wave_per_simd_items() {
  static std::atomic<uint32_t> cache[64];  // per device; the per-device worker threads share it
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 65536u;
  uint32_t v = cache[dev].load(std::memory_order_relaxed);
  if (!v) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    v = (uint32_t)cus * 256u;
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}

static uint32_t block_env(const char* name) {
  const char* e = getenv(name);
  const int b = e ? atoi(e) : COA_VERIFY_BLOCK;
  return (b == 64 || b == 128 || b == 256) ? (uint32_t)b : (uint32_t)COA_VERIFY_BLOCK;
}

hipError_t coa_launch_verify_split(const uint8_t* pks, const uint8_t* sigs, const uint8_t* msgs, uint32_t msg_len,
                                   const uint32_t* kbuf, uint32_t n, uint32_t* rec, uint8_t* flags,
                                   uint8_t* verdicts, uint32_t* scratch, uint32_t* ebp, const uint32_t* comb,
                                   const uint32_t* wcomb, hipStream_t s) {
  if (n == 0) return hipSuccess;
  // workgroup sizes (A/B: COA_PRE_BLOCK / COA_MAIN_BLOCK = 64, 128 or 256)
  static const uint32_t pre_b = block_env("COA_PRE_BLOCK"), main_b = block_env("COA_MAIN_BLOCK");
  const uint32_t blocks = (n + pre_b - 1) / pre_b;
  const int aligned = ((msg_len & 3) == 0) && (((uintptr_t)msgs & 3) == 0);
  // COA_PRE_PRIO=0: the hash/halving role at the default wave priority (A/B).
  // A library compiled with -DCOA_PRE_DIAG_BUILD also reads COA_PRE_DIAG=2 / 4:
  // skip the decompression / hash roles (role timing only, tools/pre_roles.sh;
  // verdicts are then meaningless, so release builds cannot reach it).
  // COA_PRE_PRIO=3: the raised priority also through the [e]B additions (bit
  // 8; A/B).  Bits 2 and 4 are the diagnostics below.
  static const int prio = (!getenv("COA_PRE_PRIO") ? 1
                           : atoi(getenv("COA_PRE_PRIO")) == 0 ? 0
                           : atoi(getenv("COA_PRE_PRIO")) == 3 ? (1 | 8) : 1)
#ifdef COA_PRE_DIAG_BUILD
                          | (getenv("COA_PRE_DIAG") ? atoi(getenv("COA_PRE_DIAG")) & 6 : 0)
#endif
      ;
  hipLaunchKernelGGL(k_pre_halve<3>, dim3(3 * blocks), dim3(pre_b), 0, s, pks, sigs, msgs, msg_len, aligned, kbuf, n,
                     rec, flags, scratch, ebp, comb, wcomb, blocks, prio);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // at most one wave per SIMD (65,536 items on the 256 CUs of an MI355X, the
  // C2 size): the interleaved formulas; COA_MAIN_IL=0/1 forces either (A/B)
  const char* il_env = getenv("COA_MAIN_IL");
  const bool il = il_env ? atoi(il_env) != 0 : n <= one_wave_per_simd_items();
  // an item's two chains in two waves (k_verify_main2) when the call has at
  // most a quarter wave per SIMD of items: its waves then run on SIMDs the
  // one-wave kernel leaves idle (4,096 / 16,384 items: 0.507 / 0.511 vs
  // 0.594 / 0.602 ms per call).  At 32,768 some SIMDs already get two of its
  // waves (0.82 vs 0.65 ms), and at C2's size the doubled doublings cost
  // more than the second wave per SIMD wins back (0.90 vs 0.72 ms).
  // COA_MAIN_TWO=0/1 forces either (A/B).  An explicit COA_MAIN_IL (without
  // COA_MAIN_TWO) selects the one-lane kernel it names at every size, so an
  // A/B of COA_MAIN_IL alone never measures k_verify_main2 instead.
  const char* two_s = getenv("COA_MAIN_TWO");
  const int two_env = two_s ? atoi(two_s) : (il_env ? 0 : -1);
  const bool two = ebp && (two_env >= 0 ? two_env != 0 : 4ull * n <= one_wave_per_simd_items());
  if (two)
    hipLaunchKernelGGL(k_verify_main2, dim3((n + 63) / 64), dim3(128), 0, s, rec, flags, n, verdicts, scratch, ebp);
  else if (il)
    hipLaunchKernelGGL((k_verify_main<1, true>), dim3((n + main_b - 1) / main_b), dim3(main_b), 0, s, rec, flags, n,
                       verdicts, scratch, ebp, comb, wcomb);
  else
    hipLaunchKernelGGL((k_verify_main<3, false>), dim3((n + main_b - 1) / main_b), dim3(main_b), 0, s, rec, flags, n,
                       verdicts, scratch, ebp, comb, wcomb);
  return hipGetLastError();
}

// waves: register bound of the instance (2 = 256 VGPRs, 3 = 168 with spills)
hipError_t coa_launch_verify_halved(const uint8_t* pks, const uint8_t* sigs, const uint32_t* rec, uint32_t n,
                                    uint8_t* verdicts, uint32_t* scratch, uint32_t scratch_lanes,
                                    const uint32_t* comb, const uint32_t* wcomb, int waves, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = ((uint64_t)n + COA_VERIFY_BLOCK - 1) / COA_VERIFY_BLOCK;
  const uint64_t maxb = scratch_lanes / COA_VERIFY_BLOCK;
  if (blocks > maxb) blocks = maxb;
  if (waves == 3)
    hipLaunchKernelGGL(k_verify_halved<3>, dim3((uint32_t)blocks), dim3(COA_VERIFY_BLOCK), 0, s, pks, sigs, rec, n,
                       verdicts, scratch, comb, wcomb);
  else
    hipLaunchKernelGGL(k_verify_halved<2>, dim3((uint32_t)blocks), dim3(COA_VERIFY_BLOCK), 0, s, pks, sigs, rec, n,
                       verdicts, scratch, comb, wcomb);
  return hipGetLastError();
}
