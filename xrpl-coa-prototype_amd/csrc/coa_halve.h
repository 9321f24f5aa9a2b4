// Scalar halving for ed25519 verification on gfx950 (Pornin 2020): from the
// challenge k, a short vector (c, d) of the lattice {(c, d) : c == d*k (mod
// 8l)} with d odd, by a half-gcd on (8l, k) with f64 quotient estimates.  The
// verification kernels then check [e]B - [c]A - [d]R == O (e = d*s mod l)
// with ~128-bit c and d instead of the 253-bit k (coa_halved.hip explains why
// the verdict is dalek's bit for bit).  Shared by the throughput kernels
// (coa_halved.hip) and the single-signature latency kernel (coa_latency.hip).
#pragma once
#include "coa_fe.h"
#include "coa_lehmer.h"

namespace coa_halve {

// ---------------------------------------------------------------- bigints
COA_DEV int bitlen(const uint32_t* x, int nl) {
  int bl = 0;
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (i < nl) bl = x[i] ? 32 * i + 32 - __builtin_clz(x[i]) : bl;
  return bl;
}

// out = x << s (0 <= s < 256), 8 limbs, bits above 256 dropped.
COA_DEV void shl8(uint32_t* out, const uint32_t* x, int s) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = x[i];
  const int q = s >> 5;
#pragma unroll
  for (int st = 1; st < 8; st <<= 1) {
    const bool on = (q & st) != 0;
#pragma unroll
    for (int i = 7; i >= 0; i--) t[i] = on ? (i >= st ? t[i - st] : 0u) : t[i];
  }
  const int r = s & 31;
#pragma unroll
  for (int i = 7; i >= 0; i--) {
    const uint32_t lo = i ? t[i - 1] : 0u;
    out[i] = r ? __builtin_amdgcn_alignbit(t[i], lo, 32 - r) : t[i];
  }
}

COA_DEV void shr1_8(uint32_t* x) {
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = __builtin_amdgcn_alignbit(i < 7 ? x[i + 1] : 0u, x[i], 1);
}

// 8-limb add / subtract with carry / borrow out, as one unpadded VCC chain
// (hipcc pads every VCC hand-off of __builtin_addc/subc with s_nop on gfx950;
// see coa_fe.h).  The last instruction turns VCC into the 0/1 result word.
#define COA_CHAIN8(OP0, OPC)                                                       \
  OP0 " %0, vcc, %9, %17\n\t" OPC " %1, vcc, %10, %18, vcc\n\t"                 \
  OPC " %2, vcc, %11, %19, vcc\n\t" OPC " %3, vcc, %12, %20, vcc\n\t"           \
  OPC " %4, vcc, %13, %21, vcc\n\t" OPC " %5, vcc, %14, %22, vcc\n\t"           \
  OPC " %6, vcc, %15, %23, vcc\n\t" OPC " %7, vcc, %16, %24, vcc\n\t"           \
  "v_addc_co_u32_e32 %8, vcc, 0, %25, vcc"
#define COA_CHAIN8_OPS(r, a, b, c, z)                                                                        \
  : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]), \
    "=&v"(c)                                                                                                 \
  : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(b[0]),      \
    "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(z)                      \
  : "vcc"

COA_DEV uint32_t sub8(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t o[8], bw;
  const uint32_t z = 0;
  asm(COA_CHAIN8("v_sub_co_u32_e32", "v_subb_co_u32_e32") COA_CHAIN8_OPS(o, a, b, bw, z));
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = o[i];
  return bw;
}
COA_DEV uint32_t add8(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t o[8], c;
  const uint32_t z = 0;
  asm(COA_CHAIN8("v_add_co_u32_e32", "v_addc_co_u32_e32") COA_CHAIN8_OPS(o, a, b, c, z));
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = o[i];
  return c;
}

COA_DEV double to_f64(const uint32_t* x) {
  double d = (double)x[7];
#pragma unroll
  for (int i = 6; i >= 0; i--) d = fma(d, 4294967296.0, (double)x[i]);
  return d;
}

// r = a - q*b (mod 2^256); returns 1 if a < q*b (the borrow out of the
// 288-bit subtraction, top word included).
COA_DEV uint32_t submul8(uint32_t* r, const uint32_t* a, const uint32_t* b, uint32_t q) {
  uint32_t pr[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc = (uint64_t)b[i] * q + (acc >> 32);
    pr[i] = (uint32_t)acc;
  }
  pr[8] = (uint32_t)(acc >> 32);
  uint32_t o[8], bw;
  const uint32_t z = 0;
  asm("v_sub_co_u32_e32 %0, vcc, %9, %17\n\t"
      "v_subb_co_u32_e32 %1, vcc, %10, %18, vcc\n\t"
      "v_subb_co_u32_e32 %2, vcc, %11, %19, vcc\n\t"
      "v_subb_co_u32_e32 %3, vcc, %12, %20, vcc\n\t"
      "v_subb_co_u32_e32 %4, vcc, %13, %21, vcc\n\t"
      "v_subb_co_u32_e32 %5, vcc, %14, %22, vcc\n\t"
      "v_subb_co_u32_e32 %6, vcc, %15, %23, vcc\n\t"
      "v_subb_co_u32_e32 %7, vcc, %16, %24, vcc\n\t"
      "v_subb_co_u32_e32 %8, vcc, %26, %25, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %26, vcc"
      : "=&v"(o[0]), "=&v"(o[1]), "=&v"(o[2]), "=&v"(o[3]), "=&v"(o[4]), "=&v"(o[5]), "=&v"(o[6]), "=&v"(o[7]),
        "=&v"(bw)
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(pr[0]),
        "v"(pr[1]), "v"(pr[2]), "v"(pr[3]), "v"(pr[4]), "v"(pr[5]), "v"(pr[6]), "v"(pr[7]), "v"(pr[8]), "v"(z)
      : "vcc");
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = o[i];
  return bw;
}

COA_DEV void madd5(uint32_t* r, const uint32_t* a, const uint32_t* b, uint32_t q) {  // r = a + q*b
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc = (uint64_t)b[i] * q + a[i] + (acc >> 32);
    r[i] = (uint32_t)acc;
  }
}

// Track the best lattice vector (c, t) with t odd: cost = max(bits(c), bits(t)).
COA_DEV void consider(uint32_t* c_out, uint32_t* d_out, int& best, bool& best_neg, const uint32_t* c,
                      const uint32_t* t, bool neg) {
  if (!(t[0] & 1)) return;
  const int cost = max(bitlen(c, 8), bitlen(t, 8));
  if (cost < best) {
    best = cost;
    best_neg = neg;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c_out[i] = c[i];
      d_out[i] = t[i];
    }
  }
}

// The three candidates of a remainder pair (a, b) with cofactors (ma, mb),
// mb of sign tb_neg: (b, mb), (a, ma) and (a - b, ma + mb).
COA_DEV void consider3(uint32_t* c_out, uint32_t* d_out, int& best, bool& best_neg, const uint32_t* a,
                       const uint32_t* b, const uint32_t* ma, const uint32_t* mb, bool tb_neg) {
  consider(c_out, d_out, best, best_neg, b, mb, tb_neg);
  consider(c_out, d_out, best, best_neg, a, ma, !tb_neg);
  if ((ma[0] ^ mb[0]) & 1) {
    uint32_t cd[8], dd[8];
    (void)sub8(cd, a, b);
    (void)add8(dd, ma, mb);
    consider(c_out, d_out, best, best_neg, cd, dd, !tb_neg);
  }
}

// Half-gcd on (8l, k) by the extended Euclidean algorithm: remainders
// r_i == t_i * k (mod 8l) with |r_{i-1} t_i| + |r_i t_{i-1}| = 8l, so once
// r_i < 2^128, |t_i| <= 2^127.  Quotients come from an f64 estimate of a/b
// (exact to 2^-52 relative) corrected by at most a few exact add-backs; a
// quotient >= 2^31 (probability ~2^-31 per step) takes a shift-subtract
// step instead.  Returns the lattice vector (c, |d|, sign d) with d odd that
// minimises max(bits(c), bits(d)) among the last remainders and their
// neighbours; (k, 1) if none is shorter.
// Down to 140-bit remainders the steps are taken in Lehmer blocks
// (coa_lehmer.h: the same remainders, ~6 full-width updates instead of ~70
// steps); the exact steps then walk the candidates' region one remainder at
// a time.  Remainders below 124 bits cannot beat a candidate already seen
// (their cofactors exceed 2^129), so the walk stops there.
COA_DEV void halve(uint32_t* c_out, uint32_t* d_out, int& cost_out, bool& neg_out, const uint32_t* k) {
  uint32_t a[8] = {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0, 0, 0, 0x80000000u};  // 8l
  uint32_t b[8], ma[8], mb[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    b[i] = k[i];
    ma[i] = 0;
    mb[i] = i == 0 ? 1u : 0u;
    c_out[i] = k[i];
    d_out[i] = i == 0 ? 1u : 0u;
  }
  bool tb_neg = false;  // sign of t_b; t_a has the opposite sign
  int best = max(bitlen(k, 8), 1);
  bool best_neg = false;
  int lb = bitlen(b, 8);
  double af = to_f64(a), bf = to_f64(b);  // f64 images, carried across steps
  for (int guard = 0; guard < 400; guard++) {
    if (lb <= 124) break;
    if (lb > 140) {  // a Lehmer block: several exact quotients at once
      const int nst = coa_lehmer::step(a, b, ma, mb, 140);
      if (nst) {
        if (nst & 1) tb_neg = !tb_neg;
        lb = bitlen(b, 8);
        af = to_f64(a);
        bf = to_f64(b);
        if (lb <= 136) consider3(c_out, d_out, best, best_neg, a, b, ma, mb, tb_neg);
        continue;
      }
    }
    // quotient estimate: a correctly rounded f64 division of the f64 images
    // (relative error ~2^-50), so for q < 2^31 floor() is off by at most one
    // and the fix-ups below correct it.  NOT v_rcp_f64: its approximation
    // error let a rare large quotient overshoot the fix-ups (one valid
    // signature in 4M rejected, tests/test_gpu_halve.py pins such k).
    const double qd = floor(af / bf);
    uint32_t r[8], mr[8];
    if (qd < 2147483648.0) {
      uint32_t q = (uint32_t)qd;
      if (submul8(r, a, b, q)) {  // overestimated: add b back (at most twice)
#pragma unroll 1
        for (int fix = 0; fix < 2; fix++) {
          uint32_t c = 0;
#pragma unroll
          for (int i = 0; i < 8; i++) r[i] = addc32(r[i], b[i], c, c);
          q -= 1;
          if (c) break;  // crossed back to >= 0
        }
      }
      uint32_t tmp[8];
#pragma unroll 1
      for (int fix = 0; fix < 2; fix++) {  // underestimated: r >= b
        if (sub8(tmp, r, b)) break;
#pragma unroll
        for (int i = 0; i < 8; i++) r[i] = tmp[i];
        q += 1;
      }
      madd5(mr, ma, mb, q);
    } else {  // huge quotient: one shift-subtract step, keep a as the larger
      const int s = bitlen(a, 8) - lb - 1;
      uint32_t t[8], u[8];
      shl8(t, b, s);
      (void)sub8(r, a, t);
      shl8(u, mb, s);
      (void)add8(mr, ma, u);
      uint32_t tmp[8];
      if (!sub8(tmp, r, b)) {  // still >= b: stay, the next step continues on (r, b)
#pragma unroll
        for (int i = 0; i < 8; i++) {
          a[i] = r[i];
          ma[i] = mr[i];
        }
        af = to_f64(a);
        continue;
      }
    }
    // (a, b) <- (b, r); t_r = t_a - q t_b has the sign of t_a
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a[i] = b[i];
      ma[i] = mb[i];
      b[i] = r[i];
      mb[i] = mr[i];
    }
    tb_neg = !tb_neg;
    lb = bitlen(b, 8);
    af = bf;
    bf = to_f64(b);
    if (lb <= 136) consider3(c_out, d_out, best, best_neg, a, b, ma, mb, tb_neg);
  }
  cost_out = best;
  neg_out = best_neg;
}

}  // namespace coa_halve
