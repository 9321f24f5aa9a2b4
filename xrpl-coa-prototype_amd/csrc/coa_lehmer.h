// Lehmer acceleration of the half-gcd in coa_halve.h (scalar halving,
// Pornin 2020): the Euclidean algorithm on (8l, k) run on the leading ~50
// bits of the two remainders in f64 arithmetic (every value an exact integer
// below 2^53), with Knuth's test (TAOCP 4.5.2, Algorithm L) deciding how
// many quotients of the truncated pair are provably those of the full pair;
// the 2x2 cosequence matrix (entries below 2^31) is then applied to the
// 256-bit remainders and their cofactors once.  One application replaces
// ~15 full-width Euclid steps (each a 256-bit multiply-subtract, add-back
// fix-ups and f64 re-conversions), so the ~80 steps from 256 bits down to
// the ~140-bit region cost ~6 applications plus ~80 scalar f64 steps.
//
// The result is the SAME remainder pair the full-width algorithm reaches
// (Knuth's test only accepts quotients both bracketing ratios agree on), so
// the halving's output (c, d) is unchanged; tests/test_lehmer_host.py checks
// every state against an exact big-integer Euclid on the host.
//
// Plain C++ on 32-bit limbs (no inline asm): hipcc compiles it for the
// device, and g++ for the host test (define COA_LH before including).
#pragma once
#include <math.h>
#include <stdint.h>

#ifndef COA_LH
#define COA_LH __host__ __device__ __forceinline__
#endif

namespace coa_lehmer {

COA_LH int bitlen8(const uint32_t* x) {
  int bl = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) bl = x[i] ? 32 * i + 32 - __builtin_clz(x[i]) : bl;
  return bl;
}

// floor(x / 2^s) for a value known to be below 2^53, as an exact double.
COA_LH double top_bits(const uint32_t* x, int s) {
  const int q = s >> 5, r = s & 31;
  uint64_t w = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    // limbs q, q+1, q+2 hold the window
    const int j = i - q;
    const uint64_t limb = x[i];
    if (j == 0) w |= limb >> r;
    if (j == 1) w |= r ? (limb << (32 - r)) : (limb << 32);
    if (j == 2 && r) w |= limb << (64 - r);
  }
  return (double)w;
}

// r = u*x - v*y for 8-limb x, y and u, v < 2^32, when the result is known to
// lie in [0, 2^256).
COA_LH void mul_sub(uint32_t* r, const uint32_t* x, uint32_t u, const uint32_t* y, uint32_t v) {
  uint64_t cx = 0, cy = 0;
  int64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    cx += (uint64_t)x[i] * u;
    cy += (uint64_t)y[i] * v;
    const int64_t d = (int64_t)(uint32_t)cx - (int64_t)(uint32_t)cy + br;
    r[i] = (uint32_t)d;
    br = d >> 32;  // -1 or 0 (arithmetic shift)
    cx >>= 32;
    cy >>= 32;
  }
}

// r = u*x + v*y for 8-limb x, y and u, v < 2^32 (the result fits 256 bits).
COA_LH void mul_add(uint32_t* r, const uint32_t* x, uint32_t u, const uint32_t* y, uint32_t v) {
  uint64_t cx = 0, cy = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    cx += (uint64_t)x[i] * u;
    cy += (uint64_t)y[i] * v;
    c += (uint64_t)(uint32_t)cx + (uint32_t)cy;
    r[i] = (uint32_t)c;
    c >>= 32;
    cx >>= 32;
    cy >>= 32;
  }
}

// One Lehmer step on the remainder pair a > b with cofactor magnitudes ta,
// tb (the cofactors alternate in sign along the Euclidean sequence:
// t_{i+1} = t_{i-1} - q t_i has the sign of t_{i-1}, so magnitudes add).
// Emulates as many Euclid steps as Knuth's test proves on the top 50 bits of
// a (same shift for b), but stops once the estimated b would drop to
// stop_bits or fewer bits.  Returns the number of steps applied (0: the
// caller must take one exact full-width step).
COA_LH int step(uint32_t* a, uint32_t* b, uint32_t* ta, uint32_t* tb, int stop_bits) {
  const int la = bitlen8(a);
  const int s = la > 50 ? la - 50 : 0;
  double ah = top_bits(a, s), bh = top_bits(b, s);
  double A = 1.0, B = 0.0, C = 0.0, D = 1.0;
  // stop once the truncated b is below 2^(stop_bits - s): the full b then has
  // at most stop_bits bits (plus one for the truncation error)
  const double stop = stop_bits > s ? ldexp(1.0, stop_bits - s) : 0.0;
  int n = 0;
  for (int guard = 0; guard < 64; guard++) {
    const double y1 = bh + C, y2 = bh + D;
    if (!(y1 > 0.0) || !(y2 > 0.0)) break;
    const double x1 = ah + A, x2 = ah + B;
    double q = floor(x1 / y1);
    const double r1 = fma(-q, y1, x1);  // exact: |r1| < 2 y1 < 2^53
    if (r1 < 0.0) q -= 1.0;
    else if (r1 >= y1) q += 1.0;
    // the other bracket must give the same quotient: 0 <= x2 - q y2 < y2
    const double r2 = fma(-q, y2, x2);
    if (!(r2 >= 0.0 && r2 < y2)) break;
    const double nC = fma(-q, C, A), nD = fma(-q, D, B);
    if (fabs(nC) > 2147483647.0 || fabs(nD) > 2147483647.0) break;  // entries stay below 2^31
    const double nb = fma(-q, bh, ah);
    A = C;
    B = D;
    C = nC;
    D = nD;
    ah = bh;
    bh = nb;
    n++;
    if (bh < stop) break;
  }
  if (n == 0) return 0;
  // (a, b) <- (A a + B b, C a + D b); A, B (and C, D) have opposite signs or
  // one of them is 0, so the sign of B (D) tells which product is subtracted
  uint32_t a2[8], b2[8], ta2[8], tb2[8];
  const uint32_t uA = (uint32_t)fabs(A), uB = (uint32_t)fabs(B), uC = (uint32_t)fabs(C), uD = (uint32_t)fabs(D);
  if (B > 0.0) mul_sub(a2, b, uB, a, uA);
  else mul_sub(a2, a, uA, b, uB);
  if (D > 0.0) mul_sub(b2, b, uD, a, uC);
  else mul_sub(b2, a, uC, b, uD);
  mul_add(ta2, ta, uA, tb, uB);
  mul_add(tb2, ta, uC, tb, uD);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = a2[i];
    b[i] = b2[i];
    ta[i] = ta2[i];
    tb[i] = tb2[i];
  }
  return n;
}

}  // namespace coa_lehmer
