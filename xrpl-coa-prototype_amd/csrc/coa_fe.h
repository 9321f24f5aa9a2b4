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
// them per schoolbook product beat the 100 of a 10 x 25.5-bit layout.
//
// The column (comba) accumulation keeps a 96-bit accumulator (64-bit pair +
// carry word) and takes the mad's own carry-out, so each partial product costs
// one v_mad_u64_u32 + one v_addc_co_u32.  A carry-save variant (a fresh 64-bit
// accumulator per column, high columns folded as 64-bit mads) issues 10 fewer
// instructions but 6 more mads per multiply and measured 9 % slower at one
// wave per SIMD (tools/gen_fe_cs.py, tools/ubench_fecs.hip,
// profiles/r02_ubench_fecs.txt).  The second carry fold of every product,
// add and sub is taken only when a lane needs it (a wave-uniform branch).
//
// Carry chains are inline-asm strings.  hipcc's gfx950 hazard model pads
// every VALU write of VCC/an SGPR that a later VALU reads (carry-in
// included) with two wait states, and every asm statement with one more
// before the first reader of its outputs; at one wave per SIMD those pads are
// exposed issue slots.  Here each comba column, each add/sub/fold chain and
// the squaring's diagonal add is one string whose carries pass through VCC
// between adjacent instructions (the VOP2 carry-in read).  The unpadded hand-off is checked bit-exact
// against host ports at 1, 4 and 8 waves per SIMD (tools/ubench_carry.hip,
// tools/ubench_fecs.hip; profiles/r01_ubench_*.txt, profiles/r02_ubench_fecs.txt)
// and by the whole GPU parity suite.
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

// (acc:64, c2:32) += a * b.  v_mad_u64_u32 writes its carry-out to VCC (one
// bit per lane), which the 4-byte VOP2 v_addc_co_u32 reads implicitly as its
// carry-in and folds into the third word.  A VALU VCC write read as carry-in
// needs no wait states, so nothing is padded inside the string.
COA_DEV void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(c2)
      : "v"(a), "v"(b)
      : "vcc");
}

// One whole comba column in a single asm statement: (acc, c2) = acc +
// sum_p x[p] * y[p], where c2 starts from the first product's carry-out.
// hipcc pads every inline-asm statement with an `s_nop 0` before the next
// VALU that reads its outputs; one statement per column instead of one per
// product removes ~50 of those issue slots from every fe_mul
// (tools/ubench_fe3.hip, profiles/r01_ubench_fe3.txt: 1104 -> 913 cycles per
// multiply at one wave per SIMD).  Operands: %0 acc, %1 c2, %2 a zero VGPR
// (the VOP2 addc takes its second source from a VGPR), %3.. the x/y pairs.
#define COA_MAD0(X, Y)                                   \
  "v_mad_u64_u32 %0, vcc, %" #X ", %" #Y ", %0\n\t"      \
  "v_addc_co_u32_e32 %1, vcc, 0, %2, vcc\n\t"
#define COA_MADC(X, Y)                                   \
  "v_mad_u64_u32 %0, vcc, %" #X ", %" #Y ", %0\n\t"      \
  "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
#define COA_COL_OUT "+v"(acc), "=&v"(c2)

template <int P>
COA_DEV void col(uint64_t& acc, uint32_t& c2, const uint32_t* x, const uint32_t* y) {
  const uint32_t z = 0;
  static_assert(P >= 1 && P <= 8, "column width");
  if constexpr (P == 1) {
    asm(COA_MAD0(3, 4) : COA_COL_OUT : "v"(z), "v"(x[0]), "v"(y[0]) : "vcc");
  } else if constexpr (P == 2) {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) : COA_COL_OUT : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]) : "vcc");
  } else if constexpr (P == 3) {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) COA_MADC(7, 8)
        : COA_COL_OUT
        : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]) : "vcc");
  } else if constexpr (P == 4) {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) COA_MADC(7, 8) COA_MADC(9, 10)
        : COA_COL_OUT
        : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]) : "vcc");
  } else if constexpr (P == 5) {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) COA_MADC(7, 8) COA_MADC(9, 10) COA_MADC(11, 12)
        : COA_COL_OUT
        : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]),
          "v"(y[4]) : "vcc");
  } else if constexpr (P == 6) {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) COA_MADC(7, 8) COA_MADC(9, 10) COA_MADC(11, 12) COA_MADC(13, 14)
        : COA_COL_OUT
        : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]),
          "v"(y[4]), "v"(x[5]), "v"(y[5]) : "vcc");
  } else if constexpr (P == 7) {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) COA_MADC(7, 8) COA_MADC(9, 10) COA_MADC(11, 12) COA_MADC(13, 14)
            COA_MADC(15, 16)
        : COA_COL_OUT
        : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]),
          "v"(y[4]), "v"(x[5]), "v"(y[5]), "v"(x[6]), "v"(y[6]) : "vcc");
  } else {
    asm(COA_MAD0(3, 4) COA_MADC(5, 6) COA_MADC(7, 8) COA_MADC(9, 10) COA_MADC(11, 12) COA_MADC(13, 14)
            COA_MADC(15, 16) COA_MADC(17, 18)
        : COA_COL_OUT
        : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]),
          "v"(y[4]), "v"(x[5]), "v"(y[5]), "v"(x[6]), "v"(y[6]), "v"(x[7]), "v"(y[7]) : "vcc");
  }
}

// Column k of a product: the pairs (i, k - i), 0 <= i, k - i < 8; for a
// squaring only the cross products i < k - i.
template <int K, bool SQ>
COA_DEV void mul_col(uint64_t& acc, uint32_t& c2, const fe& a, const fe& b) {
  constexpr int lo = K < 8 ? 0 : K - 7;
  constexpr int hi = SQ ? (K - 1) / 2 : (K < 8 ? K : 7);
  constexpr int P = hi - lo + 1;
  uint32_t x[P > 0 ? P : 1], y[P > 0 ? P : 1];
#pragma unroll
  for (int p = 0; p < P; p++) {
    x[p] = a.v[lo + p];
    y[p] = b.v[K - lo - p];
  }
  if constexpr (P > 0) col<P>(acc, c2, x, y);
}

template <bool SQ, int K = SQ ? 1 : 0>
COA_DEV void mul_cols(uint32_t* t, uint64_t& acc, const fe& a, const fe& b) {
  if constexpr (K < (SQ ? 14 : 15)) {
    uint32_t c2;
    mul_col<K, SQ>(acc, c2, a, b);
    t[K] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    mul_cols<SQ, K + 1>(t, acc, a, b);
  }
}

COA_DEV void fe_set(fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = 0;
}

// ------------------------------------------------------- add / sub / neg
// Carry chains are written as unpadded VOP2 strings: each v_addc/v_subb
// takes its carry-in from VCC, written by the instruction before it.  hipcc's
// own code pads every such hand-off with `s_nop 1` on gfx950; at one wave per
// SIMD (the C2 occupancy) that costs 1.6x (tools/ubench_carry.hip,
// profiles/r01_ubench_carry.txt).
#define COA_R8_INOUT(r)                                                                                    \
  "+&v"(r.v[0]), "+&v"(r.v[1]), "+&v"(r.v[2]), "+&v"(r.v[3]), "+&v"(r.v[4]), "+&v"(r.v[5]), "+&v"(r.v[6]), \
      "+&v"(r.v[7])
#define COA_B8_IN(b) \
  "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]), "v"(b.v[7])

// The rare second pass of a fold runs out of line: the common path falls
// through the s_cbranch_vccnz (no taken branch, which a lone wave pays for in
// issue cycles), and the rare block is assembled into subsection 1 of the
// function's own text section (build.py compiles with -ffunction-sections),
// after the function's code, from where it branches back.  A branch reaches
// +-128 KiB, so a translation unit with a larger kernel defines
// COA_RARE_INLINE and keeps the block inline (skipped by a taken branch).
#ifndef COA_RARE_INLINE
#define COA_RARE_BEGIN "s_cbranch_vccnz 2f\n1:\n\t.subsection 1\n2:\n\t"
#define COA_RARE_END "s_branch 1b\n\t.subsection 0"
#else
#define COA_RARE_BEGIN "s_cbranch_vccz 1f\n\t"
#define COA_RARE_END "1:"
#endif

// r = a + b (mod p), result < 2^256.  2^256 == 38: the carry out of word 7
// becomes 38 added to word 0.  That add carries on only when word 0 was
// within 38 of 2^32 (probability ~2^-26 per lane), so the propagation through
// words 1..7 runs only when some lane carried (a wave-uniform branch to the
// out-of-line block, COA_RARE_BEGIN); a carry out of that second
// pass leaves words that wrapped to values < 38, so its fold cannot carry.
COA_DEV void fe_add(fe& r, const fe& a, const fe& b) {
  fe x = a;
  uint32_t t;
  asm("v_add_co_u32_e32 %0, vcc, %0, %9\n\t"
      "v_addc_co_u32_e32 %1, vcc, %1, %10, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, %2, %11, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, %3, %12, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, %4, %13, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, %5, %14, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, %6, %15, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, %7, %16, vcc\n\t"
      "v_cndmask_b32_e64 %8, 0, 38, vcc\n\t"
      "v_add_co_u32_e32 %0, vcc, %0, %8\n\t"
      COA_RARE_BEGIN
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, 0, %4, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, 0, %5, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, 0, %6, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, 0, %7, vcc\n\t"
      "v_cndmask_b32_e64 %8, 0, 38, vcc\n\t"
      "v_add_u32_e32 %0, %0, %8\n\t"
      COA_RARE_END
      : COA_R8_INOUT(x), "=&v"(t)
      : COA_B8_IN(b)
      : "vcc");
  r = x;
}

// r = a - b (mod p), result < 2^256: a - b + 2^256 is computed, then
// 2^256 == 38 subtracted once per borrow; the second borrow pass is behind
// the same kind of wave-uniform branch as fe_add's.
COA_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  fe x = a;
  uint32_t t;
  asm("v_sub_co_u32_e32 %0, vcc, %0, %9\n\t"
      "v_subb_co_u32_e32 %1, vcc, %1, %10, vcc\n\t"
      "v_subb_co_u32_e32 %2, vcc, %2, %11, vcc\n\t"
      "v_subb_co_u32_e32 %3, vcc, %3, %12, vcc\n\t"
      "v_subb_co_u32_e32 %4, vcc, %4, %13, vcc\n\t"
      "v_subb_co_u32_e32 %5, vcc, %5, %14, vcc\n\t"
      "v_subb_co_u32_e32 %6, vcc, %6, %15, vcc\n\t"
      "v_subb_co_u32_e32 %7, vcc, %7, %16, vcc\n\t"
      "v_cndmask_b32_e64 %8, 0, 38, vcc\n\t"
      "v_sub_co_u32_e32 %0, vcc, %0, %8\n\t"
      COA_RARE_BEGIN
      "v_subbrev_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_subbrev_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_subbrev_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
      "v_subbrev_co_u32_e32 %4, vcc, 0, %4, vcc\n\t"
      "v_subbrev_co_u32_e32 %5, vcc, 0, %5, vcc\n\t"
      "v_subbrev_co_u32_e32 %6, vcc, 0, %6, vcc\n\t"
      "v_subbrev_co_u32_e32 %7, vcc, 0, %7, vcc\n\t"
      "v_cndmask_b32_e64 %8, 0, 38, vcc\n\t"
      "v_sub_u32_e32 %0, %0, %8\n\t"
      COA_RARE_END
      : COA_R8_INOUT(x), "=&v"(t)
      : COA_B8_IN(b)
      : "vcc");
  r = x;
}

// r += w (w < 2^32 - 2^10), then the carry folded as 38; result < 2^256.
COA_DEV void fe_fold_word(fe& r, uint32_t w) {
  asm("v_add_co_u32_e32 %0, vcc, %0, %8\n\t"
      "v_mov_b32_e32 %8, 0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, 0, %4, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, 0, %5, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, 0, %6, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, 0, %7, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %8, vcc\n\t"
      "v_mul_u32_u24_e32 %8, 38, %8\n\t"
      "v_add_u32_e32 %0, %0, %8"
      : COA_R8_INOUT(r), "+&v"(w)
      :
      : "vcc");
}

// s = a + b and d = a - b (mod p, results < 2^256) as two interleaved carry
// chains: the sum's carries pass through one SGPR pair, the difference's
// borrows through another (VOP3 forms), so each instruction's carry-in was
// written two instructions earlier rather than by the one before it, which a
// wave alone on its SIMD otherwise waits for.  Folds as in fe_add / fe_sub;
// both second passes run in one out-of-line block, entered when either chain
// carried (a chain that did not carry propagates zeros there).  The s_or_b64
// that joins the two carry masks writes SCC, so SCC is declared clobbered: a
// compiler-held SCC (a loop condition) live across the statement would
// otherwise be lost -- without it k_verify_main never left its digit loop.
COA_DEV void fe_addsub(fe& s, fe& d, const fe& a, const fe& b) {
  fe x = a, y = a;
  uint32_t t, u;
  uint64_t cs, cd;
  asm("v_add_co_u32_e64 %0, %[cs], %0, %[b0]\n\t"
      "v_sub_co_u32_e64 %8, %[cd], %8, %[b0]\n\t"
      "v_addc_co_u32_e64 %1, %[cs], %1, %[b1], %[cs]\n\t"
      "v_subb_co_u32_e64 %9, %[cd], %9, %[b1], %[cd]\n\t"
      "v_addc_co_u32_e64 %2, %[cs], %2, %[b2], %[cs]\n\t"
      "v_subb_co_u32_e64 %10, %[cd], %10, %[b2], %[cd]\n\t"
      "v_addc_co_u32_e64 %3, %[cs], %3, %[b3], %[cs]\n\t"
      "v_subb_co_u32_e64 %11, %[cd], %11, %[b3], %[cd]\n\t"
      "v_addc_co_u32_e64 %4, %[cs], %4, %[b4], %[cs]\n\t"
      "v_subb_co_u32_e64 %12, %[cd], %12, %[b4], %[cd]\n\t"
      "v_addc_co_u32_e64 %5, %[cs], %5, %[b5], %[cs]\n\t"
      "v_subb_co_u32_e64 %13, %[cd], %13, %[b5], %[cd]\n\t"
      "v_addc_co_u32_e64 %6, %[cs], %6, %[b6], %[cs]\n\t"
      "v_subb_co_u32_e64 %14, %[cd], %14, %[b6], %[cd]\n\t"
      "v_addc_co_u32_e64 %7, %[cs], %7, %[b7], %[cs]\n\t"
      "v_subb_co_u32_e64 %15, %[cd], %15, %[b7], %[cd]\n\t"
      "v_cndmask_b32_e64 %[t], 0, 38, %[cs]\n\t"
      "v_cndmask_b32_e64 %[u], 0, 38, %[cd]\n\t"
      "v_add_co_u32_e64 %0, %[cs], %0, %[t]\n\t"
      "v_sub_co_u32_e64 %8, %[cd], %8, %[u]\n\t"
      "s_or_b64 vcc, %[cs], %[cd]\n\t"
      COA_RARE_BEGIN
      "v_addc_co_u32_e64 %1, %[cs], 0, %1, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %9, %[cd], 0, %9, %[cd]\n\t"
      "v_addc_co_u32_e64 %2, %[cs], 0, %2, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %10, %[cd], 0, %10, %[cd]\n\t"
      "v_addc_co_u32_e64 %3, %[cs], 0, %3, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %11, %[cd], 0, %11, %[cd]\n\t"
      "v_addc_co_u32_e64 %4, %[cs], 0, %4, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %12, %[cd], 0, %12, %[cd]\n\t"
      "v_addc_co_u32_e64 %5, %[cs], 0, %5, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %13, %[cd], 0, %13, %[cd]\n\t"
      "v_addc_co_u32_e64 %6, %[cs], 0, %6, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %14, %[cd], 0, %14, %[cd]\n\t"
      "v_addc_co_u32_e64 %7, %[cs], 0, %7, %[cs]\n\t"
      "v_subbrev_co_u32_e64 %15, %[cd], 0, %15, %[cd]\n\t"
      "v_cndmask_b32_e64 %[t], 0, 38, %[cs]\n\t"
      "v_cndmask_b32_e64 %[u], 0, 38, %[cd]\n\t"
      "v_add_u32_e32 %0, %0, %[t]\n\t"
      "v_sub_u32_e32 %8, %8, %[u]\n\t"
      COA_RARE_END
      : COA_R8_INOUT(x), COA_R8_INOUT(y), [t] "=&v"(t), [u] "=&v"(u), [cs] "=&s"(cs), [cd] "=&s"(cd)
      : [b0] "v"(b.v[0]), [b1] "v"(b.v[1]), [b2] "v"(b.v[2]), [b3] "v"(b.v[3]), [b4] "v"(b.v[4]),
        [b5] "v"(b.v[5]), [b6] "v"(b.v[6]), [b7] "v"(b.v[7])
      : "vcc", "scc");  // s_or_b64 writes SCC
  s = x;
  d = y;
}

COA_DEV void fe_neg(fe& r, const fe& a) {
  fe z;
  fe_set(z, 0);
  fe_sub(r, z, a);
}

// ------------------------------------------------------------- reduction
// r = t[0..15] (512-bit) mod p, result < 2^256.  The eight limb products
// u_i = 38 t[8+i] + t[i] < 39 * 2^32 are independent mads (no carries, so
// nothing to pad); one VCC chain then adds the high words one limb up, and
// the top word (< 40) is folded as 38 into word 0.  That add carries only
// when word 0 was within 1,482 of 2^32 (~2^-21 per lane), so the
// propagation through words 1..7 runs out of line, only when some lane
// carried (COA_RARE_BEGIN); its own carry out leaves words that
// wrapped to zero, so the 38 it adds to word 0 cannot carry.
COA_DEV void fe_reduce512(fe& r, const uint32_t* t) {
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t u = (uint64_t)t[8 + i] * 38u + t[i];
    lo[i] = (uint32_t)u;
    hi[i] = (uint32_t)(u >> 32);
  }
  uint32_t w;
  asm("v_add_co_u32_e32 %1, vcc, %10, %17\n\t"
      "v_addc_co_u32_e32 %2, vcc, %11, %18, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, %12, %19, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, %13, %20, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, %14, %21, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, %15, %22, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, %16, %23, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %24, vcc\n\t"
      "v_mul_u32_u24_e32 %8, 38, %8\n\t"
      "v_add_co_u32_e32 %0, vcc, %9, %8\n\t"
      COA_RARE_BEGIN
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, 0, %4, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, 0, %5, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, 0, %6, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, 0, %7, vcc\n\t"
      "v_cndmask_b32_e64 %8, 0, 38, vcc\n\t"
      "v_add_u32_e32 %0, %0, %8\n\t"
      COA_RARE_END
      : "=&v"(r.v[0]), "=&v"(r.v[1]), "=&v"(r.v[2]), "=&v"(r.v[3]), "=&v"(r.v[4]), "=&v"(r.v[5]), "=&v"(r.v[6]),
        "=&v"(r.v[7]), "=&v"(w)
      : "v"(lo[0]), "v"(lo[1]), "v"(lo[2]), "v"(lo[3]), "v"(lo[4]), "v"(lo[5]), "v"(lo[6]), "v"(lo[7]), "v"(hi[0]),
        "v"(hi[1]), "v"(hi[2]), "v"(hi[3]), "v"(hi[4]), "v"(hi[5]), "v"(hi[6]), "v"(hi[7])
      : "vcc");
}

// ------------------------------------------------------------ multiply
COA_DEV void fe_mul(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
  mul_cols<false>(t, acc, a, b);
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

// Squaring: the 28 cross products by comba, doubled by a funnel shift (no
// carry chain), then the 8 squares added with one unpadded VCC chain (44 mads
// vs 72 for fe_mul).  The doubled cross sum is < 2^511, so the shift loses
// nothing and the final chain cannot carry out.
// The squaring after its cross columns: t[1..13] and acc hold the cross sum.
COA_DEV void sq_finish(fe& r, uint32_t* t, uint64_t acc, const fe& a) {
  t[14] = (uint32_t)acc;
  t[15] = (uint32_t)(acc >> 32);
  uint32_t u[16];
#pragma unroll
  for (int i = 15; i >= 2; i--) u[i] = __builtin_amdgcn_alignbit(t[i], t[i - 1], 31);
  u[1] = t[1] << 1;
  uint32_t d[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t p = (uint64_t)a.v[i] * a.v[i];
    d[2 * i] = (uint32_t)p;
    d[2 * i + 1] = (uint32_t)(p >> 32);
  }
  u[0] = d[0];
  asm("v_add_co_u32_e32 %0, vcc, %0, %15\n\t"
      "v_addc_co_u32_e32 %1, vcc, %1, %16, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, %2, %17, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, %3, %18, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, %4, %19, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, %5, %20, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, %6, %21, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, %7, %22, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, %8, %23, vcc\n\t"
      "v_addc_co_u32_e32 %9, vcc, %9, %24, vcc\n\t"
      "v_addc_co_u32_e32 %10, vcc, %10, %25, vcc\n\t"
      "v_addc_co_u32_e32 %11, vcc, %11, %26, vcc\n\t"
      "v_addc_co_u32_e32 %12, vcc, %12, %27, vcc\n\t"
      "v_addc_co_u32_e32 %13, vcc, %13, %28, vcc\n\t"
      "v_addc_co_u32_e32 %14, vcc, %14, %29, vcc"
      : "+&v"(u[1]), "+&v"(u[2]), "+&v"(u[3]), "+&v"(u[4]), "+&v"(u[5]), "+&v"(u[6]), "+&v"(u[7]), "+&v"(u[8]),
        "+&v"(u[9]), "+&v"(u[10]), "+&v"(u[11]), "+&v"(u[12]), "+&v"(u[13]), "+&v"(u[14]), "+&v"(u[15])
      : "v"(d[1]), "v"(d[2]), "v"(d[3]), "v"(d[4]), "v"(d[5]), "v"(d[6]), "v"(d[7]), "v"(d[8]), "v"(d[9]),
        "v"(d[10]), "v"(d[11]), "v"(d[12]), "v"(d[13]), "v"(d[14]), "v"(d[15])
      : "vcc");
  fe_reduce512(r, u);
}

COA_DEV void fe_sq(fe& r, const fe& a) {
  uint32_t t[16];
  t[0] = 0;
  uint64_t acc = 0;
  mul_cols<true>(t, acc, a, a);
  sq_finish(r, t, acc, a);
}

// ------------------------------------------- interleaved independent products
// N independent products (or squarings), issued column by column: column K
// of product 0, of product 1, ... then column K + 1.  Inside one column the
// mads are a dependency chain through the accumulator; a wave alone on its
// SIMD (the C2 occupancy of k_verify_main) otherwise waits on that chain at
// every column boundary.  tools/ubench_ilp.hip, one wave per SIMD: 888
// cycles per product as one chain, 802 with two interleaved
// (profiles/r02_ubench_ilp.txt).
template <bool SQ, int N, int K = SQ ? 1 : 0>
COA_DEV void mul_cols_n(uint32_t (&t)[N][16], uint64_t (&acc)[N], const fe (&a)[N], const fe (&b)[N]) {
  if constexpr (K < (SQ ? 14 : 15)) {
    uint32_t c2[N];
#pragma unroll
    for (int q = 0; q < N; q++) mul_col<K, SQ>(acc[q], c2[q], a[q], SQ ? a[q] : b[q]);
#pragma unroll
    for (int q = 0; q < N; q++) {
      t[q][K] = (uint32_t)acc[q];
      acc[q] = (acc[q] >> 32) | ((uint64_t)c2[q] << 32);
    }
    mul_cols_n<SQ, N, K + 1>(t, acc, a, b);
  }
}

// r[q] = a[q] * b[q]; the outputs are written after every input is read, so
// they may alias the inputs.
template <int N>
COA_DEV void fe_mul_n(fe (&r)[N], const fe (&a)[N], const fe (&b)[N]) {
  uint32_t t[N][16];
  uint64_t acc[N];
#pragma unroll
  for (int q = 0; q < N; q++) acc[q] = 0;
  mul_cols_n<false, N>(t, acc, a, b);
#pragma unroll
  for (int q = 0; q < N; q++) {
    t[q][15] = (uint32_t)acc[q];
    fe_reduce512(r[q], t[q]);
  }
}

// r[q] = a[q]^2.
template <int N>
COA_DEV void fe_sq_n(fe (&r)[N], const fe (&a)[N]) {
  uint32_t t[N][16];
  uint64_t acc[N];
#pragma unroll
  for (int q = 0; q < N; q++) {
    acc[q] = 0;
    t[q][0] = 0;
  }
  mul_cols_n<true, N>(t, acc, a, a);
#pragma unroll
  for (int q = 0; q < N; q++) sq_finish(r[q], t[q], acc[q], a[q]);
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
  fe_fold_word(r, (uint32_t)(acc >> 32) * 38u);  // c < 2^26: < 2^32 - 2^10
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
