// The round-1 field arithmetic of coa_fe.h, kept for the tools' A/B
// microbenchmarks (tools/ubench_fecs.hip): the comba product with both carry
// folds of the reduction unconditional, and the add/sub likewise; plus the
// carry-save variant of tools/gen_fe_cs.py.  Not used by the engine.
#pragma once
#include "../xrpl-coa-prototype_amd/csrc/coa_fe.h"
#include "fe_cs.h"

// ------------------------------------------------------------- reduction
// r = t[0..15] (512-bit) mod p, result < 2^256.  The eight limb products
// u_i = 38 t[8+i] + t[i] < 39 * 2^32 are independent mads (no carries, so
// nothing to pad); one VCC chain then adds the high words one limb up, and a
// second folds the top word (< 40) as 38 and its carry as 38 again.
COA_DEV void fe_reduce512_full(fe& r, const uint32_t* t) {
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
      : "=&v"(r.v[0]), "=&v"(r.v[1]), "=&v"(r.v[2]), "=&v"(r.v[3]), "=&v"(r.v[4]), "=&v"(r.v[5]), "=&v"(r.v[6]),
        "=&v"(r.v[7]), "=&v"(w)
      : "v"(lo[0]), "v"(lo[1]), "v"(lo[2]), "v"(lo[3]), "v"(lo[4]), "v"(lo[5]), "v"(lo[6]), "v"(lo[7]), "v"(hi[0]),
        "v"(hi[1]), "v"(hi[2]), "v"(hi[3]), "v"(hi[4]), "v"(hi[5]), "v"(hi[6]), "v"(hi[7])
      : "vcc");
}

// ------------------------------------------------------------ multiply
COA_DEV void fe_mul_comba(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
  mul_cols<false>(t, acc, a, b);
  t[15] = (uint32_t)acc;
  fe_reduce512_full(r, t);
}

// Squaring: the 28 cross products by comba, doubled by a funnel shift (no
// carry chain), then the 8 squares added with one unpadded VCC chain (44 mads
// vs 72 for fe_mul).  The doubled cross sum is < 2^511, so the shift loses
// nothing and the final chain cannot carry out.
COA_DEV void fe_sq_comba(fe& r, const fe& a) {
  uint32_t t[16];
  t[0] = 0;
  uint64_t acc = 0;
  mul_cols<true>(t, acc, a, a);
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
  fe_reduce512_full(r, u);
}



#define COA_FOLD38_TAIL(R0, R1, R2, R3, R4, R5, R6, R7, T, Z)               \
  "v_addc_co_u32_e32 %" #T ", vcc, 0, %" #Z ", vcc\n\t"                      \
  "v_mul_u32_u24_e32 %" #T ", 38, %" #T "\n\t"                               \
  "v_add_co_u32_e32 %" #R0 ", vcc, %" #R0 ", %" #T "\n\t"                    \
  "v_addc_co_u32_e32 %" #R1 ", vcc, 0, %" #R1 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #R2 ", vcc, 0, %" #R2 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #R3 ", vcc, 0, %" #R3 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #R4 ", vcc, 0, %" #R4 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #R5 ", vcc, 0, %" #R5 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #R6 ", vcc, 0, %" #R6 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #R7 ", vcc, 0, %" #R7 ", vcc\n\t"                    \
  "v_addc_co_u32_e32 %" #T ", vcc, 0, %" #Z ", vcc\n\t"                      \
  "v_mul_u32_u24_e32 %" #T ", 38, %" #T "\n\t"                               \
  "v_add_u32_e32 %" #R0 ", %" #R0 ", %" #T

COA_DEV void fe_add_comba(fe& r, const fe& a, const fe& b) {
  fe x = a;
  uint32_t t;
  const uint32_t z = 0;
  asm("v_add_co_u32_e32 %0, vcc, %0, %10\n\t"
      "v_addc_co_u32_e32 %1, vcc, %1, %11, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, %2, %12, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, %3, %13, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, %4, %14, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, %5, %15, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, %6, %16, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, %7, %17, vcc\n\t"
      COA_FOLD38_TAIL(0, 1, 2, 3, 4, 5, 6, 7, 8, 9)
      : COA_R8_INOUT(x), "=&v"(t)
      : "v"(z), COA_B8_IN(b)
      : "vcc");
  r = x;
}

COA_DEV void fe_sub_comba(fe& r, const fe& a, const fe& b) {
  fe x = a;
  uint32_t t;
  const uint32_t z = 0;
  asm("v_sub_co_u32_e32 %0, vcc, %0, %10\n\t"
      "v_subb_co_u32_e32 %1, vcc, %1, %11, vcc\n\t"
      "v_subb_co_u32_e32 %2, vcc, %2, %12, vcc\n\t"
      "v_subb_co_u32_e32 %3, vcc, %3, %13, vcc\n\t"
      "v_subb_co_u32_e32 %4, vcc, %4, %14, vcc\n\t"
      "v_subb_co_u32_e32 %5, vcc, %5, %15, vcc\n\t"
      "v_subb_co_u32_e32 %6, vcc, %6, %16, vcc\n\t"
      "v_subb_co_u32_e32 %7, vcc, %7, %17, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %9, vcc\n\t"
      "v_mul_u32_u24_e32 %8, 38, %8\n\t"
      "v_sub_co_u32_e32 %0, vcc, %0, %8\n\t"
      "v_subb_co_u32_e32 %1, vcc, %1, %9, vcc\n\t"
      "v_subb_co_u32_e32 %2, vcc, %2, %9, vcc\n\t"
      "v_subb_co_u32_e32 %3, vcc, %3, %9, vcc\n\t"
      "v_subb_co_u32_e32 %4, vcc, %4, %9, vcc\n\t"
      "v_subb_co_u32_e32 %5, vcc, %5, %9, vcc\n\t"
      "v_subb_co_u32_e32 %6, vcc, %6, %9, vcc\n\t"
      "v_subb_co_u32_e32 %7, vcc, %7, %9, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %9, vcc\n\t"
      "v_mul_u32_u24_e32 %8, 38, %8\n\t"
      "v_sub_u32_e32 %0, %0, %8"
      : COA_R8_INOUT(x), "=&v"(t)
      : "v"(z), COA_B8_IN(b)
      : "vcc");
  r = x;
}
