// Issue cost of multiply/add instructions at one and at eight waves per
// SIMD (C2 runs at one), eight independent chains per lane, and of
// v_mad_u64_u32 interleaved with independent cheap ops: whether a lone wave
// overlaps cheap VALU work with a mad decides the field-multiply design
// (field arithmetic; profiles/r01_ubench_mad.txt).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_mad.hip -o tools/ubench_mad
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>

#define C 8
// Each asm statement holds one instruction per chain (8 chains), so hipcc's
// one s_nop per statement costs 1/8 of an issue slot per instruction.
// V: 0 mad_u64 (sgpr sdst)  1 mad_u64 (vcc sdst)  2 mul_lo_u32  3 mul_hi_u32
//    4 mul_u32_u24  5 mul_hi_u32_u24  6 mad_u32_u24  7 add_u32  8 fma_f64
//    10/11/12 mad_u64 + 1/2/3 independent adds  13 lshl_add_u64
//    14 lshrrev_b64  15 add_co+addc pairs  16 add3_u32
//    17 alignbit_b32  18 bitop3_b32  19 mov_b32_dpp quad_perm  20 and_b32
//    (17-20: the SHA-512 lane-pair round's instruction classes, round 5)
template <int V>
__global__ void k(uint64_t* out, uint32_t a0, int n) {
  uint64_t acc[C];
  uint32_t w[C];
  uint32_t a = a0 + threadIdx.x, b = a0 ^ blockIdx.x;
  const double fa = 1.0000001 * a, fb = 0.999999 * b;
  const uint64_t wb = b;
#pragma unroll
  for (int c = 0; c < C; c++) {
    acc[c] = c;
    w[c] = c * 7;
  }
  if (V == 8)
#pragma unroll
    for (int c = 0; c < C; c++) acc[c] = __builtin_bit_cast(uint64_t, (double)c);
  for (int r = 0; r < n; r++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if constexpr (V == 0) asm volatile("v_mad_u64_u32 %0, s[20:21], %8, %9, %0\n\tv_mad_u64_u32 %1, s[20:21], %8, %9, %1\n\tv_mad_u64_u32 %2, s[20:21], %8, %9, %2\n\tv_mad_u64_u32 %3, s[20:21], %8, %9, %3\n\tv_mad_u64_u32 %4, s[20:21], %8, %9, %4\n\tv_mad_u64_u32 %5, s[20:21], %8, %9, %5\n\tv_mad_u64_u32 %6, s[20:21], %8, %9, %6\n\tv_mad_u64_u32 %7, s[20:21], %8, %9, %7" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 1) asm volatile("v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, vcc, %8, %9, %1\n\tv_mad_u64_u32 %2, vcc, %8, %9, %2\n\tv_mad_u64_u32 %3, vcc, %8, %9, %3\n\tv_mad_u64_u32 %4, vcc, %8, %9, %4\n\tv_mad_u64_u32 %5, vcc, %8, %9, %5\n\tv_mad_u64_u32 %6, vcc, %8, %9, %6\n\tv_mad_u64_u32 %7, vcc, %8, %9, %7" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 2) asm volatile("v_mul_lo_u32 %0, %0, %9\n\tv_mul_lo_u32 %1, %1, %9\n\tv_mul_lo_u32 %2, %2, %9\n\tv_mul_lo_u32 %3, %3, %9\n\tv_mul_lo_u32 %4, %4, %9\n\tv_mul_lo_u32 %5, %5, %9\n\tv_mul_lo_u32 %6, %6, %9\n\tv_mul_lo_u32 %7, %7, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 3) asm volatile("v_mul_hi_u32 %0, %0, %9\n\tv_mul_hi_u32 %1, %1, %9\n\tv_mul_hi_u32 %2, %2, %9\n\tv_mul_hi_u32 %3, %3, %9\n\tv_mul_hi_u32 %4, %4, %9\n\tv_mul_hi_u32 %5, %5, %9\n\tv_mul_hi_u32 %6, %6, %9\n\tv_mul_hi_u32 %7, %7, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 4) asm volatile("v_mul_u32_u24 %0, %0, %9\n\tv_mul_u32_u24 %1, %1, %9\n\tv_mul_u32_u24 %2, %2, %9\n\tv_mul_u32_u24 %3, %3, %9\n\tv_mul_u32_u24 %4, %4, %9\n\tv_mul_u32_u24 %5, %5, %9\n\tv_mul_u32_u24 %6, %6, %9\n\tv_mul_u32_u24 %7, %7, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 5) asm volatile("v_mul_hi_u32_u24 %0, %0, %9\n\tv_mul_hi_u32_u24 %1, %1, %9\n\tv_mul_hi_u32_u24 %2, %2, %9\n\tv_mul_hi_u32_u24 %3, %3, %9\n\tv_mul_hi_u32_u24 %4, %4, %9\n\tv_mul_hi_u32_u24 %5, %5, %9\n\tv_mul_hi_u32_u24 %6, %6, %9\n\tv_mul_hi_u32_u24 %7, %7, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 6) asm volatile("v_mad_u32_u24 %0, %8, %9, %0\n\tv_mad_u32_u24 %1, %8, %9, %1\n\tv_mad_u32_u24 %2, %8, %9, %2\n\tv_mad_u32_u24 %3, %8, %9, %3\n\tv_mad_u32_u24 %4, %8, %9, %4\n\tv_mad_u32_u24 %5, %8, %9, %5\n\tv_mad_u32_u24 %6, %8, %9, %6\n\tv_mad_u32_u24 %7, %8, %9, %7" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 7) asm volatile("v_add_u32 %0, %0, %9\n\tv_add_u32 %1, %1, %9\n\tv_add_u32 %2, %2, %9\n\tv_add_u32 %3, %3, %9\n\tv_add_u32 %4, %4, %9\n\tv_add_u32 %5, %5, %9\n\tv_add_u32 %6, %6, %9\n\tv_add_u32 %7, %7, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 8) asm volatile("v_fma_f64 %0, %10, %11, %0\n\tv_fma_f64 %1, %10, %11, %1\n\tv_fma_f64 %2, %10, %11, %2\n\tv_fma_f64 %3, %10, %11, %3\n\tv_fma_f64 %4, %10, %11, %4\n\tv_fma_f64 %5, %10, %11, %5\n\tv_fma_f64 %6, %10, %11, %6\n\tv_fma_f64 %7, %10, %11, %7" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]) : "v"(a), "v"(b), "v"(fa), "v"(fb) : "vcc", "s20", "s21");
      if constexpr (V == 13) asm volatile("v_lshl_add_u64 %0, %0, 0, %10\n\tv_lshl_add_u64 %1, %1, 0, %10\n\tv_lshl_add_u64 %2, %2, 0, %10\n\tv_lshl_add_u64 %3, %3, 0, %10\n\tv_lshl_add_u64 %4, %4, 0, %10\n\tv_lshl_add_u64 %5, %5, 0, %10\n\tv_lshl_add_u64 %6, %6, 0, %10\n\tv_lshl_add_u64 %7, %7, 0, %10" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 14) asm volatile("v_lshrrev_b64 %0, 1, %0\n\tv_lshrrev_b64 %1, 1, %1\n\tv_lshrrev_b64 %2, 1, %2\n\tv_lshrrev_b64 %3, 1, %3\n\tv_lshrrev_b64 %4, 1, %4\n\tv_lshrrev_b64 %5, 1, %5\n\tv_lshrrev_b64 %6, 1, %6\n\tv_lshrrev_b64 %7, 1, %7" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 16) asm volatile("v_add3_u32 %0, %0, %8, %9\n\tv_add3_u32 %1, %1, %8, %9\n\tv_add3_u32 %2, %2, %8, %9\n\tv_add3_u32 %3, %3, %8, %9\n\tv_add3_u32 %4, %4, %8, %9\n\tv_add3_u32 %5, %5, %8, %9\n\tv_add3_u32 %6, %6, %8, %9\n\tv_add3_u32 %7, %7, %8, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 17) asm volatile("v_alignbit_b32 %0, %0, %9, %8\n\tv_alignbit_b32 %1, %1, %9, %8\n\tv_alignbit_b32 %2, %2, %9, %8\n\tv_alignbit_b32 %3, %3, %9, %8\n\tv_alignbit_b32 %4, %4, %9, %8\n\tv_alignbit_b32 %5, %5, %9, %8\n\tv_alignbit_b32 %6, %6, %9, %8\n\tv_alignbit_b32 %7, %7, %9, %8" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 18) asm volatile("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 19) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %4, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %5, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %6, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %7, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 20) asm volatile("v_and_b32 %0, %0, %9\n\tv_and_b32 %1, %1, %9\n\tv_and_b32 %2, %2, %9\n\tv_and_b32 %3, %3, %9\n\tv_and_b32 %4, %4, %9\n\tv_and_b32 %5, %5, %9\n\tv_and_b32 %6, %6, %9\n\tv_and_b32 %7, %7, %9" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc", "s20", "s21");
      if constexpr (V == 10) asm volatile("v_mad_u64_u32 %0, s[20:21], %16, %17, %0\n\tv_add_u32 %8, %8, %17\n\tv_mad_u64_u32 %1, s[20:21], %16, %17, %1\n\tv_add_u32 %9, %9, %17\n\tv_mad_u64_u32 %2, s[20:21], %16, %17, %2\n\tv_add_u32 %10, %10, %17\n\tv_mad_u64_u32 %3, s[20:21], %16, %17, %3\n\tv_add_u32 %11, %11, %17\n\tv_mad_u64_u32 %4, s[20:21], %16, %17, %4\n\tv_add_u32 %12, %12, %17\n\tv_mad_u64_u32 %5, s[20:21], %16, %17, %5\n\tv_add_u32 %13, %13, %17\n\tv_mad_u64_u32 %6, s[20:21], %16, %17, %6\n\tv_add_u32 %14, %14, %17\n\tv_mad_u64_u32 %7, s[20:21], %16, %17, %7\n\tv_add_u32 %15, %15, %17" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]), "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b) : "s20", "s21");
      if constexpr (V == 11) asm volatile("v_mad_u64_u32 %0, s[20:21], %16, %17, %0\n\tv_add_u32 %8, %8, %17\n\tv_add_u32 %9, %9, %17\n\tv_mad_u64_u32 %1, s[20:21], %16, %17, %1\n\tv_add_u32 %9, %9, %17\n\tv_add_u32 %10, %10, %17\n\tv_mad_u64_u32 %2, s[20:21], %16, %17, %2\n\tv_add_u32 %10, %10, %17\n\tv_add_u32 %11, %11, %17\n\tv_mad_u64_u32 %3, s[20:21], %16, %17, %3\n\tv_add_u32 %11, %11, %17\n\tv_add_u32 %12, %12, %17\n\tv_mad_u64_u32 %4, s[20:21], %16, %17, %4\n\tv_add_u32 %12, %12, %17\n\tv_add_u32 %13, %13, %17\n\tv_mad_u64_u32 %5, s[20:21], %16, %17, %5\n\tv_add_u32 %13, %13, %17\n\tv_add_u32 %14, %14, %17\n\tv_mad_u64_u32 %6, s[20:21], %16, %17, %6\n\tv_add_u32 %14, %14, %17\n\tv_add_u32 %15, %15, %17\n\tv_mad_u64_u32 %7, s[20:21], %16, %17, %7\n\tv_add_u32 %15, %15, %17\n\tv_add_u32 %8, %8, %17" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]), "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b) : "s20", "s21");
      if constexpr (V == 12) asm volatile("v_mad_u64_u32 %0, s[20:21], %16, %17, %0\n\tv_add_u32 %8, %8, %17\n\tv_add_u32 %9, %9, %17\n\tv_add_u32 %10, %10, %17\n\tv_mad_u64_u32 %1, s[20:21], %16, %17, %1\n\tv_add_u32 %9, %9, %17\n\tv_add_u32 %10, %10, %17\n\tv_add_u32 %11, %11, %17\n\tv_mad_u64_u32 %2, s[20:21], %16, %17, %2\n\tv_add_u32 %10, %10, %17\n\tv_add_u32 %11, %11, %17\n\tv_add_u32 %12, %12, %17\n\tv_mad_u64_u32 %3, s[20:21], %16, %17, %3\n\tv_add_u32 %11, %11, %17\n\tv_add_u32 %12, %12, %17\n\tv_add_u32 %13, %13, %17\n\tv_mad_u64_u32 %4, s[20:21], %16, %17, %4\n\tv_add_u32 %12, %12, %17\n\tv_add_u32 %13, %13, %17\n\tv_add_u32 %14, %14, %17\n\tv_mad_u64_u32 %5, s[20:21], %16, %17, %5\n\tv_add_u32 %13, %13, %17\n\tv_add_u32 %14, %14, %17\n\tv_add_u32 %15, %15, %17\n\tv_mad_u64_u32 %6, s[20:21], %16, %17, %6\n\tv_add_u32 %14, %14, %17\n\tv_add_u32 %15, %15, %17\n\tv_add_u32 %8, %8, %17\n\tv_mad_u64_u32 %7, s[20:21], %16, %17, %7\n\tv_add_u32 %15, %15, %17\n\tv_add_u32 %8, %8, %17\n\tv_add_u32 %9, %9, %17" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]), "+v"(acc[6]), "+v"(acc[7]), "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b) : "s20", "s21");
      if constexpr (V == 15) asm volatile("v_add_co_u32 %0, vcc, %0, %9\n\tv_addc_co_u32 %1, vcc, %1, %9, vcc\n\tv_add_co_u32 %1, vcc, %1, %9\n\tv_addc_co_u32 %2, vcc, %2, %9, vcc\n\tv_add_co_u32 %2, vcc, %2, %9\n\tv_addc_co_u32 %3, vcc, %3, %9, vcc\n\tv_add_co_u32 %3, vcc, %3, %9\n\tv_addc_co_u32 %4, vcc, %4, %9, vcc\n\tv_add_co_u32 %4, vcc, %4, %9\n\tv_addc_co_u32 %5, vcc, %5, %9, vcc\n\tv_add_co_u32 %5, vcc, %5, %9\n\tv_addc_co_u32 %6, vcc, %6, %9, vcc\n\tv_add_co_u32 %6, vcc, %6, %9\n\tv_addc_co_u32 %7, vcc, %7, %9, vcc\n\tv_add_co_u32 %7, vcc, %7, %9\n\tv_addc_co_u32 %0, vcc, %0, %9, vcc" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]) : "v"(a), "v"(b), "v"(wb), "v"(wb) : "vcc");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < C; c++) s ^= acc[c] ^ w[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int V>
void run(uint64_t* d, const char* name, int per) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int n = 2000;
  float ms[2];
  const int blocks[2] = {256, 256 * 8};
  for (int w = 0; w < 2; w++) {
    hipLaunchKernelGGL(k<V>, dim3(blocks[w]), dim3(256), 0, 0, d, 3u, 10);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<V>, dim3(blocks[w]), dim3(256), 0, 0, d, 3u, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[w], e0, e1);
  }
  // per SIMD: waves * n * 64 groups of `per` instructions
  const double c1 = ms[0] * 1e-3 * 2.4e9 / (1.0 * n * 64);
  const double c8 = ms[1] * 1e-3 * 2.4e9 / (8.0 * n * 64);
  printf("%-32s 1 wave/SIMD %6.2f cyc/group (%5.2f /instr)   8 waves/SIMD %6.2f cyc/group (%5.2f /instr)\n", name, c1,
         c1 / per, c8, c8 / per);
}

int main() {
  uint64_t* d;
  hipMalloc(&d, sizeof(uint64_t) * 256 * 256 * 8);
  run<0>(d, "v_mad_u64_u32 (sgpr sdst)", 1);
  run<1>(d, "v_mad_u64_u32 (vcc sdst)", 1);
  run<2>(d, "v_mul_lo_u32", 1);
  run<3>(d, "v_mul_hi_u32", 1);
  run<4>(d, "v_mul_u32_u24", 1);
  run<5>(d, "v_mul_hi_u32_u24", 1);
  run<6>(d, "v_mad_u32_u24", 1);
  run<7>(d, "v_add_u32", 1);
  run<8>(d, "v_fma_f64", 1);
    run<10>(d, "mad_u64 + 1 add", 2);
  run<11>(d, "mad_u64 + 2 adds", 3);
  run<12>(d, "mad_u64 + 3 adds", 4);
  run<13>(d, "v_lshl_add_u64", 1);
  run<14>(d, "v_lshrrev_b64", 1);
  run<15>(d, "v_add_co + v_addc (pair)", 2);
  run<16>(d, "v_add3_u32", 1);
  run<17>(d, "v_alignbit_b32", 1);
  run<18>(d, "v_bitop3_b32", 1);
  run<19>(d, "v_mov_b32_dpp quad_perm", 1);
  run<20>(d, "v_and_b32", 1);
  return 0;
}
