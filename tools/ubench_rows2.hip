// Row squaring control flow on a lone wave (s_memtime cycles per squaring):
//   cur      the round-2 start: normalize's carry check as a loop, one
//            squaring per loop trip
//   expect   the check's rare ripple behind __builtin_expect, common path
//            straight-line
//   unroll4  expect, and the squaring loop unrolled by four
//   lean     unroll4, and the column sums start from the first product
//            (no zeroed accumulator, the first carry by v_cndmask)
//   split    unroll4, the eight multiply-accumulates as two interleaved
//            chains of four (k < 4, k >= 4) added at the end
// Every variant's result is compared with the one-lane fe_sqn (canonical).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../xrpl-coa-prototype_amd/csrc ubench_rows2.hip -o ubench_rows2
#include <cstdio>

#include "coa_fe_wave.h"

namespace v2 {
template <bool Expect>
COA_DEV uint32_t normalize(uint64_t m) {
  const uint32_t r = fw::row_lane();
  fw::wrap_step(m, r);
  if (!Expect) {
#pragma unroll 1
    while (__any((uint32_t)(m >> 32) != 0u)) fw::wrap_step(m, r);
    return (uint32_t)m;
  }
  if (__builtin_expect(__any((uint32_t)(m >> 32) != 0u), 0)) {
#pragma unroll 1
    do fw::wrap_step(m, r);
    while (__any((uint32_t)(m >> 32) != 0u));
  }
  return (uint32_t)m;
}
template <bool Expect = true, bool Lean = false, bool Split = false>
COA_DEV uint32_t mul(uint32_t a, uint32_t b) {
  uint32_t bk[8], ak[8];
  bk[0] = fw::bcast<0>(b);
  bk[1] = fw::bcast<1>(b);
  bk[2] = fw::bcast<2>(b);
  bk[3] = fw::bcast<3>(b);
  bk[4] = fw::bcast<4>(b);
  bk[5] = fw::bcast<5>(b);
  bk[6] = fw::bcast<6>(b);
  bk[7] = fw::bcast<7>(b);
  ak[0] = a;
  ak[1] = fw::shr<1>(a);
  ak[2] = fw::shr<2>(a);
  ak[3] = fw::shr<3>(a);
  ak[4] = fw::shr<4>(a);
  ak[5] = fw::shr<5>(a);
  ak[6] = fw::shr<6>(a);
  ak[7] = fw::shr<7>(a);
  uint64_t acc = 0;
  uint32_t c2 = 0;
  if (Split) {
    uint64_t acc1;
    uint32_t c3 = 0;
    asm("v_mad_u64_u32 %0, vcc, %4, %12, 0\n\t"
        "v_mad_u64_u32 %2, vcc, %8, %16, 0\n\t"
        "v_mad_u64_u32 %0, vcc, %5, %13, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
        "v_mad_u64_u32 %2, vcc, %9, %17, %2\n\t"
        "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
        "v_mad_u64_u32 %0, vcc, %6, %14, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
        "v_mad_u64_u32 %2, vcc, %10, %18, %2\n\t"
        "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
        "v_mad_u64_u32 %0, vcc, %7, %15, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
        "v_mad_u64_u32 %2, vcc, %11, %19, %2\n\t"
        "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc"
        : "+&v"(acc), "+&v"(c2), "=&v"(acc1), "+&v"(c3)
        : "v"(ak[0]), "v"(ak[1]), "v"(ak[2]), "v"(ak[3]), "v"(ak[4]), "v"(ak[5]), "v"(ak[6]), "v"(ak[7]), "v"(bk[0]),
          "v"(bk[1]), "v"(bk[2]), "v"(bk[3]), "v"(bk[4]), "v"(bk[5]), "v"(bk[6]), "v"(bk[7])
        : "vcc");
    const uint64_t sum = acc + acc1;
    c2 += c3 + (sum < acc ? 1u : 0u);
    acc = sum;
  } else if (Lean) {
    asm("v_mad_u64_u32 %0, vcc, %2, %10, 0\n\t"
        "v_cndmask_b32_e64 %1, 0, 1, vcc\n\t"
        "v_mad_u64_u32 %0, vcc, %3, %11, %0\n\t"
        "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
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
  } else
  asm("v_mad_u64_u32 %0, vcc, %2, %10, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %3, %11, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
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
      : "+v"(acc), "+v"(c2)
      : "v"(ak[0]), "v"(ak[1]), "v"(ak[2]), "v"(ak[3]), "v"(ak[4]), "v"(ak[5]), "v"(ak[6]), "v"(ak[7]), "v"(bk[0]),
        "v"(bk[1]), "v"(bk[2]), "v"(bk[3]), "v"(bk[4]), "v"(bk[5]), "v"(bk[6]), "v"(bk[7])
      : "vcc");
  const uint64_t n = (uint64_t)(uint32_t)acc + fw::shr<1>((uint32_t)(acc >> 32)) + fw::shr<2>(c2);
  const uint32_t r = fw::row_lane();
  const uint32_t up_lo = fw::shl<8>((uint32_t)n), up_hi = fw::shl<8>((uint32_t)(n >> 32));
  uint64_t m = (uint64_t)up_lo * 38u + (r < 8 ? n : 0);
  m += (uint64_t)__umul24(up_hi, 38u) << 32;
  return normalize<Expect>(m);
}
template <bool Expect>
COA_DEV uint32_t sqn(uint32_t a, int n) {
#pragma unroll 1
  for (int i = 0; i < n; i++) a = mul<Expect>(a, a);
  return a;
}
template <bool Lean = false, bool Split = false>
COA_DEV uint32_t sqn4(uint32_t a, int n) {  // n % 4 == 0
#pragma unroll 1
  for (int i = 0; i < n; i += 4) {
    a = mul<true, Lean, Split>(a, a);
    a = mul<true, Lean, Split>(a, a);
    a = mul<true, Lean, Split>(a, a);
    a = mul<true, Lean, Split>(a, a);
  }
  return a;
}
}  // namespace v2

__global__ void k(const uint32_t* in, uint32_t* out, long long* cyc) {
  fe z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.v[i] = in[i];
  const uint32_t x0 = fw::from_fe(z);
  long long t0 = clock64();
  const uint32_t a = v2::sqn<false>(x0, 100);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = clock64();
  const uint32_t b = v2::sqn<true>(x0, 100);
  long long t2 = clock64();
  const uint32_t c = v2::sqn4(x0, 100);
  long long t3 = clock64();
  const uint32_t dl = v2::sqn4<true>(x0, 100);
  long long t4 = clock64();
  const uint32_t ds = v2::sqn4<false, true>(x0, 100);
  long long t5 = clock64();
  fe y = z;
  fe_sqn(y, y, 100);
  fe ya, yb, yc, yd, ye, ref;
  fw::to_fe(yd, dl);
  fe_canon(yd, yd);
  fw::to_fe(ye, ds);
  fe_canon(ye, ye);
  fw::to_fe(ya, a);
  fw::to_fe(yb, b);
  fw::to_fe(yc, c);
  fe_canon(ref, y);
  fe_canon(ya, ya);
  fe_canon(yb, yb);
  fe_canon(yc, yc);
  uint32_t bad = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) bad |= (ya.v[i] != ref.v[i]) | ((yb.v[i] != ref.v[i]) << 1) | ((yc.v[i] != ref.v[i]) << 2) |
                                        ((yd.v[i] != ref.v[i]) << 3) | ((ye.v[i] != ref.v[i]) << 4);
  if (threadIdx.x == 0) {
    out[0] = bad;
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
    cyc[3] = t4 - t3;
    cyc[4] = t5 - t4;
  }
}

int main() {
  uint32_t h[3][8] = {{0x12345678, 0x9abcdef0, 0x0fedcba9, 0x87654321, 0x11111111, 0x22222222, 0x33333333, 0x04444444},
                      {0xffffffec, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0x7fffffff},
                      {0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff}};
  uint32_t *din, *dout;
  long long* dc;
  if (hipMalloc(&din, 32) || hipMalloc(&dout, 4) || hipMalloc(&dc, 64)) return 1;
  int rc = 0;
  for (int v = 0; v < 3; v++) {
    (void)hipMemcpy(din, h[v], 32, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; rep++) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, dc);
      long long c[5];
      uint32_t bad = 0;
      (void)hipMemcpy(c, dc, 40, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&bad, dout, 4, hipMemcpyDeviceToHost);
      printf("input %d: cycles per squaring: cur %.1f  expect %.1f  unroll4 %.1f  lean %.1f  split %.1f  mismatch mask %u\n",
             v, c[0] / 100.0, c[1] / 100.0, c[2] / 100.0, c[3] / 100.0, c[4] / 100.0, bad);
      rc |= bad != 0;
    }
  }
  return rc;
}
