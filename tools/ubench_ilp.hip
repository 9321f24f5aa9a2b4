// Is a lone wave's field product bound by issue or by the dependency chain
// inside each comba column?  One wave per SIMD (and two, for the ceiling),
// cycles per field product when each lane runs 1, 2 or 4 independent product
// chains (the compiler free to interleave the column asm statements), and
// with two products interleaved column by column by hand (fe_mul2 / fe_sq2).
// Every variant's lanes are checked against the single-chain result.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I xrpl-coa-prototype_amd/csrc \
//       tools/ubench_ilp.hip -o tools/ubench_ilp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "coa_fe.h"

namespace {
template <bool SQ, int K = SQ ? 1 : 0>
COA_DEV void mul_cols2(uint32_t* t, uint64_t& acc, const fe& a, const fe& b, uint32_t* u, uint64_t& acc2,
                       const fe& c, const fe& d) {
  if constexpr (K < (SQ ? 14 : 15)) {
    uint32_t c2, c3;
    mul_col<K, SQ>(acc, c2, a, b);
    mul_col<K, SQ>(acc2, c3, c, d);
    t[K] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    u[K] = (uint32_t)acc2;
    acc2 = (acc2 >> 32) | ((uint64_t)c3 << 32);
    mul_cols2<SQ, K + 1>(t, acc, a, b, u, acc2, c, d);
  }
}

COA_DEV void fe_mul2(fe& r, const fe& a, const fe& b, fe& r2, const fe& c, const fe& d) {
  uint32_t t[16], u[16];
  uint64_t acc = 0, acc2 = 0;
  mul_cols2<false>(t, acc, a, b, u, acc2, c, d);
  t[15] = (uint32_t)acc;
  u[15] = (uint32_t)acc2;
  fe_reduce512(r, t);
  fe_reduce512(r2, u);
}
// Probe (not in the engine): two independent subtractions interleaved through
// two SGPR carry pairs, as fe_addsub does for a + b / a - b.  Measured slower
// than two plain fe_sub chains (profiles/r02_ubench_ilp.txt).
COA_DEV void fe_sub2(fe& d1, const fe& a1, const fe& b1, fe& d2, const fe& a2, const fe& b2) {
  fe x = a1, y = a2;
  uint32_t t, u;
  uint64_t c1, c2;
  asm("v_sub_co_u32_e64 %0, %[c1], %0, %[p0]\n\t"
      "v_sub_co_u32_e64 %8, %[c2], %8, %[q0]\n\t"
      "v_subb_co_u32_e64 %1, %[c1], %1, %[p1], %[c1]\n\t"
      "v_subb_co_u32_e64 %9, %[c2], %9, %[q1], %[c2]\n\t"
      "v_subb_co_u32_e64 %2, %[c1], %2, %[p2], %[c1]\n\t"
      "v_subb_co_u32_e64 %10, %[c2], %10, %[q2], %[c2]\n\t"
      "v_subb_co_u32_e64 %3, %[c1], %3, %[p3], %[c1]\n\t"
      "v_subb_co_u32_e64 %11, %[c2], %11, %[q3], %[c2]\n\t"
      "v_subb_co_u32_e64 %4, %[c1], %4, %[p4], %[c1]\n\t"
      "v_subb_co_u32_e64 %12, %[c2], %12, %[q4], %[c2]\n\t"
      "v_subb_co_u32_e64 %5, %[c1], %5, %[p5], %[c1]\n\t"
      "v_subb_co_u32_e64 %13, %[c2], %13, %[q5], %[c2]\n\t"
      "v_subb_co_u32_e64 %6, %[c1], %6, %[p6], %[c1]\n\t"
      "v_subb_co_u32_e64 %14, %[c2], %14, %[q6], %[c2]\n\t"
      "v_subb_co_u32_e64 %7, %[c1], %7, %[p7], %[c1]\n\t"
      "v_subb_co_u32_e64 %15, %[c2], %15, %[q7], %[c2]\n\t"
      "v_cndmask_b32_e64 %[t], 0, 38, %[c1]\n\t"
      "v_cndmask_b32_e64 %[u], 0, 38, %[c2]\n\t"
      "v_sub_co_u32_e64 %0, %[c1], %0, %[t]\n\t"
      "v_sub_co_u32_e64 %8, %[c2], %8, %[u]\n\t"
      "s_or_b64 vcc, %[c1], %[c2]\n\t"
      COA_RARE_BEGIN
      "v_subbrev_co_u32_e64 %1, %[c1], 0, %1, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %9, %[c2], 0, %9, %[c2]\n\t"
      "v_subbrev_co_u32_e64 %2, %[c1], 0, %2, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %10, %[c2], 0, %10, %[c2]\n\t"
      "v_subbrev_co_u32_e64 %3, %[c1], 0, %3, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %11, %[c2], 0, %11, %[c2]\n\t"
      "v_subbrev_co_u32_e64 %4, %[c1], 0, %4, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %12, %[c2], 0, %12, %[c2]\n\t"
      "v_subbrev_co_u32_e64 %5, %[c1], 0, %5, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %13, %[c2], 0, %13, %[c2]\n\t"
      "v_subbrev_co_u32_e64 %6, %[c1], 0, %6, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %14, %[c2], 0, %14, %[c2]\n\t"
      "v_subbrev_co_u32_e64 %7, %[c1], 0, %7, %[c1]\n\t"
      "v_subbrev_co_u32_e64 %15, %[c2], 0, %15, %[c2]\n\t"
      "v_cndmask_b32_e64 %[t], 0, 38, %[c1]\n\t"
      "v_cndmask_b32_e64 %[u], 0, 38, %[c2]\n\t"
      "v_sub_u32_e32 %0, %0, %[t]\n\t"
      "v_sub_u32_e32 %8, %8, %[u]\n\t"
      COA_RARE_END
      : COA_R8_INOUT(x), COA_R8_INOUT(y), [t] "=&v"(t), [u] "=&v"(u), [c1] "=&s"(c1), [c2] "=&s"(c2)
      : [p0] "v"(b1.v[0]), [p1] "v"(b1.v[1]), [p2] "v"(b1.v[2]), [p3] "v"(b1.v[3]), [p4] "v"(b1.v[4]),
        [p5] "v"(b1.v[5]), [p6] "v"(b1.v[6]), [p7] "v"(b1.v[7]), [q0] "v"(b2.v[0]), [q1] "v"(b2.v[1]),
        [q2] "v"(b2.v[2]), [q3] "v"(b2.v[3]), [q4] "v"(b2.v[4]), [q5] "v"(b2.v[5]), [q6] "v"(b2.v[6]),
        [q7] "v"(b2.v[7])
      : "vcc", "scc");
  d1 = x;
  d2 = y;
}

}  // namespace

// V: 0 one chain, 1 two chains, 2 four chains, 3 two chains by fe_mul2,
//    4 four chains by two fe_mul2
template <int V>
__global__ void __launch_bounds__(256) k(fe* x, int n) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  fe a = x[id], b = x[id ^ 1], c = x[id ^ 2], e = x[id ^ 3], f = x[id ^ 4];
  for (int i = 0; i < n; i++) {
    if (V == 0) fe_mul(a, a, b);
    if (V == 1 || V == 2) {
      fe_mul(a, a, b);
      fe_mul(c, c, b);
    }
    if (V == 2) {
      fe_mul(e, e, b);
      fe_mul(f, f, b);
    }
    if (V == 3 || V == 4) fe_mul2(a, a, b, c, c, b);
    if (V == 4) fe_mul2(e, e, b, f, f, b);
    if (V == 5) {
      fe x[4] = {a, c, e, f}, y[4] = {b, b, b, b};
      fe_mul_n<4>(x, x, y);
      a = x[0]; c = x[1]; e = x[2]; f = x[3];
    }
    if (V == 6) fe_sq(a, a);
    if (V == 7 || V == 9) {
      fe_sq(a, a);
      fe_sq(c, c);
    }
    if (V == 9) {
      fe_sq(e, e);
      fe_sq(f, f);
    }
    if (V == 8) {
      fe x[2] = {a, c};
      fe_sq_n<2>(x, x);
      a = x[0]; c = x[1];
    }
    if (V == 10) {
      fe x[4] = {a, c, e, f};
      fe_sq_n<4>(x, x);
      a = x[0]; c = x[1]; e = x[2]; f = x[3];
    }
    if (V == 11) {
      fe s, t;
      fe_add(s, a, b);
      fe_sub(t, a, b);
      a = s;
      b = t;
    }
    if (V == 12) fe_addsub(a, b, a, b);
    if (V == 13) {
      fe s, t;
      fe_sub(s, a, b);
      fe_sub(t, b, c);
      a = s;
      b = t;
    }
    if (V == 14) fe_sub2(a, a, b, b, b, c);
  }
  if (V >= 11) fe_add(a, a, b);
  if (V >= 1 && V != 6 && V < 11) {
    fe_add(a, a, c);
    if (V == 2 || V == 4 || V == 5 || V == 9 || V == 10) {
      fe_add(a, a, e);
      fe_add(a, a, f);
    }
  }
  x[id] = a;
}

int main() {
  const int nthreads = 256 * 8 * 256;
  fe* h0 = (fe*)malloc(sizeof(fe) * nthreads);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < nthreads; i++)
    for (int j = 0; j < 8; j++) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      h0[i].v[j] = (uint32_t)s;
    }
  for (int i = 0; i < 8192; i++) {
    const int kind = i % 8;
    for (int j = 0; j < 8; j++) {
      uint32_t v = h0[i].v[j];
      if (kind == 0) v = 0xffffffffu;
      if (kind == 1) v = j == 0 ? 0xffffffedu - (i & 31) : (j == 7 ? 0x7fffffffu : 0xffffffffu);
      if (kind == 2) v = j == 0 ? 0xffffffffu - (i & 63) : 0xffffffffu;
      if (kind == 3) v = 0;
      if (kind == 4) v = j == (i / 8) % 8 ? 0xffffffffu : 0;
      if (kind == 5) v = j < 4 ? 0xffffffffu : v;
      h0[i].v[j] = v;
    }
  }
  fe *d, *ref;
  hipMalloc(&d, sizeof(fe) * nthreads);
  ref = (fe*)malloc(sizeof(fe) * nthreads);
  fe* got = (fe*)malloc(sizeof(fe) * nthreads);
  const int NV = 15;
  void (*ks[NV])(fe*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>, k<11>, k<12>, k<13>, k<14>};
  const char* names[NV] = {"mul 1 chain", "mul 2 chains", "mul 4 chains", "mul 2 by fe_mul2", "mul 4 by 2x fe_mul2",
                           "mul 4 by mul_n<4>", "sq 1 chain", "sq 2 chains", "sq 2 by sq_n<2>", "sq 4 chains",
                           "sq 4 by sq_n<4>", "add+sub", "fe_addsub", "sub+sub", "fe_sub2"};
  const int per[NV] = {1, 2, 4, 2, 4, 4, 1, 2, 2, 4, 4, 1, 1, 1, 1};
  const int cmp[NV] = {-1, -1, -1, 1, 2, 2, -1, -1, 7, -1, 9, -1, 11, -1, 13};  // variant that must agree
  // correctness: variants 1/3 and 2/4 must agree with each other
  for (int v = 0; v < NV; v++) {
    hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 5);
    hipMemcpy(got, d, sizeof(fe) * nthreads, hipMemcpyDeviceToHost);
    if (cmp[v] >= 0) {
      hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(ks[cmp[v]], dim3(nthreads / 256), dim3(256), 0, 0, d, 5);
      hipMemcpy(ref, d, sizeof(fe) * nthreads, hipMemcpyDeviceToHost);
      int bad = 0;
      for (int i = 0; i < nthreads; i++) bad += memcmp(&ref[i], &got[i], sizeof(fe)) != 0;
      printf("%-20s vs %-14s: %d lanes differ\n", names[v], names[cmp[v]], bad);
      if (bad) return 1;
    }
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int N = 1000;
  for (int waves = 1; waves <= 2; waves++) {
    for (int v = 0; v < NV; v++) {
      hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
      const int blocks = 256 * waves;
      hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, d, 10);
      hipDeviceSynchronize();
      float best = 1e30f;
      for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, d, N);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      const double ops = (double)blocks * 256 * N * per[v];
      printf("%d wave/SIMD %-20s %7.1f cyc per op per SIMD @2.4GHz\n", waves, names[v],
             (best * 1e-3) * 2.4e9 * 1024 / (ops / 64));
    }
  }
  return 0;
}
