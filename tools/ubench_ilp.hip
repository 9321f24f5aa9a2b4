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
  }
  if (V >= 1 && V != 6) {
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
  fe *d, *ref;
  hipMalloc(&d, sizeof(fe) * nthreads);
  ref = (fe*)malloc(sizeof(fe) * nthreads);
  fe* got = (fe*)malloc(sizeof(fe) * nthreads);
  const int NV = 11;
  void (*ks[NV])(fe*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>};
  const char* names[NV] = {"mul 1 chain", "mul 2 chains", "mul 4 chains", "mul 2 by fe_mul2", "mul 4 by 2x fe_mul2",
                           "mul 4 by mul_n<4>", "sq 1 chain", "sq 2 chains", "sq 2 by sq_n<2>", "sq 4 chains",
                           "sq 4 by sq_n<4>"};
  const int per[NV] = {1, 2, 4, 2, 4, 4, 1, 2, 2, 4, 4};
  const int cmp[NV] = {-1, -1, -1, 1, 2, 2, -1, -1, 7, -1, 9};  // variant that must agree
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
