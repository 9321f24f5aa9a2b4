// Field-multiply issue cost: per-product asm (one hipcc s_nop pad per
// product) vs the per-column asm of coa_fe.h, plus a column variant padded
// with `s_nop 1` between each mad and its carry read (LLVM's gfx950 model for
// VALU SGPR write -> VALU SGPR read).  Build: hipcc --offload-arch=gfx950 -O3
// -std=c++17 tools/ubench_fe3.hip -o tools/ubench_fe3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdlib>
#include "../xrpl-coa-prototype_amd/csrc/coa_fe.h"

COA_DEV void mac0_old(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t sc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, 0, %1"
      : "+v"(acc), "=&s"(sc), "=v"(c2) : "v"(a), "v"(b));
}
COA_DEV void fe_mul_old(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j < 0 || j > 7) continue;
      if (first) { mac0_old(acc, c2, a.v[i], b.v[j]); first = false; } else mac(acc, c2, a.v[i], b.v[j]); }
    t[k] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)c2 << 32);
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}
COA_DEV void mac_nop(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t sc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(sc), "+v"(c2) : "v"(a), "v"(b));
}
COA_DEV void fe_mul_nop(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint32_t c2 = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j < 0 || j > 7) continue; mac_nop(acc, c2, a.v[i], b.v[j]); }
    t[k] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)c2 << 32);
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

// VCC-carry column: the e32 addc reads VCC implicitly (no wait states in any
// model), and is a 4-byte encoding.  The first product's carry word comes from
// 0 + zero-register + carry.
#define VMAD0(X, Y) "v_mad_u64_u32 %0, vcc, %" #X ", %" #Y ", %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %2, vcc\n\t"
#define VMADC(X, Y) "v_mad_u64_u32 %0, vcc, %" #X ", %" #Y ", %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
template <int P>
COA_DEV void colv(uint64_t& acc, uint32_t& c2, const uint32_t* x, const uint32_t* y) {
  const uint32_t z = 0;
  if constexpr (P == 1) asm(VMAD0(3, 4) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]) : "vcc");
  else if constexpr (P == 2) asm(VMAD0(3, 4) VMADC(5, 6) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]) : "vcc");
  else if constexpr (P == 3) asm(VMAD0(3, 4) VMADC(5, 6) VMADC(7, 8) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]) : "vcc");
  else if constexpr (P == 4) asm(VMAD0(3, 4) VMADC(5, 6) VMADC(7, 8) VMADC(9, 10) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]) : "vcc");
  else if constexpr (P == 5) asm(VMAD0(3, 4) VMADC(5, 6) VMADC(7, 8) VMADC(9, 10) VMADC(11, 12) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]), "v"(y[4]) : "vcc");
  else if constexpr (P == 6) asm(VMAD0(3, 4) VMADC(5, 6) VMADC(7, 8) VMADC(9, 10) VMADC(11, 12) VMADC(13, 14) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]), "v"(y[4]), "v"(x[5]), "v"(y[5]) : "vcc");
  else if constexpr (P == 7) asm(VMAD0(3, 4) VMADC(5, 6) VMADC(7, 8) VMADC(9, 10) VMADC(11, 12) VMADC(13, 14) VMADC(15, 16) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]), "v"(y[4]), "v"(x[5]), "v"(y[5]), "v"(x[6]), "v"(y[6]) : "vcc");
  else asm(VMAD0(3, 4) VMADC(5, 6) VMADC(7, 8) VMADC(9, 10) VMADC(11, 12) VMADC(13, 14) VMADC(15, 16) VMADC(17, 18) : "+v"(acc), "=&v"(c2) : "v"(z), "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]), "v"(x[4]), "v"(y[4]), "v"(x[5]), "v"(y[5]), "v"(x[6]), "v"(y[6]), "v"(x[7]), "v"(y[7]) : "vcc");
}
template <int K>
COA_DEV void vcols(uint32_t* t, uint64_t& acc, const fe& a, const fe& b) {
  if constexpr (K < 15) {
    constexpr int lo = K < 8 ? 0 : K - 7, hi = K < 8 ? K : 7, P = hi - lo + 1;
    uint32_t x[P], y[P];
#pragma unroll
    for (int p = 0; p < P; p++) { x[p] = a.v[lo + p]; y[p] = b.v[K - lo - p]; }
    uint32_t c2;
    colv<P>(acc, c2, x, y);
    t[K] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c2 << 32);
    vcols<K + 1>(t, acc, a, b);
  }
}
COA_DEV void fe_mul_vcc(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0;
  vcols<0>(t, acc, a, b);
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

template <int V>
__global__ void k(fe* x, int n) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  fe a = x[id], b = x[id ^ 1];
  for (int i = 0; i < n; i++) {
    if (V == 0) fe_mul_old(a, a, b);
    if (V == 1) fe_mul(a, a, b);
    if (V == 2) fe_sq(a, a);
    if (V == 3) fe_mul_nop(a, a, b);
    if (V == 4) fe_mul_vcc(a, a, b);
  }
  x[id] = a;
}
static void ref_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  unsigned __int128 t[17] = {0};
  for (int i = 0; i < 8; i++) for (int j = 0; j < 8; j++) t[i + j] += (unsigned __int128)a[i] * b[j];
  uint32_t w[17]; unsigned __int128 c = 0;
  for (int i = 0; i < 16; i++) { c += t[i]; w[i] = (uint32_t)c; c >>= 32; }
  uint64_t x[9] = {0}; uint64_t cc = 0;
  for (int i = 0; i < 8; i++) { cc += (uint64_t)w[i] + (uint64_t)w[i + 8] * 38; x[i] = (uint32_t)cc; cc >>= 32; }
  uint64_t d = cc * 38;
  for (int i = 0; i < 8; i++) { d += x[i]; x[i] = (uint32_t)d; d >>= 32; }
  x[0] += d * 38;
  for (int rep = 0; rep < 3; rep++) {
    uint64_t top = x[7] >> 31; x[7] &= 0x7fffffff; uint64_t e = top * 19;
    for (int i = 0; i < 8; i++) { e += x[i]; x[i] = (uint32_t)e; e >>= 32; }
  }
  bool ge = (x[7] == 0x7fffffff); for (int i = 6; i >= 1 && ge; i--) ge = x[i] == 0xffffffff; if (ge) ge = x[0] >= 0xffffffed;
  if (ge) { x[0] -= 0xffffffed; for (int i = 1; i < 7; i++) x[i] = 0; x[7] = 0; }
  for (int i = 0; i < 8; i++) r[i] = (uint32_t)x[i];
}
static void canon(uint32_t* v) { uint32_t one[8] = {1,0,0,0,0,0,0,0}, t[8]; ref_mul(t, v, one); for (int i = 0; i < 8; i++) v[i] = t[i]; }
int main() {
  const int nthreads = 256 * 8 * 256;
  fe* h = (fe*)malloc(sizeof(fe) * nthreads); fe* h0 = (fe*)malloc(sizeof(fe) * nthreads);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < nthreads; i++) for (int j = 0; j < 8; j++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h0[i].v[j] = (uint32_t)s; }
  for (int i = 0; i < 64; i++) for (int j = 0; j < 8; j++) h0[i].v[j] = 0xffffffffu;
  fe* d; hipMalloc(&d, sizeof(fe) * nthreads);
  void (*ks[5])(fe*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>};
  const char* names[5] = {"mul_per_product_asm", "mul_per_column_asm", "sq_per_column_asm", "mul_snop1_padded", "mul_vcc_column"};
  int total_bad = 0;
  for (int v = 0; v < 5; v++) {
    hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 3);
    hipMemcpy(h, d, sizeof(fe) * nthreads, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 16384; i++) {
      uint32_t a[8], b[8]; for (int j = 0; j < 8; j++) { a[j] = h0[i].v[j]; b[j] = h0[i ^ 1].v[j]; }
      for (int r = 0; r < 3; r++) { uint32_t t[8]; if (v == 2) ref_mul(t, a, a); else ref_mul(t, a, b); for (int j = 0; j < 8; j++) a[j] = t[j]; }
      uint32_t g[8]; for (int j = 0; j < 8; j++) g[j] = h[i].v[j]; canon(g);
      for (int j = 0; j < 8; j++) if (g[j] != a[j]) { bad++; break; }
    }
    total_bad += bad;
    printf("%s correctness: %d bad of 16384\n", names[v], bad);
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int N = 2000;
  for (int v = 0; v < 5; v++) {
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 10); hipDeviceSynchronize();
    for (int occ = 0; occ < 1; occ++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, N);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double ops = (double)nthreads * N;
      printf("%-22s %8.2f G fe-ops/s  %7.1f cyc/wave-op/SIMD @2.4GHz\n", names[v], ops / (ms * 1e-3) / 1e9,
             (ms * 1e-3) * 2.4e9 * 1024 / (ops / 64));
    }
  }
  // one wave per SIMD (the C2 occupancy): 1024 waves
  for (int v = 0; v < 5; v++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[v], dim3(256), dim3(256), 0, 0, d, N);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double ops = 65536.0 * N;
    printf("1wave/SIMD %-22s %7.1f cyc/wave-op\n", names[v], (ms * 1e-3) * 2.4e9 * 1024 / (ops / 64));
  }
  return total_bad ? 1 : 0;
}
