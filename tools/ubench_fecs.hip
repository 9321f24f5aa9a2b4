// Field product A/B: tools/fe_comba.h (comba with a shifted 96-bit accumulator, two
// full carry folds) against coa_fe.h / coa_fe_cs.h (fresh 64-bit column accumulators
// with carry words, high columns folded by 38 as 64-bit mads, rare-branch
// top fold), plus fe_add / fe_sub with the second fold on a wave-uniform
// branch.  Every lane is checked against a host big-integer port after a
// chain of operations, on random, all-ones and near-p inputs (the latter
// drive the rare branches).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_fecs.hip -o tools/ubench_fecs
// (tools/fe_cs.h comes from tools/gen_fe_cs.py)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "fe_comba.h"

template <int V>
__global__ void k(fe* x, int n) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  fe a = x[id], b = x[id ^ 1];
  for (int i = 0; i < n; i++) {
    if (V == 0) fe_mul_comba(a, a, b);
    if (V == 1) fe_mul(a, a, b);
    if (V == 2) fecs::mul(a, a, b);
    if (V == 3) fe_sq_comba(a, a);
    if (V == 4) fe_sq(a, a);
    if (V == 5) fecs::sq(a, a);
    if (V == 6) { fe_add_comba(a, a, b); fe_add_comba(b, a, b); }
    if (V == 7) { fe_add(a, a, b); fe_add(b, a, b); }
    if (V == 8) { fe_sub_comba(a, a, b); fe_sub_comba(b, b, a); }
    if (V == 9) { fe_sub(a, a, b); fe_sub(b, b, a); }
  }
  x[id] = a;
}

// ---- host big-integer port (16 x 32-bit words, mod p)
typedef unsigned __int128 u128;
static void canon16(uint32_t* r, const uint32_t* w16) {
  // reduce a 512-bit value mod p = 2^255 - 19
  uint64_t x[17] = {0};
  for (int i = 0; i < 16; i++) x[i] = w16[i];
  for (int rep = 0; rep < 4; rep++) {
    // fold words 8..15 by 38 (2^256 == 38)
    u128 acc = 0;
    uint64_t z[17] = {0};
    for (int i = 0; i < 8; i++) {
      acc += (u128)x[i] + (u128)x[i + 8] * 38u;
      z[i] = (uint32_t)acc;
      acc >>= 32;
    }
    z[8] = (uint64_t)acc;
    for (int i = 0; i < 17; i++) x[i] = z[i];
  }
  for (int rep = 0; rep < 3; rep++) {
    uint64_t top = (x[7] >> 31) + (x[8] << 1);
    x[7] &= 0x7fffffff;
    x[8] = 0;
    u128 e = (u128)top * 19;
    for (int i = 0; i < 8; i++) {
      e += x[i];
      x[i] = (uint32_t)e;
      e >>= 32;
    }
    x[8] = (uint64_t)e;
  }
  bool ge = (x[7] == 0x7fffffff);
  for (int i = 6; i >= 1 && ge; i--) ge = x[i] == 0xffffffff;
  if (ge) ge = x[0] >= 0xffffffed;
  if (ge) {
    x[0] -= 0xffffffed;
    for (int i = 1; i < 8; i++) x[i] = 0;
  }
  for (int i = 0; i < 8; i++) r[i] = (uint32_t)x[i];
}
static void hmul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  u128 t[17] = {0};
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) t[i + j] += (u128)a[i] * b[j];
  uint32_t w[16];
  u128 c = 0;
  for (int i = 0; i < 16; i++) {
    c += t[i];
    w[i] = (uint32_t)c;
    c >>= 32;
  }
  canon16(r, w);
}
static void hadd(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t w[16] = {0};
  uint64_t c = 0;
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)a[i] + b[i];
    w[i] = (uint32_t)c;
    c >>= 32;
  }
  w[8] = (uint32_t)c;
  canon16(r, w);
}
static void hsub(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  // a + 4p - b, 4p = 2^257 - 76
  uint32_t fp[9] = {0xffffffb4u, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                    0xffffffffu, 0xffffffffu, 0xffffffffu, 1u};
  uint32_t w[16] = {0};
  int64_t c = 0;
  for (int i = 0; i < 9; i++) {
    c += (int64_t)(i < 8 ? a[i] : 0) + fp[i] - (int64_t)(i < 8 ? b[i] : 0);
    w[i] = (uint32_t)c;
    c >>= 32;
  }
  canon16(r, w);
}

int main() {
  const int nthreads = 256 * 8 * 256;
  fe* h0 = (fe*)malloc(sizeof(fe) * nthreads);
  fe* h = (fe*)malloc(sizeof(fe) * nthreads);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < nthreads; i++)
    for (int j = 0; j < 8; j++) {
      s ^= s << 13;
      s ^= s >> 7;
      s ^= s << 17;
      h0[i].v[j] = (uint32_t)s;
    }
  // carry-heavy lanes: all ones, p - small, 2^256 - small, zero, single words
  for (int i = 0; i < 4096; i++) {
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
  fe* d;
  hipMalloc(&d, sizeof(fe) * nthreads);
  const int NV = 10;
  void (*ks[NV])(fe*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>};
  const char* names[NV] = {"mul r1 (2 folds)", "mul (rare fold)", "mul carry-save", "sq r1 (2 folds)",
                           "sq (rare fold)", "sq carry-save", "add x2 r1", "add x2 rare-br",
                           "sub x2 r1", "sub x2 rare-br"};
  const int reps = 3;
  int total_bad = 0;
  for (int v = 0; v < NV; v++) {
    hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, reps);
    hipMemcpy(h, d, sizeof(fe) * nthreads, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 65536; i++) {
      uint32_t a[8], b[8];
      for (int j = 0; j < 8; j++) {
        a[j] = h0[i].v[j];
        b[j] = h0[i ^ 1].v[j];
      }
      for (int r = 0; r < reps; r++) {
        uint32_t t[8];
        if (v <= 2) hmul(t, a, b), memcpy(a, t, 32);
        else if (v <= 5) hmul(t, a, a), memcpy(a, t, 32);
        else if (v <= 7) { hadd(t, a, b); memcpy(a, t, 32); hadd(t, a, b); memcpy(b, t, 32); }
        else { hsub(t, a, b); memcpy(a, t, 32); hsub(t, b, a); memcpy(b, t, 32); }
      }
      uint32_t g[8], w16[16] = {0};
      for (int j = 0; j < 8; j++) w16[j] = h[i].v[j];
      canon16(g, w16);
      uint32_t want[8], wa[16] = {0};
      for (int j = 0; j < 8; j++) wa[j] = a[j];
      canon16(want, wa);
      if (memcmp(g, want, 32)) bad++;
    }
    total_bad += bad;
    printf("%-16s correctness: %d bad of 65536\n", names[v], bad);
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int N = 2000;
  for (int waves = 1; waves <= 8; waves *= 2) {
    for (int v = 0; v < NV; v++) {
      hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
      const int blocks = 256 * waves;
      hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, d, 10);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, d, N);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double ops = (double)blocks * 256 * N * (v >= 6 ? 2 : 1);
      printf("%d wave/SIMD %-16s %7.1f cyc/wave-op per SIMD @2.4GHz\n", waves, names[v],
             (ms * 1e-3) * 2.4e9 * 1024 / (ops / 64));
    }
  }
  return total_bad ? 1 : 0;
}
