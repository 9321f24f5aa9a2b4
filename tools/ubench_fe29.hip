// Radix-2^29 probe: 9 limbs of 29 bits (261 bits), every product column
// accumulated in 64 bits by plain v_mad_u64_u32 chains with no carry flags
// (a column holds at most 9 products < 2^60.0), against the radix-2^32 comba
// of coa_fe.h.  Reports cycles per multiply / squaring at 8 and at 1 wave per
// SIMD (the C2 occupancy) and checks results against a host big-int model.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_fe29.hip -o tools/ubench_fe29
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../xrpl-coa-prototype_amd/csrc/coa_fe.h"

struct fe9 {
  uint32_t v[9];
};
#define M29 0x1fffffffu
#define M23 0x7fffffu

COA_DEV uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// t[0..16] (column sums) -> h.  2^261 == 64 * 19 = 1216, 2^255 == 19.
// Output: limbs < 2^29 except h1 < 2^29 + 2^17 and h8 < 2^23.
COA_DEV void red9(fe9& h, uint64_t* t) {
  uint64_t t17;
#pragma unroll
  for (int k = 9; k < 16; k++) {
    t[k + 1] += t[k] >> 29;
    t[k] = (uint32_t)t[k] & M29;
  }
  t17 = t[16] >> 29;
  t[16] = (uint32_t)t[16] & M29;
#pragma unroll
  for (int k = 9; k < 17; k++) t[k - 9] = mad((uint32_t)t[k], 1216u, t[k - 9]);
  t[8] = mad((uint32_t)t17, 1216u, t[8]);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    t[k + 1] += t[k] >> 29;
    t[k] = (uint32_t)t[k] & M29;
  }
  const uint64_t c = t[8] >> 23;
  t[8] = (uint32_t)t[8] & M23;
  t[0] = mad((uint32_t)c, 19u, t[0]);
  t[1] = mad((uint32_t)(c >> 32), 152u, t[1]);
  t[1] += t[0] >> 29;
  t[0] = (uint32_t)t[0] & M29;
#pragma unroll
  for (int i = 0; i < 9; i++) h.v[i] = (uint32_t)t[i];
}

COA_DEV void fe9_mul(fe9& h, const fe9& f, const fe9& g) {
  uint64_t t[17];
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j < 0 || j > 8) continue;
      acc = mad(f.v[i], g.v[j], acc);
    }
    t[k] = acc;
  }
  red9(h, t);
}

COA_DEV void fe9_sq(fe9& h, const fe9& f) {
  uint32_t f2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) f2[i] = f.v[i] << 1;
  uint64_t t[17];
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j <= i || j > 8) continue;
      acc = mad(f2[i], f.v[j], acc);
    }
    if ((k & 1) == 0 && k / 2 <= 8) acc = mad(f.v[k / 2], f.v[k / 2], acc);
    t[k] = acc;
  }
  red9(h, t);
}

template <int V>
__global__ void k(uint32_t* x, int n) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (V < 2) {
    fe9 a, b;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a.v[i] = x[(size_t)id * 10 + i];
      b.v[i] = x[(size_t)(id ^ 1) * 10 + i];
    }
    for (int r = 0; r < n; r++) {
      if (V == 0) fe9_mul(a, a, b);
      else fe9_sq(a, a);
    }
#pragma unroll
    for (int i = 0; i < 9; i++) x[(size_t)id * 10 + i] = a.v[i];
  } else {
    fe a, b;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a.v[i] = x[(size_t)id * 10 + i];
      b.v[i] = x[(size_t)(id ^ 1) * 10 + i];
    }
    for (int r = 0; r < n; r++) {
      if (V == 2) fe_mul(a, a, b);
      else fe_sq(a, a);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) x[(size_t)id * 10 + i] = a.v[i];
  }
}

// ------------------------------------------------------------ host model
typedef unsigned __int128 u128;
static void to_int(uint64_t out[5], const uint32_t* l) {  // sum l_i 2^(29 i) < 2^320
  memset(out, 0, 40);
  for (int i = 0; i < 9; i++) {
    const int sh = 29 * i, w = sh / 64, b = sh % 64;
    u128 v = (u128)l[i] << b;
    u128 c = 0;
    for (int k = w; k < 5; k++) {
      c += (u128)out[k] + (uint64_t)v;
      out[k] = (uint64_t)c;
      c >>= 64;
      v >>= 64;
    }
  }
}
static void modp(uint64_t x[5]) {  // x < 2^320 -> x mod p
  for (int rep = 0; rep < 4; rep++) {
    uint64_t hi[3] = {(x[3] >> 63) | (x[4] << 1), x[4] >> 63, 0};
    x[3] &= 0x7fffffffffffffffull;
    x[4] = 0;
    u128 c = 0;
    for (int k = 0; k < 5; k++) {
      c += (u128)x[k] + (k < 3 ? (u128)hi[k] * 19 : 0);
      x[k] = (uint64_t)c;
      c >>= 64;
    }
  }
  const uint64_t p[4] = {0xffffffffffffffedull, ~0ull, ~0ull, 0x7fffffffffffffffull};
  bool ge = true;
  for (int k = 3; k >= 0; k--)
    if (x[k] != p[k]) {
      ge = x[k] > p[k];
      break;
    }
  if (ge) {
    uint64_t b = 0;
    for (int k = 0; k < 4; k++) {
      u128 d = (u128)x[k] - p[k] - b;
      x[k] = (uint64_t)d;
      b = (d >> 64) ? 1 : 0;
    }
  }
}
static void mulmod(uint64_t r[5], const uint64_t a[5], const uint64_t b[5]) {
  uint64_t prod[9] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a[i] * b[j] + prod[i + j];
      prod[i + j] = (uint64_t)c;
      c >>= 64;
    }
    prod[i + 4] += (uint64_t)c;
  }
  uint64_t x[5] = {0};
  u128 c = 0;
  for (int k = 0; k < 4; k++) {
    c += (u128)prod[k] + (u128)prod[k + 4] * 38;
    x[k] = (uint64_t)c;
    c >>= 64;
  }
  x[4] = (uint64_t)c;
  modp(x);
  for (int k = 0; k < 5; k++) r[k] = x[k];
}

int main() {
  const int nthreads = 256 * 8 * 256;
  uint32_t* h0 = (uint32_t*)malloc(sizeof(uint32_t) * 10 * nthreads);
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * 10 * nthreads);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < nthreads * 10; i++) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    // worst-case inputs for the 9-limb kernels: limbs up to 2^30 (a lazy sum)
    h0[i] = (uint32_t)s & ((i % 10) == 8 ? 0xffffffu : 0x3fffffffu);
  }
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * 10 * nthreads);
  void (*ks[4])(uint32_t*, int) = {k<0>, k<1>, k<2>, k<3>};
  const char* names[4] = {"fe9_mul (radix 2^29)", "fe9_sq  (radix 2^29)", "fe_mul  (radix 2^32)",
                          "fe_sq   (radix 2^32)"};
  int bad = 0;
  for (int v = 0; v < 2; v++) {
    hipMemcpy(d, h0, sizeof(uint32_t) * 10 * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 1);
    hipMemcpy(h, d, sizeof(uint32_t) * 10 * nthreads, hipMemcpyDeviceToHost);
    int b = 0, bnd = 0;
    for (int i = 0; i < nthreads; i++) {
      uint64_t a[5], bb[5], g[5];
      to_int(a, h0 + (size_t)i * 10);
      modp(a);
      to_int(bb, h0 + (size_t)(i ^ 1) * 10);
      modp(bb);
      mulmod(a, a, v == 0 ? bb : a);
      const uint32_t* o = h + (size_t)i * 10;
      to_int(g, o);
      modp(g);
      if (memcmp(a, g, 32)) b++;
      for (int l = 0; l < 9; l++)
        if (o[l] >= (l == 8 ? (1u << 23) : l == 1 ? (1u << 29) + (1u << 17) : (1u << 29))) bnd++;
    }
    printf("%s correctness: %d bad, %d out-of-bound limbs of %d (one op, worst-case inputs)\n", names[v], b, bnd,
           nthreads);
    bad += b + bnd;
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int N = 2000;
  for (int v = 0; v < 4; v++) {
    hipMemcpy(d, h0, sizeof(uint32_t) * 10 * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 10);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, N);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)nthreads * N;
    float msw[3];
    const int wv[3] = {1, 2, 4};
    for (int q = 0; q < 3; q++) {
      hipMemcpy(d, h0, sizeof(uint32_t) * 10 * nthreads, hipMemcpyHostToDevice);
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[v], dim3(256 * wv[q]), dim3(256), 0, 0, d, N);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&msw[q], e0, e1);
    }
    // cycles per op per SIMD (SIMD throughput), and per wave
    printf("%-24s SIMD cycles per op: 8 waves %6.1f | 4 waves %6.1f | 2 waves %6.1f | 1 wave %6.1f\n", names[v],
           (ms * 1e-3) * 2.4e9 * 1024 / (ops / 64), (msw[2] * 1e-3) * 2.4e9 / (4.0 * N),
           (msw[1] * 1e-3) * 2.4e9 / (2.0 * N), (msw[0] * 1e-3) * 2.4e9 / (1.0 * N));
  }
  return bad ? 1 : 0;
}
