// Radix-2^25.5 field arithmetic probe: 10 limbs (26/25 bits alternating),
// every column of a product accumulated in 64 bits by independent
// v_mad_u64_u32 chains (no carry flags), against the radix-2^32 comba of
// coa_fe.h.  Reports cycles per multiply / squaring at 8 and at 1 wave per
// SIMD (the C2 occupancy) and checks results against a host big-int model.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_fe10.hip -o tools/ubench_fe10
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../xrpl-coa-prototype_amd/csrc/coa_fe.h"

struct fe10 {
  uint32_t v[10];
};
#define M26 0x3ffffffu
#define M25 0x1ffffffu

COA_DEV uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// h = f * g mod p; inputs limbs < 2^27, output carried (limb < 2^26 / 2^25,
// limb 1 may exceed by a carry of the last fold)
COA_DEV void carry10(fe10& h, uint64_t* t) {
  // interleaved carry chains (two independent halves), as ref10
  uint64_t c;
  c = t[0] >> 26; t[1] += c; t[0] &= M26;
  c = t[4] >> 26; t[5] += c; t[4] &= M26;
  c = t[1] >> 25; t[2] += c; t[1] &= M25;
  c = t[5] >> 25; t[6] += c; t[5] &= M25;
  c = t[2] >> 26; t[3] += c; t[2] &= M26;
  c = t[6] >> 26; t[7] += c; t[6] &= M26;
  c = t[3] >> 25; t[4] += c; t[3] &= M25;
  c = t[7] >> 25; t[8] += c; t[7] &= M25;
  c = t[4] >> 26; t[5] += c; t[4] &= M26;
  c = t[8] >> 26; t[9] += c; t[8] &= M26;
  c = t[9] >> 25; t[0] += c * 19; t[9] &= M25;
  c = t[0] >> 26; t[1] += c; t[0] &= M26;
#pragma unroll
  for (int i = 0; i < 10; i++) h.v[i] = (uint32_t)t[i];
}

COA_DEV void fe10_mul(fe10& h, const fe10& f, const fe10& g) {
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  uint64_t t[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      const uint32_t fi = ((i & 1) && (j & 1)) ? f2[i] : f.v[i];
      acc = mad(fi, wrap ? g19[j] : g.v[j], acc);
    }
    t[k] = acc;
  }
  carry10(h, t);
}

COA_DEV void fe10_sq(fe10& h, const fe10& f) {
  uint32_t f2[10], f19[10], f38[10];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    f2[i] = 2u * f.v[i];
    f19[i] = 19u * f.v[i];
    f38[i] = 38u * f.v[i];
  }
  uint64_t t[10];
#pragma unroll
  for (int k = 0; k < 10; k++) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      const bool wrap = j < 0;
      if (wrap) j += 10;
      if (j < i) continue;  // each unordered pair once
      const bool odd2 = (i & 1) && (j & 1);
      if (i == j) {  // f_i^2 * (odd ? 2 : 1) * (wrap ? 19 : 1)
        const uint32_t a = odd2 ? f2[i] : f.v[i];
        acc = mad(a, wrap ? f19[i] : f.v[i], acc);
      } else {  // 2 f_i f_j * (odd ? 2 : 1) * (wrap ? 19 : 1)
        const uint32_t a = odd2 ? f2[i] : f.v[i];
        const uint32_t b = wrap ? f38[j] : f2[j];
        acc = mad(a, b, acc);
      }
    }
    t[k] = acc;
  }
  carry10(h, t);
}

template <int V>
__global__ void k(uint32_t* x, int n) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (V < 2) {
    fe10 a, b;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      a.v[i] = x[(size_t)id * 10 + i];
      b.v[i] = x[(size_t)(id ^ 1) * 10 + i];
    }
    for (int r = 0; r < n; r++) {
      if (V == 0) fe10_mul(a, a, b);
      else fe10_sq(a, a);
    }
#pragma unroll
    for (int i = 0; i < 10; i++) x[(size_t)id * 10 + i] = a.v[i];
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

// host model: value of a 10-limb element mod p as 4 x u64 (little endian)
typedef unsigned __int128 u128;
static void to_int(uint64_t out[5], const uint32_t* l) {  // sum l_i 2^ceil(25.5 i), < 2^320
  static const int sh[10] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230};
  memset(out, 0, 40);
  for (int i = 0; i < 10; i++) {
    const int w = sh[i] / 64, b = sh[i] % 64;
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
static void modp(uint64_t x[5]) {  // reduce a < 2^320 value mod p = 2^255 - 19
  for (int rep = 0; rep < 4; rep++) {
    // x = lo255 + hi * 19
    uint64_t hi[5];
    for (int k = 0; k < 5; k++) hi[k] = 0;
    for (int k = 3; k < 5; k++) {
      hi[k - 3] |= x[k] >> 63;
      if (k + 1 < 5) hi[k - 3] |= 0;  // filled below
    }
    // hi = x >> 255
    for (int k = 0; k < 2; k++) hi[k] = (x[3 + k] >> 63) | (k + 4 < 5 ? (x[4 + k] << 1) : 0);
    hi[2] = 0;
    x[3] &= 0x7fffffffffffffffull;
    x[4] = 0;
    u128 c = 0;
    for (int k = 0; k < 5; k++) {
      c += (u128)x[k] + (k < 3 ? (u128)hi[k] * 19 : 0);
      x[k] = (uint64_t)c;
      c >>= 64;
    }
  }
  // final conditional subtract
  const uint64_t p[4] = {0xffffffffffffffedull, 0xffffffffffffffffull, 0xffffffffffffffffull,
                         0x7fffffffffffffffull};
  bool ge = true;
  for (int k = 3; k >= 0; k--) {
    if (x[k] != p[k]) {
      ge = x[k] > p[k];
      break;
    }
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
  u128 t[9] = {0};
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
  (void)t;
  // prod (512 bits) mod p: lo + hi * 38
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
    h0[i] = (uint32_t)s & ((i % 10) & 1 ? M25 : M26);
  }
  uint32_t* d;
  hipMalloc(&d, sizeof(uint32_t) * 10 * nthreads);
  void (*ks[4])(uint32_t*, int) = {k<0>, k<1>, k<2>, k<3>};
  const char* names[4] = {"fe10_mul (radix 2^25.5)", "fe10_sq  (radix 2^25.5)", "fe_mul   (radix 2^32)",
                          "fe_sq    (radix 2^32)"};
  int bad = 0;
  for (int v = 0; v < 2; v++) {
    hipMemcpy(d, h0, sizeof(uint32_t) * 10 * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 3);
    hipMemcpy(h, d, sizeof(uint32_t) * 10 * nthreads, hipMemcpyDeviceToHost);
    int b = 0;
    for (int i = 0; i < 4096; i++) {
      uint64_t a[5], bb[5], g[5];
      to_int(a, h0 + (size_t)i * 10);
      modp(a);
      to_int(bb, h0 + (size_t)(i ^ 1) * 10);
      modp(bb);
      for (int r = 0; r < 3; r++) mulmod(a, a, v == 0 ? bb : a);
      to_int(g, h + (size_t)i * 10);
      modp(g);
      if (memcmp(a, g, 32)) b++;
    }
    printf("%s correctness: %d bad of 4096\n", names[v], b);
    bad += b;
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
    hipMemcpy(d, h0, sizeof(uint32_t) * 10 * nthreads, hipMemcpyHostToDevice);
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[v], dim3(256), dim3(256), 0, 0, d, N);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms1;
    hipEventElapsedTime(&ms1, e0, e1);
    printf("%-26s 8 waves/SIMD: %7.1f cyc/wave-op   1 wave/SIMD: %7.1f cyc/wave-op\n", names[v],
           (ms * 1e-3) * 2.4e9 * 1024 / (ops / 64), (ms1 * 1e-3) * 2.4e9 * 1024 / (65536.0 * N / 64));
  }
  return bad ? 1 : 0;
}
