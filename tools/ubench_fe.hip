#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
struct fe { uint32_t v[8]; };
// comba MAC: (acc:64, c2:32) += a*b using mad carry-out
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t sc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(sc), "+v"(c2) : "v"(a), "v"(b));
}
__device__ __forceinline__ void fe_reduce512(fe& r, const uint32_t* t) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) { c = (uint64_t)t[8+i] * 38u + (c >> 32) + t[i]; r.v[i] = (uint32_t)c; }
  uint64_t d = (uint32_t)(c >> 32) * 38u;
#pragma unroll
  for (int i = 0; i < 8; i++) { d += r.v[i]; r.v[i] = (uint32_t)d; d >>= 32; }
  r.v[0] += (uint32_t)d * 38u;
}
__device__ __forceinline__ void fe_mul_asm(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j < 0 || j > 7) continue; mac(acc, c2, a.v[i], b.v[j]); }
    t[k] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)c2 << 32); c2 = 0;
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}
__device__ __forceinline__ void fe_mul_c(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j < 0 || j > 7) continue;
      uint64_t p = (uint64_t)a.v[i] * b.v[j]; acc += p; c2 += (acc < p); }
    t[k] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)c2 << 32); c2 = 0;
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}
// operand scanning: row i: t[i+j] += a_i*b_j + carry
__device__ __forceinline__ void fe_mul_os(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
#pragma unroll
  for (int j = 0; j < 16; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) { c = (uint64_t)a.v[i] * b.v[j] + t[i+j] + (c >> 32); t[i+j] = (uint32_t)c; }
    t[i+8] = (uint32_t)(c >> 32);
  }
  fe_reduce512(r, t);
}
// squaring via comba: cross products doubled
__device__ __forceinline__ void fe_sq_asm(fe& r, const fe& a) {
  uint32_t t[16];
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint64_t x = 0; uint32_t x2 = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j <= i || j > 7) continue; mac(x, x2, a.v[i], a.v[j]); }
    // double cross sum (x2:x) and add to acc
    x2 = (x2 << 1) | (uint32_t)(x >> 63); x <<= 1;
    if ((k & 1) == 0) mac(x, x2, a.v[k/2], a.v[k/2]);
    uint64_t s = acc + x; x2 += c2 + (s < x); 
    t[k] = (uint32_t)s; acc = (s >> 32) | ((uint64_t)x2 << 32); c2 = 0;
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}

__device__ __forceinline__ void mac0(uint64_t& acc, uint32_t& c2, uint32_t a, uint32_t b) {
  uint64_t sc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, 0, %1"
      : "+v"(acc), "=&s"(sc), "=v"(c2) : "v"(a), "v"(b));
}
__device__ __forceinline__ void fe_mul_asm2(fe& r, const fe& a, const fe& b) {
  uint32_t t[16];
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j < 0 || j > 7) continue;
      if (first) { mac0(acc, c2, a.v[i], b.v[j]); first = false; } else mac(acc, c2, a.v[i], b.v[j]); }
    t[k] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)c2 << 32);
  }
  t[15] = (uint32_t)acc;
  fe_reduce512(r, t);
}
__device__ __forceinline__ uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t& cout) {
  unsigned int c; uint32_t r = __builtin_addc(a, b, cin, &c); cout = c; return r;
}
__device__ __forceinline__ void fe_sq2(fe& r, const fe& a) {
  uint32_t t[16];
  t[0] = 0;
  uint64_t acc = 0; uint32_t c2 = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
    bool first = true;
#pragma unroll
    for (int i = 0; i < 8; i++) { int j = k - i; if (j <= i || j > 7) continue;
      if (first) { mac0(acc, c2, a.v[i], a.v[j]); first = false; } else mac(acc, c2, a.v[i], a.v[j]); }
    t[k] = (uint32_t)acc; acc = (acc >> 32) | ((uint64_t)c2 << 32);
  }
  t[14] = (uint32_t)acc; t[15] = (uint32_t)(acc >> 32);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = addc32(t[i], t[i], c, c);
  uint32_t d[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { uint64_t p = (uint64_t)a.v[i] * a.v[i]; d[2*i] = (uint32_t)p; d[2*i+1] = (uint32_t)(p >> 32); }
  c = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) t[i] = addc32(t[i], d[i], c, c);
  fe_reduce512(r, t);
}

template <int V>
__global__ void k(fe* x, int n) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  fe a = x[id], b = x[id ^ 1];
  for (int i = 0; i < n; i++) {
    if (V == 0) fe_mul_asm(a, a, b);
    if (V == 1) fe_mul_c(a, a, b);
    if (V == 2) fe_mul_os(a, a, b);
    if (V == 3) fe_sq_asm(a, a);
    if (V == 4) fe_mul_asm2(a, a, b);
    if (V == 5) fe_sq2(a, a);
  }
  x[id] = a;
}
// host reference mul mod p via 8x32 schoolbook with __int128 then compare numerically (value mod p)
static void ref_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  // big-int via unsigned __int128 columns
  unsigned __int128 t[17] = {0};
  for (int i = 0; i < 8; i++) for (int j = 0; j < 8; j++) t[i+j] += (unsigned __int128)a[i]*b[j];
  uint32_t w[17]; unsigned __int128 c = 0;
  for (int i = 0; i < 16; i++) { c += t[i]; w[i] = (uint32_t)c; c >>= 32; }
  // reduce mod p = 2^255-19 by repeated folding using Python-like slow method: compute value as array and fold
  uint64_t x[9] = {0}; uint64_t cc = 0;
  for (int i = 0; i < 8; i++) { cc += (uint64_t)w[i] + (uint64_t)w[i+8]*38; x[i] = (uint32_t)cc; cc >>= 32; }
  // x = low + cc*2^256
  uint64_t d = cc * 38;
  for (int i = 0; i < 8; i++) { d += x[i]; x[i] = (uint32_t)d; d >>= 32; }
  x[0] += d * 38;
  // canonicalize: reduce below p
  for (int rep = 0; rep < 3; rep++) {
    // fold bit 255
    uint64_t top = x[7] >> 31; x[7] &= 0x7fffffff; uint64_t e = top * 19;
    for (int i = 0; i < 8; i++) { e += x[i]; x[i] = (uint32_t)e; e >>= 32; }
  }
  // if x >= p subtract p
  bool ge = (x[7] == 0x7fffffff); for (int i = 6; i >= 1 && ge; i--) ge = x[i] == 0xffffffff; if (ge) ge = x[0] >= 0xffffffed;
  if (ge) { x[0] -= 0xffffffed; for (int i = 1; i < 7; i++) x[i] = 0; x[7] = 0; }
  for (int i = 0; i < 8; i++) r[i] = (uint32_t)x[i];
}
static void canon(uint32_t* v) { uint32_t one[8] = {1,0,0,0,0,0,0,0}; uint32_t t[8]; ref_mul(t, v, one); for (int i=0;i<8;i++) v[i]=t[i]; }
int main() {
  const int nthreads = 256 * 8 * 256; // 2048 blocks of 256
  fe* h = (fe*)malloc(sizeof(fe) * nthreads); fe* h0 = (fe*)malloc(sizeof(fe) * nthreads);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < nthreads; i++) for (int j = 0; j < 8; j++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h0[i].v[j] = (uint32_t)s; }
  for (int i = 0; i < 64; i++) { for (int j = 0; j < 8; j++) h0[i].v[j] = 0xffffffffu; } // extremes
  fe* d; hipMalloc(&d, sizeof(fe) * nthreads);
  void (*ks[6])(fe*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
  const char* names[6] = {"mul_asm_comba", "mul_c_comba", "mul_operand_scan", "sq_asm_comba", "mul_asm2", "sq2"};
  // correctness with n=3
  for (int v = 0; v < 6; v++) {
    hipMemcpy(d, h0, sizeof(fe) * nthreads, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 3);
    hipMemcpy(h, d, sizeof(fe) * nthreads, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 4096; i++) {
      uint32_t a[8], b[8]; for (int j=0;j<8;j++){a[j]=h0[i].v[j]; b[j]=h0[i^1].v[j];}
      for (int r = 0; r < 3; r++) { uint32_t t[8]; if (v==3 || v==5) ref_mul(t, a, a); else ref_mul(t, a, b); for (int j=0;j<8;j++) a[j]=t[j]; }
      uint32_t g[8]; for (int j=0;j<8;j++) g[j]=h[i].v[j]; canon(g);
      for (int j=0;j<8;j++) if (g[j]!=a[j]) { bad++; break; }
    }
    printf("%s correctness: %d bad of 4096\n", names[v], bad);
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int N = 2000;
  for (int v = 0; v < 6; v++) {
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, 10); hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[v], dim3(nthreads / 256), dim3(256), 0, 0, d, N);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)nthreads * N;
    printf("%-20s %8.2f G fe-ops/s  %7.1f cyc/wave-op/SIMD @2.4GHz\n", names[v], ops / (ms * 1e-3) / 1e9,
           (ms * 1e-3) * 2.4e9 * 1024 / (ops / 64));
  }
  return 0;
}
