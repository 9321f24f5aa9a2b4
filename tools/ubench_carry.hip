// Carry-chain cost: a plain-C fe_add (hipcc pads each VCC carry hand-off
// with `s_nop 1` on gfx950) vs an unpadded VOP2 asm chain with separate
// outputs vs coa_fe.h's in-place asm fe_add (carry-in read straight from VCC).  Checks every lane against a host port
// after many launches at several occupancies.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_carry.hip -o tools/ubench_carry
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../xrpl-coa-prototype_amd/csrc/coa_fe.h"

// The pre-asm coa_fe.h fe_add, kept here as the padded baseline.
COA_DEV void fe_add_c(fe& r, const fe& a, const fe& b) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(a.v[i], b.v[i], c, c);
  uint32_t c2 = 0;
  r.v[0] = addc32(r.v[0], c * 38u, 0, c2);
#pragma unroll
  for (int i = 1; i < 8; i++) r.v[i] = addc32(r.v[i], 0, c2, c2);
  r.v[0] += c2 * 38u;
}

// r = a + b mod p (< 2^256), same value as fe_add.
COA_DEV void fe_add_asm(fe& r, const fe& a, const fe& b) {
  uint32_t t;
  const uint32_t z = 0;
  asm("v_add_co_u32_e32 %0, vcc, %10, %18\n\t"
      "v_addc_co_u32_e32 %1, vcc, %11, %19, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, %12, %20, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, %13, %21, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, %14, %22, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, %15, %23, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, %16, %24, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, %17, %25, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %9, vcc\n\t"
      "v_mul_u32_u24_e32 %8, 38, %8\n\t"
      "v_add_co_u32_e32 %0, vcc, %0, %8\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e32 %3, vcc, 0, %3, vcc\n\t"
      "v_addc_co_u32_e32 %4, vcc, 0, %4, vcc\n\t"
      "v_addc_co_u32_e32 %5, vcc, 0, %5, vcc\n\t"
      "v_addc_co_u32_e32 %6, vcc, 0, %6, vcc\n\t"
      "v_addc_co_u32_e32 %7, vcc, 0, %7, vcc\n\t"
      "v_addc_co_u32_e32 %8, vcc, 0, %9, vcc\n\t"
      "v_mul_u32_u24_e32 %8, 38, %8\n\t"
      "v_add_u32_e32 %0, %0, %8"
      : "=&v"(r.v[0]), "=&v"(r.v[1]), "=&v"(r.v[2]), "=&v"(r.v[3]), "=&v"(r.v[4]), "=&v"(r.v[5]), "=&v"(r.v[6]),
        "=&v"(r.v[7]), "=&v"(t)
      : "v"(z), "v"(a.v[0]), "v"(a.v[1]), "v"(a.v[2]), "v"(a.v[3]), "v"(a.v[4]), "v"(a.v[5]), "v"(a.v[6]),
        "v"(a.v[7]), "v"(b.v[0]), "v"(b.v[1]), "v"(b.v[2]), "v"(b.v[3]), "v"(b.v[4]), "v"(b.v[5]), "v"(b.v[6]),
        "v"(b.v[7])
      : "vcc");
}

template <int V>
__global__ void k(fe* x, int n) {
  int id = blockIdx.x * blockDim.x + threadIdx.x;
  fe a = x[2 * id], b = x[2 * id + 1];
  for (int i = 0; i < n; i++) {
    if (V == 0) { fe_add_c(a, a, b); fe_add_c(b, b, a); }
    if (V == 1) { fe_add_asm(a, a, b); fe_add_asm(b, b, a); }
    if (V == 2) { fe_add(a, a, b); fe_add(b, b, a); }
  }
  x[2 * id] = a;
  x[2 * id + 1] = b;
}

static void host_add(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint64_t c = 0;
  uint32_t t[8];
  for (int i = 0; i < 8; i++) { c += (uint64_t)a[i] + b[i]; t[i] = (uint32_t)c; c >>= 32; }
  uint64_t d = c * 38;
  for (int i = 0; i < 8; i++) { d += t[i]; t[i] = (uint32_t)d; d >>= 32; }
  t[0] += (uint32_t)d * 38;
  memcpy(r, t, 32);
}

int main() {
  const int maxthreads = 256 * 8 * 256;
  const int n_iter = 64;
  fe* h0 = (fe*)malloc(sizeof(fe) * 2 * maxthreads);
  fe* h = (fe*)malloc(sizeof(fe) * 2 * maxthreads);
  fe* ref = (fe*)malloc(sizeof(fe) * 2 * maxthreads);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < 2 * maxthreads; i++)
    for (int j = 0; j < 8; j++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; h0[i].v[j] = (uint32_t)s; }
  for (int i = 0; i < 256; i++) for (int j = 0; j < 8; j++) h0[i].v[j] = (i & 1) ? 0xffffffffu : (j ? 0xffffffffu : 0xffffffdau);
  for (int i = 0; i < maxthreads; i++) {
    uint32_t a[8], b[8];
    memcpy(a, h0[2 * i].v, 32); memcpy(b, h0[2 * i + 1].v, 32);
    for (int r = 0; r < n_iter; r++) { host_add(a, a, b); host_add(b, b, a); }
    memcpy(ref[2 * i].v, a, 32); memcpy(ref[2 * i + 1].v, b, 32);
  }
  fe* d; hipMalloc(&d, sizeof(fe) * 2 * maxthreads);
  void (*ks[3])(fe*, int) = {k<0>, k<1>, k<2>};
  const char* names[3] = {"fe_add_C(padded)", "fe_add_asm(unpadded)", "coa_fe.h fe_add"};
  int total_bad = 0;
  const int blocks_list[3] = {256, 1024, 2048};  // 1, 4, 8 waves per SIMD
  for (int v = 0; v < 3; v++) {
    for (int bi = 0; bi < 3; bi++) {
      int bad = 0;
      for (int rep = 0; rep < 20; rep++) {
        hipMemcpy(d, h0, sizeof(fe) * 2 * maxthreads, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(ks[v], dim3(blocks_list[bi]), dim3(256), 0, 0, d, n_iter);
        hipMemcpy(h, d, sizeof(fe) * 2 * maxthreads, hipMemcpyDeviceToHost);
        for (int i = 0; i < blocks_list[bi] * 256 * 2; i++) if (memcmp(h[i].v, ref[i].v, 32)) bad++;
      }
      total_bad += bad;
      printf("%-22s blocks=%4d correctness: %d bad of %d\n", names[v], blocks_list[bi], bad, blocks_list[bi] * 512 * 20);
    }
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int N = 20000;
  for (int bi = 0; bi < 3; bi++) {
    for (int v = 0; v < 3; v++) {
      hipLaunchKernelGGL(ks[v], dim3(blocks_list[bi]), dim3(256), 0, 0, d, 100); hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[v], dim3(blocks_list[bi]), dim3(256), 0, 0, d, N);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double waves_per_simd = blocks_list[bi] * 4.0 / 1024;
      printf("blocks=%4d %-22s %6.1f cyc/fe_add per wave\n", blocks_list[bi], names[v],
             (ms * 1e-3) * 2.4e9 / (2.0 * N * waves_per_simd));
    }
  }
  return total_bad ? 1 : 0;
}
