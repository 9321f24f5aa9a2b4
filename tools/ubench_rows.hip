// Latency of one z^((p-5)/8) chain on a lone wave: the one-lane chain of
// coa_fe.h against the 16-lane-row chain of coa_fe_wave.h (s_memtime cycles).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../xrpl-coa-prototype_amd/csrc ubench_rows.hip -o ubench_rows
#include <cstdio>

#include "coa_fe_wave.h"

__global__ void k(const uint32_t* in, uint32_t* out, long long* cyc) {
  fe z, r;
#pragma unroll
  for (int i = 0; i < 8; i++) z.v[i] = in[i];
  long long t0 = clock64();
  fe_pow_p58(r, z);
  uint32_t s = r.v[0];
  long long t1 = clock64();
  fe_pow_p58_rows(r, z);
  s ^= r.v[0];
  long long t2 = clock64();
  uint32_t x = fw::from_fe(z);
  x = fw::sqn<100>(x);
  long long t3 = clock64();
  fe y = z;
  fe_sqn(y, y, 100);
  long long t4 = clock64();
  fe q;
  fw::to_fe(q, x);
  if (threadIdx.x == 0) {
    out[0] = s ^ q.v[0] ^ y.v[0];
    cyc[0] = t1 - t0;
    cyc[1] = t2 - t1;
    cyc[2] = t3 - t2;
    cyc[3] = t4 - t3;
  }
}

int main() {
  uint32_t h[8] = {0x12345678, 0x9abcdef0, 0x0fedcba9, 0x87654321, 0x11111111, 0x22222222, 0x33333333, 0x04444444};
  uint32_t *din, *dout;
  long long* dc;
  hipMalloc(&din, 32);
  hipMalloc(&dout, 4);
  hipMalloc(&dc, 32);
  hipMemcpy(din, h, 32, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout, dc);
    long long c[4];
    hipMemcpy(c, dc, 32, hipMemcpyDeviceToHost);
    printf("pow_p58 one-lane %lld cycles, rows %lld; 100 squarings rows %lld, one-lane %lld\n", c[0], c[1], c[2],
           c[3]);
  }
  return 0;
}
