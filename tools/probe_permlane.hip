// Semantics probe of v_permlane32_swap / v_permlane16_swap on gfx950: both
// operands are the lane id; prints, for the first lane of each 16-lane row,
// the two results of each swap.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
  const unsigned x = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(x, x + 100, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(x, x + 100, false, false);
  o[threadIdx.x * 4 + 0] = a[0];
  o[threadIdx.x * 4 + 1] = a[1];
  o[threadIdx.x * 4 + 2] = b[0];
  o[threadIdx.x * 4 + 3] = b[1];
}
int main() {
  unsigned* d;
  unsigned h[256];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int l = 0; l < 64; l += 8)
    printf("lane %2d: p32 (%u, %u)  p16 (%u, %u)\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  return 0;
}
