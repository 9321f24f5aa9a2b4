// CU-mask probe: does a kernel on a stream masked to half the CUs leave the
// other half free for another stream's kernels?  Stream A (CU mask: all, the
// upper half, or the lower half) runs a ~60 ms spin kernel with enough
// workgroups to fill every CU it may use; meanwhile stream B (all CUs) runs
// 40 short kernels (64 workgroups x 256 threads, ~100 us each) one after
// another; prints B's per-kernel latency p50 / max.
//   hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe
//   tools/cumask_probe <all|upper|lower|none>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void spin(unsigned long long ticks, unsigned* out) {
  const unsigned long long t0 = wall_clock64();
  unsigned x = 0;
  while (wall_clock64() - t0 < ticks) x++;
  if (threadIdx.x == 0 && x == 0xdeadbeefu) out[0] = x;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "upper";
  if (hipSetDevice(0) != hipSuccess) return 1;
  int cus = 0, freq = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipDeviceGetAttribute(&freq, hipDeviceAttributeWallClockRate, 0);  // kHz
  std::vector<uint32_t> all((cus + 31) / 32, 0), part((cus + 31) / 32, 0);
  for (int c = 0; c < cus; c++) all[c / 32] |= 1u << (c % 32);
  for (int c = 0; c < cus; c++)
    if ((!strcmp(mode, "upper") && c >= cus / 2) || (!strcmp(mode, "lower") && c < cus / 2)) part[c / 32] |= 1u << (c % 32);
  hipStream_t a, b;
  if (!strcmp(mode, "all") || !strcmp(mode, "none"))
    hipExtStreamCreateWithCUMask(&a, all.size(), all.data());
  else
    hipExtStreamCreateWithCUMask(&a, part.size(), part.data());
  hipExtStreamCreateWithCUMask(&b, all.size(), all.data());
  unsigned* out;
  hipMalloc(&out, 64);
  spin<<<1, 64, 0, a>>>(1, out);
  spin<<<1, 64, 0, b>>>(1, out);
  hipDeviceSynchronize();
  if (strcmp(mode, "none")) spin<<<cus * 8, 256, 0, a>>>((unsigned long long)freq * 60, out);  // ~60 ms
  std::vector<double> lat;
  for (int i = 0; i < 40; i++) {
    const auto t0 = std::chrono::steady_clock::now();
    spin<<<64, 256, 0, b>>>((unsigned long long)freq / 10, out);  // ~100 us
    hipStreamSynchronize(b);
    lat.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
  hipDeviceSynchronize();
  std::vector<double> s = lat;
  std::sort(s.begin(), s.end());
  printf("{\"mode\": \"%s\", \"cus\": %d, \"b_p50_ms\": %.3f, \"b_max_ms\": %.3f, \"b_first5\": [%.3f, %.3f, %.3f, %.3f, %.3f]}\n",
         mode, cus, s[s.size() / 2], s.back(), lat[0], lat[1], lat[2], lat[3], lat[4]);
  return 0;
}
