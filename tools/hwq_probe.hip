// Hardware-queue probe: how many of a process's streams really run at once.
//
// HIP maps streams onto at most GPU_MAX_HW_QUEUES hardware queues per
// priority; streams that share a queue run one after another.  The probe opens
// `bg` plain streams first (as torch's stream and the engine contexts' streams
// are), then `n` streams of one kind, launches one ~2 ms single-wave spin
// kernel on each of the n and reports the elapsed time: ~2 ms means all n ran
// concurrently, k x 2 ms means they shared queues.
//
// kinds: plain (hipStreamCreateWithFlags), cumask (hipExtStreamCreateWithCUMask,
// every CU enabled), hi / lo (hipStreamCreateWithPriority, greatest / least).
//
//   hipcc --offload-arch=gfx950 -O2 tools/hwq_probe.hip -o tools/hwq_probe
//   tools/hwq_probe <kind> <n> <bg>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__global__ void spin(unsigned long long ticks, unsigned* out) {
  const unsigned long long t0 = wall_clock64();
  unsigned x = 0;
  while (wall_clock64() - t0 < ticks) x++;
  if (threadIdx.x == 0 && x == 0xdeadbeefu) out[0] = x;
}

#define CK(e)                                                               \
  do {                                                                      \
    hipError_t r_ = (e);                                                    \
    if (r_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(r_)); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main(int argc, char** argv) {
  const char* kind = argc > 1 ? argv[1] : "plain";
  const int n = argc > 2 ? atoi(argv[2]) : 4;
  const int bg = argc > 3 ? atoi(argv[3]) : 0;
  if (n < 1 || n > 16 || bg < 0 || bg > 16) return 2;
  CK(hipSetDevice(0));
  int cus = 0, lo = 0, hi = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  std::vector<hipStream_t> bgs(bg), ss(n);
  for (auto& s : bgs) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<uint32_t> mask((cus + 31) / 32, 0);
  for (int c = 0; c < cus; c++) mask[c / 32] |= 1u << (c % 32);
  for (auto& s : ss) {
    if (!strcmp(kind, "cumask"))
      CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    else if (!strcmp(kind, "hi"))
      CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    else if (!strcmp(kind, "lo"))
      CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, lo));
    else
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  unsigned* out;
  CK(hipMalloc(&out, 64));
  int freq = 0;
  CK(hipDeviceGetAttribute(&freq, hipDeviceAttributeWallClockRate, 0));  // kHz
  const unsigned long long ticks = (unsigned long long)freq * 2;           // 2 ms
  // warm up every stream
  for (auto& s : ss) spin<<<1, 64, 0, s>>>(1, out);
  for (auto& s : bgs) spin<<<1, 64, 0, s>>>(1, out);
  CK(hipDeviceSynchronize());
  double best = 1e30;
  for (int rep = 0; rep < 3; rep++) {
    const auto t0 = std::chrono::steady_clock::now();
    for (auto& s : ss) spin<<<1, 64, 0, s>>>(ticks, out);
    for (auto& s : ss) CK(hipStreamSynchronize(s));
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    best = ms < best ? ms : best;
  }
  const char* env = getenv("GPU_MAX_HW_QUEUES");
  printf("{\"kind\": \"%s\", \"streams\": %d, \"background_streams\": %d, \"GPU_MAX_HW_QUEUES\": \"%s\", "
         "\"prio_range\": [%d, %d], \"ms\": %.3f, \"serial_factor\": %.2f}\n",
         kind, n, bg, env ? env : "(unset)", lo, hi, best, best / 2.0);
  return 0;
}
