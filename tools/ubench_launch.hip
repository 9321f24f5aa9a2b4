// Round-trip latency of a one-item call, with the kernel's work taken out:
//   launch   hipLaunchKernelGGL of a 5-workgroup kernel whose last block
//            writes a tagged word into page-locked host memory; the host
//            polls it (the engine's latency-path protocol)
//   launch3KB the same with 3 KB of kernel arguments (the inline certificate)
//   resident the same 5 workgroups already running, each polling a job word
//            in page-locked host memory; the host writes the job, the last
//            block publishes the tagged result (a persistent kernel's
//            protocol; the grid exits on a quit job)
// p50/p99 over 2000 calls each.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_launch.hip -o tools/ubench_launch
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_once(uint32_t* res, uint32_t* ctr, uint32_t tag, uint32_t blocks) {
  if (threadIdx.x) return;
  __threadfence();
  const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 != blocks) return;
  __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(res, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Big {
  uint32_t w[768];  // 3 KB of kernel arguments, as the inline certificate launch
};
__global__ void k_once_big(Big b, uint32_t* res, uint32_t* ctr, uint32_t tag, uint32_t blocks) {
  if (threadIdx.x) return;
  const uint32_t x = b.w[blockIdx.x * 64];  // touch the argument block
  __threadfence();
  const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 != blocks) return;
  __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(res, tag + (x & 0u), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// job word: (seq << 1) | quit.  Every block waits for a new seq, then counts
// itself done; the last one publishes seq.  Exits when quit is set.
__global__ void k_resident(const uint32_t* job, uint32_t* res, uint32_t* ctr, uint32_t blocks) {
  if (threadIdx.x) return;
  uint32_t seen = 0;
  for (;;) {
    uint32_t j;
    while (((j = __hip_atomic_load(job, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) >> 1) == seen &&
           !(j & 1u))
      __builtin_amdgcn_s_sleep(1);
    if (j & 1u) return;
    seen = j >> 1;
    const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1 == blocks) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(res, seen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void report(const char* name, std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  printf("%-10s p50 %7.2f us  p99 %7.2f us  min %7.2f us\n", name, v[v.size() / 2], v[v.size() * 99 / 100], v[0]);
}

int main() {
  const uint32_t blocks = 5;
  uint32_t *res, *job, *ctr;
  if (hipHostMalloc((void**)&res, 64, hipHostMallocCoherent) != hipSuccess) return 1;
  if (hipHostMalloc((void**)&job, 64, hipHostMallocCoherent) != hipSuccess) return 1;
  if (hipMalloc((void**)&ctr, 64) != hipSuccess) return 1;
  (void)hipMemset(ctr, 0, 64);
  *res = 0;
  *job = 0;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  (void)hipDeviceSynchronize();
  const int N = 2000;
  std::vector<double> t;
  for (int i = 1; i <= N + 50; i++) {
    const double t0 = now_us();
    hipLaunchKernelGGL(k_once, dim3(blocks), dim3(192), 0, s, res, ctr, (uint32_t)i, blocks);
    while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != (uint32_t)i) {
    }
    if (i > 50) t.push_back(now_us() - t0);
  }
  report("launch", t);
  (void)hipStreamSynchronize(s);
  static Big big;
  for (int i = 0; i < 768; i++) big.w[i] = i;
  t.clear();
  for (int i = 1; i <= N + 50; i++) {
    const double t0 = now_us();
    hipLaunchKernelGGL(k_once_big, dim3(blocks), dim3(192), 0, s, big, res, ctr, (uint32_t)(i + 100000), blocks);
    while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != (uint32_t)(i + 100000)) {
    }
    if (i > 50) t.push_back(now_us() - t0);
  }
  report("launch3KB", t);
  (void)hipStreamSynchronize(s);
  *res = 0;
  hipLaunchKernelGGL(k_resident, dim3(blocks), dim3(192), 0, s, job, res, ctr, blocks);
  t.clear();
  for (uint32_t i = 1; i <= (uint32_t)N + 50; i++) {
    const double t0 = now_us();
    __atomic_store_n(job, i << 1, __ATOMIC_RELEASE);
    const double deadline = t0 + 1e6;
    while (__atomic_load_n(res, __ATOMIC_ACQUIRE) != i) {
      if (now_us() > deadline) {
        printf("resident: no answer\n");
        __atomic_store_n(job, 1u, __ATOMIC_RELEASE);
        (void)hipStreamSynchronize(s);
        return 2;
      }
    }
    if (i > 50) t.push_back(now_us() - t0);
  }
  __atomic_store_n(job, 1u, __ATOMIC_RELEASE);  // quit
  (void)hipStreamSynchronize(s);
  report("resident", t);
  return 0;
}
