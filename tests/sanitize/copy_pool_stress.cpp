// Stress of coa_runtime.cpp's CopyPool (the host copy threads that pack the
// aggregation queue's windows): 4 caller threads, each issuing 200 copies of
// 1-5 MB at once, so several jobs are in progress on the pool together; every
// copy is compared with its source.  tests/test_sanitizers.py extracts the
// class text from coa_runtime.cpp into copy_pool_class.inc (the runtime
// itself needs HIP) and builds this under TSan and under ASan + UBSan.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "copy_pool_class.inc"

int main() {
  std::vector<std::thread> th;
  std::atomic<int> bad{0};
  for (int t = 0; t < 4; t++)
    th.emplace_back([&, t] {
      for (int it = 0; it < 200; it++) {
        const size_t n = (size_t)(1 << 20) * (1 + (it + t) % 5) + 12345;
        std::vector<uint8_t> a(n), b(n, 0);
        for (size_t i = 0; i < n; i += 4093) a[i] = (uint8_t)(i * 7 + t + it);
        std::vector<CopyPool::Seg> segs;
        for (size_t o = 0; o < n; o += 300000) segs.push_back({b.data() + o, a.data() + o, std::min<size_t>(300000, n - o)});
        CopyPool::get().copy(segs);
        if (a != b) bad++;
      }
    });
  for (auto& x : th) x.join();
  printf("copy pool ok: %d bad\n", bad.load());
  return bad.load() != 0;
}
