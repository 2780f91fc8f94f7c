// Host memcpy of one 51 200-sample f32 block (409 600 B) into coherent pinned memory, single
// thread and split over 2 / 4 threads (tuning aid, not product).
//   hipcc --offload-arch=gfx950 -O2 -pthread tools/memcpy_probe.hip -o tools/memcpy_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

int main() {
  const size_t B = 409600, NB = 16;
  std::vector<char> src(B * NB, 1);
  void* dst;
  hipHostMalloc(&dst, B * 2, hipHostMallocCoherent);
  for (int nt : {1, 2, 4}) {
    for (int pass = 0; pass < 2; ++pass) {
      const int n = 2000;
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; ++i) {
        char* d = static_cast<char*>(dst) + (i & 1) * B;
        const char* s = src.data() + (i % NB) * B;
        if (nt == 1) {
          std::memcpy(d, s, B);
        } else {
          std::vector<std::thread> th;
          for (int t = 1; t < nt; ++t) th.emplace_back([=] { std::memcpy(d + t * B / nt, s + t * B / nt, B / nt); });
          std::memcpy(d, s, B / nt);
          for (auto& x : th) x.join();
        }
      }
      const auto t1 = std::chrono::steady_clock::now();
      if (pass) printf("threads %d: %.2f us per 409 600-B block (thread spawn included for > 1)\n", nt,
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / n);
    }
  }
  return 0;
}
