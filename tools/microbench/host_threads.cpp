// Host-side cost model of parallel_ranges (csrc/cviterbi.cpp) on the GPU box's CPU share:
// spawning + joining n threads that do nothing, and n threads streaming a 134 MB int32 array
// (config 5's component array) with a min / max / AND pass.  No GPU.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t n = (size_t)65536 * 512;
  std::vector<int32_t> a(n, -1);
  for (size_t i = 0; i < n; i += 1024) a[i] = (int32_t)(i % 7);
  for (int nt : {1, 2, 4, 8, 16, 32}) {
    double spawn = 1e9, scan = 1e9;
    for (int rep = 0; rep < 7; ++rep) {
      double t0 = now_ms();
      {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back([] {});
        for (auto& x : th) x.join();
      }
      spawn = std::min(spawn, now_ms() - t0);
      std::vector<int64_t> out((size_t)nt * 16, 0);
      t0 = now_ms();
      {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
          th.emplace_back([&, t] {
            const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
            int32_t mn = INT32_MAX, mx = INT32_MIN, an = -1;
            for (size_t i = lo; i < hi; ++i) {
              mn = std::min(mn, a[i]);
              mx = std::max(mx, a[i]);
              an &= a[i];
            }
            out[(size_t)t * 16] = (int64_t)mn + mx + an;
          });
        for (auto& x : th) x.join();
      }
      scan = std::min(scan, now_ms() - t0);
    }
    printf("threads %2d: spawn+join %.3f ms, scan 134 MB %.3f ms (%.1f GB/s)\n", nt, spawn, scan, n * 4 / scan / 1e6);
  }
  return 0;
}
