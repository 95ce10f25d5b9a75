// Host scan of config 5's components (hostscan.cpp) at N threads: spawn / scan / merge times.
// g++ -O2 -std=c++17 -pthread -Iconsistent-viterbi_amd/csrc tools/microbench/hostscan_bench.cpp consistent-viterbi_amd/csrc/hostscan.cpp
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>
#include <cstring>
#include <cstdlib>
#include "hostscan.hpp"
struct ConSeq { int64_t seq; std::vector<int64_t> elems; };
int main(int argc, char** argv) {
  const int nt = argc > 1 ? atoi(argv[1]) : 8;
  const int64_t nseq = 65536, T = 512;
  std::vector<int32_t> comp(nseq * T, -1);
  std::vector<int64_t> off(nseq + 1);
  for (int64_t s = 0; s <= nseq; ++s) off[s] = s * T;
  for (int64_t s = 0; s < nseq; s += 2) comp[s * T + (s * 7919) % T] = (int32_t)(s % 7);
  for (int rep = 0; rep < 5; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::vector<ConSeq>> part(nt);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        const int64_t lo = nseq * t / nt, hi = nseq * (t + 1) / nt;
        for (int64_t s = lo; s < hi; ++s) {
          auto r = cvscan::scan_sequence(comp.data() + off[s], T, 7);
          if (!r.constrained) continue;
          ConSeq q{s, {}};
          cvscan::constrained_positions(comp.data() + off[s], T, off[s], q.elems);
          part[t].push_back(std::move(q));
        }
      });
    auto t1 = std::chrono::steady_clock::now();
    for (auto& x : th) x.join();
    auto t2 = std::chrono::steady_clock::now();
    std::vector<ConSeq> cs;
    for (auto& p : part) for (auto& c : p) cs.push_back(std::move(c));
    auto t3 = std::chrono::steady_clock::now();
    printf("threads %d: spawn %.3f ms, scan+join %.3f ms, merge %.3f ms, total %.3f ms (%zu)\n", nt,
           std::chrono::duration<double, std::milli>(t1 - t0).count(), std::chrono::duration<double, std::milli>(t2 - t1).count(),
           std::chrono::duration<double, std::milli>(t3 - t2).count(), std::chrono::duration<double, std::milli>(t3 - t0).count(), cs.size());
  }
}
