// Host cost of the constrained decode's component scan (csrc/cviterbi.cpp build_conseq_checked)
// on config 5's layout (65,536 x 512, one constrained element in every other sequence), on the
// GPU box's CPU: the scan as shipped (a thread per worker range, a heap vector per constrained
// sequence) against the same scan with positions counted only, and with one flat position array
// per worker.  Links csrc/hostscan.cpp.  No GPU.
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../consistent-viterbi_amd/csrc/hostscan.hpp"

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct ConSeq {
  int64_t seq;
  std::vector<int64_t> elems;
};
template <typename F>
static void par(int nt, int64_t n, F&& f) {
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back([&, t] { f(t, n * t / nt, n * (t + 1) / nt); });
  for (auto& x : th) x.join();
}

int main() {
  const int64_t nseq = 65536, T = 512;
  std::vector<int64_t> off(nseq + 1);
  for (int64_t s = 0; s <= nseq; ++s) off[s] = s * T;
  std::vector<int32_t> comp((size_t)(nseq * T), -1);
  uint64_t x = 12345;
  for (int64_t s = 0; s < nseq; s += 2) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    comp[(size_t)(s * T + (int64_t)((x >> 33) % T))] = (int32_t)((x >> 20) % 7);
  }
  const int nt = 16;
  for (int mode = 0; mode < 3; ++mode) {
    double best = 1e9, best_cat = 1e9;
    for (int rep = 0; rep < 9; ++rep) {
      std::vector<ConSeq> cs;
      std::vector<std::vector<ConSeq>> part(nt);
      std::vector<std::vector<int64_t>> flat(nt);
      std::vector<int64_t> cnt(nt, 0);
      double t0 = now_ms();
      par(nt, nseq, [&](int t, int64_t lo, int64_t hi) {
        for (int64_t s = lo; s < hi; ++s) {
          const cvscan::SeqScan r = cvscan::scan_sequence(comp.data() + off[s], off[s + 1] - off[s], 7);
          if (r.bad >= 0 || !r.constrained) continue;
          if (mode == 0) {
            ConSeq q{s, {}};
            cvscan::constrained_positions(comp.data() + off[s], off[s + 1] - off[s], off[s], q.elems);
            part[t].push_back(std::move(q));
          } else if (mode == 1) {
            ++cnt[t];
          } else {
            cvscan::constrained_positions(comp.data() + off[s], off[s + 1] - off[s], off[s], flat[t]);
          }
        }
      });
      const double t1 = now_ms();
      if (mode == 0)
        for (auto& p : part)
          for (auto& c : p) cs.push_back(std::move(c));
      best = std::min(best, t1 - t0);
      best_cat = std::min(best_cat, now_ms() - t1);
    }
    printf("%s: workers %.3f ms, concatenation %.3f ms\n",
           mode == 0 ? "as shipped (vector per sequence)" : mode == 1 ? "scan only (count)" : "flat positions per worker",
           best, best_cat);
  }
  return 0;
}
