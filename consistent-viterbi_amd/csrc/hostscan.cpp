// hostscan.cpp -- the constrained decode's host scan of `component` (one pass per sequence:
// range check, "any constrained element", then the constrained positions), host-only.
// Config 5 reads 134 MB of components before the first launch ("Config 5's work
// floor"); the scalar loop ran at ~3 GB/s per core.  Here the checks are min / max / AND
// reductions the compiler vectorises, and the positions come from 16-element blocks whose AND is
// not -1 (with every component >= -1, a block of -1s ANDs to -1).  An AVX2 build of the same
// loops is picked at run time when the CPU has it (the library's baseline is x86-64).
#include "hostscan.hpp"

#include <algorithm>
#include <climits>

namespace cvscan {
namespace {

template <int Dummy>
inline SeqScan scan_body(const int32_t* c, int64_t n, int32_t ncomp) {
  int32_t all = -1, mn = INT32_MAX, mx = INT32_MIN;
  for (int64_t k = 0; k < n; ++k) {
    all &= c[k];
    mn = std::min(mn, c[k]);
    mx = std::max(mx, c[k]);
  }
  SeqScan r{all != -1, -1};
  if (n > 0 && (mn < -1 || mx >= ncomp))
    for (int64_t k = 0; k < n; ++k)
      if (c[k] < -1 || c[k] >= ncomp) {
        r.bad = k;
        break;
      }
  return r;
}

template <int Dummy>
inline void positions_body(const int32_t* c, int64_t n, int64_t base, std::vector<int64_t>& out) {
  for (int64_t k0 = 0; k0 < n; k0 += 16) {
    const int64_t k1 = std::min<int64_t>(n, k0 + 16);
    int32_t b = -1;
    for (int64_t k = k0; k < k1; ++k) b &= c[k];
    if (b == -1) continue;
    for (int64_t k = k0; k < k1; ++k)
      if (c[k] >= 0) out.push_back(base + k);
  }
}

SeqScan scan_generic(const int32_t* c, int64_t n, int32_t ncomp) { return scan_body<0>(c, n, ncomp); }
void positions_generic(const int32_t* c, int64_t n, int64_t base, std::vector<int64_t>& out) {
  positions_body<0>(c, n, base, out);
}
__attribute__((target("avx2"))) SeqScan scan_avx2(const int32_t* c, int64_t n, int32_t ncomp) {
  return scan_body<1>(c, n, ncomp);
}
__attribute__((target("avx2"))) void positions_avx2(const int32_t* c, int64_t n, int64_t base,
                                                    std::vector<int64_t>& out) {
  positions_body<1>(c, n, base, out);
}

bool use_avx2() {
  static const bool v = __builtin_cpu_supports("avx2");
  return v;
}
}  // namespace

SeqScan scan_sequence(const int32_t* c, int64_t n, int32_t ncomp) {
  return use_avx2() ? scan_avx2(c, n, ncomp) : scan_generic(c, n, ncomp);
}

void constrained_positions(const int32_t* c, int64_t n, int64_t base, std::vector<int64_t>& out) {
  if (use_avx2()) positions_avx2(c, n, base, out);
  else positions_generic(c, n, base, out);
}

}  // namespace cvscan
