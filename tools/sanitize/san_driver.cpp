// san_driver.cpp -- host-only AddressSanitizer + UndefinedBehaviorSanitizer run of the C++
// host units that parse untrusted input or do wide integer arithmetic:
//   hmm_json.cpp  the hmm.json reader/writer (malformed files, nulls, round trips)
//   csp.cpp       exact term accumulation (add_exact), pair lists, the component search
//   hostscan.cpp  the constrained decode's component scan vs a scalar loop (both builds)
//   exact_fixed.h nearbyint(x * 2^64) limbs for f32 and f64 vs an __int128 reference
// Built with g++ -fsanitize=address,undefined (tools/sanitize/Makefile); runs in the
// container, never on the GPU box.  Exit status 0 = every check passed with no sanitizer
// report (UBSan is built with -fno-sanitize-recover, so any report aborts).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../consistent-viterbi_amd/csrc/csp.hpp"
#include "../../consistent-viterbi_amd/csrc/exact_fixed.h"
#include "../../consistent-viterbi_amd/csrc/hmm_json.hpp"
#include "../../consistent-viterbi_amd/csrc/hostscan.hpp"

static int g_fail = 0;
static int g_csp_feasible = 0;  // CSP trials with a feasible optimum (compared)
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                            \
    }                                                                      \
  } while (0)

// reference: round-half-even of x * 2^64 in plain double arithmetic (the scaling by 2^64 is
// exact; nearbyint rounds half to even in the default mode; |y| >= 2^52 is already integral
// and converts to __int128 exactly)
static __int128 ref_units(double x) {
  const double y = std::ldexp(x, 64);
  return (__int128)(std::fabs(y) >= 0x1p52 ? y : std::nearbyint(y));
}

static __int128 limbs_value(const int64_t* l) {
  const __int128 B = (__int128)1 << 32;
  return (__int128)l[0] + (__int128)l[1] * B + (__int128)l[2] * (B * B) + (__int128)l[3] * (B * B * B);
}

static void check_exact_fixed() {
  std::mt19937_64 rng(7);
  std::vector<double> xs = {0.0, -0.0, -1.0, -0.5, -0x1p-64, -0x1p-65, -0x1.8p-65, -0x1p-66, -3.0 * 0x1p-66,
                            -0x1p31, -0x1.fffffffffffffp31, 0x1p31, -1e-300, -4.9e-324, -2.2250738585072014e-308};
  for (int i = 0; i < 200000; ++i) {
    const double m = std::ldexp((double)(rng() >> 11), -53);
    const int e = (int)(rng() % 100) - 70;
    xs.push_back(-std::ldexp(m, e));
  }
  for (double x : xs) {
    if (!cvx::term_in_range(x)) continue;
    int64_t l[4];
    cvx::fixed64_limbs(x, l);
    CHECK(limbs_value(l) == ref_units(x));
    const float f = (float)x;
    if (cvx::term_in_range((double)f)) {
      int64_t lf[4];
      cvx::fixed64_limbs(f, lf);
      CHECK(limbs_value(lf) == ref_units((double)f));
    }
  }
  CHECK(!cvx::term_in_range(-0x1p32) && !cvx::term_in_range(0x1p32) && !cvx::term_in_range(-INFINITY));
  CHECK(cvx::term_in_range(-0x1.fffffffffffffp31));
}

static void check_add_exact() {
  int64_t limbs[4] = {0, 0, 0, 0}, ninf = 0;
  __int128 want = 0;
  std::mt19937_64 rng(11);
  for (int i = 0; i < 100000; ++i) {
    const double x = -std::ldexp((double)(rng() >> 11), -22);  // up to ~2^31 in magnitude
    CHECK(cvcsp::add_exact(limbs, &ninf, x));
    want += ref_units(x);
  }
  CHECK(limbs_value(limbs) == want);
  CHECK(cvcsp::add_exact(limbs, &ninf, -INFINITY) && ninf == 1);
  CHECK(cvcsp::add_exact(limbs, &ninf, -INFINITY + 0.0f) && ninf == 2);
  // out of range: rejected, nothing added (a huge finite "impossible" value)
  CHECK(!cvcsp::add_exact(limbs, &ninf, -1e30));
  CHECK(!cvcsp::add_exact(limbs, &ninf, -1e30f));
  CHECK(!cvcsp::add_exact(limbs, &ninf, -3.4e38f));
  CHECK(limbs_value(limbs) == want && ninf == 2);
}

static void check_csp() {
  // pair list + index
  const int64_t off[4] = {0, 4, 7, 10};
  const int32_t comp[10] = {-1, 2, 0, 2, 1, -1, 0, 3, 3, -1};
  const std::vector<int32_t> p = cvcsp::component_pairs(3, off, comp);
  CHECK(p == (std::vector<int32_t>{0, 1, 0, 2}));
  CHECK(cvcsp::pair_index(p.data(), 2, 0, 2) == 1 && cvcsp::pair_index(p.data(), 2, 1, 2) == -1);
  // exact search vs brute force on random small problems, with limb carries
  std::mt19937_64 rng(3);
  const __int128 M = 0xffffffff;
  for (int trial = 0; trial < 60; ++trial) {
    const int N = 2 + (int)(rng() % 3), ncomp = 2 + (int)(rng() % 2);
    std::vector<int32_t> pairs;
    for (int c1 = 0; c1 < ncomp; ++c1)
      for (int c2 = c1 + 1; c2 < ncomp; ++c2)
        if (rng() & 1) pairs.push_back(c1), pairs.push_back(c2);
    const int64_t npairs = (int64_t)pairs.size() / 2;
    std::vector<int64_t> part((size_t)cvcsp::partial_words(N, ncomp, npairs), 0);
    std::vector<__int128> U((size_t)ncomp * N), P((size_t)npairs * N * N);
    std::vector<uint8_t> Ud((size_t)ncomp * N, 0), Pd((size_t)npairs * N * N, 0);
    auto put = [&](int64_t* w, __int128 v) {
      w[0] += (int64_t)(v & M);
      w[1] += (int64_t)((v >> 32) & M);
      w[2] += (int64_t)((v >> 64) & M);
      w[3] += (int64_t)(v >> 96);
    };
    for (int c = 0; c < ncomp; ++c) {
      int64_t* u = part.data() + (size_t)c * cvcsp::unary_words(N);
      u[5 * N] = 1;
      for (int s = 0; s < N; ++s) {
        for (int k = 0; k < 3; ++k) {
          const __int128 v = ((__int128)(int64_t)(rng() >> 2) << (rng() % 40)) - ((__int128)1 << 88);
          put(u + 4 * s, v);
          U[(size_t)c * N + s] += v;
        }
        if (rng() % 7 == 0) u[4 * N + s] += 1, Ud[(size_t)c * N + s] = 1;
      }
    }
    for (int64_t q = 0; q < npairs; ++q) {
      int64_t* w = part.data() + (size_t)ncomp * cvcsp::unary_words(N) + (size_t)q * cvcsp::pair_words(N);
      w[5 * N * N] = 1;
      for (int e = 0; e < N * N; ++e) {
        const __int128 v = (__int128)(int64_t)(rng() >> 4) - ((__int128)1 << 70);
        put(w + 4 * e, v);
        P[(size_t)q * N * N + e] = v;
        if (rng() % 9 == 0) w[4 * N * N + e] += 1, Pd[(size_t)q * N * N + e] = 1;
      }
    }
    std::vector<int32_t> got((size_t)ncomp, -2);
    const cvcsp::SolveResult r = cvcsp::solve(N, ncomp, pairs.data(), npairs, part.data(), got.data(), 1000000);
    CHECK(!r.limit_hit);
    // brute force over every assignment, lexicographically smallest among the maxima, groups
    // merged (the whole problem as one group gives the same per-component optimum only when
    // connected; compare objective values instead)
    bool have = false;
    __int128 best = 0;
    std::vector<int> st((size_t)ncomp, 0), arg;
    for (int64_t code = 0, tot = (int64_t)std::pow(N, ncomp); code < tot; ++code) {
      int64_t c2 = code;
      for (int c = ncomp - 1; c >= 0; --c) st[(size_t)c] = (int)(c2 % N), c2 /= N;
      bool ok = true;
      __int128 v = 0;
      for (int c = 0; c < ncomp && ok; ++c) {
        ok = !Ud[(size_t)c * N + st[(size_t)c]];
        v += U[(size_t)c * N + st[(size_t)c]];
      }
      for (int64_t q = 0; q < npairs && ok; ++q) {
        const size_t e = (size_t)q * N * N + (size_t)st[(size_t)pairs[2 * q]] * N + st[(size_t)pairs[2 * q + 1]];
        ok = !Pd[e];
        v += P[e];
      }
      if (ok && (!have || v > best)) have = true, best = v, arg = st;
    }
    if (have) {
      ++g_csp_feasible;
      bool all = true;
      __int128 v = 0;
      for (int c = 0; c < ncomp; ++c) all &= got[(size_t)c] >= 0;
      if (all) {
        for (int c = 0; c < ncomp; ++c) v += U[(size_t)c * N + got[(size_t)c]];
        for (int64_t q = 0; q < npairs; ++q)
          v += P[(size_t)q * N * N + (size_t)got[(size_t)pairs[2 * q]] * N + got[(size_t)pairs[2 * q + 1]]];
      }
      CHECK(all && v == best);
    }
  }
}

// cvscan::scan_sequence / constrained_positions vs the scalar definition: random lengths
// (incl. 0 and non-multiples of 16), sparse / dense constrained elements, out-of-range values
static void check_hostscan() {
  std::mt19937_64 rng(7);
  for (int trial = 0; trial < 20000; ++trial) {
    const int64_t n = (int64_t)(rng() % 300);
    const int32_t ncomp = 1 + (int32_t)(rng() % 9);
    std::vector<int32_t> c((size_t)n, -1);
    const int mode = (int)(rng() % 4);
    for (int64_t k = 0; k < n; ++k) {
      const uint64_t x = rng() % 1000;
      if (mode >= 1 && x < (mode == 1 ? 5u : mode == 2 ? 300u : 1000u)) c[(size_t)k] = (int32_t)(rng() % ncomp);
    }
    if (n > 0 && rng() % 8 == 0)  // an out-of-range value somewhere
      c[(size_t)(rng() % n)] = (rng() % 2) ? ncomp + (int32_t)(rng() % 3) : -2 - (int32_t)(rng() % 3);
    int64_t bad = -1;
    bool any = false;
    std::vector<int64_t> pos;
    for (int64_t k = 0; k < n; ++k) {
      if (bad < 0 && (c[(size_t)k] < -1 || c[(size_t)k] >= ncomp)) bad = k;
      if (c[(size_t)k] >= 0) any = true;
    }
    const cvscan::SeqScan r = cvscan::scan_sequence(c.data(), n, ncomp);
    CHECK(r.bad == bad);
    if (bad >= 0) continue;
    CHECK(r.constrained == any);
    for (int64_t k = 0; k < n; ++k)
      if (c[(size_t)k] >= 0) pos.push_back(1000 + k);
    std::vector<int64_t> got;
    cvscan::constrained_positions(c.data(), n, 1000, got);
    CHECK(got == pos);
  }
}

static void check_json() {
  const std::string good =
      "{\"a\":{\"v\":1,\"dim\":[2,2],\"data\":[-0.1549019599857432,-0.5228787452803376,null,0.0]},"
      "\"b\":{\"v\":1,\"dim\":[2],\"data\":[{\"v\":1,\"dim\":[3,1],\"data\":[-0.3010299956639812,-0.3010299956639812,null]},"
      "{\"v\":1,\"dim\":[3,1],\"data\":[null,-0.47712125471966244,-0.17609125905568124]}]},"
      "\"pi\":{\"v\":1,\"dim\":[2],\"data\":[-0.3010299956639812,-0.3010299956639812]}}";
  cvh::HmmJson h;
  std::string err;
  CHECK(cvh::parse_hmm_json(good, h, err));
  CHECK(h.nstates == 2 && h.bdims.size() == 2 && h.a.size() == 4 && h.b.size() == 6);
  CHECK(std::isinf(h.a[2]) && h.a[2] < 0 && std::isinf(h.b[2]));
  const std::string round = cvh::format_hmm_json(h.nstates, h.bdims, h.pi.data(), h.a.data(), h.b.data());
  cvh::HmmJson h2;
  CHECK(cvh::parse_hmm_json(round, h2, err));
  CHECK(std::memcmp(h.a.data(), h2.a.data(), 32) == 0 && std::memcmp(h.b.data(), h2.b.data(), 48) == 0);
  // malformed inputs: every prefix of the good file, bad shapes, bad tokens -- rejected
  // without a sanitizer report
  for (size_t n = 0; n < good.size(); ++n) {
    cvh::HmmJson x;
    CHECK(!cvh::parse_hmm_json(good.substr(0, n), x, err));
  }
  const char* bad[] = {"{", "{\"a\":1}", "[]", "{\"a\":{\"v\":1,\"dim\":[2,2],\"data\":[1,2,3]},\"b\":{\"dim\":[0],\"data\":[]},"
                       "\"pi\":{\"v\":1,\"dim\":[2],\"data\":[0,0]}}", "{\"a\":{\"v\":1,\"dim\":[-1,2],\"data\":[]}}",
                       "{\"a\":{\"v\":1,\"dim\":[99999999999,99999999999],\"data\":[]}}", "nul", "\"\\u12", "1e99999",
                       "{\"a\":{\"v\":1,\"dim\":[1,1],\"data\":[nan]}}"};
  for (const char* b : bad) {
    cvh::HmmJson x;
    CHECK(!cvh::parse_hmm_json(b, x, err));
  }
  // random byte flips of the good file: whatever the parser says, no sanitizer report
  std::mt19937_64 rng(5);
  for (int i = 0; i < 3000; ++i) {
    std::string s = good;
    for (int k = 0; k < 3; ++k) s[rng() % s.size()] = (char)(rng() & 0x7f);
    cvh::HmmJson x;
    (void)cvh::parse_hmm_json(s, x, err);
  }
}

int main() {
  check_hostscan();
  check_exact_fixed();
  check_add_exact();
  check_csp();
  check_json();
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  CHECK(g_csp_feasible >= 20);
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("sanitizer driver: all checks passed (%d feasible CSP trials vs brute force)\n", g_csp_feasible);
  return 0;
}
