// Exact component-state search (see csp.hpp).  Pure host C++, no device code.
#include "csp.hpp"
#include "exact_fixed.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>

namespace cvcsp {

template <typename REAL>
static bool add_exact_t(int64_t* limbs4, int64_t* ninf_count, REAL x) {
  if (!(x > -INFINITY)) {
    *ninf_count += 1;
    return true;
  }
  if (!cvx::term_in_range((double)x)) return false;  // |x| >= 2^32: outside the exact unit
  // the limbs of nearbyint(x * 2^64), shared with the device sums (exact_fixed.h); checked
  // bit-identical to the double -> __int128 form on 3.7e7 floats incl. every exponent
  int64_t l[4];
  cvx::fixed64_limbs(x, l);
  for (int k = 0; k < 4; ++k) limbs4[k] += l[k];
  return true;
}

bool add_exact(int64_t* limbs4, int64_t* ninf_count, float x) { return add_exact_t(limbs4, ninf_count, x); }
bool add_exact(int64_t* limbs4, int64_t* ninf_count, double x) { return add_exact_t(limbs4, ninf_count, x); }

static inline __int128 limbs_value(const int64_t* l) {
  // multiplications, not shifts: limb 3 and carried limbs may be negative (a left shift of a
  // negative value is undefined before C++20)
  const __int128 B = (__int128)1 << 32;
  return (__int128)l[0] + (__int128)l[1] * B + (__int128)l[2] * (B * B) + (__int128)l[3] * (B * B * B);
}

std::vector<int32_t> component_pairs(int64_t nseq, const int64_t* offsets, const int32_t* component) {
  std::vector<std::pair<int32_t, int32_t>> ps;
  for (int64_t q = 0; q < nseq; ++q) {
    int32_t prev = -1;
    for (int64_t e = offsets[q]; e < offsets[q + 1]; ++e) {
      const int32_t c = component[e];
      if (c < 0) continue;
      if (prev >= 0 && prev != c) ps.emplace_back(std::min(prev, c), std::max(prev, c));
      prev = c;
    }
  }
  std::sort(ps.begin(), ps.end());
  ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
  std::vector<int32_t> out;
  out.reserve(ps.size() * 2);
  for (auto& p : ps) out.push_back(p.first), out.push_back(p.second);
  return out;
}

int64_t pair_index(const int32_t* pairs, int64_t npairs, int32_t c1, int32_t c2) {
  int64_t lo = 0, hi = npairs;
  while (lo < hi) {
    const int64_t mid = (lo + hi) / 2;
    const int32_t a = pairs[2 * mid], b = pairs[2 * mid + 1];
    if (a < c1 || (a == c1 && b < c2)) lo = mid + 1;
    else hi = mid;
  }
  return (lo < npairs && pairs[2 * lo] == c1 && pairs[2 * lo + 1] == c2) ? lo : -1;
}

namespace {

struct Nbr {
  int var;      // neighbour's position in the group's variable order
  int64_t p;    // pair index
  bool row;     // this variable is the pair's c1 (row index of the table)
};

struct Group {
  int N;
  std::vector<int32_t> comps;                  // ascending component ids
  std::vector<std::vector<Nbr>> nbrs;          // per variable
  const std::vector<__int128>* U;              // [ncomp*N]
  const std::vector<uint8_t>* Ud;
  const std::vector<std::vector<__int128>>* P; // per pair [N*N]
  const std::vector<std::vector<uint8_t>>* Pd;
  // R[v][k][s] = max over feasible s' of P(v=s, nbr k = s') for later neighbours (k index
  // into nbrs[v]); Rd = no feasible s'.
  std::vector<std::vector<std::vector<__int128>>> R;
  std::vector<std::vector<std::vector<uint8_t>>> Rd;

  __int128 pv(const Nbr& nb, int s_self, int s_other) const {
    const auto& t = (*P)[nb.p];
    return nb.row ? t[(size_t)s_self * N + s_other] : t[(size_t)s_other * N + s_self];
  }
  bool pd(const Nbr& nb, int s_self, int s_other) const {
    const auto& t = (*Pd)[nb.p];
    return nb.row ? t[(size_t)s_self * N + s_other] : t[(size_t)s_other * N + s_self];
  }
};

struct Search {
  const Group& g;
  uint64_t limit;
  uint64_t nodes = 0, explored = 0;
  bool limit_hit = false;
  std::vector<int> st;
  bool have = false;
  __int128 best = 0;
  std::vector<int> inc;

  explicit Search(const Group& gr, uint64_t lim) : g(gr), limit(lim), st(gr.comps.size(), -1) {}

  // value of variable v at state s given assigned variables [0, L): unary + pairs with
  // assigned neighbours (+ R of later neighbours when with_later).  false if infeasible.
  bool score(int v, int s, int L, bool with_later, __int128& val, __int128& inc_val) const {
    const int N = g.N;
    const size_t ui = (size_t)g.comps[v] * N + s;
    if ((*g.Ud)[ui]) return false;
    __int128 x = (*g.U)[ui];
    __int128 later = 0;
    const auto& nb = g.nbrs[v];
    for (size_t k = 0; k < nb.size(); ++k) {
      const int u = nb[k].var;
      if (u < L) {
        if (g.pd(nb[k], s, st[u])) return false;
        x += g.pv(nb[k], s, st[u]);
      } else if (u > v && with_later) {
        if (g.Rd[v][k][s]) return false;
        later += g.R[v][k][s];
      }
    }
    inc_val = x;
    val = x + later;
    return true;
  }

  bool lex_le_incumbent(int len) const {  // st[0..len) <= inc[0..len) lexicographically
    for (int i = 0; i < len; ++i) {
      if (st[i] < inc[i]) return true;
      if (st[i] > inc[i]) return false;
    }
    return true;
  }

  void dfs(int L, __int128 pv) {
    if (limit_hit) return;
    if (++nodes > limit) {
      limit_hit = true;
      return;
    }
    const int G = (int)g.comps.size();
    const int N = g.N;
    if (L == G) {
      if (!have || pv > best || (pv == best && std::lexicographical_compare(st.begin(), st.end(), inc.begin(),
                                                                           inc.end()))) {
        have = true;
        best = pv;
        inc = st;
      }
      return;
    }
    // optimistic bound of the free variables (L+1..G): free-free pairs charged to the earlier one
    __int128 rest = 0;
    for (int v = L + 1; v < G; ++v) {
      bool any = false;
      __int128 m = 0;
      for (int s = 0; s < N; ++s) {
        __int128 val, iv;
        if (!score(v, s, L, true, val, iv)) continue;
        if (!any || val > m) m = val, any = true;
      }
      if (!any) return;  // some free variable has no feasible state
      rest += m;
    }
    std::vector<std::pair<__int128, int>> cand;
    std::vector<__int128> incv(N);
    cand.reserve(N);
    for (int s = 0; s < N; ++s) {
      __int128 val, iv;
      if (!score(L, s, L, true, val, iv)) continue;
      incv[s] = iv;
      cand.emplace_back(val, s);
    }
    explored += (uint64_t)N;
    std::sort(cand.begin(), cand.end(), [](const std::pair<__int128, int>& a, const std::pair<__int128, int>& b) {
      return a.first > b.first || (a.first == b.first && a.second < b.second);
    });
    for (const auto& c : cand) {
      const __int128 ub = pv + c.first + rest;
      if (have && ub < best) break;  // sorted: every later candidate is bounded lower
      st[L] = c.second;
      if (have && ub == best && !lex_le_incumbent(L + 1)) {
        st[L] = -1;
        continue;
      }
      dfs(L + 1, pv + incv[c.second]);
      st[L] = -1;
      if (limit_hit) return;
    }
  }
};

}  // namespace

SolveResult solve(int N, int32_t ncomp, const int32_t* pairs, int64_t npairs, const int64_t* partials,
                  int32_t* comp_state_out, uint64_t node_limit) {
  SolveResult res;
  const int64_t uw = unary_words(N), pw = pair_words(N);
  std::vector<__int128> U((size_t)ncomp * N);
  std::vector<uint8_t> Ud((size_t)ncomp * N);
  std::vector<uint8_t> used(ncomp);
  for (int32_t c = 0; c < ncomp; ++c) {
    const int64_t* pc = partials + c * uw;
    used[c] = pc[5 * N] != 0;
    comp_state_out[c] = -1;
    for (int s = 0; s < N; ++s) {
      U[(size_t)c * N + s] = limbs_value(pc + 4 * s);
      Ud[(size_t)c * N + s] = pc[4 * N + s] != 0;
    }
  }
  std::vector<std::vector<__int128>> P(npairs);
  std::vector<std::vector<uint8_t>> Pd(npairs);
  std::vector<uint8_t> pused(npairs);
  const int64_t* pbase = partials + (int64_t)ncomp * uw;
  for (int64_t p = 0; p < npairs; ++p) {
    const int64_t* pp = pbase + p * pw;
    pused[p] = pp[5 * (int64_t)N * N] != 0;
    if (!pused[p]) continue;
    P[p].resize((size_t)N * N);
    Pd[p].resize((size_t)N * N);
    for (int64_t e = 0; e < (int64_t)N * N; ++e) {
      P[p][e] = limbs_value(pp + 4 * e);
      Pd[p][e] = pp[4 * (int64_t)N * N + e] != 0;
    }
  }
  // connected groups of used components
  std::vector<int32_t> parent(ncomp);
  std::iota(parent.begin(), parent.end(), 0);
  auto find = [&](int32_t x) {
    while (parent[x] != x) x = parent[x] = parent[parent[x]];
    return x;
  };
  for (int64_t p = 0; p < npairs; ++p)
    if (pused[p]) parent[find(pairs[2 * p])] = find(pairs[2 * p + 1]);
  std::vector<std::vector<int32_t>> groups(ncomp);
  for (int32_t c = 0; c < ncomp; ++c)
    if (used[c]) groups[find(c)].push_back(c);
  for (auto& comps : groups) {
    if (comps.empty()) continue;  // ascending by construction
    Group g;
    g.N = N;
    g.comps = comps;
    g.U = &U;
    g.Ud = &Ud;
    g.P = &P;
    g.Pd = &Pd;
    const int G = (int)comps.size();
    g.nbrs.resize(G);
    for (int64_t p = 0; p < npairs; ++p) {
      if (!pused[p]) continue;
      const auto i1 = std::lower_bound(comps.begin(), comps.end(), pairs[2 * p]);
      if (i1 == comps.end() || *i1 != pairs[2 * p]) continue;
      const int v1 = (int)(i1 - comps.begin());
      const int v2 = (int)(std::lower_bound(comps.begin(), comps.end(), pairs[2 * p + 1]) - comps.begin());
      g.nbrs[v1].push_back({v2, p, true});
      g.nbrs[v2].push_back({v1, p, false});
    }
    g.R.resize(G);
    g.Rd.resize(G);
    for (int v = 0; v < G; ++v) {
      g.R[v].resize(g.nbrs[v].size());
      g.Rd[v].resize(g.nbrs[v].size());
      for (size_t k = 0; k < g.nbrs[v].size(); ++k) {
        if (g.nbrs[v][k].var < v) continue;
        auto& r = g.R[v][k];
        auto& rd = g.Rd[v][k];
        r.assign(N, 0);
        rd.assign(N, 1);
        for (int s = 0; s < N; ++s)
          for (int s2 = 0; s2 < N; ++s2) {
            if (g.pd(g.nbrs[v][k], s, s2)) continue;
            const __int128 x = g.pv(g.nbrs[v][k], s, s2);
            if (rd[s] || x > r[s]) r[s] = x, rd[s] = 0;
          }
      }
    }
    Search S(g, node_limit > res.nodes ? node_limit - res.nodes : 0);
    S.dfs(0, 0);
    res.nodes += S.nodes;
    res.explored += S.explored;
    if (S.limit_hit) {
      res.limit_hit = true;
      return res;
    }
    if (S.have)
      for (int v = 0; v < G; ++v) comp_state_out[comps[v]] = S.inc[v];
  }
  return res;
}

}  // namespace cvcsp
