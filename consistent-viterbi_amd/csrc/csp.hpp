// Exact component-state search for the consistency-constrained decode (host side).
//
// The constrained objective decomposes over the constrained positions of each sequence
// (the cfn.rs:11-34 segment pattern): with positions t_1 < ... < t_m
// holding components c_1..c_m,
//   V(s_1..s_m) = alpha(s_1) + sum_k M_k(s_k, s_{k+1}) + beta(s_m)     (m >= 2)
//   V(s)        = mu(s) = f32(delta_{t}(s) + beta(s))                   (m == 1)
// alpha = forward row at t_1, M_k = segment table (start in s at t_k with score 0, run to
// t_{k+1}), beta = best continuation after t_m.  Summed over sequences this is a weighted
// CSP with unary terms U_c(s) and pairwise terms P_{c,c'}(s,s') only.  Every term is
// accumulated as an exact integer in units of 2^-64 (base-2^32 limbs in int64 words, so
// partials of disjoint shards add with one all-reduce SUM); -inf terms are counted.
//
// Partials layout (int64 words), N = states, pairs sorted (c1 < c2):
//   unary c:  [4N limbs (state-major)] [N -inf counts] [1 element count]        5N+1 words
//   pair p:   [4N^2 limbs, entry s1*N+s2] [N^2 -inf counts] [1 sequence count]  5N^2+1 words
#pragma once
#include <cstdint>
#include <vector>

namespace cvcsp {

inline int64_t unary_words(int N) { return 5 * (int64_t)N + 1; }
inline int64_t pair_words(int N) { return 5 * (int64_t)N * N + 1; }
inline int64_t partial_words(int N, int ncomp, int64_t npairs) {
  return (int64_t)ncomp * unary_words(N) + npairs * pair_words(N);
}

// Adds the exact value of x (units of 2^-64) into 4 limbs, or counts it as -inf; false (and
// nothing added) when |x| >= 2^32, outside the exact unit's range (exact_fixed.h).
bool add_exact(int64_t* limbs4, int64_t* ninf_count, float x);
bool add_exact(int64_t* limbs4, int64_t* ninf_count, double x);

// Pairs (c1 < c2) of different components that are consecutive constrained elements of
// some sequence, sorted and unique.
std::vector<int32_t> component_pairs(int64_t nseq, const int64_t* offsets, const int32_t* component);

// Index of pair (c1, c2), c1 < c2, in a sorted pair list, or -1.
int64_t pair_index(const int32_t* pairs, int64_t npairs, int32_t c1, int32_t c2);

struct SolveResult {
  uint64_t explored = 0;  // (component, state) candidates scored by the search
  uint64_t nodes = 0;
  bool limit_hit = false;
};

// Exact maximisation of sum_c U_c(s_c) + sum_p P_p(s_c1, s_c2) over the components that
// have constrained elements, one connected group (components linked by pairs) at a time.
// Ties: the lexicographically smallest state vector in component order (first argmax
// for a lone component).  comp_state_out[c] = -1 for unused components and for every
// component of a group without a feasible assignment.  Branch and bound, depth-first in
// decreasing optimistic value; stops with limit_hit after node_limit nodes.
SolveResult solve(int N, int32_t ncomp, const int32_t* pairs, int64_t npairs, const int64_t* partials,
                  int32_t* comp_state_out, uint64_t node_limit);

}  // namespace cvcsp
