// wide.h -- the candidate loop of the wide super-sequence chain (cp_chain_wide_step in
// trellis64.hip): one state per thread, its predecessors' values staged through LDS, the table
// column streamed from L2 / HBM with the loads pipelined (per element at N = 10,240: 1.13 ->
// 0.73 ms, 4,096: 0.33 -> 0.23 ms against the plain unrolled loop; the batch decode's
// generic_wide_step keeps the plain loop, which won at few sequences).
#pragma once
#include <hip/hip_runtime.h>

namespace cvk {

// The candidate loop: the S previous rows staged through LDS in tiles of
// 256 (the next tile's values loaded a tile ahead), the table column in two rings of U loads,
// one ring in flight while the other is compared -- a plain loop waited one L2 / HBM round trip
// per U candidates.  Entries past N are -inf in the
// tile (their table loads clamped): never strictly above the maximum, so the first index
// still wins and the results are generic_fwd's.  Every thread of the workgroup runs it (the
// barriers); DP: c = (a + e) + d, else s = d + a.
// col == nullptr: every table value is kval (the super-sequence chain's sequence start, where
// the predecessor term is the constant pi[j], utils.rs:32-38).
template <typename REAL, int S, bool DP>
__device__ __forceinline__ void wide_candidates(const REAL* __restrict__ col, int N, const REAL* const (&prev)[S],
                                                const REAL (&e)[S], REAL (&best)[S], int (&arg)[S], REAL* tile,
                                                REAL kval = REAL(0)) {
  constexpr int U = 8;
  const int tid = threadIdx.x;
  const REAL ninf = -__builtin_inf();
  REAL ra[U], rb[U], tn[S];
  auto load_a = [&](int i0, REAL(&r)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = col ? col[(size_t)min(i0 + u, N - 1) * N] : kval;
  };
  auto load_t = [&](int i0) {
#pragma unroll
    for (int s = 0; s < S; ++s) tn[s] = i0 + tid < N ? prev[s][i0 + tid] : ninf;
  };
  auto cmp = [&](const REAL(&r)[U], int i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const REAL d = tile[s * 256 + ((i0 + u) & 255)];
        const REAL x = DP ? (r[u] + e[s]) + d : d + r[u];
        if (x > best[s]) {
          best[s] = x;
          arg[s] = i0 + u;
        }
      }
    }
  };
#pragma unroll
  for (int s = 0; s < S; ++s) {
    best[s] = ninf;
    arg[s] = 0;
  }
  load_t(0);
  load_a(0, ra);
  load_a(U, rb);
  for (int i0 = 0; i0 < N; i0 += 2 * U) {
    if ((i0 & 255) == 0) {  // a new tile: the values loaded a tile ago
      __syncthreads();
#pragma unroll
      for (int s = 0; s < S; ++s) tile[s * 256 + tid] = tn[s];
      __syncthreads();
      load_t(i0 + 256);
    }
    cmp(ra, i0);
    load_a(i0 + 2 * U, ra);
    cmp(rb, i0 + U);
    load_a(i0 + 3 * U, rb);
  }
}

}  // namespace cvk
