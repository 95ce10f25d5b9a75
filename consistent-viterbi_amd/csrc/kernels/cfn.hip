// cfn.hip -- segment rows of the cost-function-network export (viterbi_solver/cfn.rs:11-80,
// SURVEY.md §8f rank 1).  write_cfn needs, for every pair of consecutive constraint
// boundaries and every start state n1, the f64 max-plus row of the super-sequence segment
// that starts at (t_from, n1) with score 0 (longest_path, cfn.rs:11-34), plus the start
// (cfn.rs:36-53) and end (cfn.rs:55-80) unary rows.  One workgroup per (segment, start state)
// job, one thread per state, the row double-buffered in LDS; every step is the reference's
// elementwise (row + transitions) -> max -> + emission in f64 (built with
// -ffp-contract=off; adds and max only, so the result is bit-identical to the Rust loop).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "cfn.h"

namespace cvcfn {

__global__ __launch_bounds__(256) void cfn_rows_f64(CfnArgs g) {
  extern __shared__ double smem[];  // two rows of N
  const CfnJob job = g.jobs[blockIdx.x];
  const int N = g.nstates;
  double* cur = smem;
  double* nxt = smem + N;
  const double NEG = -INFINITY;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    if (job.mode == kCfnStart)  // init_probs(sequence[0]) = pi + b[:, o] (hmm.rs:215-218)
      cur[j] = g.pi[j] + g.et[(size_t)g.obs[job.t_begin] * N + j];
    else  // score 0 at the start state, -inf elsewhere (cfn.rs:12-13, 60-61)
      cur[j] = (j == job.state) ? 0.0 : NEG;
  }
  __syncthreads();
  for (int64_t t = job.t_begin + 1; t <= job.t_end; ++t) {
    // constrained elements take the start state: inside the segment (cfn.rs:16-18) or up to
    // and including the last element for the end cost (cfn.rs:63-67); never for the start
    // cost (cfn.rs:44-50)
    const bool forced = g.comp[t] >= 0 && job.mode != kCfnStart && (t < job.t_end || job.mode == kCfnEnd);
    const bool first = g.seq_start[t] != 0;  // MetaElements::transitions at t == 0: pi (utils.rs:32-38)
    const double* et = g.et + (size_t)g.obs[t] * N;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      double v = NEG;
      if (!forced || j == job.state) {
        double m = NEG;
        for (int i = 0; i < N; ++i) {
          const double x = cur[i] + (first ? g.pi[j] : g.a[(size_t)i * N + j]);
          m = x > m ? x : m;
        }
        v = m + et[j];
      }
      nxt[j] = v;
    }
    __syncthreads();
    double* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  for (int j = threadIdx.x; j < N; j += blockDim.x) g.out[(size_t)blockIdx.x * N + j] = cur[j];
}

hipError_t launch_cfn_rows(const CfnArgs& g, int64_t njobs, hipStream_t stream) {
  if (njobs <= 0) return hipSuccess;
  const size_t lds = 2 * (size_t)g.nstates * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cfn_rows_f64), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(cfn_rows_f64, dim3((unsigned)njobs), dim3(256), lds, stream, g);
  return hipGetLastError();
}

}  // namespace cvcfn
