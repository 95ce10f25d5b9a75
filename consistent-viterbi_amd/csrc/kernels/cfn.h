// cfn.h -- job list and launcher of the CFN segment-row kernel (cfn.hip).
// Internal to libcviterbi; the public entry point is cv_solver_write_cfn (include/cviterbi.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvcfn {

// job modes: the three row computations of cfn.rs
constexpr int32_t kCfnSegment = 0;  // longest_path (cfn.rs:11-34): start (t_begin, state) = 0,
                                    // constrained elements before t_end forced to state
constexpr int32_t kCfnEnd = 1;      // get_unary_end_cost (cfn.rs:55-80): same, forced through t_end
constexpr int32_t kCfnStart = 2;    // get_unary_start_cost (cfn.rs:36-53): init_probs at t_begin

struct CfnJob {
  int64_t t_begin, t_end;  // super-sequence element range; the row at t_end is the output
  int32_t state;           // start state (unused for kCfnStart)
  int32_t mode;
};

struct CfnArgs {
  const CfnJob* jobs;
  const int32_t* obs;        // [elements] observation index
  const int32_t* comp;       // [elements] active constraint component, -1 = none
  const uint8_t* seq_start;  // [elements] 1 at the first element of each sequence
  const double* a;           // [N][N] log10, from-major
  const double* et;          // [V][N] log10 emissions, transposed
  const double* pi;          // [N]
  int nstates;
  double* out;               // [jobs][N]
};

hipError_t launch_cfn_rows(const CfnArgs& g, int64_t njobs, hipStream_t stream);

}  // namespace cvcfn
