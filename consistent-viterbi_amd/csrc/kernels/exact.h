// exact.h -- device exact sums of the constrained decode's unary terms (exact.hip).
// Internal to libcviterbi.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvx {

constexpr int kUnarySumMaxComp = 15;  // components summed on the device (one launch per kUnarySumGroup)

struct UnarySumArgs {
  const void* mu;     // [nc][np] suffix max-marginal rows (float, or double when f64)
  const void* dl;     // [nc][np] prefix last rows (multi-position sequences)
  const int32_t* c1;  // [nc] component of the first constrained element
  const int32_t* cm;  // [nc] component of the last constrained element
  int64_t nc, n1;     // sequences [0, n1) have one constrained element
  int np, nstates, ncomp;
  int f64;            // terms are double
  int64_t uw;         // int64 words per component (5N + 1)
  long long* part;    // [ncomp][uw], accumulated into
  unsigned* bad;      // set to nonzero when a term is outside the exact unit's range
  int cbase, cgroup;  // set by launch_unary_sums: one launch per kUnarySumGroup components
};
constexpr int kUnarySumGroup = 2;

hipError_t launch_unary_sums(const UnarySumArgs& g, int nblocks, hipStream_t stream);

}  // namespace cvx
