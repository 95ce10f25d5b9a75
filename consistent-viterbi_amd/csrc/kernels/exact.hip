// exact.hip -- unary terms of the constrained decode summed exactly on the device
// (the host form is constrained_partials_locked's loop over
// cvcsp::add_exact).  For every constrained sequence i and state s the term row (max-
// marginal mu for single-position sequences; prefix row delta and suffix mu for the first
// and last component of multi-position ones) is added, as the integer nearbyint(x * 2^64)
// in 4 limbs (exact_fixed.h), to its component's words: one thread per state accumulates a
// block's share of the sequences in LDS (thread-private columns, no atomics), then adds its
// words into the output with 64-bit atomics.  Integer sums: the result is the same words as
// the host loop, in any order.  f32 (the f32 trellis) or f64 (the exact-f64 trellis) terms; a
// term outside the exact unit's range (|x| >= 2^32) sets *bad instead of being added.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "../exact_fixed.h"
#include "exact.h"

namespace cvx {

template <typename REAL>
__global__ __launch_bounds__(256) void unary_sums(UnarySumArgs g) {
  extern __shared__ long long acc[];  // [cgroup][5][256]: 4 limbs + the -inf count, state-minor
  const int s = threadIdx.x;
  const int ncomp = g.cgroup;  // this launch's components [cbase, cbase + cgroup)
  for (int q = 0; q < ncomp * 5; ++q) acc[q * 256 + s] = 0;
  const int64_t per = (g.nc + gridDim.x - 1) / gridDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * per, i1 = min(g.nc, i0 + per);
  const REAL* mu = static_cast<const REAL*>(g.mu);
  const REAL* dl = static_cast<const REAL*>(g.dl);
  bool bad = false;
  auto add = [&](int c, REAL x) {
    c -= g.cbase;
    if ((unsigned)c >= (unsigned)ncomp) return;  // another launch's component
    long long* a = acc + (size_t)c * 5 * 256 + s;
    if (!(x > -INFINITY)) {
      a[4 * 256] += 1;
      return;
    }
    if (!term_in_range((double)x)) {  // outside the exact unit: the host reports CV_EINVAL
      bad = true;
      return;
    }
    int64_t l[4];
    fixed64_limbs(x, l);
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k * 256] += l[k];
  };
  if (s < g.nstates) {
    for (int64_t i = i0; i < i1; ++i) {
      const REAL m = mu[(size_t)i * g.np + s];
      if (i < g.n1) {
        add(g.c1[i], m);
      } else {
        add(g.c1[i], dl[(size_t)i * g.np + s]);
        add(g.cm[i], m);
      }
    }
    for (int c = 0; c < ncomp; ++c) {
      const long long* a = acc + (size_t)c * 5 * 256 + s;
      unsigned long long* u = reinterpret_cast<unsigned long long*>(g.part + (size_t)(g.cbase + c) * g.uw);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (a[k * 256]) atomicAdd(u + 4 * s + k, (unsigned long long)a[k * 256]);
      if (a[4 * 256]) atomicAdd(u + 4 * (size_t)g.nstates + s, (unsigned long long)a[4 * 256]);
    }
  }
  if (bad) atomicOr(g.bad, 1u);
}

hipError_t launch_unary_sums(const UnarySumArgs& g, int nblocks, hipStream_t stream) {
  if (g.nc <= 0) return hipSuccess;
  if (g.ncomp > kUnarySumMaxComp || g.nstates > 256 || !g.bad) return hipErrorInvalidValue;
  // kUnarySumGroup components per launch: 20 KiB of LDS, so the launches co-reside with the
  // workgroups of a long decode on the same CUs (eight-wave f64 forward: 128.5 KiB of the
  // CU's 160) instead of waiting for whole CUs (config 5: 21 ms -> ...)
  for (int cb = 0; cb < g.ncomp; cb += kUnarySumGroup) {
    UnarySumArgs q = g;
    q.cbase = cb;
    q.cgroup = std::min(kUnarySumGroup, g.ncomp - cb);
    const size_t lds = (size_t)q.cgroup * 5 * 256 * sizeof(long long);
    if (g.f64)
      hipLaunchKernelGGL(unary_sums<double>, dim3((unsigned)nblocks), dim3(256), lds, stream, q);
    else
      hipLaunchKernelGGL(unary_sums<float>, dim3((unsigned)nblocks), dim3(256), lds, stream, q);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace cvx
