// fit.hip -- MI355X (gfx950) kernels for fitting the HMM:
//   mle_counts     exact integer counts of hmm.rs:30-62 (maximum_likelihood_estimation)
//   bw_forward     scaled, tag-clamped forward pass of hmm.rs:78-100 (train)
//   bw_backward    scaled, tag-clamped backward pass of hmm.rs:102-121
//   bw_stats       gamma (hmm.rs:124-131), xi (hmm.rs:133-143) and the E-step sums of
//                  hmm.rs:145-170, accumulated per sequence and added to global sums
// f64 throughout, probability space, like the reference.  One workgroup (256 threads) per
// sequence; thread i < N owns state i.  The transition matrix is read from L2 (row-major A
// for the forward step, A^T for the backward and xi steps, so every read is coalesced
// across the threads of a row).  bw_stats keeps the sequence's xi sum (N x N) in LDS up to
// N = 128 (the reference trains POS taggers: N = 12; it has no limit on N).  For N <= 64 the
// one-wave-per-sequence kernels below (bw_fwd_wave, bw_bwd_stats_wave) replace all three.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "fit.h"
#include "../tuning.h"

namespace cvf {

typedef double f64x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double block_sum(double v, double* red) {
  // 256 threads = 4 waves: wave shuffle-reduce, then across the 4 waves through LDS
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // red[] may still be read by the previous call
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// normalize (hmm.rs:274-282): v / sum, or 1/len when the sum is 0
#ifndef CVF_ABL_NODIV
__device__ __forceinline__ double normalized(double v, double s, int n) { return s != 0.0 ? v / s : 1.0 / n; }
#else
__device__ __forceinline__ double normalized(double v, double s, int n) { return s != 0.0 ? v * s : 1.0 / n; }
#endif

// xi without overflow.  The reference normalises each xi_t entry by entry (hmm.rs:135-141:
// A o (alpha_t (x) u_{t+1}) / c_t, every entry <= 1); the kernels factor it as
// A o sum_t (alpha_t / c_t) (x) u_{t+1}, and alpha / c overflows once c_t is subnormal (an EM
// run drifting to tiny emissions: seen at N = 256 after ~250 iterations).  So the factors are
// balanced by a power of two: r = alpha / (c 2^k), u' = u 2^k with 2^k ~ 1 / sqrt(c max u) --
// exact scalings whose product is the same; both factors stay below ~2^540.
__device__ __forceinline__ int xi_scale(double c, double umax) {
  if (!(c > 0.0) || !(umax > 0.0)) return 0;
  return -(ilogb(c) + ilogb(umax)) / 2;
}

// a select of two computed values: without the empty asm the compiler turns a per-lane `?:`
// with arithmetic on one side into an exec-masked branch, and a branch here waits for every
// outstanding load (vmcnt(0))
__device__ __forceinline__ double sel(bool c, double a, double b) {
  asm("" : "+v"(a));
  asm("" : "+v"(b));
  return c ? a : b;
}

__device__ __forceinline__ double block_max(double v, double* red) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

__global__ __launch_bounds__(256) void mle_counts(MleArgs g) {
  const int64_t seq = blockIdx.x;
  const int64_t e0 = g.offsets[seq], e1 = g.offsets[seq + 1];
  const int N = g.nstates;
  if (e1 <= e0) return;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
    const int s = g.tags[e];
    atomicAdd(reinterpret_cast<unsigned long long*>(&g.b_cnt[(size_t)s * g.nobs + g.obs[e]]), 1ull);
    atomicAdd(reinterpret_cast<unsigned long long*>(&g.seen[s]), 1ull);
    if (e + 1 < e1) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&g.a_cnt[(size_t)s * N + g.tags[e + 1]]), 1ull);
    } else {
      atomicAdd(reinterpret_cast<unsigned long long*>(&g.end[s]), 1ull);
    }
    if (e == e0) atomicAdd(reinterpret_cast<unsigned long long*>(&g.pi_cnt[s]), 1ull);
  }
}

__global__ __launch_bounds__(256) void bw_forward(BwArgs g) {
  __shared__ double x[256];
  __shared__ double red[4];
  const int64_t seq = blockIdx.x;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const int N = g.nstates;
  const int i = threadIdx.x;
  if (T <= 0) return;
  double* al = g.alpha + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  const int32_t* tag = g.tags + e0;
  // t = 0 (hmm.rs:81-88): tagged -> one-hot, else normalize(pi * b(o_0))
  {
    const int tg = tag[0];
    const double y = (i < N) ? g.pi[i] * g.et[(size_t)obs[0] * N + i] : 0.0;
    const double s = block_sum(y, red);
    if (i < N) al[i] = tg >= 0 ? (i == tg ? 1.0 : 0.0) : normalized(y, s, N);
  }
  for (int t = 1; t < T; ++t) {
    const int tg = tag[t];  // uniform
    if (tg >= 0) {          // hmm.rs:91
      if (i < N) al[(size_t)t * N + i] = (i == tg) ? 1.0 : 0.0;
      continue;
    }
    // (alpha[t-1] * b(o_t)) . A  -- hmm.rs:93-94, emission applied as written
    __syncthreads();
    if (i < N) x[i] = al[(size_t)(t - 1) * N + i] * g.et[(size_t)obs[t] * N + i];
    __syncthreads();
    double y = 0.0;
    if (i < N)
      for (int k = 0; k < N; ++k) y += x[k] * g.a[(size_t)k * N + i];
    const double s = block_sum(y, red);
    if (i < N) al[(size_t)t * N + i] = normalized(y, s, N);
  }
}

__global__ __launch_bounds__(256) void bw_backward(BwArgs g) {
  __shared__ double x[256];
  __shared__ double red[4];
  const int64_t seq = blockIdx.x;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const int N = g.nstates;
  const int i = threadIdx.x;
  if (T <= 0) return;
  double* be = g.beta + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  const int32_t* tag = g.tags + e0;
  {  // t = T-1 (hmm.rs:105-108): tagged -> one-hot, else ones
    const int tg = tag[T - 1];
    if (i < N) be[(size_t)(T - 1) * N + i] = tg >= 0 ? (i == tg ? 1.0 : 0.0) : 1.0;
  }
  for (int t = T - 2; t >= 0; --t) {
    const int tg = tag[t];
    if (tg >= 0) {
      if (i < N) be[(size_t)t * N + i] = (i == tg) ? 1.0 : 0.0;
      continue;
    }
    // (beta[t+1] * b(o_{t+1})) . A^T  -- hmm.rs:113-116
    __syncthreads();
    if (i < N) x[i] = be[(size_t)(t + 1) * N + i] * g.et[(size_t)obs[t + 1] * N + i];
    __syncthreads();
    double y = 0.0;
    if (i < N)
      for (int k = 0; k < N; ++k) y += x[k] * g.at[(size_t)k * N + i];
    const double s = block_sum(y, red);
    if (i < N) be[(size_t)t * N + i] = normalized(y, s, N);
  }
}

// ---- N > 256 (up to kBwMaxStates): the per-sequence kernels with the states strided over the
// 256 threads (thread i owns states i, i + 256, ...), the vector operand and (stats) the owned
// states' gamma sums in dynamic LDS; the xi sum is the GEMM over the rows, as for N <= 256.
// One workgroup per sequence and all of A per step: a correctness path for large models (the
// reference trains any N, hmm.rs:69-190), not a tuned one.  GS: the vectors in global scratch
// (g.gscratch, 4 N doubles per workgroup: N > kBwLdsMaxStates), the same values.
template <bool GS>
__global__ __launch_bounds__(256) void bw_forward_g(BwArgs g) {
  extern __shared__ double xs_lds[];
  double* xs = GS ? g.gscratch + (size_t)blockIdx.x * 4 * g.nstates : xs_lds;  // [N]
  __shared__ double red[4];
  const int64_t e0 = g.offsets[blockIdx.x];
  const int T = (int)(g.offsets[blockIdx.x + 1] - e0);
  const int N = g.nstates, tid = threadIdx.x;
  if (T <= 0) return;
  double* al = g.alpha + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  const int32_t* tag = g.tags + e0;
  {  // t = 0 (hmm.rs:81-88)
    const int tg = tag[0];
    double part = 0.0;
    for (int i = tid; i < N; i += 256) {
      const double y = g.pi[i] * g.et[(size_t)obs[0] * N + i];
      al[i] = y;
      part += y;
    }
    const double s = block_sum(part, red);
    for (int i = tid; i < N; i += 256) al[i] = tg >= 0 ? (i == tg ? 1.0 : 0.0) : normalized(al[i], s, N);
  }
  for (int t = 1; t < T; ++t) {
    const int tg = tag[t];  // uniform
    double* row = al + (size_t)t * N;
    if (tg >= 0) {  // hmm.rs:91
      for (int i = tid; i < N; i += 256) row[i] = (i == tg) ? 1.0 : 0.0;
      continue;
    }
    __syncthreads();  // xs free
    for (int i = tid; i < N; i += 256) xs[i] = row[i - N] * g.et[(size_t)obs[t] * N + i];
    __syncthreads();
    double part = 0.0;
    for (int i = tid; i < N; i += 256) {  // (alpha[t-1] * b(o_t)) . A  -- hmm.rs:93-94
      double y = 0.0;
      for (int k = 0; k < N; ++k) y += xs[k] * g.a[(size_t)k * N + i];
      row[i] = y;
      part += y;
    }
    const double s = block_sum(part, red);
    for (int i = tid; i < N; i += 256) row[i] = normalized(row[i], s, N);
  }
}

template <bool GS>
__global__ __launch_bounds__(256) void bw_backward_g(BwArgs g) {
  extern __shared__ double xs_lds[];
  double* xs = GS ? g.gscratch + (size_t)blockIdx.x * 4 * g.nstates : xs_lds;  // [N]
  __shared__ double red[4];
  const int64_t e0 = g.offsets[blockIdx.x];
  const int T = (int)(g.offsets[blockIdx.x + 1] - e0);
  const int N = g.nstates, tid = threadIdx.x;
  if (T <= 0) return;
  double* be = g.beta + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  const int32_t* tag = g.tags + e0;
  {  // t = T-1 (hmm.rs:105-108)
    const int tg = tag[T - 1];
    for (int i = tid; i < N; i += 256) be[(size_t)(T - 1) * N + i] = tg >= 0 ? (i == tg ? 1.0 : 0.0) : 1.0;
  }
  for (int t = T - 2; t >= 0; --t) {
    const int tg = tag[t];
    double* row = be + (size_t)t * N;
    if (tg >= 0) {
      for (int i = tid; i < N; i += 256) row[i] = (i == tg) ? 1.0 : 0.0;
      continue;
    }
    __syncthreads();
    for (int i = tid; i < N; i += 256) xs[i] = row[i + N] * g.et[(size_t)obs[t + 1] * N + i];
    __syncthreads();
    double part = 0.0;
    for (int i = tid; i < N; i += 256) {  // (beta[t+1] * b(o_{t+1})) . A^T  -- hmm.rs:113-116
      double y = 0.0;
      for (int k = 0; k < N; ++k) y += xs[k] * g.at[(size_t)k * N + i];
      row[i] = y;
      part += y;
    }
    const double s = block_sum(part, red);
    for (int i = tid; i < N; i += 256) row[i] = normalized(row[i], s, N);
  }
}

// gamma and xi of one sequence (as bw_stats_rows): r_t over alpha's row t, u_{t+1} 2^k over
// beta's row t, zeros at the last step; the gamma sums of the owned states in LDS
template <bool GS>
__global__ __launch_bounds__(256) void bw_stats_rows_g(BwArgs g) {
  extern __shared__ double sm_lds[];
  double* sm = GS ? g.gscratch + (size_t)blockIdx.x * 4 * g.nstates : sm_lds;  // ps[N] | pi_acc[N] | a_den[N] | b_den[N]
  __shared__ double red[4];
  const int64_t e0 = g.offsets[blockIdx.x];
  const int T = (int)(g.offsets[blockIdx.x + 1] - e0);
  const int N = g.nstates, tid = threadIdx.x;
  if (T <= 0) return;
  double *ps = sm, *sp = sm + N, *sa = sm + 2 * N, *sb = sm + 3 * N;
  for (int i = tid; i < N; i += 256) sp[i] = sa[i] = sb[i] = 0.0;
  double* al = g.alpha + (e0 - g.elem_base) * N;
  double* be = g.beta + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  double z = 0.0;
  for (int t = 0; t < T; ++t) {
    double* ar = al + (size_t)t * N;
    double* br = be + (size_t)t * N;
    double part = 0.0;
    for (int i = tid; i < N; i += 256) part += ar[i] * br[i];
    const double s = block_sum(part, red);
    for (int i = tid; i < N; i += 256) {  // gamma_t (hmm.rs:127-129) into the sums
      const double gm = normalized(ar[i] * br[i], s, N);
      if (t == 0) sp[i] += gm;
      if (t < T - 1) sa[i] += gm;
      sb[i] += gm;
      unsafeAtomicAdd(&g.b_num[(size_t)obs[t] * N + i], gm);  // hmm.rs:155-163
    }
    if (t + 1 < T) {
      __syncthreads();  // ps free
      for (int i = tid; i < N; i += 256) ps[i] = g.et[(size_t)obs[t + 1] * N + i] * br[i + N];
      __syncthreads();
      double pc = 0.0, pu = 0.0;
      for (int i = tid; i < N; i += 256) {  // w_i = sum_j A[i][j] u_j; c = alpha_t . w
        double w = 0.0;
        for (int j = 0; j < N; ++j) w += g.at[(size_t)j * N + i] * ps[j];
        pc += ar[i] * w;
        pu = fmax(pu, ps[i]);
      }
      const double c = block_sum(pc, red);
      const int ks = xi_scale(c, block_max(pu, red));  // balanced factors
      for (int i = tid; i < N; i += 256) {
        const double r = c != 0.0 ? ar[i] / __builtin_ldexp(c, ks) : 0.0;
        const double u = __builtin_ldexp(ps[i], ks);
        ar[i] = r;
        br[i] = u;
      }
      if (tid == 0 && c == 0.0) z += 1.0;  // xi_t uniform (hmm.rs:306-317)
    } else {
      for (int i = tid; i < N; i += 256) ar[i] = br[i] = 0.0;
    }
  }
  for (int i = tid; i < N; i += 256) {
    unsafeAtomicAdd(&g.pi_acc[i], sp[i]);
    unsafeAtomicAdd(&g.a_den[i], sa[i]);
    unsafeAtomicAdd(&g.b_den[i], sb[i]);
  }
  if (tid == 0 && z != 0.0) unsafeAtomicAdd(g.xi_zero, z);
}

// E-step sums of one sequence.  xi_t = normalize(A o (alpha_t (x) u_{t+1})), u = b(o_{t+1}) o
// beta_{t+1} (hmm.rs:135-141); its sum c_t = alpha_t . (A u_{t+1}), so sum_t xi_t =
// A o S + z / N^2 with S = sum over c_t != 0 of (alpha_t / c_t) (x) u_{t+1} and z = #{c_t == 0}
// (those xi_t are uniform).  S is kept in LDS: S[k][i] with thread i owning column i.
__global__ __launch_bounds__(256) void bw_stats(BwArgs g) {
  extern __shared__ double smem[];  // S[N*N] | p[256] | red[4]
  const int64_t seq = blockIdx.x;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const int N = g.nstates;
  const int i = threadIdx.x;
  if (T <= 0) return;
  double* S = smem;
  double* p = smem + (size_t)N * N;
  double* red = p + 256;
  for (int k = i; k < N * N; k += blockDim.x) S[k] = 0.0;
  const double* al = g.alpha + (e0 - g.elem_base) * N;
  const double* be = g.beta + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  double pi_acc = 0.0, a_den = 0.0, b_den = 0.0, z = 0.0;
  for (int t = 0; t < T; ++t) {
    // gamma_t = normalize(alpha_t * beta_t)  (hmm.rs:127-129)
    const double ab = (i < N) ? al[(size_t)t * N + i] * be[(size_t)t * N + i] : 0.0;
    const double s = block_sum(ab, red);
    if (i < N) {
      const double gm = normalized(ab, s, N);
      if (t == 0) pi_acc += gm;
      if (t < T - 1) a_den += gm;
      b_den += gm;
      unsafeAtomicAdd(&g.b_num[(size_t)obs[t] * N + i], gm);  // new_b[state][obs] += gamma (hmm.rs:155-163)
    }
    if (t + 1 < T) {
      // u_j = b(o_{t+1})[j] * beta_{t+1}[j];  w_i = sum_j A[i][j] u_j;  c = alpha_t . w
      __syncthreads();
      if (i < N) p[i] = g.et[(size_t)obs[t + 1] * N + i] * be[(size_t)(t + 1) * N + i];
      __syncthreads();
      double w = 0.0;
      if (i < N)
        for (int k = 0; k < N; ++k) w += g.at[(size_t)k * N + i] * p[k];
      const double ai = (i < N) ? al[(size_t)t * N + i] : 0.0;
      const double c = block_sum(ai * w, red);
      if (c != 0.0) {
        // S[k][j] += (alpha_t[k] / c) * u_j: thread j = i owns column i; alpha/c via LDS,
        // both factors balanced by 2^k (xi_scale)
        const int ks = xi_scale(c, block_max((i < N) ? p[i] : 0.0, red));
        const double uj = (i < N) ? __builtin_ldexp(p[i], ks) : 0.0;
        __syncthreads();
        if (i < N) p[i] = ai / __builtin_ldexp(c, ks);
        __syncthreads();
        if (i < N)
          for (int k = 0; k < N; ++k) S[(size_t)k * N + i] += p[k] * uj;
      } else {
        z += 1.0;
      }
    }
  }
  __syncthreads();
  if (i < N) {
    unsafeAtomicAdd(&g.pi_acc[i], pi_acc);
    unsafeAtomicAdd(&g.a_den[i], a_den);
    unsafeAtomicAdd(&g.b_den[i], b_den);
  }
  for (int k = i; k < N * N; k += blockDim.x) unsafeAtomicAdd(&g.xi_s[k], S[k]);
  if (i == 0 && z != 0.0) unsafeAtomicAdd(g.xi_zero, z);
}

// ---- 128 < N <= 256: the xi sum as a GEMM ---------------------------------------------------
// S (N x N, 512 KiB at N = 256) no longer fits LDS.  bw_stats_rows computes the same per-step
// quantities as bw_stats but, instead of the rank-1 update S += r_t (x) u_{t+1}, writes
// r_t = alpha_t / c_t (0 when c_t == 0) over alpha's row t and u_{t+1} over beta's row t (both
// rows are dead by then: alpha_t and beta_t were last read for gamma_t and xi_t; beta_{t+1} is
// read in this step, rewritten in the next), and zeros at the last step of each sequence.  Then
// sum_t S_t = R^T U over all rows of the chunk: bw_xi_gemm, on the matrix cores.
__global__ __launch_bounds__(256) void bw_stats_rows(BwArgs g) {
  __shared__ double p[256];
  __shared__ double red[4];
  const int64_t seq = blockIdx.x;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const int N = g.nstates;
  const int i = threadIdx.x;
  if (T <= 0) return;
  double* al = g.alpha + (e0 - g.elem_base) * N;
  double* be = g.beta + (e0 - g.elem_base) * N;
  const int32_t* obs = g.obs + e0;
  double pi_acc = 0.0, a_den = 0.0, b_den = 0.0, z = 0.0;
  for (int t = 0; t < T; ++t) {
    // gamma_t = normalize(alpha_t * beta_t)  (hmm.rs:127-129)
    const double ai = (i < N) ? al[(size_t)t * N + i] : 0.0;
    const double ab = (i < N) ? ai * be[(size_t)t * N + i] : 0.0;
    const double s = block_sum(ab, red);
    if (i < N) {
      const double gm = normalized(ab, s, N);
      if (t == 0) pi_acc += gm;
      if (t < T - 1) a_den += gm;
      b_den += gm;
      unsafeAtomicAdd(&g.b_num[(size_t)obs[t] * N + i], gm);  // hmm.rs:155-163
    }
    double r = 0.0, u = 0.0;
    if (t + 1 < T) {
      // u_j = b(o_{t+1})[j] * beta_{t+1}[j];  w_i = sum_j A[i][j] u_j;  c = alpha_t . w
      __syncthreads();
      if (i < N) p[i] = g.et[(size_t)obs[t + 1] * N + i] * be[(size_t)(t + 1) * N + i];
      __syncthreads();
      double w = 0.0;
      if (i < N)
        for (int k = 0; k < N; ++k) w += g.at[(size_t)k * N + i] * p[k];
      const double c = block_sum(ai * w, red);
      const int ks = xi_scale(c, block_max((i < N) ? p[i] : 0.0, red));  // balanced factors
      u = (i < N) ? __builtin_ldexp(p[i], ks) : 0.0;
      if (c != 0.0) r = ai / __builtin_ldexp(c, ks);
      else z += 1.0;  // xi_t uniform (hmm.rs:306-317), counted separately
    }
    if (i < N) {
      al[(size_t)t * N + i] = r;
      be[(size_t)t * N + i] = u;
    }
  }
  if (i < N) {
    unsafeAtomicAdd(&g.pi_acc[i], pi_acc);
    unsafeAtomicAdd(&g.a_den[i], a_den);
    unsafeAtomicAdd(&g.b_den[i], b_den);
  }
  if (i == 0 && z != 0.0) unsafeAtomicAdd(g.xi_zero, z);
}

// xi_s[m][n] += sum_r R[r][m] U[r][n] over rows [0, nrows) (R = alpha rows, U = beta rows of
// bw_stats_rows / bw_bwd_mm).  One wave per (16 TM)^2 output tile and row range: per 4 rows,
// lane l feeds R[r + l/16][m0 + 16 mt + l%16] and U[...][n0 + 16 nt + l%16] into TM^2
// v_mfma_f64_16x16x4_f64 (TM = 4: 16 MFMAs per 8 loads, each row of R and U read by N/64
// waves); one atomic flush of the tile at the end.
template <int TM, int ST>
__global__ __launch_bounds__(64, 2) void bw_xi_gemm(BwArgs g, int64_t nrows, int64_t rows_per_wave) {
  constexpr int TS = 16 * TM;
  const int N = g.nstates;
  const int ntt = (N + TS - 1) / TS;
  // XCD-aware: workgroup b runs on XCD b % 8 (round-robin dispatch), so the ntt^2 tiles of one
  // row range are the blocks b = 8 (part / 8 * ntt^2 + tile) + part % 8 -- one XCD, dispatched
  // together: the range's rows come from HBM once into that XCD's L2 and serve every tile
#ifndef CVF_GEMM_NOXCD
  const int64_t b = blockIdx.x, j = b / 8;
  const int tile = (int)(j % (ntt * ntt));
  const int64_t part = (j / (ntt * ntt)) * 8 + b % 8;
#else
  const int tile = blockIdx.x % (ntt * ntt);
  const int64_t part = blockIdx.x / (ntt * ntt);
#endif
  const int m0 = TS * (tile / ntt), n0 = TS * (tile % ntt);
  const int l = threadIdx.x, kk = l >> 4, cl = l & 15;
  const int64_t r0 = part * rows_per_wave, r1 = r0 + rows_per_wave < nrows ? r0 + rows_per_wave : nrows;
  if (r0 >= nrows) return;  // padding blocks of the XCD mapping (wave-uniform)
  f64x4_t acc[TM][TM];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f64x4_t{0.0, 0.0, 0.0, 0.0};
  int cm[TM], cn[TM];
  bool vm[TM], vn[TM];
#pragma unroll
  for (int q = 0; q < TM; ++q) {
    cm[q] = m0 + 16 * q + cl;
    cn[q] = n0 + 16 * q + cl;
    vm[q] = cm[q] < N;
    vn[q] = cn[q] < N;
    cm[q] = min(cm[q], N - 1);
    cn[q] = min(cn[q], N - 1);
  }
  // per 4 rows: TM loads of R and of U (lane l: row r + l/16, column l%16 of each 16-wide
  // tile), masked loads (a select on a loaded value cost ~30% here); ST = 2 issues the next 4
  // rows' loads before the current rows' MFMAs
  auto mma = [&](const double (&av)[TM], const double (&bv)[TM]) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
  };
#define CVF_GEMM_LOAD(RR, AV, BV)                                            \
  {                                                                          \
    const int64_t row_ = (RR) + kk;                                          \
    const bool vr_ = row_ < r1;                                              \
    const double* R_ = g.alpha + (size_t)(vr_ ? row_ : r0) * N;              \
    const double* U_ = g.beta + (size_t)(vr_ ? row_ : r0) * N;               \
    const double rs_ = g.rscale ? g.rscale[vr_ ? row_ : r0] : 1.0;           \
    _Pragma("unroll") for (int q = 0; q < TM; ++q) {                         \
      AV[q] = (vr_ && vm[q]) ? R_[cm[q]] * rs_ : 0.0;                        \
      BV[q] = (vr_ && vn[q]) ? U_[cn[q]] : 0.0;                              \
    }                                                                        \
  }
  if constexpr (ST == 2) {
    double a0[TM], b0[TM], a1[TM], b1[TM];
    CVF_GEMM_LOAD(r0, a0, b0)
    for (int64_t r = r0; r < r1; r += 8) {
      CVF_GEMM_LOAD(r + 4, a1, b1)
      mma(a0, b0);
      CVF_GEMM_LOAD(r + 8, a0, b0)
      mma(a1, b1);
    }
  } else {
    for (int64_t r = r0; r < r1; r += 4) {
      double av[TM], bv[TM];
      CVF_GEMM_LOAD(r, av, bv)
      mma(av, bv);
    }
  }
#undef CVF_GEMM_LOAD
  // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 16 * a + (l >> 4) + 4 * q, col = n0 + 16 * b + (l & 15);
        if (row < N && col < N && acc[a][b][q] != 0.0) unsafeAtomicAdd(&g.xi_s[(size_t)row * N + col], acc[a][b][q]);
      }
}

// The same sum with 128 x 128 output tiles per workgroup (four waves of 64 x 64): 16 rows of R
// and U at a time go through LDS (double-buffered, 64 KiB), so each row segment comes from L2
// once per workgroup instead of once per wave -- half the L2 traffic of bw_xi_gemm<4> at 256
// states.  Row ranges and the XCD-aware block map as above.
constexpr int kGemmKB = 16;  // rows per LDS stage
__global__ __launch_bounds__(256, 2) void bw_xi_gemm_lds(BwArgs g, int64_t nrows, int64_t rows_per_wg) {
  constexpr int TS = 128, KB = kGemmKB, LS = TS + 2;  // LS: row stride (doubles) of a stage
  __shared__ __attribute__((aligned(16))) double rs[2][KB * LS], us[2][KB * LS];
  const int N = g.nstates;
  const int ntt = (N + TS - 1) / TS;
  const int64_t b = blockIdx.x, j = b / 8;
  const int tile = (int)(j % (ntt * ntt));
  const int64_t part = (j / (ntt * ntt)) * 8 + b % 8;
  const int m0 = TS * (tile / ntt), n0 = TS * (tile % ntt);
  const int64_t r0 = part * rows_per_wg;
  if (r0 >= nrows) return;  // workgroup-uniform (padding blocks)
  const int64_t r1 = r0 + rows_per_wg < nrows ? r0 + rows_per_wg : nrows;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, kk = l >> 4, cl = l & 15;
  const int wm = w >> 1, wn = w & 1;
  // staging: thread tid copies row (tid >> 4) of R and U, 8 doubles from column 8 (tid & 15);
  // A/B: 16-byte loads of strided column pairs with forced selects (2-way LDS write conflicts)
  // 98 vs 79 ms, 8-byte strided loads 109 ms
  const int srow = tid >> 4, scol = 8 * (tid & 15);
  double rsc = 1.0;  // the staged row's R scale
  auto stage_load = [&](int64_t rb, double (&ra)[8], double (&ua)[8]) {
    const int64_t row = rb + srow;
    const bool vr = row < r1;
    const double* R = g.alpha + (size_t)(vr ? row : r0) * N;
    const double* U = g.beta + (size_t)(vr ? row : r0) * N;
    rsc = g.rscale ? g.rscale[vr ? row : r0] : 1.0;  // R = alpha rscale (bw_bwd_mm), applied at the LDS write
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int cm = m0 + scol + q, cn = n0 + scol + q;
      ra[q] = (vr && cm < N) ? R[cm] : 0.0;
      ua[q] = (vr && cn < N) ? U[cn] : 0.0;
    }
  };
  auto stage_store = [&](int buf, const double (&ra)[8], const double (&ua)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      rs[buf][srow * LS + scol + q] = ra[q] * rsc;
      us[buf][srow * LS + scol + q] = ua[q];
    }
  };
  f64x4_t acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f64x4_t{0.0, 0.0, 0.0, 0.0};
  double ra[8], ua[8];
  stage_load(r0, ra, ua);
  stage_store(0, ra, ua);
  __syncthreads();
  int buf = 0;
  for (int64_t rb = r0; rb < r1; rb += KB) {
    const bool next = rb + KB < r1;  // workgroup-uniform
    if (next) stage_load(rb + KB, ra, ua);  // in flight during this stage's products
#pragma unroll
    for (int ks = 0; ks < KB / 4; ++ks) {
      const int row = 4 * ks + kk;
      double av[4], bv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) av[a] = rs[buf][row * LS + 64 * wm + 16 * a + cl];
#pragma unroll
      for (int c = 0; c < 4; ++c) bv[c] = us[buf][row * LS + 64 * wn + 16 * c + cl];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[a][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[c], acc[a][c], 0, 0, 0);
    }
    if (next) stage_store(buf ^ 1, ra, ua);
    __syncthreads();  // the next stage complete; this one free
    buf ^= 1;
  }
  // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 64 * wm + 16 * a + (l >> 4) + 4 * q, col = n0 + 64 * wn + 16 * c + (l & 15);
        if (row < N && col < N && acc[a][c][q] != 0.0) unsafeAtomicAdd(&g.xi_s[(size_t)row * N + col], acc[a][c][q]);
      }
}

// ---- N <= 64: one wave per sequence ---------------------------------------------------------
// Lane i owns state i.  The transition matrix lives in VGPRs (forward: column i, backward:
// row i), the vector being multiplied is broadcast through a per-wave LDS slot (ds_read_b128,
// all lanes same address), and the three per-step sums are wave reductions (DPP inside a row
// of 16, readlane across the 4 rows) -- no workgroup barrier anywhere.  LDS accesses of one
// wave complete in order, so the slot is rewritten each step without a fence.  The observation
// and tag of each step come from a 64-step block held one element per lane (readlane).

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double readlane_f64(double v, int k) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)u, k);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(u >> 32), k);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// sum over the 64 lanes, the identical value in every lane
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror: quad q <-> 1-q within 8
  v += dpp_f64<0x140>(v);  // row_mirror: half h <-> 1-h within 16
  return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// maximum over the 64 lanes, the identical value in every lane
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  v = fmax(v, dpp_f64<0x140>(v));
  return fmax(fmax(readlane_f64(v, 0), readlane_f64(v, 16)), fmax(readlane_f64(v, 32), readlane_f64(v, 48)));
}

// two independent sums with their latencies overlapped
__device__ __forceinline__ void wave_sum2(double& a, double& b) {
  a += dpp_f64<0xB1>(a);
  b += dpp_f64<0xB1>(b);
  a += dpp_f64<0x4E>(a);
  b += dpp_f64<0x4E>(b);
  a += dpp_f64<0x141>(a);
  b += dpp_f64<0x141>(b);
  a += dpp_f64<0x140>(a);
  b += dpp_f64<0x140>(b);
  a = (readlane_f64(a, 0) + readlane_f64(a, 16)) + (readlane_f64(a, 32) + readlane_f64(a, 48));
  b = (readlane_f64(b, 0) + readlane_f64(b, 16)) + (readlane_f64(b, 32) + readlane_f64(b, 48));
}

// Memory operations in the step loops are all unconditional (clamped indices; lanes without
// a state store to / add into a per-lane dump slot): a load, store or atomic under a branch
// makes the compiler's wait-count tracking give up and wait for every outstanding load
// (vmcnt(0)) at the next use, which would expose the full HBM latency on every step.  The step
// loops are unrolled with a static slot per step, so no loaded register is copied across the
// loop edge either (a copy is a use, i.e. a wait for the load just issued).

// a value loaded through a vector load but equal in all lanes, as a scalar (uniform control
// flow and addresses downstream)
__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// four independent sums with their latencies overlapped
__device__ __forceinline__ void wave_sum4(double& a, double& b, double& c, double& d) {
#define CVF_LVL(CTRL)          \
  a += dpp_f64<CTRL>(a);       \
  b += dpp_f64<CTRL>(b);       \
  c += dpp_f64<CTRL>(c);       \
  d += dpp_f64<CTRL>(d);
  CVF_LVL(0xB1)
  CVF_LVL(0x4E)
  CVF_LVL(0x141)
  CVF_LVL(0x140)
#undef CVF_LVL
  a = (readlane_f64(a, 0) + readlane_f64(a, 16)) + (readlane_f64(a, 32) + readlane_f64(a, 48));
  b = (readlane_f64(b, 0) + readlane_f64(b, 16)) + (readlane_f64(b, 32) + readlane_f64(b, 48));
  c = (readlane_f64(c, 0) + readlane_f64(c, 16)) + (readlane_f64(c, 32) + readlane_f64(c, 48));
  d = (readlane_f64(d, 0) + readlane_f64(d, 16)) + (readlane_f64(d, 32) + readlane_f64(d, 48));
}

// y = sum_j p[j] * m[j], p broadcast from LDS, 4 partial sums (fused multiply-add)
template <int NP>
__device__ __forceinline__ double dot_lds_fma(const double* p, const double (&m)[NP]) {
  double y0 = 0.0, y1 = 0.0, y2 = 0.0, y3 = 0.0;
#pragma unroll
  for (int j = 0; j < NP; j += 4) {
    const double2 u = *reinterpret_cast<const double2*>(p + j);
    const double2 v = *reinterpret_cast<const double2*>(p + j + 2);
    y0 = __builtin_fma(u.x, m[j], y0);
    y1 = __builtin_fma(u.y, m[j + 1], y1);
    y2 = __builtin_fma(v.x, m[j + 2], y2);
    y3 = __builtin_fma(v.y, m[j + 3], y3);
  }
  return (y0 + y1) + (y2 + y3);
}

// Sequence order: ord[k] is the k-th sequence to start (longest first, see the host), so the
// first resident waves take the long chains and short ones fill in behind them.
template <int NP>
__global__ __launch_bounds__(256) void bw_fwd_wave(BwArgs g, int64_t nseq) {
  __shared__ __attribute__((aligned(16))) double slot[4][NP];
  const int w = threadIdx.x >> 6, i = threadIdx.x & 63;
  const int64_t kq = (int64_t)blockIdx.x * 4 + w;
  if (kq >= nseq) return;  // wave-uniform
  const int64_t seq = uniform64(g.order ? g.order[kq] : kq);
  const int N = g.nstates;
  const bool act = i < N;
  const int ic = act ? i : N - 1;  // state index inactive lanes load with (always in bounds)
  double* p = slot[w];
  double acol[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) acol[j] = (act && j < N) ? g.a[(size_t)j * N + i] : 0.0;
  const int64_t e0 = uniform64(g.offsets[seq]);
  const int T = __builtin_amdgcn_readfirstlane((int)(g.offsets[seq + 1] - e0));
  if (T <= 0) return;
  double* al = g.alpha + (e0 - g.elem_base) * N;
  double* const dump = g.dump + (size_t)(kq & (kBwDumpWaves - 1)) * 64 + i;
  const int32_t* obs = g.obs + e0;
  const int32_t* tag = g.tags + e0;
  const double* et = g.et;
  // t = 0 (hmm.rs:81-88)
  double cur;
  {
    const int o = obs[0], tg = tag[0];
    const double y = act ? g.pi[i] * et[(size_t)o * N + i] : 0.0;
    const double s = wave_sum(y);
    cur = tg >= 0 ? (i == tg ? 1.0 : 0.0) : (act ? normalized(y, s, N) : 0.0);
    *(act ? al + i : dump) = cur;
  }
  // observation index and tag of step s fetched 6 steps ahead (slot s mod 8), b(o_s) 3 steps
  // ahead (slot s mod 4) from the index fetched 3 steps before that; all indices clamped.
  int po[8], ptg[8];
  double pe[4];
  auto fetch_ot = [&](int s, int k8) {
    const int sc = min(s, T - 1);
    po[k8] = obs[sc];
    ptg[k8] = tag[sc];
  };
#pragma unroll
  for (int k = 0; k < 6; ++k) fetch_ot(1 + k, k);  // steps 1..6
#pragma unroll
  for (int k = 0; k < 3; ++k) pe[k] = et[(size_t)po[k] * N + ic];  // steps 1..3
  for (int t0 = 1; t0 < T; t0 += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int t = t0 + k;
      if (t >= T) break;
      fetch_ot(t + 6, (k + 6) & 7);
      pe[(k + 3) & 3] = et[(size_t)po[(k + 3) & 7] * N + ic];
      const int tg = __builtin_amdgcn_readfirstlane(ptg[k]);
      if (tg >= 0) {  // hmm.rs:91
        cur = (i == tg) ? 1.0 : 0.0;
      } else {        // (alpha[t-1] * b(o_t)) . A  -- hmm.rs:93-94
        if (i < NP) p[i] = act ? cur * pe[k & 3] : 0.0;
        __builtin_amdgcn_wave_barrier();
        const double y = dot_lds_fma<NP>(p, acol);
        __builtin_amdgcn_wave_barrier();
        const double sy = wave_sum(y);
        cur = act ? normalized(y, sy, N) : 0.0;
      }
      *(act ? al + (size_t)t * N + i : dump) = cur;
    }
  }
}

// Backward pass fused with the E-step sums: beta is never stored.  At step t the backward
// product w = A u_{t+1} (u = b(o_{t+1}) o beta_{t+1}) is also xi's row sum, so
// c_t = alpha_t . w, S += (alpha_t / c_t) (x) u_{t+1} and beta_t = normalize(w) (or one-hot).
// Each wave runs TWO sequences side by side (consecutive in the longest-first order, so of
// similar length, aligned at their last element): their chains are independent, which hides
// the latency of the reductions and divisions, and one pass over lane i's row of A (in LDS)
// serves both products.  u_{t+1} is the LDS row every lane reads for w anyway; r_t =
// alpha_t / c_t goes to a second LDS row; every 2 steps the rank-4 update S += R^T U (2 steps
// x 2 sequences) runs on the matrix cores (v_mfma_f64_16x16x4_f64), S being (NP/16)^2
// accumulator tiles.  A wave walks pairs w, w + nwaves, ... keeping S and the gamma sums in
// registers; one atomic flush at the end.
template <int NP>
__global__ __launch_bounds__(256) void bw_bwd_stats_wave(BwArgs g, int64_t nseq, int64_t nwaves) {
  constexpr int NT = NP / 16;
  __shared__ __attribute__((aligned(16))) double uu[4][4][NP];  // [wave][2 * (step & 1) + seq][state]
  __shared__ __attribute__((aligned(16))) double rr[4][4][NP];
  const int w = threadIdx.x >> 6, i = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * 4 + w;
  const int N = g.nstates;
  const bool act = i < N;
  const int ic = act ? i : N - 1;
  double* const dump = g.dump + (size_t)(gw & (kBwDumpWaves - 1)) * 64 + i;
  const double* et = g.et;
  // A lives in LDS, row i read by lane i (row stride AS = 2 mod 32 doubles: the 16 lanes of a
  // ds_read_b128 phase hit 16 distinct 4-bank groups); registers go to S and the fetch slots
  constexpr int AS = (NP + 31) / 32 * 32 + 2;
  __shared__ __attribute__((aligned(16))) double As[NP * AS];
  for (int k = threadIdx.x; k < NP * AS; k += 256) {
    const int r = k / AS, c = k - r * AS;
    As[k] = (r < N && c < N) ? g.a[(size_t)r * N + c] : 0.0;
  }
  __syncthreads();  // every wave of the block loads its share of A before any leaves
  if (gw >= nwaves) return;
  const double* arow = As + (i < NP ? i : 0) * AS;
  typedef double double4_t __attribute__((ext_vector_type(4)));
  double4_t S[NT][NT];
#pragma unroll
  for (int m = 0; m < NT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) S[m][n] = double4_t{0.0, 0.0, 0.0, 0.0};
  if (i < NP)
#pragma unroll
    for (int q = 0; q < 4; ++q) uu[w][q][i] = rr[w][q][i] = 0.0;
  // rank-4 update from the 4 staged rows: lane l supplies R[k = l>>4][m = 16 mt + (l&15)] as
  // A and U[k][n = 16 nt + (l&15)] as B
  auto mfma_update = [&]() {
    __builtin_amdgcn_wave_barrier();
    double av[NT], bv[NT];
#pragma unroll
    for (int m = 0; m < NT; ++m) {
      av[m] = rr[w][i >> 4][16 * m + (i & 15)];
      bv[m] = uu[w][i >> 4][16 * m + (i & 15)];
    }
#pragma unroll
    for (int m = 0; m < NT; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n) S[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m], bv[n], S[m][n], 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
  };
  double pi_acc = 0.0, a_den = 0.0, b_den = 0.0, z = 0.0;
  const int64_t npairs = (nseq + 1) / 2;
  for (int64_t pq = gw; pq < npairs; pq += nwaves) {
    // the two sequences; a missing second one (odd count) runs as T = 0 on the first's arrays
    const double* al[2];
    const int32_t* obs[2];
    const int32_t* tag[2];
    int T[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int64_t kq = 2 * pq + x < nseq ? 2 * pq + x : 2 * pq;
      const int64_t seq = uniform64(g.order ? g.order[kq] : kq);
      const int64_t e0 = uniform64(g.offsets[seq]);
      T[x] = 2 * pq + x < nseq ? __builtin_amdgcn_readfirstlane((int)(g.offsets[seq + 1] - e0)) : 0;
      al[x] = g.alpha + (e0 - g.elem_base) * N;
      obs[x] = g.obs + e0;
      tag[x] = g.tags + e0;
    }
    // t = T-1 (hmm.rs:105-108)
    double beta[2], pe[2][4], pa[2][4];
    int po[2][8], ptg[2][8];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const bool valid = T[x] > 0;
      const int tl = valid ? T[x] - 1 : 0;
      const int o = obs[x][tl], tg = tag[x][tl];
      beta[x] = tg >= 0 ? (i == tg ? 1.0 : 0.0) : (act ? 1.0 : 0.0);
      const double alt = (act && valid) ? al[x][(size_t)tl * N + i] : 0.0;
      pe[x][3] = act ? et[(size_t)o * N + i] : 0.0;  // b(o_{T-1}), used by step T-2
      const double ab = alt * beta[x];
      const double gm = normalized(ab, wave_sum(ab), N);
      const bool on = act && valid;
      if (on) {
        b_den += gm;
        if (T[x] == 1) pi_acc += gm;
      }
      unsafeAtomicAdd(on ? &g.b_num[(size_t)o * N + i] : dump, on ? gm : 0.0);
    }
    // observation index and tag of step s fetched 6 steps ahead (slot by step mod 8), b(o_s)
    // and alpha_s 2 steps ahead (slot mod 4); all indices clamped into the sequence.
    auto fetch_ot = [&](int x, int s, int k8) {
      const int sc = min(max(s, 0), max(T[x] - 1, 0));
#ifndef CVF_ABL_NOIDX
      po[x][k8] = obs[x][sc];
      ptg[x][k8] = tag[x][sc];
#else
      po[x][k8] = sc & 1023;
      ptg[x][k8] = (sc % 5 == 0) ? 3 : -1;
#endif
    };
    auto fetch_ea = [&](int x, int s, int k8, int k4) {
      const int sc = min(max(s, 0), max(T[x] - 1, 0));
#ifndef CVF_ABL_NOLOAD
      pe[x][k4] = et[(size_t)po[x][k8] * N + ic];
      pa[x][k4] = al[x][(size_t)sc * N + ic];
#else
      pe[x][k4] = 1e-3 * (double)(po[x][k8] + ic);
      pa[x][k4] = 1e-2 * (double)(sc + ic);
#endif
    };
#pragma unroll
    for (int x = 0; x < 2; ++x) {
#pragma unroll
      for (int k = 0; k < 6; ++k) fetch_ot(x, T[x] - 2 - k, k);  // steps T-2 .. T-7
      fetch_ea(x, T[x] - 2, 0, 0);
      fetch_ea(x, T[x] - 3, 1, 1);
    }
    const int L = max(T[0], T[1]);
    // step r of the pair is step t = T[x] - 2 - r of sequence x (inactive once t < 0)
    for (int r0 = 0; r0 < L - 1; r0 += 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = r0 + k;
        if (r >= L - 1) break;
        double alt[2], wv[2], uval[2];
        bool valid[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          const int t = T[x] - 2 - r;
          valid[x] = t >= 0;
          fetch_ot(x, t - 6, (k + 6) & 7);
          fetch_ea(x, t - 2, (k + 2) & 7, (k + 2) & 3);
          alt[x] = (act && valid[x]) ? pa[x][k & 3] : 0.0;
          // u_{t+1} = b(o_{t+1}) o beta_{t+1}  (hmm.rs:113-116, 135-141)
          uval[x] = (act && valid[x]) ? pe[x][(k + 3) & 3] * beta[x] : 0.0;
          if (i < NP) uu[w][2 * (k & 1) + x][i] = uval[x];
        }
        __builtin_amdgcn_wave_barrier();
        {  // w_x[i] = sum_j A[i][j] u_x[j], one pass over the row of A for both sequences
          const double* u0 = uu[w][2 * (k & 1)];
          const double* u1 = uu[w][2 * (k & 1) + 1];
          double y0 = 0.0, y1 = 0.0, y2 = 0.0, y3 = 0.0;
#pragma unroll
          for (int j = 0; j < NP; j += 2) {
            const double2 av = *reinterpret_cast<const double2*>(arow + j);
            const double2 p0 = *reinterpret_cast<const double2*>(u0 + j);
            const double2 p1 = *reinterpret_cast<const double2*>(u1 + j);
            y0 = __builtin_fma(p0.x, av.x, y0);
            y1 = __builtin_fma(p0.y, av.y, y1);
            y2 = __builtin_fma(p1.x, av.x, y2);
            y3 = __builtin_fma(p1.y, av.y, y3);
          }
          wv[0] = y0 + y1;
          wv[1] = y2 + y3;
        }
        double c0 = alt[0] * wv[0], sw0 = wv[0], c1 = alt[1] * wv[1], sw1 = wv[1];
        wave_sum4(c0, sw0, c1, sw1);
        const double c[2] = {c0, c1}, sw[2] = {sw0, sw1};
        double ab[2];
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          z += (valid[x] && c[x] == 0.0) ? 1.0 : 0.0;  // xi_t uniform (hmm.rs:306-317), counted separately
          // r = alpha / (c 2^k) and u' = u 2^k (xi_scale): the row of u the MFMA update reads
          // is rescaled in place (this lane's own entry; w above used the unscaled one)
          const int ks = xi_scale(c[x], wave_max(uval[x]));
          if (i < NP) {
            rr[w][2 * (k & 1) + x][i] = c[x] != 0.0 ? alt[x] / __builtin_ldexp(c[x], ks) : 0.0;
            uu[w][2 * (k & 1) + x][i] = __builtin_ldexp(uval[x], ks);
          }
          const int tg = ptg[x][k];
          const double nb = tg >= 0 ? (i == tg ? 1.0 : 0.0) : (act ? normalized(wv[x], sw[x], N) : 0.0);
          beta[x] = valid[x] ? nb : beta[x];
          ab[x] = alt[x] * beta[x];
        }
#ifndef CVF_ABL_NOMFMA
        if (k & 1) mfma_update();  // 2 steps x 2 sequences staged
#endif
        double s0 = ab[0], s1 = ab[1];
        wave_sum2(s0, s1);  // hmm.rs:127-129
        const double sab[2] = {s0, s1};
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          const double gm = normalized(ab[x], sab[x], N);
          const bool on = act && valid[x];
          if (on) {
            a_den += gm;
            b_den += gm;
            if (T[x] - 2 - r == 0) pi_acc += gm;
          }
#ifndef CVF_ABL_NOATOMIC
          unsafeAtomicAdd(on ? &g.b_num[(size_t)po[x][k] * N + i] : dump, on ? gm : 0.0);
#else
          b_den += on ? gm * (double)po[x][k] : 0.0;
#endif
        }
      }
    }
    if ((L - 1) & 1) {  // flush the odd last step: zero the rows of the missing one
      if (i < NP) uu[w][2][i] = uu[w][3][i] = rr[w][2][i] = rr[w][3][i] = 0.0;
      mfma_update();
    }
  }
  if (act) {
    unsafeAtomicAdd(&g.pi_acc[i], pi_acc);
    unsafeAtomicAdd(&g.a_den[i], a_den);
    unsafeAtomicAdd(&g.b_den[i], b_den);
  }
  // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int m = 0; m < NT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * m + (i >> 4) + 4 * r, col = 16 * n + (i & 15);
        if (row < N && col < N) unsafeAtomicAdd(&g.xi_s[(size_t)row * N + col], S[m][n][r]);
      }
  if (i == 0 && z != 0.0) unsafeAtomicAdd(g.xi_zero, z);
}

// ---- 64 < N <= 256: 64 sequences per workgroup, each step's products on the matrix cores ----
// The workgroup kernels above give every sequence its own workgroup, so every sequence step
// streams all of A (512 KiB at N = 256) through L1/L2 for N^2 FMAs: ~5 TFLOP/s.  Here a
// workgroup advances 64 sequences (consecutive in the longest-first order) in lock step and
// one step is the product X (64 x NP) . A (NP x NP) on v_mfma_f64_16x16x4_f64: each A value
// read serves 64 sequences.  Wave w owns the output columns [64 w, 64 w + 64) (CT = NP / 64
// tiles of 16) for all 64 sequences (4 tiles of 16): 16 CT independent accumulators, lane l
// holding Y[g = 16 m + (l >> 4) + 4 r][i = 16 (w CT + n) + (l & 15)] (f64 C/D layout).  The
// next step's operand X goes through LDS transposed, X^T[k][g] (xt_at: a padded row stride).  Row sums (normalisation, c_t, gamma) reduce in registers over the wave's tiles,
// by DPP over the 16 lanes of a row, then over the 4 waves through LDS -- one order, so runs
// repeat bit for bit.  A's indices are clamped into [0, N): rows k >= N meet X entries that
// are 0, columns >= N are dropped.

__device__ __forceinline__ double row16_sum(double v) {  // sum over the 16 lanes of a DPP row
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  v += dpp_f64<0x140>(v);
  return v;
}
__device__ __forceinline__ double row16_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  v = fmax(v, dpp_f64<0x140>(v));
  return v;
}
// normalize by a reciprocal taken once per sequence step: v / s to within an ulp (the sums run
// in another order than the reference's anyway).  Both scaled by 2^64, so a subnormal s (tiny
// emissions) still has a finite reciprocal; every v here is one of s's non-negative terms.
__device__ __forceinline__ double recip64(double s) { return 1.0 / (s * 0x1p64); }
// s != 0: v / s (to an ulp, by the reciprocal); s == 0: 1 / n (hmm.rs:274-282)
__device__ __forceinline__ double normalized_r(double v, double s, double inv, double inv_n) {
  return sel(s != 0.0, (v * 0x1p64) * inv, inv_n);
}

// X^T[k][g] with a row stride of G + 1 doubles: one ds_write_b64 (16 lanes: 16 consecutive k,
// one g) spreads over 16 bank pairs; an operand read (16 consecutive g at k and k + 1) is a
// 2-way conflict.  Additive, so every (tile, register) offset is a compile-time constant the
// LDS instructions carry (an XOR swizzle kept 16-32 per-lane addresses live and spilled).
template <int G>
__device__ __forceinline__ int xt_at(int k, int g) { return k * (G + 1) + g; }

// the WV waves' partials of sequence gi (red[w * G + gi]) added in one fixed (pairwise) order
template <int WV>
__device__ __forceinline__ double wsum(const double* red, int G, int gi) {
  if constexpr (WV == 4) return (red[gi] + red[G + gi]) + (red[2 * G + gi] + red[3 * G + gi]);
  else return wsum<WV / 2>(red, G, gi) + wsum<WV / 2>(red + (WV / 2) * G, G, gi);
}
template <int WV>
__device__ __forceinline__ double wmax(const double* red, int G, int gi) {
  double v = red[gi];
#pragma unroll
  for (int w = 1; w < WV; ++w) v = fmax(v, red[w * G + gi]);
  return v;
}

template <int NP, int MT, int WV, class Pre>
__device__ __forceinline__ void mm_step(const double* __restrict__ xt, const double* __restrict__ M, int N, int w,
                                        int l, f64x4_t (&acc)[MT][NP / (16 * WV)], Pre&& pre) {
#ifndef CVF_MM_PF
  constexpr int PF = 4;
#else
  constexpr int PF = CVF_MM_PF;
#endif
  constexpr int CT = NP / (16 * WV), NK = NP / 4, G = 16 * MT;
  const int cl = l & 15, kq = l >> 4;
  int col[CT];
#pragma unroll
  for (int n = 0; n < CT; ++n) col[n] = min(16 * (w * CT + n) + cl, N - 1);
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < CT; ++n) acc[m][n] = f64x4_t{0.0, 0.0, 0.0, 0.0};
  // A rows PF k-blocks ahead (L2), the LDS operand one k-block ahead
  // the products at a higher issue priority than the other workgroup's phase-E VALU work on
  // the SIMD (A/B: forward 77.8 vs 79.1 ms, backward 110.0 vs 110.8 ms at config-4 shape)
#ifndef CVF_MM_NOPRIO
  __builtin_amdgcn_s_setprio(2);
#endif
  double ring[PF][CT];
#define CVF_MM_LOAD(KK, DST)                                                  \
  {                                                                           \
    const int k_ = min(4 * (KK) + kq, N - 1);                                 \
    _Pragma("unroll") for (int n = 0; n < CT; ++n) DST[n] = M[(size_t)k_ * N + col[n]]; \
  }
#pragma unroll
  for (int p = 0; p < PF; ++p) CVF_MM_LOAD(p, ring[p])
  // loads the caller wants in flight during the products: issued after the ring's first
  // blocks, so the in-order wait for those does not wait for them
  pre();
  double av[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) av[m] = xt[xt_at<G>(kq, 16 * m + cl)];
#pragma unroll 1
  for (int kk0 = 0; kk0 < NK; kk0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int kk = kk0 + p;
      double bv[CT], an[MT];
#pragma unroll
      for (int n = 0; n < CT; ++n) bv[n] = ring[p][n];
      CVF_MM_LOAD(min(kk + PF, NK - 1), ring[p])
      const int kn = 4 * min(kk + 1, NK - 1) + kq;
#pragma unroll
      for (int m = 0; m < MT; ++m) an[m] = xt[xt_at<G>(kn, 16 * m + cl)];
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < CT; ++n) acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m], bv[n], acc[m][n], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = an[m];
    }
  }
#ifndef CVF_MM_NOPRIO
  __builtin_amdgcn_s_setprio(0);
#endif
#undef CVF_MM_LOAD
}

// the group's sequences: element offset, length, and the longest length
template <int G>
__device__ __forceinline__ void mm_setup(const BwArgs& g, int64_t nseq, int64_t* s_e0, int* s_T, int* s_tmax) {
  const int tid = threadIdx.x;
  if (tid < G) {
    const int64_t k = (int64_t)blockIdx.x * G + tid;
    int64_t e0 = 0;
    int T = 0;
    if (k < nseq) {
      const int64_t s = g.order ? g.order[k] : k;
      e0 = g.offsets[s];
      T = (int)(g.offsets[s + 1] - e0);
    }
    s_e0[tid] = e0 - g.elem_base;
    s_T[tid] = T;
  }
  __syncthreads();
  if (tid == 0) {
    int tm = 0;
    for (int k = 0; k < G; ++k) tm = max(tm, s_T[k]);
    *s_tmax = tm;
  }
  __syncthreads();
}

// forward (hmm.rs:78-100) of 16 MT sequences: alpha rows to g.alpha (observation slots two
// steps ahead: slot t & 3 holds step t, written at step t - 2 behind two barriers).
template <int NP, int MT, int WV>
__global__ __launch_bounds__(64 * WV, (MT == 4 ? 1 : 2) * WV / 4) void bw_fwd_mm(BwArgs g, int64_t nseq) {
  constexpr int CT = NP / (16 * WV), G = 16 * MT;
  __shared__ __attribute__((aligned(16))) double xt[NP * (G + 1)];
  __shared__ double red[WV][G];
  __shared__ int64_t s_e0[G];
  __shared__ int s_T[G], s_ob[4][G], s_tg[4][G];
  __shared__ int s_tmax;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, cl = l & 15;
  const int N = g.nstates;
  const double inv_n = 1.0 / N;
  double* const dump = g.dump + (size_t)((blockIdx.x * WV + (tid >> 6)) & (kBwDumpWaves - 1)) * 64 + (tid & 63);
  mm_setup<G>(g, nseq, s_e0, s_T, &s_tmax);
  const int tmax = s_tmax;
  if (tmax <= 0) return;  // workgroup-uniform
  auto fetch = [&](int t) {  // observation and tag of step t into slot t & 3
    if (tid < G) {
      const bool v = t < s_T[tid];
      const int64_t e = (int64_t)s_e0[tid] + g.elem_base + (v ? t : 0);
      s_ob[t & 3][tid] = v ? g.obs[e] : 0;
      s_tg[t & 3][tid] = v ? g.tags[e] : -1;
    }
  };
  fetch(0);
  fetch(1);
  fetch(2);
  __syncthreads();
  int col[CT], cc[CT];
#pragma unroll
  for (int n = 0; n < CT; ++n) {
    col[n] = 16 * (w * CT + n) + cl;
    cc[n] = min(col[n], N - 1);
  }
  f64x4_t acc[MT][CT];
  // t = 0 (hmm.rs:81-88): y = pi * b(o_0)
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = s_ob[0][16 * m + (l >> 4) + 4 * r];
#pragma unroll
      for (int n = 0; n < CT; ++n) acc[m][n][r] = g.pi[cc[n]] * g.et[(size_t)o * N + cc[n]];
    }
  for (int t = 0;; ++t) {
    if (t > 0) {
      fetch(t + 2);  // slot (t + 2) & 3 held step t - 2, last read before step t - 1's closing barrier
      // (alpha_{t-1} o b(o_t)) . A  (hmm.rs:93-94)
      mm_step<NP, MT, WV>(xt, g.a, N, w, l, acc, [] {});
    }
    // row sums of y over the N states
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double v = 0.0;
#pragma unroll
        for (int n = 0; n < CT; ++n) v += col[n] < N ? acc[m][n][r] : 0.0;
        v = row16_sum(v);
        if (cl == 0) red[w][16 * m + (l >> 4) + 4 * r] = v;
      }
    __syncthreads();
    const bool more = t + 1 < tmax;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 16 * m + (l >> 4) + 4 * r;
        const double sum = wsum<WV>(&red[0][0], G, gi);
        const double inv = recip64(sum);
        const int tg = s_tg[t & 3][gi];
        const bool on = t < s_T[gi];
        const bool on1 = t + 1 < s_T[gi];
        double* arow = g.alpha + (size_t)(s_e0[gi] + t) * N;
#pragma unroll
        for (int n = 0; n < CT; ++n) {
          const int c = col[n];
          const double a = sel(tg >= 0, c == tg ? 1.0 : 0.0, normalized_r(acc[m][n][r], sum, inv, inv_n));
          *((on && c < N) ? arow + c : dump) = a;  // branch-free: dead lanes store to their dump slot
          acc[m][n][r] = sel(on1 && c < N, a, 0.0);
        }
      }
    // the next operand alpha_t o b(o_{t+1}): all emission loads (L2 hits) issued together
    if (more) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gi = 16 * m + (l >> 4) + 4 * r;
          const double* er = g.et + (size_t)s_ob[(t + 1) & 3][gi] * N;  // b(o_{t+1})
#pragma unroll
          for (int n = 0; n < CT; ++n) xt[xt_at<G>(col[n], gi)] = acc[m][n][r] * er[cc[n]];
        }
    }
    __syncthreads();  // xt complete; red free
    if (!more) break;
  }
}

// backward (hmm.rs:102-121) fused with gamma / xi of hmm.rs:124-143 for 16 MT sequences,
// aligned at their last elements: step r is t = T_g - 1 - r of sequence g.  W_t = A u_{t+1}
// (u_{t+1} = b(o_{t+1}) o beta_{t+1}, in xt) gives c_t = alpha_t . W_t and beta_t =
// normalize(W_t); r_t = alpha_t / (c_t 2^k) and u'_{t+1} = u_{t+1} 2^k overwrite alpha's and
// beta's row t for bw_xi_gemm (zeros at t = T - 1), as bw_stats_rows writes them.  One
// reduction round per step: gamma_t = normalize(alpha_t o beta_t) needs sum_i alpha_i beta_i,
// which is c_t / sum W_t for an untagged step (beta = W / sum W), 1 at a tagged one (alpha_t and
// beta_t both one-hot at the tag: the forward wrote alpha_t so), and sum alpha_t at t = T - 1
// (beta = 1) or where sum W_t = 0 (beta uniform, / N).  alpha_t's loads are in flight during
// the step's products with -DCVF_BWD_PREFETCH (its registers spill at N = 256).
template <int NP, int MT, int WV>
__global__ __launch_bounds__(64 * WV, (MT == 4 ? 1 : 2) * WV / 4) void bw_bwd_mm(BwArgs g, int64_t nseq) {
  constexpr int CT = NP / (16 * WV), G = 16 * MT;
  __shared__ __attribute__((aligned(16))) double xt[NP * (G + 1)];
  __shared__ double red[4][WV][G];  // c, sum W, max u_{t+1}, sum alpha -- per wave
  __shared__ double s_den[3][NP];   // the workgroup's pi_acc, a_den, b_den (LDS atomics)
  __shared__ int64_t s_e0[G];
  __shared__ int s_T[G], s_ob[2][G], s_tg[2][G];
  __shared__ int s_tmax;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, cl = l & 15;
  const int N = g.nstates;
  const double inv_n = 1.0 / N;
  mm_setup<G>(g, nseq, s_e0, s_T, &s_tmax);
  const int tmax = s_tmax;
  if (tmax <= 0) return;
  auto fetch = [&](int r) {  // observation and tag of step r (t = T - 1 - r) into slot r & 1
    if (tid < G) {
      const int t = s_T[tid] - 1 - r;
      const int64_t e = (int64_t)s_e0[tid] + g.elem_base + (t >= 0 ? t : 0);
      s_ob[r & 1][tid] = t >= 0 ? g.obs[e] : 0;
      s_tg[r & 1][tid] = t >= 0 ? g.tags[e] : -1;
    }
  };
  fetch(0);
  for (int i = tid; i < 3 * NP; i += 64 * WV) (&s_den[0][0])[i] = 0.0;
  __syncthreads();
  int col[CT], cc[CT];
#pragma unroll
  for (int n = 0; n < CT; ++n) {
    col[n] = 16 * (w * CT + n) + cl;
    cc[n] = min(col[n], N - 1);
  }
  f64x4_t acc[MT][CT];
  double al[MT][CT][4];
  auto load_alpha = [&](int r) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gi = 16 * m + (l >> 4) + 4 * q;
        const int t = s_T[gi] - 1 - r;
        const double* arow = g.alpha + (size_t)(s_e0[gi] + max(t, 0)) * N;
#pragma unroll
        for (int n = 0; n < CT; ++n) {
          // unconditional (clamped row): a load under a per-lane branch is waited for at once
#ifndef CVF_ABL_NOALPHA
          al[m][n][q] = sel(t >= 0 && col[n] < N, arow[cc[n]], 0.0);
#else
          al[m][n][q] = (t >= 0 && col[n] < N) ? 1e-3 * (double)(t + col[n] + (arow - g.alpha) % 7) : 0.0;
#endif
        }
      }
  };
  double z = 0.0;
  double* const dump = g.dump + (size_t)((blockIdx.x * WV + w) & (kBwDumpWaves - 1)) * 64 + l;
  for (int r = 0; r < tmax; ++r) {
    if (r > 0) {
      fetch(r);  // slot r & 1 held step r - 2, read before step r - 1's closing barrier
      // W_t[i] = sum_j A[i][j] u_{t+1}[j]  (hmm.rs:113-116)
#ifdef CVF_BWD_PREFETCH
      mm_step<NP, MT, WV>(xt, g.at, N, w, l, acc, [&] { load_alpha(r); });
#else
      mm_step<NP, MT, WV>(xt, g.at, N, w, l, acc, [] {});
      load_alpha(r);
#endif
    } else {
      load_alpha(0);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < CT; ++n) acc[m][n] = f64x4_t{0.0, 0.0, 0.0, 0.0};
    }
    // the reduction round: c_t, sum W_t, max u_{t+1} (r > 0), sum alpha_t
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gi = 16 * m + (l >> 4) + 4 * q;
        double c = 0.0, sw = 0.0, um = 0.0, sa = 0.0;
#pragma unroll
        for (int n = 0; n < CT; ++n) {
          const double wv = col[n] < N ? acc[m][n][q] : 0.0;
          c += al[m][n][q] * wv;
          sw += wv;
          sa += al[m][n][q];
          if (r > 0) um = fmax(um, xt[xt_at<G>(col[n], gi)]);  // u_{t+1} (0 beyond N)
        }
        c = row16_sum(c);
        sw = row16_sum(sw);
        um = row16_max(um);
        sa = row16_sum(sa);
        if (cl == 0) {
          red[0][w][gi] = c;
          red[1][w][gi] = sw;
          red[2][w][gi] = um;
          red[3][w][gi] = sa;
        }
      }
    __syncthreads();
    double gb[CT], gp[CT];  // this step's gamma sums over the lane's sequences (all; t == 0)
#pragma unroll
    for (int n = 0; n < CT; ++n) gb[n] = gp[n] = 0.0;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      // b(o_t) for u_t, this tile's loads (L2 hits) issued before its stores and atomics; one
      // M-tile at a time (sched_barrier): both at once spill at 256 states
      __builtin_amdgcn_sched_barrier(0);
      double ev[CT][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double* er = g.et + (size_t)s_ob[r & 1][16 * m + (l >> 4) + 4 * q] * N;
#pragma unroll
        for (int n = 0; n < CT; ++n) ev[n][q] = er[cc[n]];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gi = 16 * m + (l >> 4) + 4 * q;
        const double c = wsum<WV>(&red[0][0][0], G, gi);
        const double sw = wsum<WV>(&red[1][0][0], G, gi);
        const double umax = wmax<WV>(&red[2][0][0], G, gi);
        const double sa = wsum<WV>(&red[3][0][0], G, gi);
        const int t = s_T[gi] - 1 - r;
        const bool on = t >= 0;
        const int tg = s_tg[r & 1][gi];
        const int o = s_ob[r & 1][gi];
        const double isw = recip64(sw);
        const int ks = xi_scale(c, umax);  // balanced factors (xi_scale)
        const double ics = recip64(__builtin_ldexp(c, ks));  // r = alpha / (c 2^k), by one reciprocal
        // sum_i alpha_i beta_i (see above); tagged steps take gamma = one-hot directly
        const double sab = r == 0 ? sa : sel(sw != 0.0, (c * 0x1p64) * isw, sa * inv_n);
        const double isab = recip64(sab);
        double* urow = g.beta + (size_t)(s_e0[gi] + max(t, 0)) * N;
        if (r > 0 && on && c == 0.0 && cl == 0 && w == 0) z += 1.0;  // xi_t uniform (hmm.rs:306-317)
        // R's row t is alpha_t (left in place) times this scalar: 2^64 ics = 1 / (c 2^k), 0 where
        // c = 0 or at t = T - 1 -- the same product (alpha 2^64) ics the GEMM used to read
        if (on && cl == 0 && w == 0) g.rscale[s_e0[gi] + t] = (r > 0 && c != 0.0) ? ics * 0x1p64 : 0.0;
#pragma unroll
        for (int n = 0; n < CT; ++n) {
          const int k = col[n];
          const bool onk = on && k < N;
          double beta;
          // rows for bw_xi_gemm; t = T - 1 (r = 0): zero rows (branch-free: dead lanes store
          // to their dump slot)
          double uv = 0.0;
          if (r > 0) {  // workgroup-uniform
            uv = __builtin_ldexp(xt[xt_at<G>(k, gi)], ks);  // u_{t+1} 2^k
            beta = sel(tg >= 0, k == tg ? 1.0 : 0.0, sel(k < N, normalized_r(acc[m][n][q], sw, isw, inv_n), 0.0));
          } else {  // t = T - 1 (hmm.rs:105-108): tagged -> one-hot, else ones
            beta = tg >= 0 ? (k == tg ? 1.0 : 0.0) : (k < N ? 1.0 : 0.0);
          }
#ifndef CVF_ABL_NOROWS
          *(onk ? urow + k : dump) = uv;
#else
          gb[n] += uv * 1e-300;
#endif
          // gamma_t (hmm.rs:127-129)
          const double gm = sel(tg >= 0, k == tg ? 1.0 : 0.0, normalized_r(al[m][n][q] * beta, sab, isab, inv_n));
          const double gon = onk ? gm : 0.0;
          gb[n] += gon;
          gp[n] += t == 0 ? gon : 0.0;
#ifndef CVF_ABL_NOBNUM
          unsafeAtomicAdd(onk ? &g.b_num[(size_t)o * N + k] : dump, onk ? gm : 0.0);  // hmm.rs:155-163
#else
          gb[n] += onk ? gm * (double)o : 0.0;
#endif
          // u_t = b(o_t) o beta_t, the next step's operand (this lane read u_{t+1} there above)
          xt[xt_at<G>(k, gi)] = sel(t >= 1 && k < N, ev[n][q] * beta, 0.0);
        }
      }
    }
    // the sums of gamma (hmm.rs:145-170): b_den over every step, a_den over t < T - 1 (r > 0),
    // pi over t == 0 -- into the workgroup's LDS sums (no loop-carried registers)
#pragma unroll
    for (int n = 0; n < CT; ++n)
      if (col[n] < N) {
        atomicAdd(&s_den[2][col[n]], gb[n]);
        if (r > 0) atomicAdd(&s_den[1][col[n]], gb[n]);
        atomicAdd(&s_den[0][col[n]], gp[n]);
      }
    __syncthreads();  // xt = u_t complete; red and the step-r slot free
  }
  // the workgroup's gamma sums: one atomic per state
  for (int i = tid; i < N; i += 64 * WV) {
    unsafeAtomicAdd(&g.pi_acc[i], s_den[0][i]);
    unsafeAtomicAdd(&g.a_den[i], s_den[1][i]);
    unsafeAtomicAdd(&g.b_den[i], s_den[2][i]);
  }
  if (w == 0) {
    z += __shfl_xor(z, 16);
    z += __shfl_xor(z, 32);
    if (l == 0 && z != 0.0) unsafeAtomicAdd(g.xi_zero, z);
  }
}

// ---- tiny arcs (cv_hmm_fit_train runs the E-step on A 2^K while A has one) --------------------
// the bits of the smallest positive entry (positive doubles order like their bit patterns)
__global__ __launch_bounds__(256) void bw_amin(const double* __restrict__ a, int64_t n, unsigned long long* out) {
  double mn = __builtin_inf();
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) {
    const double v = a[k];
    mn = v > 0.0 ? fmin(mn, v) : mn;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) mn = fmin(mn, __shfl_xor(mn, off));
  if ((threadIdx.x & 63) == 0 && mn < __builtin_inf()) atomicMin(out, (unsigned long long)__double_as_longlong(mn));
}

__global__ __launch_bounds__(256) void bw_scale(const double* __restrict__ src, double* __restrict__ dst, int64_t n,
                                                double scale) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)gridDim.x * 256) dst[k] = src[k] * scale;
}

hipError_t launch_bw_amin(const double* a, int64_t n, unsigned long long* out, hipStream_t stream) {
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (n + 255) / 256));
  hipLaunchKernelGGL(bw_amin, dim3(blocks), dim3(256), 0, stream, a, n, out);
  return hipGetLastError();
}

hipError_t launch_bw_scale(const double* src, double* dst, int64_t n, double scale, hipStream_t stream) {
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (n + 255) / 256));
  hipLaunchKernelGGL(bw_scale, dim3(blocks), dim3(256), 0, stream, src, dst, n, scale);
  return hipGetLastError();
}

// ---- M-step on the device (hmm.rs:145-175) ---------------------------------------------------
// Parameters stay resident between iterations: pi, a (and its transpose at), et = b^T.  The
// convergence sum d = sum |new - old| is reduced per block into part[]; the host adds the
// parts in a fixed order.  Built with -ffp-contract=off: same roundings as the host M-step.

__device__ __forceinline__ double block_sum_any(double v, double* red) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// m.parts_a blocks (1 up to kBwLdsMaxStates: the parts add in the same order as ever); block 0
// also updates pi
__global__ __launch_bounds__(256) void bw_mstep_pa(MstepArgs m) {
  __shared__ double red[4];
  const int N = m.nstates;
  const double* pi_acc = m.acc;
  const double* a_den = m.acc + N;
  const double* xs = m.acc + 3 * N + (size_t)m.nobs * N;
  const double zu = xs[(size_t)N * N] / ((double)N * (double)N);
  double d = 0.0;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
      const double np = pi_acc[i] / (double)m.nseq;
      d += fabs(np - m.pi[i]);
      m.pi[i] = np;
    }
  const int64_t nn = (int64_t)N * N;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nn; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = k / N, j = k - i * N;
    // The factored sum S = sum_t alpha_t u_t+1 / c_t can exceed DBL_MAX exactly where A is 0
    // or subnormal (each xi_t entry A alpha u / c is <= 1, hmm.rs:135-141, so alpha u / c <=
    // 1 / A): a == 0 takes no term (the reference's entries are 0 there; 0 * inf would be NaN),
    // and S is clamped to DBL_MAX as a last guard.  While A has an arc below kBwTinyArc the
    // E-step runs on A 2^K (m.ascale = 2^K, every arc >= kBwTinyArc there), which leaves
    // S' = S / 2^K in range, so the count is (a 2^K) S' -- exact scalings of the same products
    const double ak = m.ascale != 0.0 ? m.a[k] * m.ascale : m.a[k];
    const double na = ((m.a[k] != 0.0 ? ak * fmin(xs[k], 1.7976931348623157e308) : 0.0) + zu) / a_den[i];
    d += fabs(na - m.a[k]);
    m.a[k] = na;
    m.at[(size_t)j * N + i] = na;
  }
  d = block_sum_any(d, red);
  if (threadIdx.x == 0) m.part[blockIdx.x] = d;
}

__global__ __launch_bounds__(256) void bw_mstep_b(MstepArgs m) {
  __shared__ double red[4];
  const int N = m.nstates;
  const double* b_den = m.acc + 2 * N;
  const double* b_num = m.acc + 3 * N;
  const size_t n = (size_t)m.nobs * N;
  double d = 0.0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (size_t)gridDim.x * blockDim.x) {
    const double nb = b_num[k] / b_den[k % N];
    d += fabs(nb - m.et[k]);
    m.et[k] = nb;
  }
  d = block_sum_any(d, red);
  if (threadIdx.x == 0) m.part[m.parts_a + blockIdx.x] = d;
}

hipError_t launch_mle_counts(const MleArgs& g, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(mle_counts, dim3((unsigned)nseq), dim3(256), 0, stream, g);
  return hipGetLastError();
}

template <int NP>
static void launch_wave_estep(const BwArgs& g, int64_t nseq, int64_t nwaves, hipStream_t stream) {
  hipLaunchKernelGGL((bw_fwd_wave<NP>), dim3((unsigned)((nseq + 3) / 4)), dim3(256), 0, stream, g, nseq);
  hipLaunchKernelGGL((bw_bwd_stats_wave<NP>), dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0, stream, g, nseq,
                     nwaves);
}

// sequences per workgroup of the 64 < N <= 256 kernels: 16 MT; MT = 2 runs two workgroups per
// CU, so one's reductions and barriers overlap the other's matrix products (MT = 4, one
// workgroup of 64 per CU, and eight forward waves per workgroup -- 82.4 vs 79.2 ms at config 4
// -- measured slower in round 4 and removed in round 6 with the GEMM's one-wave-tile,
// double-buffered and 32 x 32 variants)
template <int NP, int MT, int WVF, int WVB>
static void launch_mm(const BwArgs& g, int64_t nseq, hipStream_t stream, hipEvent_t fwd_done) {
  const dim3 grid((unsigned)((nseq + 16 * MT - 1) / (16 * MT)));
  hipLaunchKernelGGL((bw_fwd_mm<NP, MT, WVF>), grid, dim3(64 * WVF), 0, stream, g, nseq);
  if (fwd_done) (void)hipEventRecord(fwd_done, stream);
  hipLaunchKernelGGL((bw_bwd_mm<NP, MT, WVB>), grid, dim3(64 * WVB), 0, stream, g, nseq);
}

// tuning key bw_perseq = 1 keeps one workgroup per sequence (A/B and tests)
static bool bw_per_seq() { return cvk::tuning().bw_perseq == 1; }

bool bw_estep_mm(int nstates) { return nstates > kBwWaveStates && nstates <= kBwMmStates && !bw_per_seq(); }

// tuning key bw_gemm_path = 1 takes the xi GEMM path at every N (A/B and tests)
bool bw_gemm_path() { return cvk::tuning().bw_gemm_path == 1; }

hipError_t launch_bw_estep(const BwArgs& g, int64_t nseq, int64_t max_waves, hipStream_t stream, int64_t nrows,
                           hipEvent_t fwd_done) {
  if (nseq <= 0) return hipSuccess;
  if (g.nstates > kBwMaxStates) return hipErrorInvalidValue;
  if (g.nstates > kBwMmStates) {  // N > 256: the strided per-sequence kernels, then the xi GEMM
    if (g.gscratch) {  // their vectors in global scratch, kBwScratchSeqs sequences per launch
      for (int64_t s0 = 0; s0 < nseq; s0 += kBwScratchSeqs) {
        BwArgs gb = g;
        gb.offsets = g.offsets + s0;  // rows stay at (element - elem_base)
        const unsigned n = (unsigned)std::min<int64_t>(kBwScratchSeqs, nseq - s0);
        hipLaunchKernelGGL(bw_forward_g<true>, dim3(n), dim3(256), 0, stream, gb);
        hipLaunchKernelGGL(bw_backward_g<true>, dim3(n), dim3(256), 0, stream, gb);
        hipLaunchKernelGGL(bw_stats_rows_g<true>, dim3(n), dim3(256), 0, stream, gb);
      }
    } else {  // in LDS (N <= kBwLdsMaxStates)
      if (g.nstates > kBwLdsMaxStates) return hipErrorInvalidValue;
      const size_t l1 = (size_t)g.nstates * 8, l4 = 4 * l1;
      for (const void* k :
           {reinterpret_cast<const void*>(&bw_forward_g<false>), reinterpret_cast<const void*>(&bw_backward_g<false>)})
        if (l1 > 64 * 1024) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l1);
      if (l4 > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bw_stats_rows_g<false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)l4);
      hipLaunchKernelGGL(bw_forward_g<false>, dim3((unsigned)nseq), dim3(256), l1, stream, g);
      hipLaunchKernelGGL(bw_backward_g<false>, dim3((unsigned)nseq), dim3(256), l1, stream, g);
      hipLaunchKernelGGL(bw_stats_rows_g<false>, dim3((unsigned)nseq), dim3(256), l4, stream, g);
    }
    const int nt = (g.nstates + 127) / 128;
    const int64_t parts2 = std::max<int64_t>(1, std::min<int64_t>(512 / (nt * nt), (nrows + 255) / 256));
    const int64_t per2 = ((nrows + parts2 - 1) / parts2 + kGemmKB - 1) / kGemmKB * kGemmKB;
    const int64_t np2 = (nrows + per2 - 1) / per2;
    hipLaunchKernelGGL(bw_xi_gemm_lds, dim3((unsigned)((np2 + 7) / 8 * 8 * nt * nt)), dim3(256), 0, stream, g, nrows,
                       per2);
    return hipGetLastError();
  }
  const bool mm = bw_estep_mm(g.nstates);
  if (g.nstates > kBwLdsStates || mm || bw_gemm_path()) {  // the xi sum as R^T U on the matrix cores
    BwArgs gg = g;
    if (!mm) gg.rscale = nullptr;  // the per-sequence kernels store R over alpha
    if (mm) {  // 16 MT sequences per workgroup, the step products on the matrix cores
      // waves per workgroup: forward / backward (the backward's per-step state needs the
      // registers of four waves at 256 states)
      if (g.nstates <= 128) launch_mm<128, 2, 4, 4>(g, nseq, stream, fwd_done);
      else if (g.nstates <= 192) launch_mm<192, 2, 4, 4>(g, nseq, stream, fwd_done);
      else launch_mm<256, 2, 4, 4>(g, nseq, stream, fwd_done);
    } else {
      hipLaunchKernelGGL(bw_forward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
      hipLaunchKernelGGL(bw_backward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
      hipLaunchKernelGGL(bw_stats_rows, dim3((unsigned)nseq), dim3(256), 0, stream, g);
    }
    // 64 x 64 tiles per wave above 128 states (32 x 32 below); ~4,096 waves: row ranges of a
    // multiple of 4 rows per output tile
    const bool t64 = g.nstates > 128;
    const int ts = t64 ? 64 : 32, ntt = (g.nstates + ts - 1) / ts;
    const int64_t parts = std::max<int64_t>(1, std::min<int64_t>(4096 / (ntt * ntt), (nrows + 255) / 256));
    const int64_t per = ((nrows + parts - 1) / parts + 3) / 4 * 4;
    const int64_t np = (nrows + per - 1) / per;
    // a multiple of 8 row ranges (empty ones exit): the XCD-aware block mapping of bw_xi_gemm
    const dim3 grid((unsigned)((np + 7) / 8 * 8 * ntt * ntt)), block(64);
    if (t64) {
      // 128 x 128 per workgroup: ~2 workgroups per CU over 256 CUs
      const int nt = (g.nstates + 127) / 128;
      const int64_t parts2 = std::max<int64_t>(1, std::min<int64_t>(512 / (nt * nt), (nrows + 255) / 256));
      const int64_t per2 = ((nrows + parts2 - 1) / parts2 + kGemmKB - 1) / kGemmKB * kGemmKB;
      const int64_t np2 = (nrows + per2 - 1) / per2;
      hipLaunchKernelGGL(bw_xi_gemm_lds, dim3((unsigned)((np2 + 7) / 8 * 8 * nt * nt)), dim3(256), 0, stream, gg, nrows,
                         per2);
    } else {
      hipLaunchKernelGGL((bw_xi_gemm<2, 1>), grid, block, 0, stream, gg, nrows, per);
    }
    return hipGetLastError();
  }
  if (g.nstates <= kBwWaveStates) {
    const int64_t nwaves = std::max<int64_t>(1, std::min<int64_t>((nseq + 1) / 2, max_waves));  // pairs
    if (g.nstates <= 16) launch_wave_estep<16>(g, nseq, nwaves, stream);
    else if (g.nstates <= 32) launch_wave_estep<32>(g, nseq, nwaves, stream);
    else if (g.nstates <= 48) launch_wave_estep<48>(g, nseq, nwaves, stream);
    else launch_wave_estep<64>(g, nseq, nwaves, stream);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(bw_forward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
  hipLaunchKernelGGL(bw_backward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
  const size_t lds = ((size_t)g.nstates * g.nstates + 256 + 4) * sizeof(double);
  if (lds > 64 * 1024)  // per device: set on every launch that needs it (cheap)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bw_stats), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  hipLaunchKernelGGL(bw_stats, dim3((unsigned)nseq), dim3(256), lds, stream, g);
  return hipGetLastError();
}

hipError_t launch_bw_mstep(const MstepArgs& m, int nparts_b, hipStream_t stream) {
  hipLaunchKernelGGL(bw_mstep_pa, dim3((unsigned)std::max(m.parts_a, 1)), dim3(256), 0, stream, m);
  hipLaunchKernelGGL(bw_mstep_b, dim3((unsigned)nparts_b), dim3(256), 0, stream, m);
  return hipGetLastError();
}

}  // namespace cvf
