// fit.hip -- MI355X (gfx950) kernels for fitting the HMM:
//   mle_counts     exact integer counts of hmm.rs:30-62 (maximum_likelihood_estimation)
//   bw_forward     scaled, tag-clamped forward pass of hmm.rs:78-100 (train)
//   bw_backward    scaled, tag-clamped backward pass of hmm.rs:102-121
//   bw_stats       gamma (hmm.rs:124-131), xi (hmm.rs:133-143) and the E-step sums of
//                  hmm.rs:145-170, accumulated per sequence and added to global sums
// f64 throughout, probability space, like the reference.  One workgroup (256 threads) per
// sequence; thread i < N owns state i.  The transition matrix is read from L2 (row-major A
// for the forward step, A^T for the backward and xi steps, so every read is coalesced
// across the threads of a row).  bw_stats keeps the sequence's xi sum (N x N) in LDS, so
// the trainer covers N <= 128 (the reference trains POS taggers: N = 12).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fit.h"

namespace cvf {

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
__device__ __forceinline__ double normalized(double v, double s, int n) { return s != 0.0 ? v / s : 1.0 / n; }

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
        // S[k][j] += (alpha_t[k] / c) * u_j: thread j = i owns column i; alpha/c via LDS
        const double uj = (i < N) ? p[i] : 0.0;
        __syncthreads();
        if (i < N) p[i] = ai / c;
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

hipError_t launch_mle_counts(const MleArgs& g, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(mle_counts, dim3((unsigned)nseq), dim3(256), 0, stream, g);
  return hipGetLastError();
}

hipError_t launch_bw_estep(const BwArgs& g, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  if (g.nstates > kBwMaxStates) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bw_forward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
  hipLaunchKernelGGL(bw_backward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
  const size_t lds = ((size_t)g.nstates * g.nstates + 256 + 4) * sizeof(double);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&bw_stats), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(bw_stats, dim3((unsigned)nseq), dim3(256), lds, stream, g);
  return hipGetLastError();
}

}  // namespace cvf
