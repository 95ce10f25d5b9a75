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

#include <algorithm>

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
// bw_stats_rows).  One wave per 32 x 32 output tile and row range: per 4 rows, lane l feeds
// R[r + l/16][m0 + 16 mt + l%16] and U[...][n0 + 16 nt + l%16] into four
// v_mfma_f64_16x16x4_f64 (2 x 2 tiles); one atomic flush of the tile at the end.
__global__ __launch_bounds__(64) void bw_xi_gemm(BwArgs g, int64_t nrows, int64_t rows_per_wave) {
  const int N = g.nstates;
  const int nt32 = (N + 31) / 32;
  const int tile = blockIdx.x % (nt32 * nt32);
  const int64_t part = blockIdx.x / (nt32 * nt32);
  const int m0 = 32 * (tile / nt32), n0 = 32 * (tile % nt32);
  const int l = threadIdx.x, kk = l >> 4, cl = l & 15;
  const int64_t r0 = part * rows_per_wave, r1 = r0 + rows_per_wave < nrows ? r0 + rows_per_wave : nrows;
  typedef double double4_t __attribute__((ext_vector_type(4)));
  double4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = double4_t{0.0, 0.0, 0.0, 0.0};
  const int cm[2] = {m0 + cl, m0 + 16 + cl}, cn[2] = {n0 + cl, n0 + 16 + cl};
  const bool vm[2] = {cm[0] < N, cm[1] < N}, vn[2] = {cn[0] < N, cn[1] < N};
  for (int64_t r = r0; r < r1; r += 4) {
    const int64_t row = r + kk;
    const bool vr = row < r1;
    const double* R = g.alpha + (size_t)(vr ? row : r0) * N;
    const double* U = g.beta + (size_t)(vr ? row : r0) * N;
    double av[2], bv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      av[q] = (vr && vm[q]) ? R[cm[q]] : 0.0;
      bv[q] = (vr && vn[q]) ? U[cn[q]] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
  }
  // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + 16 * a + (l >> 4) + 4 * q, col = n0 + 16 * b + (l & 15);
        if (row < N && col < N && acc[a][b][q] != 0.0) unsafeAtomicAdd(&g.xi_s[(size_t)row * N + col], acc[a][b][q]);
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

__global__ __launch_bounds__(256) void bw_mstep_pa(MstepArgs m) {
  __shared__ double red[4];
  const int N = m.nstates;
  const double* pi_acc = m.acc;
  const double* a_den = m.acc + N;
  const double* xs = m.acc + 3 * N + (size_t)m.nobs * N;
  const double zu = xs[(size_t)N * N] / ((double)N * (double)N);
  double d = 0.0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const double np = pi_acc[i] / (double)m.nseq;
    d += fabs(np - m.pi[i]);
    m.pi[i] = np;
  }
  for (int k = threadIdx.x; k < N * N; k += blockDim.x) {
    const int i = k / N, j = k - i * N;
    // The factored sum S = sum_t alpha_t u_t+1 / c_t can exceed DBL_MAX exactly where A is 0
    // or subnormal (each xi_t entry A alpha u / c is <= 1, hmm.rs:135-141, so alpha u / c <=
    // 1 / A): a == 0 takes no term (the reference's entries are 0 there; 0 * inf would be NaN),
    // and S is clamped to DBL_MAX (finite for a subnormal a; never reached for a normal one
    // unless ~1/a summed over steps overflows)
    const double na =
        ((m.a[k] != 0.0 ? m.a[k] * fmin(xs[k], 1.7976931348623157e308) : 0.0) + zu) / a_den[i];
    d += fabs(na - m.a[k]);
    m.a[k] = na;
    m.at[(size_t)j * N + i] = na;
  }
  d = block_sum_any(d, red);
  if (threadIdx.x == 0) m.part[0] = d;
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
  if (threadIdx.x == 0) m.part[1 + blockIdx.x] = d;
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

hipError_t launch_bw_estep(const BwArgs& g, int64_t nseq, int64_t max_waves, hipStream_t stream, int64_t nrows) {
  if (nseq <= 0) return hipSuccess;
  if (g.nstates > kBwMaxStates) return hipErrorInvalidValue;
  if (g.nstates > kBwLdsStates) {  // the xi sum as R^T U on the matrix cores
    hipLaunchKernelGGL(bw_forward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
    hipLaunchKernelGGL(bw_backward, dim3((unsigned)nseq), dim3(256), 0, stream, g);
    hipLaunchKernelGGL(bw_stats_rows, dim3((unsigned)nseq), dim3(256), 0, stream, g);
    const int nt32 = (g.nstates + 31) / 32;
    // ~4,096 waves: row ranges of a multiple of 4 rows per output tile
    const int64_t parts = std::max<int64_t>(1, std::min<int64_t>(4096 / (nt32 * nt32), (nrows + 255) / 256));
    const int64_t per = ((nrows + parts - 1) / parts + 3) / 4 * 4;
    const int64_t np = (nrows + per - 1) / per;
    hipLaunchKernelGGL(bw_xi_gemm, dim3((unsigned)(np * nt32 * nt32)), dim3(64), 0, stream, g, nrows, per);
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
  hipLaunchKernelGGL(bw_mstep_pa, dim3(1), dim3(256), 0, stream, m);
  hipLaunchKernelGGL(bw_mstep_b, dim3((unsigned)nparts_b), dim3(256), 0, stream, m);
  return hipGetLastError();
}

}  // namespace cvf
