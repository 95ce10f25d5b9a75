// fit.h -- argument blocks and launchers of the HMM-fitting kernels (fit.hip).
// Internal to libcviterbi; the public boundary is include/cviterbi.h (cv_hmm_fit_*).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvf {

constexpr int kBwLdsStates = 128;  // bw_stats keeps a sequence's N x N xi sum in LDS up to here
constexpr int kBwMmStates = 256;   // up to here: the matrix-core step kernels (bw_*_mm)
constexpr int kBwLdsMaxStates = 4096;  // beyond kBwMmStates: states strided over 256 threads, the
                                       // step's vector and 3 gamma sums in LDS (4 N doubles)
constexpr int kBwMaxStates = 65535;    // beyond kBwLdsMaxStates: the same vectors in global
                                       // scratch (BwArgs::gscratch), kBwScratchSeqs per launch
constexpr int kBwScratchSeqs = 2048;

struct MleArgs {
  const int64_t* offsets;
  const int32_t* obs;   // [sum T] flattened observation index
  const int32_t* tags;  // [sum T] state of every element (all >= 0)
  int nstates;
  int64_t nobs;
  uint64_t* pi_cnt;     // [N]
  uint64_t* a_cnt;      // [N][N]
  uint64_t* b_cnt;      // [N][V]
  uint64_t* seen;       // [N]
  uint64_t* end;        // [N]
};

struct BwArgs {
  const int64_t* offsets;
  const int32_t* obs;
  const int32_t* tags;  // -1 = untagged (None)
  int64_t elem_base;    // element offset that maps to row 0 of alpha / beta
  const int64_t* order; // N <= 64 kernels: processing order of the sequences (nullable)
  int nstates;
  const double* pi;     // [N]
  const double* a;      // [N][N] row-major (from, to)
  const double* at;     // [N][N] transposed
  const double* et;     // [V][N] emissions transposed
  double* alpha;        // [elements][N] workspace
  double* beta;         // [elements][N] workspace
  double* rscale;       // [elements] N > 64 matrix-core path: row t of R = alpha_t * rscale[t]
                        // (1 / (c_t 2^k), 0 where c_t = 0 or t = T - 1); null: R is stored over alpha
  double* gscratch;     // [kBwScratchSeqs][4 N] N > kBwLdsMaxStates (or tuning key bw_global above 256):
                        // the strided kernels' per-sequence vectors in global memory
  double* dump;         // [kBwDumpWaves][64] N <= 64 kernels: target of the stores / atomic adds
                        // of lanes without a state (one row per wave: no shared hot line)
  // E-step sums (accumulated across sequences; zeroed by the host per iteration)
  double* pi_acc;       // [N]  sum of gamma_0
  double* a_den;        // [N]  sum of gamma_t, t < T-1
  double* b_den;        // [N]  sum of gamma_t
  double* b_num;        // [V][N] sum of gamma_t at o_t
  double* xi_s;         // [N][N] sum of (alpha_t / c_t) (x) u_{t+1}
  double* xi_zero;      // [1] number of steps with c_t == 0 (uniform xi)
};

// An arc below this (2^-960) can make the factored xi sum of its entry overflow (its per-step
// terms are ~xi / a) and, when subnormal, leaves the step normaliser c_t = fl(a u) with a few
// significant bits; cv_hmm_fit_train then runs the E-step on A 2^K (MstepArgs::ascale)
constexpr double kBwTinyArc = 0x1p-960;

constexpr int kBwWaveStates = 64;  // N <= 64: one wave per sequence (bw_*_wave)
constexpr int kBwDumpWaves = 4096;

// M-step: acc = [pi_acc N | a_den N | b_den N | b_num V*N | xi_s N*N | xi_zero 1]
struct MstepArgs {
  const double* acc;
  int nstates;
  int64_t nobs;
  int64_t nseq;
  double* pi;    // [N]     updated in place
  double* a;     // [N][N]  updated in place
  double* at;    // [N][N]  transposed copy, rewritten
  double* et;    // [V][N]  b^T, updated in place
  double* part;  // [parts_a + nparts_b] per-block sums of |new - old|
  int parts_a;   // blocks of the pi / a M-step (1; 1,024 above kBwLdsMaxStates: N^2 entries)
  double ascale;  // the E-step ran on A 2^K (tiny arcs): count = (a ascale) S; 0: unscaled
};

hipError_t launch_mle_counts(const MleArgs& g, int64_t nseq, hipStream_t stream);
// forward, backward and the E-step sums of sequences [0, nseq) of g.offsets; the N <= 64
// backward kernel runs at most max_waves waves (each walks several sequences)
// nrows: the chunk's elements (alpha / beta rows from elem_base), for the GEMM path (N > 128)
// fwd_done (64 < N <= 256, the matrix-core kernels): recorded on `stream` right after the
// forward launch when non-null
hipError_t launch_bw_estep(const BwArgs& g, int64_t nseq, int64_t max_waves, hipStream_t stream, int64_t nrows,
                           hipEvent_t fwd_done = nullptr);
// the E-step runs the matrix-core kernels (64 < N <= 256; tuning key bw_perseq = 1: not)
bool bw_estep_mm(int nstates);
// tuning key bw_gemm_path = 1: the per-sequence kernels + xi GEMM at every N (A/B and tests;
// tiny arcs no longer select it: since round 5 the E-step runs on A 2^K on whichever path N
// picks, cv_hmm_fit_train)
bool bw_gemm_path();
// *out = the bits of the smallest positive a[k], k < n (*out preset to +inf's bits by the caller)
hipError_t launch_bw_amin(const double* a, int64_t n, unsigned long long* out, hipStream_t stream);
// dst[k] = src[k] * scale (a power of two: exact), k < n
hipError_t launch_bw_scale(const double* src, double* dst, int64_t n, double scale, hipStream_t stream);
hipError_t launch_bw_mstep(const MstepArgs& m, int nparts_b, hipStream_t stream);

}  // namespace cvf
