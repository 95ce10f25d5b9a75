// chain.hip -- CPSolver's super-sequence decode, chained exactly, for N <= 256 (gfx950).
//
// The reference decodes a whole batch as ONE super-sequence (utils.rs:62-103): at a sequence
// start the candidate term is the constant pi[j] (MetaElements::transitions, utils.rs:32-38),
// so every value of sequence k carries the running total of sequences 0..k-1 and rounds
// accordingly.  Per element t and state j (cp.rs:70-79):
//   psi = first argmax_i (d[i] + tr(i, j)),   tr = first ? pi[j] : a[i][j]
//   d'[j] = d[psi] + (tr(psi, j) + b[j][o_t])
// then the first argmax of the last row and the backtrack through psi (cp.rs:85-93, 140).
// The element loop is a strict recurrence, so ONE workgroup walks it: thread (g, j) scans the
// candidate rows [g R, g R + R) of column j (R = NP / G), the G partial (max, first index)
// pairs are combined in row order (first index kept on ties: identical to the serial scan),
// and d' goes back through LDS.  A (NP^2 f64 = 512 KiB at N = 256) is spread over the
// workgroup's registers (RREG rows per thread), its LDS (RLDS rows) and L2 (RGLB rows, loaded
// at the start of each element, consumed last); at NP <= 128 all candidate rows sit in
// registers and a full copy of A in LDS serves the value's a[psi][j].
// The backtrack is parallel over segments: pass 1 maps each segment's last-element state to
// the state before its first element for ALL NP states at once (one lane per state); the
// host walks the segment maps from the final state; pass 2 writes every segment's path.
#include "chain.h"

namespace cvk {
namespace {

// AFULL: a full copy of A in LDS after the row slices (NP <= 128), so the value's a[psi][j]
// is an LDS read instead of an L2 round trip on the element's critical path.
template <int NP, int G, int RREG, int RLDS, int RGLB, bool AFULL>
__global__ __launch_bounds__(NP * G) void cp_chain_wg(CpChainWgArgs g) {
  constexpr int R = NP / G;
  static_assert(RREG + RLDS + RGLB == R, "every candidate row has one home");
  static_assert(NP % 64 == 0, "a wave holds one candidate group");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* prev = sm;                    // [NP]
  double* cur = sm + NP;                // [NP]
  double* pm = sm + 2 * NP;             // [G][NP] partial maxima
  int* pa = reinterpret_cast<int*>(sm + 2 * NP + G * NP);  // [G][NP] their first indices
  double* al = sm + 2 * NP + G * NP + G * NP / 2;          // [G][RLDS][NP] LDS rows of A
  double* afull = al + G * RLDS * NP;                      // [NP][NP] when AFULL
  const int tid = threadIdx.x;
  const int c = tid % NP;
  const int grp = __builtin_amdgcn_readfirstlane(tid / NP);  // wave-uniform (NP % 64 == 0)
  const int i0 = grp * R;
  double areg[RREG > 0 ? RREG : 1];
#pragma unroll
  for (int r = 0; r < RREG; ++r) areg[r] = g.a[(size_t)(i0 + r) * NP + c];
  for (int r = 0; r < RLDS; ++r) al[(grp * RLDS + r) * NP + c] = g.a[(size_t)(i0 + RREG + r) * NP + c];
  const double* aglb = g.a + (size_t)(i0 + RREG + RLDS) * NP + c;
  if constexpr (AFULL)
    for (int k = tid; k < NP * NP; k += NP * G) afull[k] = g.a[k];
  if (grp == 0) prev[c] = g.pi[c] + g.et[(size_t)g.obs[0] * NP + c];  // init_probs (cp.rs:66-68)
  __syncthreads();
  const int64_t L = g.len;
  for (int64_t t = 1; t < L; ++t) {
    const bool first = g.first[t] != 0;
    const int o = g.obs[t];
    double m;
    int arg;
    if (first) {  // transitions = the constant pi[j] (utils.rs:32-35)
      const double pj = g.pi[c];
      m = prev[i0] + pj;
      arg = i0;
#pragma unroll 8
      for (int r = 1; r < R; ++r) {
        const double x = prev[i0 + r] + pj;
        if (x > m) {
          m = x;
          arg = i0 + r;
        }
      }
    } else {
      double ag[RGLB > 0 ? RGLB : 1];
#pragma unroll
      for (int r = 0; r < RGLB; ++r) ag[r] = aglb[(size_t)r * NP];
      m = prev[i0] + areg[0];
      arg = i0;
#pragma unroll
      for (int r = 1; r < RREG; ++r) {
        const double x = prev[i0 + r] + areg[r];
        if (x > m) {
          m = x;
          arg = i0 + r;
        }
      }
#pragma unroll 8
      for (int r = 0; r < RLDS; ++r) {
        const double x = prev[i0 + RREG + r] + al[(grp * RLDS + r) * NP + c];
        if (x > m) {
          m = x;
          arg = i0 + RREG + r;
        }
      }
#pragma unroll
      for (int r = 0; r < RGLB; ++r) {
        const double x = prev[i0 + RREG + RLDS + r] + ag[r];
        if (x > m) {
          m = x;
          arg = i0 + RREG + RLDS + r;
        }
      }
    }
    pm[grp * NP + c] = m;
    pa[grp * NP + c] = arg;
    __syncthreads();
    if (grp == 0) {
      double M = pm[c];
      int A = pa[c];
#pragma unroll
      for (int q = 1; q < G; ++q) {
        const double x = pm[q * NP + c];
        if (x > M) {  // strict: the earlier rows keep their ties (first index overall)
          M = x;
          A = pa[q * NP + c];
        }
      }
      const double tr = first ? g.pi[c] : AFULL ? afull[A * NP + c] : g.a[(size_t)A * NP + c];
      cur[c] = prev[A] + (tr + g.et[(size_t)o * NP + c]);  // cp.rs:75-77
      g.psi[(size_t)t * NP + c] = (uint16_t)A;
    }
    __syncthreads();
    double* tmp = prev;
    prev = cur;
    cur = tmp;
  }
  if (tid == 0) {  // cp.rs:86 / 140: first argmax and max of the last row
    int cs = 0;
    double obj = prev[0];
    for (int i = 1; i < g.nstates; ++i)
      if (prev[i] > obj) {
        obj = prev[i];
        cs = i;
      }
    *g.objective = obj;
    *g.final_state = cs;
  }
}

template <int NP, int G, int RREG, int RLDS, int RGLB, bool AFULL>
size_t chain_lds() {
  return (size_t)(2 * NP + G * NP + G * NP / 2 + G * RLDS * NP + (AFULL ? NP * NP : 0)) * sizeof(double);
}

template <int NP, int G, int RREG, int RLDS, int RGLB, bool AFULL>
hipError_t chain_launch(const CpChainWgArgs& g, hipStream_t stream) {
  const size_t lds = chain_lds<NP, G, RREG, RLDS, RGLB, AFULL>();
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cp_chain_wg<NP, G, RREG, RLDS, RGLB, AFULL>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((cp_chain_wg<NP, G, RREG, RLDS, RGLB, AFULL>), dim3(1), dim3(NP * G), lds, stream, g);
  return hipGetLastError();
}

constexpr int kBtRows = 32;  // psi rows per LDS chunk in the backtrack passes

// pass 1: segment k >= 1, lane s = a state at the segment's last element e1 - 1; walk psi
// down to e0 (inclusive): the state at e0 - 1 on the best path through s
template <int NP>
__global__ __launch_bounds__(NP) void cp_chain_seg_map(CpChainBtArgs g) {
  __shared__ uint16_t rows[kBtRows][NP];
  const int64_t k = (int64_t)blockIdx.x + 1;
  const int64_t e0 = k * g.seg, e1 = e0 + g.seg < g.len ? e0 + g.seg : g.len;
  const int j = threadIdx.x;
  int cs = j;
  for (int64_t hi = e1 - 1; hi >= e0; hi -= kBtRows) {
    const int64_t lo = hi - kBtRows + 1 > e0 ? hi - kBtRows + 1 : e0;
    const int n = (int)(hi - lo + 1);
    __syncthreads();  // the previous chunk is consumed
    for (int r = 0; r < n; ++r) rows[r][j] = g.psi[(size_t)(lo + r) * NP + j];
    __syncthreads();
    for (int r = n - 1; r >= 0; --r) cs = rows[r][cs];
  }
  g.map[(size_t)k * NP + j] = (uint16_t)cs;
}

// pass 2: one wave per segment follows psi from the resolved end state, lane 0 walking
// through the LDS chunk, the wave storing the chunk's path
template <int NP>
__global__ __launch_bounds__(64) void cp_chain_seg_path(CpChainBtArgs g) {
  __shared__ uint16_t rows[kBtRows][NP];
  __shared__ int32_t pc[kBtRows];
  const int64_t k = blockIdx.x;
  const int64_t e0 = k * g.seg, e1 = e0 + g.seg < g.len ? e0 + g.seg : g.len;
  const int lane = threadIdx.x;
  int cs = g.end_state[k];
  for (int64_t hi = e1 - 1; hi >= e0; hi -= kBtRows) {
    const int64_t lo = hi - kBtRows + 1 > e0 ? hi - kBtRows + 1 : e0;
    const int n = (int)(hi - lo + 1);
    __syncthreads();
    for (int r = 0; r < n; ++r)
      for (int j = lane; j < NP; j += 64) rows[r][j] = g.psi[(size_t)(lo + r) * NP + j];
    __syncthreads();
    if (lane == 0) {
      for (int r = n - 1; r >= 0; --r) {  // path[t] = cs; cs = psi[t][cs] (cp.rs:88-92)
        pc[r] = cs;
        cs = rows[r][cs];
      }
    }
    __syncthreads();
    for (int r = lane; r < n; r += 64) g.path[lo + r] = pc[r];
  }
}

}  // namespace

size_t cp_chain_wg_lds(int np) {
  switch (np) {
    case 64: return chain_lds<64, 4, 16, 0, 0, true>();
    case 128: return chain_lds<128, 4, 32, 0, 0, true>();
    case 192: return chain_lds<192, 4, 32, 16, 0, false>();
    case 256: return chain_lds<256, 4, 47, 17, 0, false>();
    default: return 0;
  }
}

hipError_t launch_cp_chain_wg(int np, const CpChainWgArgs& g, hipStream_t stream) {
  if (g.len <= 0) return hipSuccess;
  switch (np) {
    case 64: return chain_launch<64, 4, 16, 0, 0, true>(g, stream);
    case 128: return chain_launch<128, 4, 32, 0, 0, true>(g, stream);
    case 192: return chain_launch<192, 4, 32, 16, 0, false>(g, stream);
    case 256: return chain_launch<256, 4, 47, 17, 0, false>(g, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_cp_chain_seg_map(const CpChainBtArgs& g, hipStream_t stream) {
  if (g.nseg <= 1) return hipSuccess;
  const dim3 grid((unsigned)(g.nseg - 1));
  switch (g.np) {
    case 64: hipLaunchKernelGGL(cp_chain_seg_map<64>, grid, dim3(64), 0, stream, g); break;
    case 128: hipLaunchKernelGGL(cp_chain_seg_map<128>, grid, dim3(128), 0, stream, g); break;
    case 192: hipLaunchKernelGGL(cp_chain_seg_map<192>, grid, dim3(192), 0, stream, g); break;
    case 256: hipLaunchKernelGGL(cp_chain_seg_map<256>, grid, dim3(256), 0, stream, g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_cp_chain_seg_path(const CpChainBtArgs& g, hipStream_t stream) {
  if (g.nseg <= 0) return hipSuccess;
  const dim3 grid((unsigned)g.nseg);
  switch (g.np) {
    case 64: hipLaunchKernelGGL(cp_chain_seg_path<64>, grid, dim3(64), 0, stream, g); break;
    case 128: hipLaunchKernelGGL(cp_chain_seg_path<128>, grid, dim3(64), 0, stream, g); break;
    case 192: hipLaunchKernelGGL(cp_chain_seg_path<192>, grid, dim3(64), 0, stream, g); break;
    case 256: hipLaunchKernelGGL(cp_chain_seg_path<256>, grid, dim3(64), 0, stream, g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace cvk
