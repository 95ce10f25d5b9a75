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

#include <algorithm>
#include "trellis.h"
#include "trellis64.h"
#include "wave64.h"

namespace cvk {
namespace {

// AFULL: a full copy of A in LDS after the row slices (NP <= 128), so the value's a[psi][j]
// is an LDS read instead of an L2 round trip on the element's critical path.
template <int NP, int G, int RREG, int RLDS, int RGLB, bool AFULL>
constexpr size_t chain_lds_bytes() {
  return (size_t)(2 * NP + G * NP + G * NP / 2 + G * RLDS * NP + (AFULL ? NP * NP : 0)) * sizeof(double);
}

template <int NP, int G, int RREG, int RLDS, int RGLB, bool AFULL, bool BATCH = false>
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
  const int32_t* obs = g.obs;
  uint16_t* psi = g.psi;
  int64_t L = g.len;
  int64_t e0 = 0;
  if constexpr (BATCH) {
    e0 = g.soff[blockIdx.x];
    L = g.soff[blockIdx.x + 1] - e0;
    obs += e0;
    psi += e0 * NP;
    if (L <= 0) return;  // uniform over the workgroup
  }
  const int i0 = grp * R;
  double areg[RREG > 0 ? RREG : 1];
#pragma unroll
  for (int r = 0; r < RREG; ++r) areg[r] = g.a[(size_t)(i0 + r) * NP + c];
  for (int r = 0; r < RLDS; ++r) al[(grp * RLDS + r) * NP + c] = g.a[(size_t)(i0 + RREG + r) * NP + c];
  const double* aglb = g.a + (size_t)(i0 + RREG + RLDS) * NP + c;
  if constexpr (AFULL)
    for (int k = tid; k < NP * NP; k += NP * G) afull[k] = g.a[k];
  if (grp == 0) {  // init_probs (cp.rs:66-68), or the row before this part of the chain
    if constexpr (BATCH)
      prev[c] = g.sinit[blockIdx.x] + (g.pi[c] + g.et[(size_t)obs[0] * NP + c]);
    else
      prev[c] = g.init_row ? g.init_row[c] : g.pi[c] + g.et[(size_t)obs[0] * NP + c];
  }
  __syncthreads();
  for (int64_t t = (!BATCH && g.init_row) ? 0 : 1; t < L; ++t) {
    // BATCH passes first = nullptr: the branch stays (without it the compiler's schedule of the
    // candidate loop spills 42 VGPRs at N = 256)
    const bool first = BATCH ? (g.first && g.first[t] != 0) : g.first[t] != 0;
    const int o = obs[t];
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
      psi[(size_t)t * NP + c] = (uint16_t)A;
    }
    __syncthreads();
    double* tmp = prev;
    prev = cur;
    cur = tmp;
  }
  if constexpr (BATCH) {
    if (grp == 0 && c < g.nstates) g.final_row[(size_t)blockIdx.x * g.nstates + c] = prev[c];
    // the path: first argmax of the last row (cp.rs:86), then psi back to element 0, the psi
    // rows staged through the LDS the A rows no longer need (after both row buffers), walked by
    // one thread (a dependent LDS read per element instead of an L2 round trip)
    constexpr int64_t kCap = (int64_t)((chain_lds_bytes<NP, G, RREG, RLDS, RGLB, AFULL>() - 2 * NP * sizeof(double)) /
                                       (NP * sizeof(uint16_t))) / 8 * 8;
    static_assert(kCap >= 8, "psi staging rows");
    uint16_t* ps = reinterpret_cast<uint16_t*>(sm + 2 * NP);
    int32_t* path = g.path + e0;
    int cs = 0;
    if (tid == 0) {
      double m = prev[0];
      for (int i = 1; i < g.nstates; ++i)
        if (prev[i] > m) {
          m = prev[i];
          cs = i;
        }
      path[L - 1] = cs;
    }
    __threadfence();  // this workgroup's psi stores, read back below
    __syncthreads();
    for (int64_t hi = L; hi > 1;) {  // rows [lo, hi) hold psi for elements lo .. hi - 1
      const int64_t lo = hi - 1 > kCap ? hi - kCap : 1;
      const uint4* src = reinterpret_cast<const uint4*>(psi + lo * NP);
      uint4* dst = reinterpret_cast<uint4*>(ps);
      for (int64_t q = tid; q < (hi - lo) * NP / 8; q += NP * G) dst[q] = src[q];
      __syncthreads();
      if (tid == 0)
        for (int64_t t = hi - 1; t >= lo; --t) {
          cs = ps[(t - lo) * NP + cs];
          path[t - 1] = cs;
        }
      __syncthreads();
      hi = lo;
    }
    return;
  }
  if (g.final_row && grp == 0) g.final_row[c] = prev[c];
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
  return chain_lds_bytes<NP, G, RREG, RLDS, RGLB, AFULL>();
}

template <int NP, int G, int RREG, int RLDS, int RGLB, bool AFULL, bool BATCH = false>
hipError_t chain_launch(const CpChainWgArgs& g, hipStream_t stream, int64_t nblocks = 1) {
  const size_t lds = chain_lds<NP, G, RREG, RLDS, RGLB, AFULL>();
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cp_chain_wg<NP, G, RREG, RLDS, RGLB, AFULL, BATCH>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((cp_chain_wg<NP, G, RREG, RLDS, RGLB, AFULL, BATCH>), dim3((unsigned)nblocks), dim3(NP * G), lds,
                     stream, g);
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

// ---- the parallel CPSolver chain (cv_decode_superseq_cp; DESIGN.md §3 "parallel chain") ----
// The chain's sequence k starts from the running maximum M of sequences 0..k-1 (utils.rs:24-38:
// at t == 0 the candidates are prev[i] + pi[j], so every start value is fl(M + fl(pi + b)) when
// the previous row's maximum is clean), and every later value carries M.  With all finite model
// entries in [-2^80, 0], every value the chain computes for sequence k that can still reach its
// optimum lies in [M + S_k - 1, M] (S_k = the sequence's own optimum), so each of its roundings
// is at most half of U = 2^-52 (|M| + |S_k| + 16): the chain's values stay within 1.5 (t + 1) U
// of the exact ones on the CP arcs w = fl(a + b) after t steps (one rounding for the value add,
// one for each candidate of the argmax), and its argmax at step t keeps the exact one whenever
// the exact gap exceeds (3t + 1) U.  The row-A0 decode at offset 0 (trellis_fwd_f64) gives
// those gaps up to its own error, (4t + 1) u0 with u0 = 2^-51 (|S_k| + 16).  cp_cert_f64 turns
// the path's gaps into ONE number per sequence,
//   rho = min( min_t (gap_t - (4t + 1) u0) / (3t + 1),  (gapF - 4T u0) / (3T + 2) )
// (gap_t = on-path candidate minus the best other candidate of step t, gapF = top-2 gap of the
// last row), so the host certifies sequence k at any offset M by rho > U: then the chain's path
// in sequence k IS the row-A0 path, its end state is the unique first argmax of its last row,
// and its maximum is the CP fold along that path from M (computed exactly on the host, or as
// M + the quantised sum of cp_quant_f64).  gF = gapF - 4T u0 bounds the exact final gap for
// the next sequence's boundary test.  rho = -1: some step is a tie (or the status is not OK) --
// the host runs the chain itself over that sequence.
template <int KP>
__global__ __launch_bounds__(256) void cp_cert_f64(CpCert64Args g) {
  constexpr int NP = 64 * KP;
  constexpr uint32_t NINF_HI = 0xFFF00000u;
  const int lane = threadIdx.x & 63;
  const int64_t slot = g.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= g.seq_end) return;
  const int64_t seq = g.order ? (int64_t)g.order[slot] : slot;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  if (T <= 0 || g.status[seq] != CVK_SEQ_OK) {
    if (lane == 0) g.out[2 * seq] = -1.0, g.out[2 * seq + 1] = -1.0;
    return;
  }
  const uint32_t* __restrict__ rows = reinterpret_cast<const uint32_t*>(g.delta) + (e0 - g.delta_elem_base) * (2 * NP);
  const int32_t* __restrict__ path = g.path + e0;
  bool valid[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) valid[k] = (lane + 64 * k) < g.nstates;
  auto load_row = [&](int r, uint32_t (&h)[KP], uint32_t (&l)[KP]) {
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      h[k] = valid[k] ? __builtin_nontemporal_load(rows + (size_t)r * (2 * NP) + lane + 64 * k) : NINF_HI;
      l[k] = valid[k] ? __builtin_nontemporal_load(rows + (size_t)r * (2 * NP) + NP + lane + 64 * k) : 0u;
    }
  };
  // top, first argmax and the best OTHER value of x (candidate i = lane + 64k)
  auto top2 = [&](const double (&x)[KP], int& arg, double& m1, double& m2) {
    double m = (-__builtin_inf());
#pragma unroll
    for (int k = 0; k < KP; ++k) m = fmax(m, x[k]);
    m1 = wave_max_d_dpp(m);
    arg = -1;
#pragma unroll
    for (int k = KP - 1; k >= 0; --k) {
      const unsigned long long mask = __ballot(valid[k] && x[k] == m1);
      if (mask) arg = 64 * k + __builtin_ctzll(mask);
    }
    double o = (-__builtin_inf());
#pragma unroll
    for (int k = 0; k < KP; ++k) o = fmax(o, (64 * k + lane == arg) ? (-__builtin_inf()) : x[k]);
    m2 = wave_max_d_dpp(o);
  };
  uint32_t ch[KP], cl[KP];
  load_row(T - 1, ch, cl);
  double x[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) x[k] = valid[k] ? from_words(ch[k], cl[k]) : (-__builtin_inf());
  int arg;
  double m1, m2;
  top2(x, arg, m1, m2);
  const double u0 = (__builtin_fabs(m1) + 16.0) * 0x1p-51;
  bool ok = m1 > (-__builtin_inf()) && arg == path[T - 1];
  const double gF = m1 - m2 - 4.0 * (double)T * u0;  // +inf when the row has one finite entry
  double rho = gF / (double)(3 * T + 2);
  if (ok && T > 1) load_row(T - 2, ch, cl);
  for (int t = T - 1; ok && t >= 1; --t) {
    uint32_t nh[KP], nl[KP];
    if (t >= 2) load_row(t - 2, nh, nl);  // the next step's row, a step ahead
    const int j = path[t], p = path[t - 1];
    const double* __restrict__ acol = g.at + (size_t)j * NP + lane;
#pragma unroll
    for (int k = 0; k < KP; ++k) x[k] = valid[k] ? from_words(ch[k], cl[k]) + acol[64 * k] : (-__builtin_inf());
    top2(x, arg, m1, m2);
    ok = arg == p && m1 > (-__builtin_inf());  // the path's predecessor is the strict first argmax
    rho = fmin(rho, (m1 - m2 - (double)(4 * t + 1) * u0) / (double)(3 * t + 1));
#pragma unroll
    for (int k = 0; k < KP; ++k) ch[k] = nh[k], cl[k] = nl[k];
  }
  if (lane == 0) {
    // the divisions and subtractions above round: a relative 2^-50 covers them
    const bool pass = ok && rho > 0.0;
    g.out[2 * seq] = pass ? rho * (1.0 - 0x1p-50) : -1.0;
    g.out[2 * seq + 1] = pass ? gF * (1.0 - 0x1p-50) : -1.0;
  }
}

// Quantised CP fold of a certified path at a predicted binade e (cp_cert_f64 above): while
// every value of the chain's sequence lies in [2^e, 2^(e+1)) in magnitude, each value is a
// multiple of g = 2^(e-52) and fl(d + w) = d + rint(w / g) g unless w / g has fractional part
// exactly 1/2 (a tie, where round-to-even depends on d).  So the fold from M is
// M + q g with q = sum_t rint(w_t / g) over the arcs w_0 = fl(pi + b), w_t = fl(a + b) of the
// path -- exact, one add per sequence on the host.  tie = 1: some w_t is a tie or out of range
// (the host folds that sequence element by element).
__global__ __launch_bounds__(256) void cp_quant_f64(CpQuant64Args g) {
  const int lane = threadIdx.x & 63;
  const int64_t seq = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (seq >= g.nseq) return;
  const int e = g.ebin[seq];
  if (e == CVK_NO_BINADE) return;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const double scale = __builtin_ldexp(1.0, 52 - e);
  const int NP = g.np;
  long long q = 0;
  bool tie = false;
  for (int t = lane; t < T; t += 64) {
    const int P = g.path[e0 + t];
    const double b = g.et[(size_t)g.obs[e0 + t] * NP + P];
    const double w = t == 0 ? g.pi[P] + b : g.a[(size_t)g.path[e0 + t - 1] * NP + P] + b;
    const double xs = w * scale;  // exact: a power-of-two scale of a normal f64
    if (!(__builtin_fabs(xs) < 0x1p61)) {
      tie = true;
      continue;
    }
    tie |= xs - __builtin_floor(xs) == 0.5;
    q += (long long)__builtin_rint(xs);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) q += __shfl_xor(q, off);
  const bool anytie = __ballot(tie) != 0;
  if (lane == 0) {
    g.q[seq] = q;
    g.tie[seq] = anytie ? 1 : 0;
  }
}

// N > 256 (the serial chain's runs, cp_superseq_chain): the two backtrack passes above with a
// runtime row width and psi read straight from global memory (no LDS staging: a row of u16 at
// N = 10,240 is 20 KiB).  pass 1: thread j walks segment k's state j down to e0.
__global__ __launch_bounds__(1024) void cp_chain_seg_map_g(CpChainBtArgs g) {
  const int64_t k = (int64_t)blockIdx.x + 1;
  const int64_t e0 = k * g.seg, e1 = e0 + g.seg < g.len ? e0 + g.seg : g.len;
  const int np = g.np;
  for (int j = threadIdx.x; j < np; j += blockDim.x) {
    int cs = j;
    for (int64_t t = e1 - 1; t >= e0; --t) cs = g.psi[t * np + cs];
    g.map[k * np + j] = (uint16_t)cs;
  }
}

// pass 2: one thread per segment follows psi from its resolved end state (cp.rs:88-92)
__global__ __launch_bounds__(64) void cp_chain_seg_path_g(CpChainBtArgs g) {
  const int64_t k = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (k >= g.nseg) return;
  const int64_t e0 = k * g.seg, e1 = e0 + g.seg < g.len ? e0 + g.seg : g.len;
  int cs = g.end_state[k];
  for (int64_t t = e1 - 1; t >= e0; --t) {
    g.path[t] = cs;
    cs = g.psi[t * g.np + cs];
  }
}

// cp_cert_f64 for N > 256: the same certificate (rho, gF) over the rows of any row-A0 decode --
// SPLIT: the f64 trellis's split-plane rows (NP = 512 / 1,024, width W = NP, a^T [NP][NP]);
// otherwise the generic kernels' plain f64 rows (width W = N, a^T [N][N]).  Each lane keeps the
// top two of its candidates i = lane + 64 k (first index on ties: a later equal candidate
// becomes the runner-up, gap 0); the wave's maximum, its lane and the best OTHER value follow
// (a tie across lanes leaves the runner-up equal to the maximum: gap 0, no certificate -- the
// only case where the arg below is not the first index, and then the result fails anyway).
template <bool SPLIT>
__global__ __launch_bounds__(256) void cp_cert_rows(CpCert64Args g, int W) {
  const int lane = threadIdx.x & 63;
  const int64_t slot = g.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= g.seq_end) return;
  const int64_t seq = g.order ? (int64_t)g.order[slot] : slot;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  if (T <= 0 || g.status[seq] != CVK_SEQ_OK) {
    if (lane == 0) g.out[2 * seq] = -1.0, g.out[2 * seq + 1] = -1.0;
    return;
  }
  const int N = g.nstates;
  const int64_t r0 = e0 - g.delta_elem_base;
  auto rowval = [&](int r, int i) -> double {
    if constexpr (SPLIT) {
      const uint32_t* row = reinterpret_cast<const uint32_t*>(g.delta) + (r0 + r) * (int64_t)(2 * W);
      return from_words(__builtin_nontemporal_load(row + i), __builtin_nontemporal_load(row + W + i));
    } else {
      return __builtin_nontemporal_load(g.delta + (r0 + r) * (int64_t)W + i);
    }
  };
  auto finish = [&](double m1l, int a1l, double m2l, int& arg, double& m1, double& m2) {
    m1 = wave_max_d_dpp(m1l);
    const unsigned long long mask = __ballot(a1l >= 0 && m1l == m1);
    const int wl = mask ? __builtin_ctzll(mask) : 0;
    arg = mask ? __shfl(a1l, wl) : -1;
    m2 = wave_max_d_dpp((mask && lane == wl) ? m2l : m1l);
  };
  int arg;
  double m1, m2;
  {
    double a = -__builtin_inf(), b = -__builtin_inf();
    int ia = -1;
#pragma unroll 4
    for (int i = lane; i < N; i += 64) {
      const double x = rowval(T - 1, i);
      if (x > a) {
        b = a;
        a = x;
        ia = i;
      } else {
        b = fmax(b, x);
      }
    }
    finish(a, ia, b, arg, m1, m2);
  }
  const int32_t* __restrict__ path = g.path + e0;
  const double u0 = (__builtin_fabs(m1) + 16.0) * 0x1p-51;
  bool ok = m1 > (-__builtin_inf()) && arg == path[T - 1];
  const double gF = m1 - m2 - 4.0 * (double)T * u0;  // +inf when the row has one finite entry
  double rho = gF / (double)(3 * T + 2);
  for (int t = T - 1; ok && t >= 1; --t) {
    const int j = path[t], p = path[t - 1];
    const double* __restrict__ acol = g.at + (size_t)j * W;
    double a = -__builtin_inf(), b = -__builtin_inf();
    int ia = -1;
#pragma unroll 4
    for (int i = lane; i < N; i += 64) {
      const double x = rowval(t - 1, i) + acol[i];
      if (x > a) {
        b = a;
        a = x;
        ia = i;
      } else {
        b = fmax(b, x);
      }
    }
    finish(a, ia, b, arg, m1, m2);
    ok = arg == p && m1 > (-__builtin_inf());  // the path's predecessor is the strict first argmax
    rho = fmin(rho, (m1 - m2 - (double)(4 * t + 1) * u0) / (double)(3 * t + 1));
  }
  if (lane == 0) {
    const bool pass = ok && rho > 0.0;
    g.out[2 * seq] = pass ? rho * (1.0 - 0x1p-50) : -1.0;
    g.out[2 * seq + 1] = pass ? gF * (1.0 - 0x1p-50) : -1.0;
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

hipError_t launch_cp_chain_wg_batch(int np, const CpChainWgArgs& g, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  if (!g.soff || !g.sinit || !g.path || !g.final_row || nseq > 0x7fffffff) return hipErrorInvalidValue;
  switch (np) {
    case 64: return chain_launch<64, 4, 16, 0, 0, true, true>(g, stream, nseq);
    case 128: return chain_launch<128, 4, 32, 0, 0, true, true>(g, stream, nseq);
    case 192: return chain_launch<192, 4, 32, 16, 0, false, true>(g, stream, nseq);
    case 256: return chain_launch<256, 4, 47, 17, 0, false, true>(g, stream, nseq);
    default: return hipErrorInvalidValue;
  }
}

// A loads in flight per thread (16: 78 VGPRs, measured no faster beside the forward)
#ifndef CVK_SPEC_UNROLL
#define CVK_SPEC_UNROLL 8
#endif
template <int NP>
__global__ __launch_bounds__(NP) void cp_spec_psi(CpSpecArgs g) {
  constexpr int kRows = 32;  // psi rows per LDS staging block of the path walk
  __shared__ __attribute__((aligned(16))) double dl[2][NP];
  __shared__ __attribute__((aligned(16))) uint16_t ps[kRows * NP];
  const int j = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t e0 = g.soff[b], T = g.soff[b + 1] - e0;
  if (T <= 0) return;  // uniform over the workgroup
  if (g.prio == 1) __builtin_amdgcn_s_setprio(1);
  if (g.prio == 2) __builtin_amdgcn_s_setprio(2);
  if (g.prio >= 3) __builtin_amdgcn_s_setprio(3);
  const int32_t* obs = g.obs + e0;
  uint16_t* psi = g.psi + e0 * NP;
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g.a), 0, NP * NP * 8, 0x00020000);
  auto aload = [&](int i) {  // a[i][j]: the row offset in a scalar register, no per-lane address math
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(ra, (uint32_t)j * 8u, (uint32_t)i * NP * 8u, 0));
  };
  dl[0][j] = g.sinit[b] + (g.pi[j] + g.et[(size_t)obs[0] * NP + j]);  // utils.rs:32-35 after a clean boundary
  __syncthreads();
  for (int64_t t = 1; t < T; ++t) {
    const double* dp = dl[(t - 1) & 1];
    const double e = g.et[(size_t)obs[t] * NP + j];
    double best = dp[0] + aload(0);
    int arg = 0;
#pragma unroll CVK_SPEC_UNROLL
    for (int i = 1; i < NP; ++i) {
      const double x = dp[i] + aload(i);
      arg = x > best ? i : arg;  // strict: the first argmax (cp.rs:70-79)
      best = __builtin_fmax(best, x);
    }
    const double v = dp[arg] + (aload(arg) + e);  // cp.rs:75-77
    psi[t * NP + j] = (uint16_t)arg;
    dl[t & 1][j] = v;
    __syncthreads();
  }
  const double* lr = dl[(T - 1) & 1];
  if (j < g.nstates) g.last[b * g.nstates + j] = lr[j];
  int32_t* path = g.path + e0;
  int cs = 0;
  if (j == 0) {  // cp.rs:86
    double m = lr[0];
    for (int i = 1; i < g.nstates; ++i)
      if (lr[i] > m) {
        m = lr[i];
        cs = i;
      }
    path[T - 1] = cs;
  }
  __threadfence();  // this workgroup's psi stores, read back below
  __syncthreads();
  for (int64_t hi = T; hi > 1;) {  // rows [lo, hi) hold psi for elements lo .. hi - 1
    const int64_t lo = hi - 1 > kRows ? hi - kRows : 1;
    const uint4* src = reinterpret_cast<const uint4*>(psi + lo * NP);
    uint4* dst = reinterpret_cast<uint4*>(ps);
    for (int64_t q = j; q < (hi - lo) * NP / 8; q += NP) dst[q] = src[q];
    __syncthreads();
    if (j == 0)
      for (int64_t t = hi - 1; t >= lo; --t) {
        cs = ps[(t - lo) * NP + cs];
        path[t - 1] = cs;
      }
    __syncthreads();
    hi = lo;
  }
}

hipError_t launch_cp_spec_psi(int np, const CpSpecArgs& g, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  if (nseq > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nseq);
  switch (np) {
    case 64: hipLaunchKernelGGL(cp_spec_psi<64>, grid, dim3(64), 0, stream, g); break;
    case 128: hipLaunchKernelGGL(cp_spec_psi<128>, grid, dim3(128), 0, stream, g); break;
    case 192: hipLaunchKernelGGL(cp_spec_psi<192>, grid, dim3(192), 0, stream, g); break;
    case 256: hipLaunchKernelGGL(cp_spec_psi<256>, grid, dim3(256), 0, stream, g); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_cp_chain_seg_map(const CpChainBtArgs& g, hipStream_t stream) {
  if (g.nseg <= 1) return hipSuccess;
  const dim3 grid((unsigned)(g.nseg - 1));
  switch (g.np) {
    case 64: hipLaunchKernelGGL(cp_chain_seg_map<64>, grid, dim3(64), 0, stream, g); break;
    case 128: hipLaunchKernelGGL(cp_chain_seg_map<128>, grid, dim3(128), 0, stream, g); break;
    case 192: hipLaunchKernelGGL(cp_chain_seg_map<192>, grid, dim3(192), 0, stream, g); break;
    case 256: hipLaunchKernelGGL(cp_chain_seg_map<256>, grid, dim3(256), 0, stream, g); break;
    default:
      if (g.np <= 0 || g.np > kChainMaxStates) return hipErrorInvalidValue;
      hipLaunchKernelGGL(cp_chain_seg_map_g, grid, dim3((unsigned)std::min(1024, (g.np + 63) / 64 * 64)), 0, stream, g);
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
    default:
      if (g.np <= 0 || g.np > kChainMaxStates) return hipErrorInvalidValue;
      hipLaunchKernelGGL(cp_chain_seg_path_g, dim3((unsigned)((g.nseg + 63) / 64)), dim3(64), 0, stream, g);
  }
  return hipGetLastError();
}

hipError_t launch_cp_cert(int np, const CpCert64Args& a, hipStream_t stream) {
  const int64_t n = a.seq_end - a.seq_begin;
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 3) / 4)), block(256);
  switch (np) {
    case 64: hipLaunchKernelGGL(cp_cert_f64<1>, grid, block, 0, stream, a); break;
    case 128: hipLaunchKernelGGL(cp_cert_f64<2>, grid, block, 0, stream, a); break;
    case 192: hipLaunchKernelGGL(cp_cert_f64<3>, grid, block, 0, stream, a); break;
    case 256: hipLaunchKernelGGL(cp_cert_f64<4>, grid, block, 0, stream, a); break;
    case 512:
    case 1024: hipLaunchKernelGGL(cp_cert_rows<true>, grid, block, 0, stream, a, np); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_cp_cert_plain(const CpCert64Args& a, hipStream_t stream) {
  const int64_t n = a.seq_end - a.seq_begin;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(cp_cert_rows<false>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, a, a.nstates);
  return hipGetLastError();
}

// the parallel chain's host walk without the whole path on the host: every sequence's end
// state (its last element; -1 for an empty sequence) ...
__global__ void cp_seq_ends(const int32_t* __restrict__ path, const int64_t* __restrict__ offsets, int64_t nseq,
                            int32_t* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nseq) return;
  const int64_t e1 = offsets[k + 1];
  out[k] = e1 > offsets[k] ? path[e1 - 1] : -1;
}

// ... and the paths of the sequences it may fold element by element, packed: sequence ids[i]'s
// path to out[dst[i] ..] (one workgroup per sequence, coalesced)
__global__ __launch_bounds__(256) void cp_gather_paths(const int32_t* __restrict__ path,
                                                       const int64_t* __restrict__ offsets,
                                                       const int64_t* __restrict__ ids, const int64_t* __restrict__ dst,
                                                       int32_t* __restrict__ out) {
  const int64_t k = ids[blockIdx.x];
  const int64_t e0 = offsets[k], T = offsets[k + 1] - e0, d = dst[blockIdx.x];
  for (int64_t t = threadIdx.x; t < T; t += 256) out[d + t] = path[e0 + t];
}

hipError_t launch_cp_seq_ends(const int32_t* path, const int64_t* offsets, int64_t nseq, int32_t* out,
                              hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(cp_seq_ends, dim3((unsigned)((nseq + 255) / 256)), dim3(256), 0, stream, path, offsets, nseq, out);
  return hipGetLastError();
}

hipError_t launch_cp_gather_paths(const int32_t* path, const int64_t* offsets, const int64_t* ids, const int64_t* dst,
                                  int64_t n, int32_t* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (n > (int64_t)INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cp_gather_paths, dim3((unsigned)n), dim3(256), 0, stream, path, offsets, ids, dst, out);
  return hipGetLastError();
}

hipError_t launch_cp_quant(const CpQuant64Args& a, hipStream_t stream) {
  if (a.nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(cp_quant_f64, dim3((unsigned)((a.nseq + 3) / 4)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace cvk
