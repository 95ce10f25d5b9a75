// trellis64.hip -- exact-f64 Viterbi trellis for N <= 256 (gfx950).
//
// The reference solvers compute in f64 (hmm.rs:10-18 stores Array2<f64>; viterbi.rs:13-18,
// cp.rs:70-79).  This is the row-A0 recurrence of SURVEY.md §8a in f64:
//   d0[j] = pi[j] + b[j,o0]                 (hmm.rs:215-218, cp.rs:66-68)
//   m     = max_i (d[i] + a[i,j])            (viterbi.rs:15-16)
//   d'[j] = m + b[j,o]                       (viterbi.rs:17)
// with the first-index argmax (ndarray-stats 0.5 argmax) recovered in the backtrack by the
// same f64 adds, so paths and scores are bit-identical to the f64 oracle.
//
// trellis_fwd_f64<C, S>: ONE WAVE decodes S sequences in lock step.  Lane l owns the C
// consecutive columns [C*l, C*l + C) of NP = 64*C padded states for all S sequences
// (acc = C*S f64 accumulators).  A (NP*NP f64 = 512 KiB at N = 256) fits neither the
// register file nor LDS, so each A row is streamed from L2 (2 KiB per row, coalesced, a
// PF-deep register ring) and reused by the S sequences: 8/S bytes of L2 traffic per
// (from,to) pair.  delta_{t-1} of the S sequences lives in the wave's own LDS slice as
// [row][S] and is broadcast with ds_read_b128 (2 sequences per read, same address in every
// lane).  Per pair: one v_add_f64 + one v_max_f64, both full rate on gfx950
// (profiles/r01_f64_rates.txt: ~59 lane-ops/clk/CU at 4 waves/SIMD, ~53 at 2).  No barrier:
// the wave is its own workgroup.  No argmax in the forward pass: each f64 delta row goes
// to HBM (8*NP B per sequence step) for the backtrack.
//
// backtrack_f64<KP>: one wave per sequence, candidates i = lane + 64k; recomputes
// s_i = d_{t-1}[i] + a[i, path[t]] in f64 and takes the first argmax (cp.rs:85-93).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "trellis.h"
#include "trellis64.h"

namespace cvk {

namespace {

__device__ __forceinline__ double ninf_d() { return -__builtin_inf(); }

// C consecutive f64 of one A row (16-byte aligned for even C: dwordx4 loads)
template <int C>
__device__ __forceinline__ void load_a(const double* p, double (&a)[C]) {
  if constexpr (C % 2 == 0) {
    const double2* q = reinterpret_cast<const double2*>(p);
#pragma unroll
    for (int c = 0; c < C / 2; ++c) {
      const double2 v = q[c];
      a[2 * c] = v.x;
      a[2 * c + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) a[c] = p[c];
  }
}

// DPA: DPSolver's association (dp.rs:147-177): d'[j] = max_i ((a[i,j] + b[j,o]) + d[i]); the
// emission enters every candidate, so it is loaded before the row loop (S <= 4: registers)
template <int C, int S, int PF, bool DPA = false>  // PF: A rows in flight
__global__ __launch_bounds__(64) void trellis_fwd_f64(T64FwdArgs g) {
  constexpr int NP = 64 * C;
  static_assert(S % 2 == 0, "S sequences are read from LDS two at a time");
  static_assert(PF % 2 == 0, "the delta register double buffer alternates with the row parity");
  __shared__ __attribute__((aligned(16))) double dl[NP * S];  // delta_{t-1}: [row][S]
  const int lane = threadIdx.x;
  const int j0 = lane * C;
  const int64_t slot0 = g.seq_begin + (int64_t)blockIdx.x * S;
  const int64_t slot_end = g.seq_begin + g.nslots;
  const double ninf = ninf_d();

  int64_t seq[S], e0[S];
  int T[S];
  int Tmax = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t slot = slot0 + s;
    if (slot < slot_end) {
      seq[s] = g.order ? (int64_t)g.order[slot] : slot;
      e0[s] = g.offsets[seq[s]];
      T[s] = (int)(g.offsets[seq[s] + 1] - e0[s]);
    } else {
      seq[s] = -1;
      e0[s] = 0;
      T[s] = 0;
    }
    Tmax = T[s] > Tmax ? T[s] : Tmax;
  }
  if (Tmax <= 0) return;
  const unsigned V = (unsigned)g.nobs;
  unsigned bad = 0;  // bit s: sequence s saw an out-of-range observation

  // emission columns [j0, j0+C) of observation o (or -inf when o is out of range)
  auto emis = [&](int s, int t, double (&e)[C]) {
    int o = 0;
    if (t < T[s]) o = g.obs[e0[s] + t];
    const bool ok = (unsigned)o < V;
    if (t < T[s] && !ok) bad |= 1u << s;
    const double* row = g.et + (size_t)(ok ? o : 0) * NP + j0;
#pragma unroll
    for (int c = 0; c < C; ++c) e[c] = ok ? row[c] : ninf;
  };
  auto store_row = [&](int s, int t, const double (&v)[C]) {
    if (t < T[s]) {
      double* dst = g.delta + (e0[s] + t - g.delta_elem_base) * NP + j0;
#pragma unroll
      for (int c = 0; c < C; ++c) dst[c] = v[c];
    }
  };

  // t = 0: d0 = pi + b[:, o0]
#pragma unroll
  for (int s = 0; s < S; ++s) {
    double e[C], v[C];
    emis(s, 0, e);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      v[c] = g.zero_init ? 0.0 : g.pi[j0 + c] + e[c];
      dl[(j0 + c) * S + s] = v[c];
    }
    store_row(s, 0, v);
  }
  __syncthreads();

  // forward waves win issue arbitration over co-resident backtrack waves of the previous
  // chunk (overlap mode), as in trellis_fwd2_f32
  __builtin_amdgcn_s_setprio(3);
  const double* __restrict__ arow = g.a + j0;
  double acc[C][S];  // after a step: delta_t of the S sequences (stored at the next step)
  for (int t = 1; t < Tmax; ++t) {
    double ar[PF][C];
#pragma unroll
    for (int u = 0; u < PF; ++u) load_a(arow + (size_t)u * NP, ar[u]);
    // delta_{t-1} rows go to HBM only now: the ring loads above were issued first, so waiting
    // for them (in-order vmcnt) does not wait for these stores
    if (t > 1) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        double v[C];
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = acc[c][s];
        store_row(s, t - 1, v);
      }
    }
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int s = 0; s < S; ++s) acc[c][s] = ninf;
    double ecur[DPA ? S : 1][C];
    if constexpr (DPA) {
#pragma unroll
      for (int s = 0; s < S; ++s) emis(s, t, ecur[s]);
    }
    // delta rows double-buffered in registers (dv[u & 1] = row i): row i+1's broadcast reads
    // are in flight while row i computes
    double2 dv[2][S / 2];
#pragma unroll
    for (int s2 = 0; s2 < S / 2; ++s2) dv[0][s2] = reinterpret_cast<const double2*>(dl)[s2];
#pragma nounroll
    for (int i0 = 0; i0 < NP; i0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = i0 + u;
        {
          const double2* nrow = reinterpret_cast<const double2*>(dl + min(i + 1, NP - 1) * S);
#pragma unroll
          for (int s2 = 0; s2 < S / 2; ++s2) dv[(u + 1) & 1][s2] = nrow[s2];
        }
#pragma unroll
        for (int s2 = 0; s2 < S / 2; ++s2) {
          const double2 d = dv[u & 1][s2];
#pragma unroll
          for (int c = 0; c < C; ++c) {
            if constexpr (DPA) {
              acc[c][2 * s2] = fmax(acc[c][2 * s2], (ar[u][c] + ecur[2 * s2][c]) + d.x);
              acc[c][2 * s2 + 1] = fmax(acc[c][2 * s2 + 1], (ar[u][c] + ecur[2 * s2 + 1][c]) + d.y);
            } else {
              acc[c][2 * s2] = fmax(acc[c][2 * s2], d.x + ar[u][c]);
              acc[c][2 * s2 + 1] = fmax(acc[c][2 * s2 + 1], d.y + ar[u][c]);
            }
          }
        }
        // refill this ring slot with row i + PF (clamped: the last rows reload row NP-1) only
        // after its last use, into the same registers: no copies, and the in-flight loads
        // cross the loop back-edge without a vmcnt(0) drain
        const int nr = min(i + PF, NP - 1);
        load_a(arow + (size_t)nr * NP, ar[u]);
      }
    }
    __syncthreads();  // every lane has read delta_{t-1} before it is overwritten
#pragma unroll
    for (int s = 0; s < S; ++s) {
      double e[C], v[C];
      if constexpr (!DPA) emis(s, t, e);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        v[c] = DPA ? acc[c][s] : acc[c][s] + e[c];
        acc[c][s] = v[c];
        dl[(j0 + c) * S + s] = v[c];
      }
    }
    __syncthreads();
  }
  if (Tmax > 1) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      double v[C];
#pragma unroll
      for (int c = 0; c < C; ++c) v[c] = acc[c][s];
      store_row(s, Tmax - 1, v);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (bad & (1u << s)) g.status[seq[s]] = CVK_SEQ_BADOBS;
  }
}

// CP association (CPSolver, cp.rs:70-79 via utils.rs:24-38, hmm.rs:220-222):
//   psi = first argmax_i (d[i] + a[i,j]);  d'[j] = d[psi] + (a[psi,j] + b[j,o])
// The value depends on psi, so the forward pass tracks the first argmax: per pair one add,
// one compare, one max and one index select (4 VALU vs 2 for row A0), then per column one
// LDS gather of d[psi] and one L2 gather of a[psi,j].  psi (u16) and the last row go out in
// generic_fwd's layout; generic_backtrack<double> follows them (cp.rs:85-93).  Same wave
// layout as trellis_fwd_f64 (S sequences per wave, A rows streamed through a register ring).
template <int C, int S, int PF>
__global__ __launch_bounds__(64) void trellis_cp_f64(T64FwdArgs g) {
  constexpr int NP = 64 * C;
  static_assert(S % 2 == 0 && PF % 2 == 0, "pairs of sequences / rows");
  __shared__ __attribute__((aligned(16))) double dl[NP * S];  // delta_{t-1}: [row][S]
  const int lane = threadIdx.x;
  const int j0 = lane * C;
  const int N = g.nstates;
  const int64_t slot0 = g.seq_begin + (int64_t)blockIdx.x * S;
  const int64_t slot_end = g.seq_begin + g.nslots;
  const double ninf = ninf_d();

  int64_t seq[S], e0[S];
  int T[S];
  int Tmax = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t slot = slot0 + s;
    if (slot < slot_end) {
      seq[s] = g.order ? (int64_t)g.order[slot] : slot;
      e0[s] = g.offsets[seq[s]];
      T[s] = (int)(g.offsets[seq[s] + 1] - e0[s]);
    } else {
      seq[s] = -1;
      e0[s] = 0;
      T[s] = 0;
    }
    Tmax = T[s] > Tmax ? T[s] : Tmax;
  }
  if (Tmax <= 0) return;
  const unsigned V = (unsigned)g.nobs;
  unsigned bad = 0;
  auto emis = [&](int s, int t, double (&e)[C]) {
    int o = 0;
    if (t < T[s]) o = g.obs[e0[s] + t];
    const bool ok = (unsigned)o < V;
    if (t < T[s] && !ok) bad |= 1u << s;
    const double* row = g.et + (size_t)(ok ? o : 0) * NP + j0;
#pragma unroll
    for (int c = 0; c < C; ++c) e[c] = ok ? row[c] : ninf;
  };
  // row t of sequence s: psi (t >= 1) and, at t = T-1, the last row
  auto emit = [&](int s, int t, const double (&v)[C], const int (&p)[C]) {
    if (t >= T[s]) return;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (j0 + c < N) {
        if (t > 0) g.psi[(e0[s] + t - g.delta_elem_base) * (int64_t)N + j0 + c] = (uint16_t)p[c];
        if (t == T[s] - 1) g.last_row[(slot0 + s - g.seq_begin) * (int64_t)N + j0 + c] = v[c];
      }
    }
  };

#pragma unroll
  for (int s = 0; s < S; ++s) {  // t = 0: pi + b (cp.rs:66-68)
    double e[C], v[C];
    int p[C] = {};
    emis(s, 0, e);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      v[c] = g.pi[j0 + c] + e[c];
      dl[(j0 + c) * S + s] = v[c];
    }
    emit(s, 0, v, p);
  }
  __syncthreads();

  __builtin_amdgcn_s_setprio(3);
  const double* __restrict__ arow = g.a + j0;
  for (int t = 1; t < Tmax; ++t) {
    double acc[C][S];
    int idx[C][S];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        acc[c][s] = ninf;
        idx[c][s] = 0;
      }
    double ar[PF][C];
#pragma unroll
    for (int u = 0; u < PF; ++u) load_a(arow + (size_t)u * NP, ar[u]);
    double2 dv[2][S / 2];
#pragma unroll
    for (int s2 = 0; s2 < S / 2; ++s2) dv[0][s2] = reinterpret_cast<const double2*>(dl)[s2];
#pragma nounroll
    for (int i0 = 0; i0 < NP; i0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = i0 + u;
        {
          const double2* nrow = reinterpret_cast<const double2*>(dl + min(i + 1, NP - 1) * S);
#pragma unroll
          for (int s2 = 0; s2 < S / 2; ++s2) dv[(u + 1) & 1][s2] = nrow[s2];
        }
#pragma unroll
        for (int s2 = 0; s2 < S / 2; ++s2) {
          const double2 d = dv[u & 1][s2];
#pragma unroll
          for (int c = 0; c < C; ++c) {
            // strict '>' from acc = -inf, idx = 0: the first maximal index, and 0 when every
            // candidate is -inf (generic_fwd's "!any || s > best")
            const double x0 = d.x + ar[u][c], x1 = d.y + ar[u][c];
            idx[c][2 * s2] = x0 > acc[c][2 * s2] ? i : idx[c][2 * s2];
            acc[c][2 * s2] = fmax(acc[c][2 * s2], x0);
            idx[c][2 * s2 + 1] = x1 > acc[c][2 * s2 + 1] ? i : idx[c][2 * s2 + 1];
            acc[c][2 * s2 + 1] = fmax(acc[c][2 * s2 + 1], x1);
          }
        }
        const int nr = min(i + PF, NP - 1);
        load_a(arow + (size_t)nr * NP, ar[u]);
      }
    }
    // CP value d[psi] + (a[psi,j] + b[j,o]): gathers of d (this wave's LDS) and a (L2)
    double v[S][C];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      double e[C];
      emis(s, t, e);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const int p = idx[c][s];
        v[s][c] = dl[p * S + s] + (g.a[(size_t)p * NP + j0 + c] + e[c]);
      }
    }
    __syncthreads();  // every lane has read delta_{t-1} before it is overwritten
#pragma unroll
    for (int s = 0; s < S; ++s) {
      int p[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        dl[(j0 + c) * S + s] = v[s][c];
        p[c] = idx[c][s];
      }
      emit(s, t, v[s], p);
    }
    __syncthreads();
  }
  if (lane == 0) {
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (bad & (1u << s)) g.status[seq[s]] = CVK_SEQ_BADOBS;
  }
}

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}

// PF: delta rows in flight per wave.  The backtrack streams 2 KiB f64 rows from HBM, and at
// NP >= 192 occupancy hides the latency better than a deeper ring: config 4 (NP = 256, serial
// schedule) 14.3 ms at PF = 2 (8 waves/SIMD) vs 15.3 (PF = 4, 74 VGPRs, 6 waves/SIMD),
// 16.9 (PF = 8) and 21.9 (PF = 16) -- profiles/r01_t64_bt_pf.txt.
template <int KP, int PF>
__global__ __launch_bounds__(256) void backtrack_f64(T64BtArgs g) {
  constexpr int NP = 64 * KP;
  const int lane = threadIdx.x & 63;
  const int64_t slot = g.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= g.seq_end) return;
  const int64_t seq = g.order ? (int64_t)g.order[slot] : slot;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const int N = g.nstates;
  if (T <= 0) {
    if (lane == 0) {
      g.score[seq] = 0.0;
      g.status[seq] = CVK_SEQ_EMPTY;
    }
    return;
  }
  int32_t* __restrict__ path = g.path + e0;
  const double* __restrict__ drow = g.delta + (e0 - g.delta_elem_base) * NP;
  bool valid[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) valid[k] = (lane + 64 * k) < N;
  auto load_row = [&](int r, double (&dst)[KP]) {
#pragma unroll
    for (int k = 0; k < KP; ++k) dst[k] = (r >= 0 && valid[k]) ? drow[(size_t)r * NP + lane + 64 * k] : ninf_d();
  };
  auto first_argmax = [&](const double (&s)[KP], double& M) {
    double m = s[0];
#pragma unroll
    for (int k = 1; k < KP; ++k) m = fmax(m, s[k]);
    M = wave_max_d(m);
    int idx = 0;
#pragma unroll
    for (int k = KP - 1; k >= 0; --k) {
      const unsigned long long mask = __ballot(valid[k] && s[k] == M);
      if (mask) idx = 64 * k + __builtin_ctzll(mask);
    }
    return idx;
  };
  double bv;
  int cur;
  {
    double last[KP];
    load_row(T - 1, last);
    cur = first_argmax(last, bv);  // cp.rs:86
  }
  const uint8_t prior = g.status[seq];
  if (!(bv > ninf_d()) || prior == CVK_SEQ_BADOBS) {
    for (int t = lane; t < T; t += 64) path[t] = 0;
    if (lane == 0) {
      g.score[seq] = ninf_d();
      g.status[seq] = prior == CVK_SEQ_BADOBS ? CVK_SEQ_BADOBS : CVK_SEQ_INFEASIBLE;
    }
    return;
  }
  int pathreg = 0;
  if (lane == ((T - 1) & 63)) pathreg = cur;
  if (((T - 1) & 63) == 0 && lane == 0) path[T - 1] = cur;
  double ring[PF][KP];
#pragma unroll
  for (int u = 0; u < PF; ++u) load_row(T - 2 - u, ring[u]);
  for (int base = T - 1; base >= 1; base -= PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int t = base - u;
      if (t >= 1) {
        const double* acol = g.at + (size_t)cur * NP + lane;
        double s[KP];
        if (g.dp_assoc) {  // (a[i,cur] + b[cur,o_t]) + d_{t-1}[i]  (dp.rs:149 arc_p, then + cost)
          const double e = g.et[(size_t)g.obs[e0 + t] * NP + cur];
#pragma unroll
          for (int k = 0; k < KP; ++k) s[k] = valid[k] ? (acol[64 * k] + e) + ring[u][k] : ninf_d();
        } else {
#pragma unroll
          for (int k = 0; k < KP; ++k) s[k] = valid[k] ? ring[u][k] + acol[64 * k] : ninf_d();
        }
        double M;
        cur = first_argmax(s, M);
        const int tp = t - 1;
        if (lane == (tp & 63)) pathreg = cur;
        if ((tp & 63) == 0 && tp + lane < T) path[tp + lane] = pathreg;
      }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) load_row(base - PF - 1 - u, ring[u]);
  }
  if (lane == 0) {
    g.score[seq] = bv;
    g.status[seq] = CVK_SEQ_OK;
  }
}

template <int C, int S>
hipError_t fwd_cs(const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  const int64_t blocks = (nseq + S - 1) / S;
  static const int pf = [] {  // tuning knob (bit-identical): A rows in flight, 8 (default) or 4
    const char* e = getenv("CV_T64_PF");
    return e ? atoi(e) : 8;
  }();
  // PF = 8 measured 183 vs 208 ms (PF = 4) per config-4 forward; S = 6 / PF = 6 lost too
  // (176 / 170 vs 164 ms, profiles/r01_t64_sweep.txt)
  if (fa.dp_assoc) {
    if constexpr (S <= 4)
      hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8, true>), dim3((unsigned)blocks), dim3(64), 0, stream, fa);
    else
      return hipErrorInvalidValue;
  } else if (pf == 4)
    hipLaunchKernelGGL((trellis_fwd_f64<C, S, 4>), dim3((unsigned)blocks), dim3(64), 0, stream, fa);
  else
    hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8>), dim3((unsigned)blocks), dim3(64), 0, stream, fa);
  return hipGetLastError();
}

template <int C>
hipError_t fwd_c(const T64FwdArgs& fa, int s, int64_t nseq, hipStream_t stream) {
  switch (s) {
    case 2: return fwd_cs<C, 2>(fa, nseq, stream);
    case 4: return fwd_cs<C, 4>(fa, nseq, stream);
    case 8: return fwd_cs<C, 8>(fa, nseq, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

template <int C>
hipError_t cp_c(const T64FwdArgs& fa, int s, int64_t nseq, hipStream_t stream) {
  const dim3 block(64);
  switch (s) {
    case 2: hipLaunchKernelGGL((trellis_cp_f64<C, 2, 4>), dim3((unsigned)((nseq + 1) / 2)), block, 0, stream, fa); break;
    case 4: hipLaunchKernelGGL((trellis_cp_f64<C, 4, 4>), dim3((unsigned)((nseq + 3) / 4)), block, 0, stream, fa); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_t64_cp_fwd(int np, int s, const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  s = s > 4 ? 4 : s;  // the argmax state (idx) costs registers: at most 4 sequences per wave
  switch (np) {
    case 64: return cp_c<1>(fa, s, nseq, stream);
    case 128: return cp_c<2>(fa, s, nseq, stream);
    case 192: return cp_c<3>(fa, s, nseq, stream);
    case 256: return cp_c<4>(fa, s, nseq, stream);
    default: return hipErrorInvalidValue;
  }
}

int t64_padded_states(int n) { return (n >= 1 && n <= 256) ? 64 * ((n + 63) / 64) : 0; }

int t64_seqs_per_wave(int64_t nseq, int cus) {
  // fill at least two waves per SIMD (4 SIMDs per CU), then prefer the larger S: each A row
  // streamed from L2 serves S sequences
  if (const char* e = getenv("CV_T64_S")) {  // tuning knob (bit-identical for every value)
    const int s = atoi(e);
    if (s == 2 || s == 4 || s == 8) return s;
  }
  const int64_t simd_waves = 2 * 4 * (int64_t)(cus > 0 ? cus : 256);
  if (nseq >= 8 * simd_waves) return 8;
  if (nseq >= 4 * simd_waves) return 4;
  return 2;
}

hipError_t launch_t64_fwd(int np, int s, const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  if (fa.dp_assoc && s > 4) s = 4;  // the emissions of every sequence stay in registers
  switch (np) {
    case 64: return fwd_c<1>(fa, s, nseq, stream);
    case 128: return fwd_c<2>(fa, s, nseq, stream);
    case 192: return fwd_c<3>(fa, s, nseq, stream);
    case 256: return fwd_c<4>(fa, s, nseq, stream);
    default: return hipErrorInvalidValue;
  }
}

template <int PF>
hipError_t bt_pf(int np, const T64BtArgs& ba, dim3 grid, dim3 block, hipStream_t stream) {
  switch (np) {
    case 64: hipLaunchKernelGGL((backtrack_f64<1, PF>), grid, block, 0, stream, ba); break;
    case 128: hipLaunchKernelGGL((backtrack_f64<2, PF>), grid, block, 0, stream, ba); break;
    case 192: hipLaunchKernelGGL((backtrack_f64<3, PF>), grid, block, 0, stream, ba); break;
    case 256: hipLaunchKernelGGL((backtrack_f64<4, PF>), grid, block, 0, stream, ba); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_t64_bt(int np, const T64BtArgs& ba, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  const dim3 grid((unsigned)((nseq + 3) / 4)), block(256);
  static const int pf_env = [] {  // tuning knob (bit-identical): 2, 4, 8 or 16 rows in flight
    const char* e = getenv("CV_T64_BT_PF");
    return e ? atoi(e) : 0;
  }();
  const int pf = pf_env ? pf_env : np >= 192 ? 2 : 8;
  switch (pf) {
    case 2: return bt_pf<2>(np, ba, grid, block, stream);
    case 4: return bt_pf<4>(np, ba, grid, block, stream);
    case 16: return bt_pf<16>(np, ba, grid, block, stream);
    default: return bt_pf<8>(np, ba, grid, block, stream);
  }
}

}  // namespace cvk
