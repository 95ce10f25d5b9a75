// trellis.hip -- MI355X (gfx950) Viterbi trellis kernels.
//
// Hot path of the reference's viterbi_solver forward pass:
//   d0[j] = pi[j] + b[j,o0]                            (hmm/hmm.rs:215-218, cp.rs:66-68)
//   s_i   = d[i] + a[i,j];  m = max_i s_i                (viterbi.rs:13-16, cp.rs:71-74)
//   psi   = first i with s_i == m                       (ndarray-stats argmax)
//   d'[j] = m + b[j,o]                                  (viterbi.rs:17)
// followed by the backtrack of cp.rs:85-93 / viterbi.rs:24-31.
//
// Kernels
//   trellis_fwd_f32<NP>   one sequence per workgroup (NP/16 waves).  A is REGISTER
//                         RESIDENT: lane (rg = lane&7, cp = lane>>3) of wave w owns
//                         columns j0 = 16w + 2cp, j0+1 and rows [rg*R, rg*R+R), R = NP/8.
//                         delta_{t-1} is broadcast from LDS with ds_read_b128 (8 distinct
//                         row-group addresses per instruction, padded so the 8 spans hit
//                         disjoint banks); per pair one v_add_f32 and half a v_max3_f32
//                         (4 VALU cycles per wave-pair: profiles/r01_valu_rates.txt shows
//                         DPP-broadcast adds and v_pk_add_f32 issue at half rate, so the
//                         broadcast goes through LDS instead).  The 8 row-group partial
//                         maxima of a column are folded with three DPP max steps inside
//                         the wave, so one barrier per time step suffices.  No argmax in
//                         the forward pass: delta rows go to HBM and the backtrack
//                         recomputes psi only along the decoded path, with the same f32
//                         adds, which is bit-identical.
//   backtrack_f32<NP>     one wave per sequence: first-argmax of the last row, then for
//                         t = T-1..1 recompute s_i = delta_{t-1}[i] + a[i, path[t]] and
//                         take the first argmax; optional f64 re-score along the path.
//   generic_fwd<REAL>     any N, f32 or f64, every association mode of the reference
//                         (VITERBI row A0, CP cp.rs:70-78, DP dp.rs:127-177, DECODE
//                         viterbi.rs:5-32) with inline first-argmax; writes u16 psi.
//   generic_backtrack<REAL>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "trellis.h"
#include "../tuning.h"

namespace cvk {

__device__ __forceinline__ float ninf_f() { return -__builtin_inff(); }

// max over the 8 lanes of an aligned lane octet (lane & 7 varies); result in all 8.
// One v_max_f32_dpp per level (the DPP read of a VGPR written by the previous VALU op
// needs 2 wait states, hence the s_nop inside the asm).
__device__ __forceinline__ float octet_max(float x) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(x));
  return x;
}

// max of x over lane pairs (l, l^16) or (l, l^32).  Inline asm: hipcc (ROCm 7.2) folds
// __builtin_amdgcn_permlane*_swap(x, x) to its first result only, which is right in half
// of the lanes (tools/debug/reduce_check.hip measured it on the device).
__device__ __forceinline__ float swap_max(float x, bool sixteen) {
  // a = vdst, b = src, both = x.  After the swap a holds the low half's values (row pair)
  // in both halves and b the high half's, so max(a, b) = max(x[l], x[l^16|32]) in every lane.
  float a = x, b = x;
  if (sixteen)
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  else
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return fmaxf(a, b);
}

// max over all 64 lanes, result in every lane: DPP inside rows of 16, then permlane swaps.
__device__ __forceinline__ float wave_max(float x) {
  x = octet_max(x);
  asm volatile(
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(x));
  x = swap_max(x, true);
  return swap_max(x, false);
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also emits the workgroup
// release fence, which waits (vmcnt) for this wave's outstanding GLOBAL stores -- the
// delta row just written for the backtrack -- adding a store round trip to every step.
// Nothing in the kernel reads those stores back, so only the LDS writes are drained.
// The wait is the s_waitcnt builtin (not inline asm) so the compiler's waitcnt pass knows
// lgkmcnt is 0 after it -- otherwise a scalar load issued before the barrier makes it
// insert lgkmcnt(0) after the next LDS reads; the empty asm statements keep the compiler
// from moving memory operations across (the s_barrier builtin itself is not a fence).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // gfx9 encoding: lgkmcnt(0), vmcnt/expcnt unconstrained
#ifndef CVK_ABLATE_NOBAR  // tools/microbench/fwd_ablate.hip only: timing without the barrier
  __builtin_amdgcn_s_barrier();
#endif
  asm volatile("" ::: "memory");
}

// Padded LDS stride (floats) of one row-group block of delta: conflict-free
// ds_read_b128 for the 8 row-group addresses of a lane group (checked exhaustively).
template <int NP>
struct TrellisGeom {
  static constexpr int WAVES = NP / 16;
  static constexpr int THREADS = NP * 4;
  static constexpr int R = NP / 8;  // rows per lane
  static constexpr int S = (R % 16 == 0) ? R + 4 : R;
  static constexpr int LDS_FLOATS = 8 * S;  // one delta buffer
  static_assert(NP % 32 == 0 && NP >= 32 && NP <= 256, "NP must be a multiple of 32 in [32,256]");
};

// slot -> (sequence id, first element, length): CSR offsets (+ optional schedule) or an
// explicit element range per slot (constrained decode: prefixes / reversed suffixes).
template <bool EXT>
__device__ __forceinline__ void seq_range(const TrellisFwdArgs& args, int64_t slot, int64_t& seq, int64_t& e0,
                                          int& T) {
  if (EXT && args.ranges) {
    seq = slot;
    e0 = args.ranges[2 * slot];
    T = (int)(args.ranges[2 * slot + 1] - e0);
  } else {
    seq = args.order ? (int64_t)args.order[slot] : slot;
    e0 = args.offsets[seq];
    T = (int)(args.offsets[seq + 1] - e0);
  }
}

// Column fold of the forward kernels: a lane's two column partials are folded
// together -- lanes rg < 4 end with column j0, rg >= 4 with column j0+1; the first level
// (row_half_mirror pairs rg with 7-rg, i.e. the other half) brings in the other column --
// so 3 DPP maxima + 2 selects replace octet_max on both columns (6 DPP maxima).
__device__ __forceinline__ float dpp_max_mirror(float mine, float other) {
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %0 row_half_mirror row_mask:0xf bank_mask:0xf"
               : "+v"(mine)
               : "v"(other));
  return mine;
}
__device__ __forceinline__ float dpp_max_xor1(float x) {
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x));
  return x;
}
__device__ __forceinline__ float dpp_max_xor1_other(float mine, float other) {
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
               : "+v"(mine)
               : "v"(other));
  return mine;
}
__device__ __forceinline__ float dpp_max_xor2_other(float mine, float other) {
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %1, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf"
               : "+v"(mine)
               : "v"(other));
  return mine;
}
__device__ __forceinline__ float dpp_max_xor2(float x) {
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(x));
  return x;
}

// EXT = false: the plain decode (no forced states, CSR ranges, forward order, no final-row
// output) -- the extra features cost registers, so they are a separate instantiation.
template <int NP, bool EXT>
__global__ __launch_bounds__(NP * 4) void trellis_fwd_f32(TrellisFwdArgs args) {
  using G = TrellisGeom<NP>;
  constexpr int R = G::R;
  constexpr int S = G::S;
  __shared__ __attribute__((aligned(16))) float lds_delta[2][G::LDS_FLOATS];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int rg = lane & 7;
  const int cp = lane >> 3;
  const int j0 = 16 * w + 2 * cp;
  const bool hi = rg >= 4;  // column of this lane after the fold: j0 + hi
  const int jw = j0 + (hi ? 1 : 0);
  const bool writer = (rg & 3) == 0;  // rg 0 stores column j0, rg 4 column j0 + 1

  const int64_t slot =
      (EXT && args.slot_order) ? (int64_t)args.slot_order[blockIdx.x] : args.seq_begin + (int64_t)blockIdx.x;
  const bool second = EXT && args.split > 0 && slot >= args.split;  // second pass of a two-pass launch
  int64_t seq, e0;
  int T;
  seq_range<EXT>(args, slot, seq, e0, T);
  if (T <= 0) return;
  // constant address space: uniform loads become s_load (SMEM), off the vmcnt queue.
  // A reversed range walks obs[end-1], obs[end-2], ... (ob_step = -1).
  const bool rev = EXT && (args.reverse || second);
  const int ob_step = rev ? -1 : 1;
  const int64_t ob0 = rev ? e0 + T - 1 : e0;
  const __attribute__((address_space(4))) int32_t* obs =
      (const __attribute__((address_space(4))) int32_t*)(args.obs + ob0);
  const __attribute__((address_space(4))) int32_t* frc =
      (const __attribute__((address_space(4))) int32_t*)((EXT && args.forced) ? args.forced + ob0 : nullptr);
  float* __restrict__ drow = !EXT ? args.delta + (e0 - args.delta_elem_base) * NP + jw
                             : (args.delta && !second)
                                 ? args.delta + (args.row_base ? args.row_base[slot] : e0 - args.delta_elem_base) * NP + jw
                                 : nullptr;
  float* __restrict__ lrow = !EXT ? nullptr
                             : second ? args.last_row2 + (slot - args.split) * NP + jw
                             : args.last_row ? args.last_row + (slot - args.seq_begin) * NP + jw : nullptr;
  const float* __restrict__ pi = second ? args.pi2 : args.pi;
  const float* __restrict__ etj = args.et + jw;
  const unsigned V = (unsigned)args.nobs;

  // A register image: float4 q of a lane = (A[rg*R+2q][j0], A[rg*R+2q][j0+1],
  // A[rg*R+2q+1][j0], A[rg*R+2q+1][j0+1]); each wave-instruction reads 1 KiB contiguous.
  // Forward waves win issue arbitration over co-resident backtrack waves (overlap mode):
  // the backtrack has slack, the forward pass is the critical path.
  __builtin_amdgcn_s_setprio(3);
  float a_reg[2 * R];
  {
    const float4* img = reinterpret_cast<const float4*>(second ? args.a_img2 : args.a_img) + (size_t)w * (R / 2) * 64 + lane;
#pragma unroll
    for (int q = 0; q < R / 2; ++q) {
      const float4 v = img[q * 64];
      a_reg[4 * q + 0] = v.x;
      a_reg[4 * q + 1] = v.y;
      a_reg[4 * q + 2] = v.z;
      a_reg[4 * q + 3] = v.w;
    }
  }

  // Observations are read with uniform (scalar) loads one step ahead of the emission
  // row they select; an out-of-range index flags the sequence and is clamped so no
  // load leaves the table.
  unsigned bad = 0;
  auto obs_s = [&](int t) -> unsigned {
    const unsigned o = (unsigned)obs[t * ob_step];
    bad |= (o >= V);
    return o < V ? o : 0u;
  };
  auto frc_s = [&](int t) -> int { return (EXT && frc) ? frc[t * ob_step] : -1; };
  auto et_row = [&](unsigned o) -> float { return etj[(size_t)o * NP]; };
  // forced state (consistency constraint): every other state of that element is impossible
  auto force = [&](float d, int f) -> float { return (EXT && f >= 0 && jw != f) ? ninf_f() : d; };

  const int lds_w = (j0 / R) * S + (j0 % R) + (hi ? 1 : 0);
  // ---- t = 0: d0 = pi + b[:,o0]  (hmm.rs:215-218, cp.rs:66-68) ----
  {
    const float e = et_row(obs_s(0));
    float d0 = pi[jw] + e;
    if (EXT && args.start) {  // segment table column: start in state s, score 0 (cfn.rs:11-34 pattern)
      const int s = args.start[slot - args.seq_begin];
      if (s >= 0) d0 = (jw == s) ? 0.0f : ninf_f();
    }
    int f0 = frc_s(0);
    if (EXT && f0 <= -2) {  // resume: row t_1 of the prefix pass, already forced
      d0 = args.resume_rows[(size_t)(-2 - f0) * NP + jw];
      f0 = -1;
    }
    d0 = force(d0, f0);
    if (writer) {
      lds_delta[0][lds_w] = d0;
      if (!EXT || drow) *drow = d0;
      if (EXT && lrow && T == 1) *lrow = d0;
    }
  }
  int f_next = frc_s(T > 1 ? 1 : 0);
  unsigned o_next = obs_s(T > 1 ? 1 : 0);
  float eA = et_row(o_next);  // emission row of t = 1
  o_next = obs_s(T > 2 ? 2 : T - 1);
  float eB;
  lds_barrier();

  // One trellis step t: consumes e_use (row of o_t, loaded one step earlier), issues the
  // load of the row of o_{t+1} into e_pref and the scalar load of o_{t+2}.
  auto step = [&](int t, const float& e_use, float& e_pref) {
    e_pref = et_row(o_next);
    const int cur = (t - 1) & 1;
    const float* dsrc = &lds_delta[cur][rg * S];
    float m0a = ninf_f(), m0b = ninf_f(), m1a = ninf_f(), m1b = ninf_f();
    // the lane's R delta rows stream through a window of three float4 blocks (block q+3 is
    // loaded once block q is consumed) instead of R registers
    constexpr int NB = R / 4;
    float4 win[3];
#pragma unroll
    for (int q = 0; q < 3 && q < NB; ++q) win[q] = *reinterpret_cast<const float4*>(dsrc + 4 * q);
#pragma unroll
    for (int q4 = 0; q4 < NB; ++q4) {
      const float4 d = win[q4 % 3];
      const int k = 4 * q4;
      // s_i = d[i] + a[i,j]  (viterbi.rs:15) for rows k..k+3 of this lane, columns j0, j0+1
      const float s00 = d.x + a_reg[2 * k + 0], s01 = d.x + a_reg[2 * k + 1];
      const float s10 = d.y + a_reg[2 * k + 2], s11 = d.y + a_reg[2 * k + 3];
      const float s20 = d.z + a_reg[2 * k + 4], s21 = d.z + a_reg[2 * k + 5];
      const float s30 = d.w + a_reg[2 * k + 6], s31 = d.w + a_reg[2 * k + 7];
      if (q4 == 0) {
        m0a = fmaxf(s00, s10);
        m1a = fmaxf(s01, s11);
        m0b = fmaxf(s20, s30);
        m1b = fmaxf(s21, s31);
      } else {
        m0a = fmaxf(fmaxf(m0a, s00), s10);
        m1a = fmaxf(fmaxf(m1a, s01), s11);
        m0b = fmaxf(fmaxf(m0b, s20), s30);
        m1b = fmaxf(fmaxf(m1b, s21), s31);
      }
      if (q4 + 3 < NB) {
        // keep the block's adds here (inputs only: an asm output would be canonicalised)
        asm volatile("" ::"v"(m0a), "v"(m0b), "v"(m1a), "v"(m1b));
        win[q4 % 3] = *reinterpret_cast<const float4*>(dsrc + 4 * (q4 + 3));
      }
    }
    const int f_use = f_next;
    o_next = obs_s(t + 2 < T ? t + 2 : T - 1);
    f_next = frc_s(t + 1 < T ? t + 1 : T - 1);
    const float m0 = fmaxf(m0a, m0b);
    const float m1 = fmaxf(m1a, m1b);
    // fold the 8 row groups; column j0 + hi ends in this lane
    float m = dpp_max_mirror(hi ? m1 : m0, hi ? m0 : m1);
    m = dpp_max_xor1(m);
    m = dpp_max_xor2(m);
    float dn = m + e_use;  // (d + a) + b -- viterbi.rs:15-17 association
    dn = force(dn, f_use);
    if (writer) {
      lds_delta[cur ^ 1][lds_w] = dn;
      if (!EXT || drow) drow[(size_t)t * NP] = dn;
      if (EXT && lrow && t == T - 1) *lrow = dn;
    }
    lds_barrier();
  };

  int t = 1;
  if ((T - 1) & 1) {  // odd number of steps: peel one so the pair loop is straight-line
    step(t, eA, eB);
    eA = eB;
    ++t;
  }
  for (; t + 1 < T; t += 2) {
    step(t, eA, eB);
    step(t + 1, eB, eA);
  }
  if (bad && lane == 0 && w == 0) args.status[seq] = CVK_SEQ_BADOBS;
}

// ---------------------------------------------------------------------------------
// trellis_fwd2_f32<NP>: the same recurrence for TWO sequences (X, Y) of equal length per
// workgroup, in alternating half-steps X(t), Y(t), one barrier after each.  Each half-step
// reads the first half of the lane's delta rows from registers prefetched during the
// previous half-step (the other sequence's data, complete since the last barrier), so the
// LDS latency after a barrier -- the bubble of the one-sequence kernel, where all four
// waves of a SIMD wait for their first ds_read together -- is hidden; the second half is
// loaded at the start of the half-step behind the first half's adds.  Plain decode, plus
// forced states (FRC: the consistency-constrained final decode) -- no other EXT features;
// the host pairs equal-length sequences and runs leftovers through trellis_fwd_f32.
// NP % 64 == 0 so that the delta blocks are whole float4s.
// ONEBAR (round 5): one workgroup barrier per STEP instead of per half-step.  Each sequence
// keeps its own double-buffered delta, so X(t) only needs X(t-1) complete (the barrier closing
// step t-1) and Y(t) only Y(t-1) (same barrier); the price is that Y(t) can no longer prefetch
// X's delta_t (not complete until the barrier), so that block is read right after it.
template <int NP, bool FRC, bool ONEBAR = false>
__global__ __launch_bounds__(NP * 4) void trellis_fwd2_f32(TrellisFwdArgs args) {
  using G = TrellisGeom<NP>;
  constexpr int R = G::R;
  constexpr int S = G::S;
  constexpr int H = R / 2;
  static_assert(H % 4 == 0, "pair kernel needs NP % 64 == 0");
  __shared__ __attribute__((aligned(16))) float lds[2][2][G::LDS_FLOATS];  // [X/Y][buffer]

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int rg = lane & 7;
  const int cp = lane >> 3;
  const int j0 = 16 * w + 2 * cp;
  const bool hi = rg >= 4;  // column of this lane after the fold: j0 + hi
  const unsigned jw = (unsigned)(j0 + (hi ? 1 : 0));  // uniform base (SGPRs) + 32-bit VGPR offset
  const bool writer = (rg & 3) == 0;                  // rg 0 stores column j0, rg 4 column j0 + 1

  const int64_t slot = args.seq_begin + 2 * (int64_t)blockIdx.x;
  int64_t seq[2], e0[2];
  int Ts[2];
  seq_range<false>(args, slot, seq[0], e0[0], Ts[0]);
  seq_range<false>(args, slot + 1, seq[1], e0[1], Ts[1]);
  const int T = Ts[0];  // host guarantees Ts[0] == Ts[1]
  if (T <= 0) return;
  typedef const __attribute__((address_space(4))) int32_t* cobs_t;
  const cobs_t obsX = (cobs_t)(args.obs + e0[0]);
  const cobs_t obsY = (cobs_t)(args.obs + e0[1]);
  const cobs_t frcX = (cobs_t)(FRC ? args.forced + e0[0] : nullptr);
  const cobs_t frcY = (cobs_t)(FRC ? args.forced + e0[1] : nullptr);
  // uniform row bases (SGPRs); the lane adds j0
  float* const dX = args.delta + (e0[0] - args.delta_elem_base) * NP;
  float* const dY = args.delta + (e0[1] - args.delta_elem_base) * NP;
  const unsigned V = (unsigned)args.nobs;

  // Forward waves win issue arbitration over co-resident backtrack waves (overlap mode):
  // the backtrack has slack, the forward pass is the critical path.
  __builtin_amdgcn_s_setprio(3);
  float a_reg[2 * R];
  {
    const float4* img = reinterpret_cast<const float4*>(args.a_img) + (size_t)w * (R / 2) * 64 + lane;
#pragma unroll
    for (int q = 0; q < R / 2; ++q) {
      const float4 v = img[q * 64];
      a_reg[4 * q + 0] = v.x;
      a_reg[4 * q + 1] = v.y;
      a_reg[4 * q + 2] = v.z;
      a_reg[4 * q + 3] = v.w;
    }
  }
#ifndef CVK_F32_NO_AWAIT
  // the A image is resident before the step loop: without this wait the compiler's waitcnt
  // pass, merging the loop's back edge with the preheader, kept in-loop vmcnt waits for these
  // loads, and those in-order waits also drained this wave's delta-row stores every half-step
  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0), expcnt/lgkmcnt unconstrained
#endif
  unsigned bad = 0;  // bit 0: X, bit 1: Y
  // CVK_F32_ABL_*: timing-only ablations (results wrong; tools/build_variant_f32.sh):
  // OBS = observations from arithmetic instead of scalar loads, NOE = no emission loads
  auto obs_x = [&](int t) -> unsigned {
#ifdef CVK_F32_ABL_OBS
    return ((unsigned)t * 7u + (unsigned)e0[0]) % V;
#endif
    const unsigned o = (unsigned)obsX[t];
    bad |= (o >= V) ? 1u : 0u;
    return o < V ? o : 0u;
  };
  auto obs_y = [&](int t) -> unsigned {
#ifdef CVK_F32_ABL_OBS
    return ((unsigned)t * 5u + (unsigned)e0[1]) % V;
#endif
    const unsigned o = (unsigned)obsY[t];
    bad |= (o >= V) ? 2u : 0u;
    return o < V ? o : 0u;
  };
  auto et_row = [&](unsigned o) -> float {
#ifdef CVK_F32_ABL_NOE
    return -1.0f * (float)(o & 3u);
#endif
    const float* row = args.et + (size_t)o * NP;  // uniform
    return row[jw];
  };
  const int lds_w = (j0 / R) * S + (j0 % R) + (hi ? 1 : 0);
  auto clampT = [&](int t) { return t < T ? t : T - 1; };
  // forced state (consistency constraint): every other state of that element is impossible
  auto force = [&](float d, int f) -> float { return (FRC && f >= 0 && (int)jw != f) ? ninf_f() : d; };

  // ---- t = 0 for both sequences ----
  {
    const float ex = et_row(obs_x(0)), ey = et_row(obs_y(0));
    const float p = args.pi[jw];
    int fx = FRC ? frcX[0] : -1, fy = FRC ? frcY[0] : -1;
    float dx = p + ex, dy = p + ey;
    if (FRC && fx <= -2) {  // resume: row t_1 of the prefix pass, already forced
      dx = args.resume_rows[(size_t)(-2 - fx) * NP + jw];
      fx = -1;
    }
    if (FRC && fy <= -2) {
      dy = args.resume_rows[(size_t)(-2 - fy) * NP + jw];
      fy = -1;
    }
    dx = force(dx, fx);
    dy = force(dy, fy);
    if (writer) {
      lds[0][0][lds_w] = dx;
      lds[1][0][lds_w] = dy;
      dX[jw] = dx;
      dY[jw] = dy;
    }
  }
  // Emission rows are loaded one HALF-step ahead (during the other sequence's half-step):
  // eX is loaded in Y(t-1) and used in X(t), eY loaded in X(t) and used in Y(t), so at each
  // use exactly two newer vector-memory ops are in flight (vmcnt(2), no store drain).  The
  // scalar obs loads are issued at the END of a half-step, so the barrier's lgkmcnt(0)
  // retires them and the compiler's own wait for them (at the next emission load) comes
  // before that half-step's LDS reads -- an SMEM load in flight would otherwise force an
  // lgkmcnt(0) on the prefetched rows and expose the LDS latency again.
  float eX = et_row(obs_x(clampT(1)));  // X at t = 1
  float eY;
  unsigned oY = obs_y(clampT(1));  // o_Y(t) for the coming X(t)
  unsigned oX = obs_x(clampT(2));  // o_X(t+1) for the coming Y(t)
  // forced state of the coming half-step, loaded (SMEM) at the end of the previous one
  int f_nx = FRC ? frcX[clampT(1)] : -1;
  lds_barrier();
  // delta rows stream through a rolling window of two 8-row blocks (P, Q): block k of the
  // lane's R rows lives in P for even k, Q for odd k, and each block is refilled with block
  // k+2 as soon as it is consumed, so a load always has the next block's adds to hide
  // behind.  Block 0 of the NEXT half-step (the other sequence's delta, complete since the
  // last barrier) goes into P while this half-step's last block is processed.  16 VGPRs of
  // delta instead of 32: 4 waves x <=112 VGPRs leave a backtrack wave room on every SIMD.
  constexpr int KB = R / 8;  // 8-row blocks per lane
  static_assert(R % 8 == 0, "pair kernel needs NP % 64 == 0");
#ifndef CVK_F32_ABL_NOLDS
  auto ld8 = [&](const float* src, float4 (&dst)[2]) {
    dst[0] = *reinterpret_cast<const float4*>(src);
    dst[1] = *reinterpret_cast<const float4*>(src + 4);
  };
#else  // timing only: no LDS reads in the loop -- the block registers are declared changed by
       // an empty asm (no instructions), so the adds stay in the loop (results wrong)
  bool abl_first = true;
  auto ld8 = [&](const float* src, float4 (&dst)[2]) {
    if (abl_first) {
      dst[0] = *reinterpret_cast<const float4*>(src);
      dst[1] = *reinterpret_cast<const float4*>(src + 4);
      abl_first = false;
    }
    asm volatile("" : "+v"(dst[0].x), "+v"(dst[0].y), "+v"(dst[0].z), "+v"(dst[0].w), "+v"(dst[1].x), "+v"(dst[1].y),
                 "+v"(dst[1].z), "+v"(dst[1].w));
  };
#endif
  float4 P[2], Q[2];
  ld8(&lds[0][0][rg * S], P);

  // One half-step at step t: dsrc = this sequence's delta_{t-1} block, nsrc = the block the
  // next half-step reads first; e_use = this half-step's emission row, e_load <- the next
  // half-step's (row o_load); then o_load <- obs(t_obs) of the sequence `is_y`.
  auto half = [&](const float* dsrc, const float* nsrc, float* ldst, float* drow, int t, const float& e_use,
                  float& e_load, unsigned& o_load, bool is_y, int t_obs) {
    const bool sync = !ONEBAR || is_y;  // ONEBAR: the barrier closes the step (after Y)
    const int f_use = f_nx;
    e_load = et_row(o_load);
    if (KB > 1) ld8(dsrc + 8, Q);
    float m0a = ninf_f(), m0b = ninf_f(), m1a = ninf_f(), m1b = ninf_f();
    auto rows4 = [&](const float4& dd, int k, bool first) {
      // s_i = d[i] + a[i,j]  (viterbi.rs:15) for rows k..k+3 of this lane, columns j0, j0+1
      const float s00 = dd.x + a_reg[2 * k + 0], s01 = dd.x + a_reg[2 * k + 1];
      const float s10 = dd.y + a_reg[2 * k + 2], s11 = dd.y + a_reg[2 * k + 3];
      const float s20 = dd.z + a_reg[2 * k + 4], s21 = dd.z + a_reg[2 * k + 5];
      const float s30 = dd.w + a_reg[2 * k + 6], s31 = dd.w + a_reg[2 * k + 7];
      if (first) {
        m0a = fmaxf(s00, s10);
        m1a = fmaxf(s01, s11);
        m0b = fmaxf(s20, s30);
        m1b = fmaxf(s21, s31);
      } else {
        m0a = fmaxf(fmaxf(m0a, s00), s10);
        m1a = fmaxf(fmaxf(m1a, s01), s11);
        m0b = fmaxf(fmaxf(m0b, s20), s30);
        m1b = fmaxf(fmaxf(m1b, s21), s31);
      }
    };
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      float4(&B)[2] = (k & 1) ? Q : P;
      rows4(B[0], 8 * k, k == 0);
      rows4(B[1], 8 * k + 4, false);
      __builtin_amdgcn_sched_barrier(0);
      if (k + 2 < KB)
        ld8(dsrc + 8 * (k + 2), B);
      else if (!(k & 1) && (k + 2 == KB || k + 1 == KB) && !(ONEBAR && is_y))
        ld8(nsrc, P);  // next half-step's block 0 (KB odd: no adds left to hide it)
      __builtin_amdgcn_sched_barrier(0);
    }

    const float m0 = fmaxf(m0a, m0b);
    const float m1 = fmaxf(m1a, m1b);
    // fold the 8 row groups; column j0 + hi ends in this lane
    float m = dpp_max_mirror(hi ? m1 : m0, hi ? m0 : m1);
    m = dpp_max_xor1(m);
    m = dpp_max_xor2(m);
    const float dn = force(m + e_use, f_use);  // (d + a) + b, viterbi.rs:15-17
    __builtin_amdgcn_sched_barrier(0);
    o_load = is_y ? obs_y(t_obs) : obs_x(t_obs);
    // X(t) is followed by Y(t), Y(t) by X(t+1)
    if (FRC) f_nx = is_y ? frcY[clampT(t)] : frcX[clampT(t + 1)];
    // every lane stores (the 4 lanes of a column half hold the same value, so the duplicate
    // stores coalesce): under the old `if (writer)` the compiler could not count the store
    // in the in-order vmcnt queue, so the next half-step's wait for its emission row
    // (vmcnt(1) instead of vmcnt(2)) also drained this store
#ifndef CVK_F32_WRITER_STORES
    ldst[lds_w] = dn;
    float* row = drow + (size_t)t * NP;  // uniform
#ifndef CVK_F32_ABL_NOSTORE
    row[jw] = dn;
#else
    if (dn == 12345.0f) row[jw] = dn;  // timing only: no delta-row stores
#endif
#else  // A/B: the round-4 form
    if (writer) {
      ldst[lds_w] = dn;
      float* row = drow + (size_t)t * NP;  // uniform
      row[jw] = dn;
    }
#endif
    if (sync) lds_barrier();
    if (ONEBAR && is_y) ld8(nsrc, P);  // X's delta_t, complete since the barrier
  };
  // step t: X(t) prefetches Y's delta_{t-1} and loads e_Y(t); Y(t) prefetches X's delta_t and
  // loads e_X(t+1)
  auto step = [&](int t) {
    const int cur = (t - 1) & 1, nxt = t & 1;
    half(&lds[0][cur][rg * S], &lds[1][cur][rg * S], &lds[0][nxt][0], dX, t, eX, eY, oY, true, clampT(t + 1));
    half(&lds[1][cur][rg * S], &lds[0][nxt][rg * S], &lds[1][nxt][0], dY, t, eY, eX, oX, false, clampT(t + 2));
  };
  int t = 1;
  if ((T - 1) & 1) step(t++);
  for (; t + 1 < T; t += 2) {
    step(t);
    step(t + 1);
  }
  if (bad && lane == 0 && w == 0) {
    if (bad & 1u) args.status[seq[0]] = CVK_SEQ_BADOBS;
    if (bad & 2u) args.status[seq[1]] = CVK_SEQ_BADOBS;
  }
}

// ---------------------------------------------------------------------------------
// Wave-level first-argmax: (v, i) pairs, larger v wins, ties -> smaller i.
__device__ __forceinline__ void wave_argmax_first(float& v, int& i) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const float ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(i, off);
    const bool take = (ov > v) || (ov == v && oi < i);
    v = take ? ov : v;
    i = take ? oi : i;
  }
}
__device__ __forceinline__ void wave_argmax_first_d(double& v, int& i) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const double ov = __shfl_xor(v, off);
    const int oi = __shfl_xor(i, off);
    const bool take = (ov > v) || (ov == v && oi < i);
    v = take ? ov : v;
    i = take ? oi : i;
  }
}

__device__ __forceinline__ int load_path_l2(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// f64 re-score of the decoded path with the row-A0 association, one wave, sequential
// rounding exactly as the reference's f64 recurrence would produce along this path.
__device__ double rescore_path_f64(const int32_t* path, const int32_t* obs, int T, const double* pi64,
                                   const double* a64, const double* et64, int N, int lane) {
  // path was written by this wave with plain stores; drain them to L2, read back with
  // L1-bypassing (agent-scope) loads.
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) expcnt(0)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  double d = 0.0;
  for (int base = 0; base < T; base += 64) {
    const int t = base + lane;
    double av = 0.0, bv = 0.0;
    if (t < T) {
      const int p = load_path_l2(path + t);
      const int o = obs[t];
      bv = et64[(size_t)o * N + p];
      if (t == 0) {
        av = pi64[p];
      } else {
        const int pp = load_path_l2(path + t - 1);
        av = a64[(size_t)pp * N + p];
      }
    }
    const int cnt = min(64, T - base);
    for (int k = 0; k < cnt; ++k) {
      const double ak = __builtin_bit_cast(
          double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, av) >> 32), k) << 32) |
                      (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned long long, av), k));
      const double bk = __builtin_bit_cast(
          double, ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(__builtin_bit_cast(unsigned long long, bv) >> 32), k) << 32) |
                      (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned long long, bv), k));
      if (base + k == 0)
        d = ak + bk;  // pi[p0] + b[p0,o0]
      else
        d = (d + ak) + bk;  // (d + a) + b
    }
  }
  return d;
}

// One wave per sequence.  delta rows are independent of the path, so they are loaded PF
// rows at a time into a register ring; only the transition column a[:, path[t]] is a
// dependent (L2-resident) load.  First argmax = DPP/permlane wave max, then a ballot of
// the lanes holding it (lowest lane of the lowest k = lowest state index).
template <int NP>
__global__ __launch_bounds__(256) void backtrack_f32(BacktrackArgs args) {
  constexpr int KP = (NP + 63) / 64;
  constexpr int PF = 8;
  const int lane = threadIdx.x & 63;
  const int64_t slot = args.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= args.seq_end) return;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  const int N = args.nstates;
  if (T <= 0) {
    if (lane == 0) {
      args.score[seq] = 0.0;
      args.status[seq] = CVK_SEQ_EMPTY;
    }
    return;
  }
  int32_t* __restrict__ path = args.path + e0;
  const float* __restrict__ drow = args.delta + (e0 - args.delta_elem_base) * NP;
  bool valid[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) valid[k] = (lane + 64 * k) < N;
  auto load_row = [&](int r, float (&dst)[KP]) {
#pragma unroll
    for (int k = 0; k < KP; ++k) dst[k] = (r >= 0 && valid[k]) ? drow[(size_t)r * NP + lane + 64 * k] : ninf_f();
  };
  // first argmax of the last row (cp.rs:86)
  int cur;
  float bv;
  {
    float last[KP];
    load_row(T - 1, last);
    float m = last[0];
#pragma unroll
    for (int k = 1; k < KP; ++k) m = fmaxf(m, last[k]);
    bv = wave_max(m);
    cur = 0;
#pragma unroll
    for (int k = KP - 1; k >= 0; --k) {
      const unsigned long long mask = __ballot(valid[k] && last[k] == bv);
      if (mask) cur = 64 * k + __builtin_ctzll(mask);
    }
  }
  const uint8_t prior = args.status[seq];
  if (!(bv > ninf_f()) || prior == CVK_SEQ_BADOBS) {
    for (int t = lane; t < T; t += 64) path[t] = 0;
    if (lane == 0) {
      args.score[seq] = (double)ninf_f();
      args.status[seq] = prior == CVK_SEQ_BADOBS ? CVK_SEQ_BADOBS : CVK_SEQ_INFEASIBLE;
    }
    return;
  }
  const float score32 = bv;
  int pathreg = 0;
  if (lane == ((T - 1) & 63)) pathreg = cur;
  if (((T - 1) & 63) == 0 && lane == 0) path[T - 1] = cur;
  const float* __restrict__ at = args.at;
  float ring[PF][KP];
#pragma unroll
  for (int u = 0; u < PF; ++u) load_row(T - 2 - u, ring[u]);
  for (int base = T - 1; base >= 1; base -= PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int t = base - u;
      if (t >= 1) {
        // s_i = d_{t-1}[i] + a[i, cur]  -- the forward pass's exact f32 add
        const float* acol = at + (size_t)cur * NP + lane;
        float s[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) s[k] = valid[k] ? ring[u][k] + acol[64 * k] : ninf_f();
        float m = s[0];
#pragma unroll
        for (int k = 1; k < KP; ++k) m = fmaxf(m, s[k]);
        const float M = wave_max(m);
        int nxt = 0;
#pragma unroll
        for (int k = KP - 1; k >= 0; --k) {
          const unsigned long long mask = __ballot(valid[k] && s[k] == M);
          if (mask) nxt = 64 * k + __builtin_ctzll(mask);
        }
        cur = nxt;
        const int tp = t - 1;
        if (lane == (tp & 63)) pathreg = cur;
        if ((tp & 63) == 0 && tp + lane < T) path[tp + lane] = pathreg;  // flush a 64-entry block
      }
    }
    // Refill the whole ring once per block.  Vector-memory loads retire in order, so a
    // per-step refill would make every step's dependent a-column load wait for the
    // previous step's HBM row load; in bulk, only the block's first step waits for HBM.
#pragma unroll
    for (int u = 0; u < PF; ++u) load_row(base - PF - 1 - u, ring[u]);
  }
  if (lane == 0) {
    args.status[seq] = CVK_SEQ_OK;
    args.score[seq] = (double)score32;  // f64 re-score: rescore_f64_lanes (after this kernel)
    if (args.score32) args.score32[seq] = score32;
  }
}

// backtrack_v_f32<NP> (NP % 64 == 0): the same backtrack with VL = NP/64 CONSECUTIVE states
// per lane (lane l owns states VL*l .. VL*l+VL-1), so a delta row and a column of A^T are
// one dwordx{VL} load per lane instead of VL dword loads: 4x fewer vector-memory
// instructions at N = 256 and 16-byte requests.  First argmax: wave max, ballot of the lanes
// holding it (lowest lane = lowest state block), then that lane's first k (readlane).
template <int VL>
__device__ __forceinline__ void ld_vl(const float* p, float (&d)[VL]) {
  if constexpr (VL == 4) {
    const float4 x = *reinterpret_cast<const float4*>(p);
    d[0] = x.x, d[1] = x.y, d[2] = x.z, d[3] = x.w;
  } else if constexpr (VL == 2) {
    const float2 x = *reinterpret_cast<const float2*>(p);
    d[0] = x.x, d[1] = x.y;
  } else {
#pragma unroll
    for (int k = 0; k < VL; ++k) d[k] = p[k];
  }
}

template <int VL>
__device__ __forceinline__ int first_argmax_vl(const float (&s)[VL], float M, int lane) {
  int fk = VL;
#pragma unroll
  for (int k = VL - 1; k >= 0; --k) fk = (s[k] == M) ? k : fk;
  const unsigned long long mask = __ballot(fk < VL);
  const int L = (int)__builtin_ctzll(mask);  // mask != 0: M is one of the s values
  return VL * L + __builtin_amdgcn_readlane(fk, L);
}

// Backtrack of ONE sequence by one wave (lane l owns states VL*l .. VL*l+VL-1): drow / at
// point at this lane's first state of delta row 0 / of A^T row 0; badobs: the forward pass
// flagged the sequence.  Shared by backtrack_v_f32 and the fused small-N kernel.
template <int VL, int NP>
__device__ __forceinline__ void backtrack_one(const BacktrackArgs& args, int64_t seq, int64_t e0, int T, int lane,
                                              const float* __restrict__ drow, const float* __restrict__ at,
                                              bool badobs, int fixed_last = -1, bool record = true) {
  constexpr int PF = 8;
  // NP < 64 (one-wave kernels with 16/32/48 padded states): lanes >= NP hold no state
  const bool own = NP >= 64 * VL || lane < NP;
  int32_t* __restrict__ path = args.path + e0;
  // padded states (>= N) hold -inf in delta and A^T, so they never win a feasible argmax
  auto load_row = [&](int r, float (&dst)[VL]) {
    if (r >= 0 && own) {
      ld_vl<VL>(drow + (size_t)r * NP, dst);
    } else {
#pragma unroll
      for (int k = 0; k < VL; ++k) dst[k] = ninf_f();
    }
  };
  auto lane_max = [&](const float (&v)[VL]) {
    float m = v[0];
#pragma unroll
    for (int k = 1; k < VL; ++k) m = fmaxf(m, v[k]);
    return m;
  };
  // first argmax of the last row (cp.rs:86)
  int cur;
  float bv;
  if (fixed_last >= 0) {  // prefix of a resumed sequence: the forced state, known feasible
    cur = fixed_last;
    bv = 0.0f;
  } else {
    float last[VL];
    load_row(T - 1, last);
    bv = wave_max(lane_max(last));
    cur = (bv > ninf_f()) ? first_argmax_vl<VL>(last, bv, lane) : 0;
  }
  if (!(bv > ninf_f()) || badobs) {
    for (int t = lane; t < T; t += 64) path[t] = 0;
    if (lane == 0) {
      args.score[seq] = (double)ninf_f();
      args.status[seq] = badobs ? CVK_SEQ_BADOBS : CVK_SEQ_INFEASIBLE;
    }
    return;
  }
  const float score32 = bv;
  int pathreg = 0;
  if (lane == ((T - 1) & 63)) pathreg = cur;
  if (((T - 1) & 63) == 0 && lane == 0) path[T - 1] = cur;
  float ring[PF][VL];
#pragma unroll
  for (int u = 0; u < PF; ++u) load_row(T - 2 - u, ring[u]);
  for (int base = T - 1; base >= 1; base -= PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int t = base - u;
      if (t >= 1) {
        // s_i = d_{t-1}[i] + a[i, cur]  -- the forward pass's exact f32 add
        float acol[VL], sv[VL];
        if (own) {
          ld_vl<VL>(at + (size_t)cur * NP, acol);
        } else {
#pragma unroll
          for (int k = 0; k < VL; ++k) acol[k] = ninf_f();
        }
#pragma unroll
        for (int k = 0; k < VL; ++k) sv[k] = ring[u][k] + acol[k];
        const float M = wave_max(lane_max(sv));
        cur = first_argmax_vl<VL>(sv, M, lane);
        const int tp = t - 1;
        if (lane == (tp & 63)) pathreg = cur;
        if ((tp & 63) == 0 && tp + lane < T) path[tp + lane] = pathreg;  // flush a 64-entry block
      }
    }
    // refill the whole ring once per block (in-order vmcnt: see backtrack_f32)
#pragma unroll
    for (int u = 0; u < PF; ++u) load_row(base - PF - 1 - u, ring[u]);
  }
  if (record && lane == 0) {
    args.status[seq] = CVK_SEQ_OK;
    args.score[seq] = (double)score32;  // f64 re-score: rescore_f64_lanes (after this kernel)
    if (args.score32) args.score32[seq] = score32;
  }
}

template <int NP>
__global__ __launch_bounds__(256) void backtrack_v_f32(BacktrackArgs args) {
  constexpr int VL = NP / 64;
  static_assert(NP % 64 == 0, "backtrack_v_f32 needs NP % 64 == 0");
  const int lane = threadIdx.x & 63;
  const int64_t slot = args.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= args.seq_end) return;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  if (T <= 0) {
    if (lane == 0) {
      args.score[seq] = 0.0;
      args.status[seq] = CVK_SEQ_EMPTY;
    }
    return;
  }
  backtrack_one<VL, NP>(args, seq, e0, T, lane, args.delta + (e0 - args.delta_elem_base) * NP + VL * lane,
                        args.at + VL * lane, args.status[seq] == CVK_SEQ_BADOBS);
}

// ---------------------------------------------------------------------------------
// trellis_wave_f32<NPW, FRC>: small N (NPW = 16, 32, 48 or 64 padded states) -- ONE WAVE per
// sequence, forward pass and backtrack fused, no workgroup barrier and no cross-wave anything.
// Forward: lane = 4cq + rg holds rows [R·rg, R·rg + R) (R = NPW/4) of the C = NPW/16 columns
// C·cq .. C·cq + C-1 of A (R·C = NPW²/64 VGPRs, from the row-major table `a_rm`); delta_{t-1}
// is read from the wave's own LDS row with R/4 ds_read_b128 (4 distinct addresses, padded
// stride R+4: conflict-free); per pair one v_add_f32 and half a v_max3_f32; the 4 row-group
// partials of the C columns are folded across the lane quad with DPP maxima (xor1 then xor2;
// C = 4: xor1 keeps a column pair, xor2 one column; C = 3: xor1 keeps column p plus the shared
// column 2, xor2 picks one; C ≤ 2: plain butterflies), so every lane ends with one column jw
// (C < 4: some lanes hold the same column and store the same value).  Padding N to the next
// multiple of 16 instead of 32 or 64 (N = 45: 48, not 64) cuts the per-step VALU work by
// (48/64)² = 0.56.  LDS instructions of one wave execute in order, so the next step's reads
// see this step's writes without a barrier.  A workgroup holds 4 independent waves.
// Backtrack (after an agent-scope acquire, so the delta rows this wave stored are read back
// from L2): backtrack_v_f32's loop with VL = 1 (lanes >= NPW idle), A^T read from LDS.  The f64 re-score runs
// afterwards (rescore_f64_lanes).  Roofline: VALU issue / per-step latency (small batches).
template <int NPW, bool FRC>
__global__ __launch_bounds__(256) void trellis_wave_f32(TrellisFwdArgs args, BacktrackArgs bargs) {
  constexpr int C = NPW / 16;  // columns per lane
  constexpr int R = NPW / 4;   // rows per lane
  constexpr int LS = R + 4;    // padded LDS stride of a row group
  static_assert(NPW % 16 == 0 && NPW >= 16 && NPW <= 64, "NPW in {16, 32, 48, 64}");
  __shared__ __attribute__((aligned(16))) float lds_all[4][2][4 * LS];
  // A^T for the backtrack's dependent per-step read (at[cur][.]): an LDS round trip instead
  // of an L1/L2 one; filled by the whole workgroup before any wave starts
  __shared__ __attribute__((aligned(16))) float at_lds[NPW * NPW];
  for (int k = threadIdx.x; k < NPW * NPW; k += 256) at_lds[k] = bargs.at[k];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  // wave-uniform in a scalar register, so the sequence bounds, the step loop and the
  // observation reads are scalar (s_load) rather than per-lane
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rg = lane & 3, cq = lane >> 2;
  const int p = rg & 1, q = rg >> 1;
  // this lane's column after the fold
  const int jw = C == 4 ? 4 * cq + 2 * p + q : C == 3 ? 3 * cq + (q ? 2 : p) : C == 2 ? 2 * cq + p : cq;
  const int64_t slot = args.seq_begin + 4 * (int64_t)blockIdx.x + wv;
  if (slot >= bargs.seq_end) return;
  int64_t seq, e0;
  int T;
  seq_range<false>(args, slot, seq, e0, T);
  if (T <= 0) {
    if (lane == 0) {
      bargs.score[seq] = 0.0;
      bargs.status[seq] = CVK_SEQ_EMPTY;
    }
    return;
  }
  float(*lds)[4 * LS] = lds_all[wv];
  typedef const __attribute__((address_space(4))) int32_t* cobs_t;
  const cobs_t obs = (cobs_t)(args.obs + e0);
  const cobs_t frc = (cobs_t)(FRC ? args.forced + e0 : nullptr);
  float* __restrict__ drow = args.delta + (e0 - args.delta_elem_base) * NPW;
  const unsigned V = (unsigned)args.nobs;
  float a_reg[R * C];  // a_reg[C·r + k] = A[R·rg + r][C·cq + k]
  if constexpr (C == 4) {
    const float4* src = reinterpret_cast<const float4*>(args.a_img) + (size_t)(R * rg) * (NPW / 4) + cq;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float4 v = src[r * (NPW / 4)];
      a_reg[4 * r + 0] = v.x;
      a_reg[4 * r + 1] = v.y;
      a_reg[4 * r + 2] = v.z;
      a_reg[4 * r + 3] = v.w;
    }
  } else {
    const float* src = args.a_img + (size_t)(R * rg) * NPW + C * cq;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < C; ++k) a_reg[C * r + k] = src[(size_t)r * NPW + k];
  }
  unsigned bad = 0;
  auto obs_s = [&](int t) -> unsigned {
    const unsigned o = (unsigned)obs[t];
    bad |= (o >= V);
    return o < V ? o : 0u;
  };
  auto force = [&](float d, int f) -> float { return (FRC && f >= 0 && jw != f) ? ninf_f() : d; };
  const int wofs = (jw / R) * LS + (jw % R);  // where this lane's column lives in an LDS row
  // ---- t = 0 ----
  {
    const float d0 = force(args.pi[jw] + args.et[(size_t)obs_s(0) * NPW + jw], FRC ? frc[0] : -1);
    lds[0][wofs] = d0;
    drow[jw] = d0;
  }
  // Steps unrolled by 4 with a static slot per step (k = (t-1) mod 4): the emission of step t
  // is loaded 4 steps ahead (at the end of step t-4, from the observation read 4 steps before
  // that by a scalar load), all indices clamped into the sequence so every load is issued
  // unconditionally -- no loaded register is copied across the loop edge, so the wave never
  // waits on the load it just issued (one-step-ahead prefetch exposed the full memory latency
  // every step).
  const int Tm1 = T - 1;
  unsigned so[4];
  float pe[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    pe[k] = args.et[(size_t)obs_s(min(1 + k, Tm1)) * NPW + jw];  // steps 1..4
    so[k] = obs_s(min(5 + k, Tm1));                              // observations of steps 5..8
  }
  for (int t0 = 1; t0 < T; t0 += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = t0 + k;
      if (t >= T) break;
      const int f_use = FRC ? frc[t] : -1;
      const float* src = &lds[(t - 1) & 1][rg * LS];
      float4 d[R / 4];
#pragma unroll
      for (int b = 0; b < R / 4; ++b) d[b] = *reinterpret_cast<const float4*>(src + 4 * b);
      float c[C];
#pragma unroll
      for (int kc = 0; kc < C; ++kc) {
        // s_i = d[i] + a[i,j]  (viterbi.rs:15), R rows of column C·cq + kc
        float m = fmaxf(d[0].x + a_reg[0 * C + kc], d[0].y + a_reg[1 * C + kc]);
        m = fmaxf(fmaxf(m, d[0].z + a_reg[2 * C + kc]), d[0].w + a_reg[3 * C + kc]);
#pragma unroll
        for (int b = 1; b < R / 4; ++b) {
          m = fmaxf(fmaxf(m, d[b].x + a_reg[(4 * b + 0) * C + kc]), d[b].y + a_reg[(4 * b + 1) * C + kc]);
          m = fmaxf(fmaxf(m, d[b].z + a_reg[(4 * b + 2) * C + kc]), d[b].w + a_reg[(4 * b + 3) * C + kc]);
        }
        c[kc] = m;
      }
      // fold the 4 row groups of the lane quad 4cq .. 4cq+3 into this lane's column jw
      float kk;
      if constexpr (C == 4) {  // xor1 keeps columns {2p, 2p+1}, xor2 keeps 2p+q
        float k0 = p ? c[2] : c[0], k1 = p ? c[3] : c[1];
        const float g0 = p ? c[0] : c[2], g1 = p ? c[1] : c[3];
        k0 = dpp_max_xor1_other(k0, g0);
        k1 = dpp_max_xor1_other(k1, g1);
        kk = q ? k1 : k0;
        const float gg = q ? k0 : k1;
        kk = dpp_max_xor2_other(kk, gg);
      } else if constexpr (C == 3) {  // xor1 keeps column p and the shared column 2, xor2 one
        float k0 = p ? c[1] : c[0];
        const float g0 = p ? c[0] : c[1];
        k0 = dpp_max_xor1_other(k0, g0);
        const float k2 = dpp_max_xor1(c[2]);
        kk = q ? k2 : k0;
        const float gg = q ? k0 : k2;
        kk = dpp_max_xor2_other(kk, gg);
      } else if constexpr (C == 2) {  // xor1 keeps column p, xor2 completes it
        float k0 = p ? c[1] : c[0];
        const float g0 = p ? c[0] : c[1];
        k0 = dpp_max_xor1_other(k0, g0);
        kk = dpp_max_xor2(k0);
      } else {
        kk = dpp_max_xor2(dpp_max_xor1(c[0]));
      }
#ifndef CVK_ABLATE_NOEMIT
      const float e_use = pe[k];
#else
      const float e_use = -0.5f * (float)(t & 7);
#endif
      const float dn = force(kk + e_use, f_use);  // (d + a) + b -- viterbi.rs:15-17
      lds[t & 1][wofs] = dn;
      drow[(size_t)t * NPW + jw] = dn;
#ifndef CVK_ABLATE_NOEMIT
      pe[k] = args.et[(size_t)so[k] * NPW + jw];  // step t+4
      so[k] = obs_s(min(t + 8, Tm1));            // observation of step t+8
#endif
    }
  }
  // ---- backtrack (cp.rs:85-93) of this wave's own sequence: the delta rows were stored
  // by other lanes of this wave -- make them visible (release to L2, then acquire) ----
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#ifndef CVK_ABLATE_NOBT
  backtrack_one<1, NPW>(bargs, seq, e0, T, lane, drow + lane, at_lds + lane, bad != 0);
#endif
}

// rescore_f64_lanes: the f64 re-score of rescore_path_f64, but one LANE per sequence, so the
// sequential fold (its rounding order is the definition) runs in 64 sequences at once per
// wave instead of one lane of a wave doing 4 readlanes per step.  The path/obs reads and the
// a/b gathers of 8 steps are issued before the 16 dependent adds that use them.
__global__ __launch_bounds__(64) void rescore_f64_lanes(RescoreArgs r) {
  const int64_t slot = r.seq_begin + (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (slot >= r.seq_end) return;
  const int64_t seq = r.order ? (int64_t)r.order[slot] : slot;
  if (r.status[seq] != CVK_SEQ_OK) return;
  const int64_t e0 = r.offsets[seq];
  const int T = (int)(r.offsets[seq + 1] - e0);
  const int32_t* __restrict__ path = r.path + e0;
  const int32_t* __restrict__ obs = r.obs + e0;
  const int N = r.nstates;
  int pp = path[0];
  double d = r.pi64[pp] + r.et64[(size_t)obs[0] * N + pp];  // init_prob: pi + b (hmm.rs:215-218)
  int t = 1;
  constexpr int U = 8;
  for (; t + U <= T; t += U) {
    int p[U], o[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      p[k] = path[t + k];
      o[k] = obs[t + k];
    }
    double av[U], bv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      av[k] = r.a64[(size_t)(k ? p[k - 1] : pp) * N + p[k]];
      bv[k] = r.et64[(size_t)o[k] * N + p[k]];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) d = (d + av[k]) + bv[k];  // (d + a) + b, viterbi.rs:15-17
    pp = p[U - 1];
  }
  for (; t < T; ++t) {
    const int p = path[t];
    d = (d + r.a64[(size_t)pp * N + p]) + r.et64[(size_t)obs[t] * N + p];
    pp = p;
  }
  r.score[seq] = d;
}

hipError_t launch_rescore_f64(const RescoreArgs& r, int64_t nseq, hipStream_t stream, int lds_reserve) {
  if (nseq <= 0) return hipSuccess;
  if (lds_reserve > 0) {  // overlap mode: at most one re-score wave per CU beside the forward pass
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&rescore_f64_lanes),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
  }
  hipLaunchKernelGGL(rescore_f64_lanes, dim3((unsigned)((nseq + 63) / 64)), dim3(64), (size_t)lds_reserve, stream,
                     r);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// Candidate loops of the generic kernels unrolled (round 5): with one load of A per candidate
// and the compare / select after it, the rolled loop waited for every load in turn -- a few
// sequences (the parallel chain's speculative re-decodes above N = 256) then ran at one L2
// round trip per candidate.  Only generic_fwd_ms<S = 1> in psi mode (a handful of sequences;
// large batches run S = 2 / 4 at full occupancy, and the unrolled rows mode, 84 vs 40 VGPRs,
// lost 37% at N = 600: profiles/r05_ab_generic_unroll.txt).  A/B: -DCVK_GEN_UNROLL=1.
#ifndef CVK_GEN_UNROLL
#define CVK_GEN_UNROLL 8
#endif

// Generic kernel: one workgroup (256 threads) per sequence, any N, f32/f64, all modes.
template <typename REAL>
__global__ __launch_bounds__(256) void generic_fwd(GenericFwdArgs<REAL> args) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  REAL* dbuf = reinterpret_cast<REAL*>(smem_raw);  // [2][N]
  const int N = args.nstates;
  const int64_t slot = args.seq_begin + blockIdx.x;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  if (T <= 0) return;
  const int32_t* obs = args.obs + e0;
  uint16_t* psi = args.psi + (e0 - args.psi_elem_base) * (int64_t)N;
  const REAL ninf = -__builtin_inf();
  const int V = args.nobs;
  const int assoc = args.assoc;
  int bad = 0;
  {
    const int o = obs[0];
    const bool ok = (unsigned)o < (unsigned)V;
    bad |= !ok;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      const REAL e = ok ? args.et[(size_t)o * N + j] : ninf;
      REAL d;
      if (assoc == CVK_ASSOC_DECODE)
        d = (REAL)0;
      else if (assoc == CVK_ASSOC_DP)
        d = (e > ninf) ? (REAL)(args.pi[j] + e) : ninf;
      else
        d = args.cp_init ? args.cp_init[seq] + (args.pi[j] + e) : args.pi[j] + e;
      if (args.forced && args.forced[e0] >= 0 && j != args.forced[e0]) d = ninf;
      dbuf[j] = d;
    }
  }
  __syncthreads();
  for (int t = 1; t < T; ++t) {
    const REAL* prev = dbuf + ((t - 1) & 1) * N;
    REAL* cur = dbuf + (t & 1) * N;
    const int o = obs[t];
    const bool ok = (unsigned)o < (unsigned)V;
    bad |= !ok;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      const REAL e = ok ? args.et[(size_t)o * N + j] : ninf;
      REAL best = ninf;
      int arg = 0;
      bool any = false;
      if (assoc == CVK_ASSOC_DP) {
        if (e > ninf) {
          for (int i = 0; i < N; ++i) {
            const REAL c = (args.a[(size_t)i * N + j] + e) + prev[i];
            if (c > best) {
              best = c;
              arg = i;
            }
          }
        }
        cur[j] = best;
      } else {
        for (int i = 0; i < N; ++i) {
          const REAL s = prev[i] + args.a[(size_t)i * N + j];
          if (!any || s > best) {
            best = s;
            arg = i;
            any = true;
          }
        }
        if (assoc == CVK_ASSOC_CP)
          cur[j] = prev[arg] + (args.a[(size_t)arg * N + j] + e);
        else
          cur[j] = best + e;
        if (assoc == CVK_ASSOC_DECODE && !(e > ninf)) {
          cur[j] = ninf;
          arg = 0;
        }
      }
      if (args.forced && args.forced[e0 + t] >= 0 && j != args.forced[e0 + t]) cur[j] = ninf;
      psi[(size_t)t * N + j] = (uint16_t)arg;
    }
    __syncthreads();
  }
  const REAL* last = dbuf + ((T - 1) & 1) * N;
  REAL* lastout = args.last_row + (slot - args.seq_begin) * (int64_t)N;
  for (int j = threadIdx.x; j < N; j += blockDim.x) lastout[j] = last[j];
  if (args.cp_last)
    for (int j = threadIdx.x; j < N; j += blockDim.x) args.cp_last[seq * N + j] = last[j];
  if (bad && threadIdx.x == 0) args.status[seq] = CVK_SEQ_BADOBS;
}

// generic_wide_step<REAL, S>: step t of the generic decode with each sequence's states spread
// over ceil(N / 256) workgroups, S consecutive slots per workgroup (each table element loaded
// once for the S), the rows in global memory (args.grows) -- where one workgroup per sequence
// would stream the N x N table (>= 134 MB at N = 4,096 f64) through a single CU every step.
// XCD-aware when the column blocks come in eights (xcd = 1): blocks b and b + 8 share an XCD
// (MI355X_MICROARCH.md: dealt round-robin), so block b takes column block jb = b % 8 + 8 k and
// each XCD's L2 serves a fixed eighth of the table's columns to every slot group; otherwise
// (xcd = 0) jb = b % nblk (padding to eights put every block of N <= 256 on one XCD: 165 us
// per step at 620 sequences).  The candidate loop keeps the previous rows on the scalar path and
// no barriers (the pipelined LDS-tile loop of wide.h, tried here: slower at few sequences,
// 6.7 vs 5.6 ms at N = 10,240 x 4).  The same candidates in the same order per state as generic_fwd
// (viterbi.rs:5-32, cp.rs:70-79, dp.rs, decode), so the same values, back-pointers and statuses
// bit for bit.  t = 0 seeds row 0; the step at t = T - 1 also writes the sequence's last row.
template <typename REAL, int S>
__global__ __launch_bounds__(256) void generic_wide_step(GenericFwdArgs<REAL> args, int t, int nblk, int xcd,
                                                        int64_t nslots) {
  const int N = args.nstates;
  int jb;
  int64_t grp;
  if (xcd) {
    const int64_t k = (int64_t)(blockIdx.x >> 3);
    jb = (int)(blockIdx.x & 7) + 8 * (int)(k % (nblk >> 3));
    grp = k / (nblk >> 3);
  } else {
    jb = (int)(blockIdx.x % (unsigned)nblk);
    grp = (int64_t)(blockIdx.x / (unsigned)nblk);
  }
  const int64_t g0 = grp * S;  // first local slot of the group
  const int j = jb * 256 + (int)threadIdx.x;
  if (j >= N) return;
  const REAL ninf = -__builtin_inf();
  const int assoc = args.assoc;
  int64_t seq[S], e0[S];
  int T[S];
  bool act[S], ok[S];
  REAL e[S];
  const REAL* prev[S];
  bool any = false;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t ls = g0 + s;
    act[s] = false;
    seq[s] = 0;
    e0[s] = 0;
    T[s] = 0;
    ok[s] = true;
    e[s] = ninf;
    prev[s] = args.grows;
    if (ls < nslots) {
      const int64_t slot = args.seq_begin + ls;
      seq[s] = args.order ? (int64_t)args.order[slot] : slot;
      e0[s] = args.offsets[seq[s]];
      T[s] = (int)(args.offsets[seq[s] + 1] - e0[s]);
      act[s] = t < T[s];
    }
    if (act[s]) {
      const int o = args.obs[e0[s] + t];
      ok[s] = (unsigned)o < (unsigned)args.nobs;
      e[s] = ok[s] ? args.et[(size_t)o * N + j] : ninf;
      prev[s] = args.grows + ls * 2 * N + ((t & 1) ^ 1) * N;
    }
    any |= act[s];
  }
  if (!any) return;
  const REAL* __restrict__ col = args.a + j;
  REAL d[S];
  int arg[S];
#pragma unroll
  for (int s = 0; s < S; ++s) arg[s] = 0;
  if (t == 0) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (assoc == CVK_ASSOC_DECODE)
        d[s] = (REAL)0;
      else if (assoc == CVK_ASSOC_DP)
        d[s] = (e[s] > ninf) ? (REAL)(args.pi[j] + e[s]) : ninf;
      else
        d[s] = args.cp_init ? args.cp_init[seq[s]] + (args.pi[j] + e[s]) : args.pi[j] + e[s];
    }
  } else if (assoc == CVK_ASSOC_DP) {
    // e = -inf: every candidate is -inf, the maximum stays -inf at index 0 (generic_fwd skips it)
#pragma unroll
    for (int s = 0; s < S; ++s) d[s] = ninf;
#pragma unroll 8
    for (int i = 0; i < N; ++i) {
      const REAL aij = col[(size_t)i * N];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const REAL c = (aij + e[s]) + prev[s][i];
        if (c > d[s]) {
          d[s] = c;
          arg[s] = i;
        }
      }
    }
  } else {
    REAL best[S];
#pragma unroll
    for (int s = 0; s < S; ++s) best[s] = prev[s][0] + col[0];  // i = 0 seeds the maximum (generic_fwd's `!any`)
#pragma unroll 8
    for (int i = 1; i < N; ++i) {
      const REAL aij = col[(size_t)i * N];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const REAL x = prev[s][i] + aij;
        if (x > best[s]) {
          best[s] = x;
          arg[s] = i;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      d[s] = assoc == CVK_ASSOC_CP ? prev[s][arg[s]] + (col[(size_t)arg[s] * N] + e[s]) : best[s] + e[s];
      if (assoc == CVK_ASSOC_DECODE && !(e[s] > ninf)) {
        d[s] = ninf;
        arg[s] = 0;
      }
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (!act[s]) continue;
    const int64_t ls = g0 + s;
    if (args.forced && args.forced[e0[s] + t] >= 0 && j != args.forced[e0[s] + t]) d[s] = ninf;
    args.grows[ls * 2 * N + (t & 1) * N + j] = d[s];
    if (t > 0) args.psi[(e0[s] - args.psi_elem_base + t) * (int64_t)N + j] = (uint16_t)arg[s];
    if (t == T[s] - 1) {
      args.last_row[ls * N + j] = d[s];
      if (args.cp_last) args.cp_last[seq[s] * N + j] = d[s];
    }
    if (!ok[s] && j == 0) args.status[seq[s]] = CVK_SEQ_BADOBS;
  }
}

// slots per wide workgroup: 4 once that still gives >= one workgroup per CU (256 CUs), else 1
// (S = 2 was never the fastest: profiles/r05_wide_crossover.txt); tuning key wide_s = k sets it
// (1, 2 or 4; A/B and tests, bit-identical)
inline int generic_wide_seqs(int n, int64_t nseq) {
  if (const int k = tuning().wide_s; k > 0) return k >= 4 ? 4 : k >= 2 ? 2 : 1;
  return (nseq + 3) / 4 * ((n + 255) / 256) >= 256 ? 4 : 1;
}

template <typename REAL, int S>
hipError_t launch_generic_wide_s(const GenericFwdArgs<REAL>& fa, int64_t nseq, hipStream_t stream) {
  const int nblk = (fa.nstates + 255) / 256;
  // XCD-aware column blocks when they come in eights (no measurable difference at N = 10,240,
  // 273.5 vs 273.3 ms; the CV_WIDE_XCD A/B knob was removed in round 6)
  const int xcd = nblk % 8 == 0 ? 1 : 0;
  const int64_t grid = (nseq + S - 1) / S * nblk;
  if (grid > (int64_t)INT32_MAX) return hipErrorInvalidValue;
  for (int64_t t = 0; t < fa.wide_steps; ++t) {
    hipLaunchKernelGGL((generic_wide_step<REAL, S>), dim3((unsigned)grid), dim3(256), 0, stream, fa, (int)t, nblk, xcd,
                       nseq);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

template <typename REAL>
hipError_t launch_generic_wide(const GenericFwdArgs<REAL>& fa, int64_t nseq, hipStream_t stream) {
  if (fa.rows || !fa.grows || fa.nstates > kGenericGlobalMaxStates) return hipErrorInvalidValue;
  switch (generic_wide_seqs(fa.nstates, nseq)) {
    case 4: return launch_generic_wide_s<REAL, 4>(fa, nseq, stream);
    case 2: return launch_generic_wide_s<REAL, 2>(fa, nseq, stream);
    default: return launch_generic_wide_s<REAL, 1>(fa, nseq, stream);
  }
}

bool generic_wide(int n, int real_bytes, int64_t nseq, bool cp) {
  if (n > generic_max_states(real_bytes)) return true;
  if (const int m = tuning().generic_wide_min; m > 0) return n >= m;  // tuning keys (A/B and tests)
  if (tuning().generic_wide == 0) return false;
  return n > 1024 && (cp || nseq < 4096 || n > 3072);
}

// generic_fwd_ms<REAL, S, ROWS>: S sequences per workgroup (consecutive slots of the
// longest-first schedule, so near-equal lengths), every A element loaded once for all S -- the
// one-sequence kernel above streams A from L2 once per sequence step and is bound by that
// stream -- and 64 * ceil(N / 64) threads (<= 1,024), one state each where N <= 1,024.
//   ROWS = false: argmax inline, u16 psi: same values, arguments and statuses as generic_fwd,
//                 bit for bit (the same candidates in the same order per sequence);
//   ROWS = true (VITERBI, DECODE, DP): the maximum only (add + max per candidate: a max is exact
//                 in any order) and every delta row stored; generic_bt_rows recomputes the
//                 first argmax along the path from those rows, so the paths equal generic_fwd's.
// A finished sequence's rows stay untouched.
template <typename REAL, int S, bool ROWS>
__global__ __launch_bounds__(1024) void generic_fwd_ms(GenericFwdArgs<REAL> args, int64_t nslots) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  REAL* dbuf = reinterpret_cast<REAL*>(smem_raw);  // [2][S][N]
  const int N = args.nstates;
  const int V = args.nobs;
  const int assoc = args.assoc;
  const REAL ninf = -__builtin_inf();
  // candidate loops unrolled in psi mode only (see CVK_GEN_UNROLL): a rolled walk waits out one
  // L2 latency per candidate.  Four-sequence workgroups too since round 5: psi CP at N = 300,
  // 8,192 x 128, forward 28.6 -> 25.5 ms; the chain's speculative batch at S = 4 21.0 -> 12.1
  // ms (profiles/r05_ab_unroll_s4.txt).  A/B builds: -DCVK_GEN_UNROLL_S=2 (or 1)
#ifndef CVK_GEN_UNROLL_S
#define CVK_GEN_UNROLL_S 4
#endif
  constexpr int kCandUnroll = (S <= CVK_GEN_UNROLL_S && !ROWS) ? CVK_GEN_UNROLL : 1;
  int64_t e0[S], slot[S], seq[S];
  int T[S];
  int Tmax = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t k = (int64_t)blockIdx.x * S + s;
    slot[s] = args.seq_begin + k;
    seq[s] = -1;
    T[s] = 0;
    e0[s] = 0;
    if (k < nslots) {
      seq[s] = args.order ? (int64_t)args.order[slot[s]] : slot[s];
      e0[s] = args.offsets[seq[s]];
      T[s] = (int)(args.offsets[seq[s] + 1] - e0[s]);
    }
    Tmax = T[s] > Tmax ? T[s] : Tmax;
  }
  if (Tmax <= 0) return;
  if (args.prio) __builtin_amdgcn_s_setprio(3);
  auto row = [&](int buf, int s) -> REAL* { return dbuf + ((size_t)buf * S + s) * N; };
  auto grow = [&](int s, int t) -> REAL* { return args.rows + (e0[s] + t - args.psi_elem_base) * (int64_t)N; };
  int bad = 0;  // bit s: sequence s saw an observation outside [0, V)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (T[s] <= 0) continue;
    const int o = args.obs[e0[s]];
    const bool ok = (unsigned)o < (unsigned)V;
    bad |= ok ? 0 : 1 << s;
    const int fs = args.forced ? args.forced[e0[s]] : -1;
    REAL* d0 = row(0, s);
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      const REAL e = ok ? args.et[(size_t)o * N + j] : ninf;
      REAL d;
      if (assoc == CVK_ASSOC_DECODE)
        d = (REAL)0;
      else if (assoc == CVK_ASSOC_DP)
        d = (e > ninf) ? (REAL)(args.pi[j] + e) : ninf;
      else
        d = args.cp_init ? args.cp_init[seq[s]] + (args.pi[j] + e) : args.pi[j] + e;
      if (fs >= 0 && j != fs) d = ninf;
      d0[j] = d;
      if constexpr (ROWS) grow(s, 0)[j] = d;
    }
  }
  __syncthreads();
  for (int t = 1; t < Tmax; ++t) {
    int o[S], fs[S];
    bool act[S], ok[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      act[s] = t < T[s];
      o[s] = act[s] ? args.obs[e0[s] + t] : 0;
      ok[s] = (unsigned)o[s] < (unsigned)V;
      if (act[s] && !ok[s]) bad |= 1 << s;
      fs[s] = (act[s] && args.forced) ? args.forced[e0[s] + t] : -1;
    }
    const int pb = (t - 1) & 1, cb = t & 1;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      REAL e[S], best[S];
      int arg[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        e[s] = ok[s] ? args.et[(size_t)o[s] * N + j] : ninf;
        best[s] = ninf;
        arg[s] = 0;
      }
      const REAL* col = args.a + j;
      if (assoc == CVK_ASSOC_DP) {
        bool live[S];  // a -inf emission leaves the column at -inf (dp.rs:147-177)
#pragma unroll
        for (int s = 0; s < S; ++s) live[s] = act[s] && e[s] > ninf;
        #pragma unroll kCandUnroll
        for (int i = 0; i < N; ++i) {
          const REAL aij = col[(size_t)i * N];
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const REAL c = (aij + e[s]) + row(pb, s)[i];
            if constexpr (ROWS) {
              best[s] = fmax(best[s], c);
            } else if (live[s] && c > best[s]) {
              best[s] = c;
              arg[s] = i;
            }
          }
        }
#pragma unroll
        for (int s = 0; s < S; ++s)
          if (act[s]) {
            REAL v = live[s] ? best[s] : ninf;
            if (fs[s] >= 0 && j != fs[s]) v = ninf;
            row(cb, s)[j] = v;
            if constexpr (ROWS)
              grow(s, t)[j] = v;
            else
              args.psi[(e0[s] + t - args.psi_elem_base) * (int64_t)N + j] = (uint16_t)arg[s];
          }
      } else {
        {  // i = 0 seeds the maximum (generic_fwd's `!any` case)
          const REAL a0 = col[0];
#pragma unroll
          for (int s = 0; s < S; ++s) best[s] = row(pb, s)[0] + a0;
        }
        #pragma unroll kCandUnroll
        for (int i = 1; i < N; ++i) {
          const REAL aij = col[(size_t)i * N];
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const REAL x = row(pb, s)[i] + aij;
            if constexpr (ROWS) {
              best[s] = fmax(best[s], x);
            } else if (x > best[s]) {
              best[s] = x;
              arg[s] = i;
            }
          }
        }
#pragma unroll
        for (int s = 0; s < S; ++s)
          if (act[s]) {
            REAL v;
            int ag = arg[s];
            if (!ROWS && assoc == CVK_ASSOC_CP)
              v = row(pb, s)[ag] + (col[(size_t)ag * N] + e[s]);
            else
              v = best[s] + e[s];
            if (assoc == CVK_ASSOC_DECODE && !(e[s] > ninf)) {
              v = ninf;
              ag = 0;
            }
            if (fs[s] >= 0 && j != fs[s]) v = ninf;
            row(cb, s)[j] = v;
            if constexpr (ROWS)
              grow(s, t)[j] = v;
            else
              args.psi[(e0[s] + t - args.psi_elem_base) * (int64_t)N + j] = (uint16_t)ag;
          }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (T[s] <= 0) continue;
    const REAL* last = row((T[s] - 1) & 1, s);
    REAL* lastout = args.last_row + (slot[s] - args.seq_begin) * (int64_t)N;
    for (int j = threadIdx.x; j < N; j += blockDim.x) lastout[j] = last[j];
    if (args.cp_last)
      for (int j = threadIdx.x; j < N; j += blockDim.x) args.cp_last[seq[s] * N + j] = last[j];
    if ((bad >> s) & 1 && threadIdx.x == 0) args.status[seq[s]] = CVK_SEQ_BADOBS;
  }
}

// generic_fwd_split<REAL, K>: generic_fwd_ms<REAL, 1, false> (one sequence per workgroup,
// u16 psi) with K threads per state.  A few sequences (the parallel chain's speculative
// re-decodes: ~600 at config-4 size) leave most of the chip idle, and each step is one thread's
// latency-bound walk over all N candidates; here thread (q, j) walks candidates
// [q C, (q + 1) C) of state j (C = ceil(N / K)) and thread (0, j) merges the K partial
// maxima in range order, taking a later range's only when strictly greater -- the first index
// of the maximum, as the sequential walk finds it -- so the values, arguments and statuses are
// generic_fwd_ms's bit for bit.  64 ceil(N / 64) K <= 1,024 threads.
template <typename REAL, int K>
__global__ __launch_bounds__(1024) void generic_fwd_split(GenericFwdArgs<REAL> args, int64_t nslots) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int N = args.nstates;
  const int NT = (int)blockDim.x / K;  // threads per range: 64 ceil(N / 64)
  REAL* dbuf = reinterpret_cast<REAL*>(smem_raw);  // [2][N]
  REAL* pbest = dbuf + 2 * (size_t)N;               // [K - 1][NT] partial maxima of ranges 1..K-1
  int* parg = reinterpret_cast<int*>(pbest + (size_t)(K - 1) * NT);  // [K - 1][NT] their arguments
  const int V = args.nobs;
  const int assoc = args.assoc;
  const REAL ninf = -__builtin_inf();
  const int64_t k = blockIdx.x;
  if (k >= nslots) return;
  const int64_t slot = args.seq_begin + k;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  if (T <= 0) return;  // workgroup-uniform
  const int q = (int)threadIdx.x / NT, j = (int)threadIdx.x - q * NT;
  const int C = (N + K - 1) / K, i0 = q * C, i1 = min(N, i0 + C);
  int bad = 0;
  {
    const int o = args.obs[e0];
    const bool ok = (unsigned)o < (unsigned)V;
    bad = ok ? 0 : 1;
    const int fs = args.forced ? args.forced[e0] : -1;
    if (q == 0 && j < N) {
      const REAL e = ok ? args.et[(size_t)o * N + j] : ninf;
      REAL d;
      if (assoc == CVK_ASSOC_DECODE)
        d = (REAL)0;
      else if (assoc == CVK_ASSOC_DP)
        d = (e > ninf) ? (REAL)(args.pi[j] + e) : ninf;
      else
        d = args.cp_init ? args.cp_init[seq] + (args.pi[j] + e) : args.pi[j] + e;
      if (fs >= 0 && j != fs) d = ninf;
      dbuf[j] = d;
    }
  }
  __syncthreads();
  for (int t = 1; t < T; ++t) {
    const int o = args.obs[e0 + t];
    const bool ok = (unsigned)o < (unsigned)V;
    if (!ok) bad = 1;
    const int fs = args.forced ? args.forced[e0 + t] : -1;
    const REAL* prow = dbuf + (size_t)((t - 1) & 1) * N;
    REAL* crow = dbuf + (size_t)(t & 1) * N;
    REAL e = ninf, best = ninf;
    int arg = 0;
    const REAL* col = args.a + (j < N ? j : 0);
    if (j < N) {
      e = ok ? args.et[(size_t)o * N + j] : ninf;
      if (assoc == CVK_ASSOC_DP) {
        const bool live = e > ninf;  // a -inf emission leaves the column at -inf (dp.rs:147-177)
        #pragma unroll 16
        for (int i = i0; i < i1; ++i) {
          const REAL c = (col[(size_t)i * N] + e) + prow[i];
          if (live && c > best) {
            best = c;
            arg = i;
          }
        }
      } else {
        int ib = i0;
        if (q == 0) {  // i = 0 seeds the maximum (generic_fwd's `!any` case)
          best = prow[0] + col[0];
          ib = 1;
        }
        #pragma unroll 16
        for (int i = ib; i < i1; ++i) {
          const REAL x = prow[i] + col[(size_t)i * N];
          if (x > best) {
            best = x;
            arg = i;
          }
        }
      }
      if (q > 0) {
        pbest[(size_t)(q - 1) * NT + j] = best;
        parg[(size_t)(q - 1) * NT + j] = arg;
      }
    }
    __syncthreads();
    if (q == 0 && j < N) {
#pragma unroll
      for (int r = 0; r < K - 1; ++r) {
        const REAL pb = pbest[(size_t)r * NT + j];
        if (pb > best) {
          best = pb;
          arg = parg[(size_t)r * NT + j];
        }
      }
      REAL v;
      int ag = arg;
      if (assoc == CVK_ASSOC_DP)
        v = (e > ninf) ? best : ninf;
      else if (assoc == CVK_ASSOC_CP)
        v = prow[ag] + (col[(size_t)ag * N] + e);
      else
        v = best + e;
      if (assoc == CVK_ASSOC_DECODE && !(e > ninf)) {
        v = ninf;
        ag = 0;
      }
      if (fs >= 0 && j != fs) v = ninf;
      crow[j] = v;
      args.psi[(e0 + t - args.psi_elem_base) * (int64_t)N + j] = (uint16_t)ag;
    }
    __syncthreads();
  }
  if (q == 0 && j < N) {
    const REAL* last = dbuf + (size_t)((T - 1) & 1) * N;
    args.last_row[(slot - args.seq_begin) * (int64_t)N + j] = last[j];
    if (args.cp_last) args.cp_last[seq * N + j] = last[j];
  }
  if (bad && threadIdx.x == 0) args.status[seq] = CVK_SEQ_BADOBS;
}

template <typename REAL>
__global__ __launch_bounds__(256) void generic_backtrack(GenericBtArgs<REAL> args) {
  const int lane = threadIdx.x & 63;
  const int64_t slot = args.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= args.seq_end) return;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  const int N = args.nstates;
  if (T <= 0) {
    if (lane == 0) {
      args.score[seq] = 0.0;
      args.status[seq] = CVK_SEQ_EMPTY;
    }
    return;
  }
  const REAL ninf = -__builtin_inf();
  const REAL* last = args.last_row + (slot - args.seq_begin) * (int64_t)N;
  double bv = (double)ninf;
  int bi = 0x7fffffff;
  for (int i = lane; i < N; i += 64) {
    const double v = (double)last[i];
    if (bi == 0x7fffffff || v > bv) {
      bv = v;
      bi = i;
    }
  }
  wave_argmax_first_d(bv, bi);
  int32_t* path = args.path + e0;
  const uint8_t prior = args.status[seq];
  if (!(bv > (double)ninf) || prior == CVK_SEQ_BADOBS) {
    if (args.decode_bt && prior != CVK_SEQ_BADOBS) {
      // viterbi::decode backtracks an infeasible sequence too: from argmax 0 of the all -inf
      // last row through bt (0 where the emission is -inf), viterbi.rs:19-21, 24-30
      if (lane == 0) {
        const uint16_t* psi = args.psi + (e0 - args.psi_elem_base) * (int64_t)N;
        int cs = bi;
        for (int t = T - 1; t >= 0; --t) {
          path[t] = cs;
          if (t > 0) cs = psi[(size_t)t * N + cs];
        }
      }
    } else {
      for (int t = lane; t < T; t += 64) path[t] = 0;
    }
    if (lane == 0) {
      args.score[seq] = -__builtin_inf();
      args.status[seq] = prior == CVK_SEQ_BADOBS ? CVK_SEQ_BADOBS : CVK_SEQ_INFEASIBLE;
    }
    return;
  }
  if (lane == 0) {
    const uint16_t* psi = args.psi + (e0 - args.psi_elem_base) * (int64_t)N;
    int cs = bi;
    for (int t = T - 1; t >= 0; --t) {
      path[t] = cs;
      if (t > 0) cs = psi[(size_t)t * N + cs];
    }
    args.status[seq] = CVK_SEQ_OK;
    if (!args.rescore_f64) args.score[seq] = bv;
  }
  if (args.rescore_f64) {
    const double d = rescore_path_f64(path, args.obs + e0, T, args.pi64, args.a64, args.et64, N, lane);
    if (lane == 0) args.score[seq] = d;
  }
}

// generic_bt_rows<REAL>: the backtrack of generic_fwd_ms<.., ROWS = true>, one wave per
// sequence.  At step t the predecessor of state s is the FIRST argmax over i of the forward's
// own candidate values, recomputed from the stored row t-1 and a^T[s][.] (coalesced):
// VITERBI / DECODE prev[i] + a[i][s] (index 0 when every candidate is -inf, and for DECODE
// when b_s(o_t) is -inf), DP (a[i][s] + b_s(o_t)) + prev[i] over the candidates above -inf
// (index 0 when none) -- exactly generic_fwd's psi.  Statuses, scores and the infeasible /
// bad-observation paths as generic_backtrack.
template <typename REAL>
__global__ __launch_bounds__(256) void generic_bt_rows(GenericBtArgs<REAL> args) {
  const int lane = threadIdx.x & 63;
  const int64_t slot = args.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot >= args.seq_end) return;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  const int N = args.nstates;
  if (T <= 0) {
    if (lane == 0) {
      args.score[seq] = 0.0;
      args.status[seq] = CVK_SEQ_EMPTY;
    }
    return;
  }
  const REAL ninf = -__builtin_inf();
  const REAL* last = args.last_row + (slot - args.seq_begin) * (int64_t)N;
  double bv = (double)ninf;
  int bi = 0x7fffffff;
  for (int i = lane; i < N; i += 64) {
    const double v = (double)last[i];
    if (bi == 0x7fffffff || v > bv) {
      bv = v;
      bi = i;
    }
  }
  wave_argmax_first_d(bv, bi);
  int32_t* path = args.path + e0;
  const uint8_t prior = args.status[seq];
  const bool feasible = bv > (double)ninf && prior != CVK_SEQ_BADOBS;
  if (!feasible && !(args.decode_bt && prior != CVK_SEQ_BADOBS)) {
    for (int t = lane; t < T; t += 64) path[t] = 0;
    if (lane == 0) {
      args.score[seq] = -__builtin_inf();
      args.status[seq] = prior == CVK_SEQ_BADOBS ? CVK_SEQ_BADOBS : CVK_SEQ_INFEASIBLE;
    }
    return;
  }
  const REAL* rows = args.rows + (e0 - args.psi_elem_base) * (int64_t)N;
  const int32_t* obs = args.obs + e0;
  const bool dp = args.assoc == CVK_ASSOC_DP, dec = args.assoc == CVK_ASSOC_DECODE;
  int cs = bi;
  for (int t = T - 1; t >= 0; --t) {
    if (lane == 0) path[t] = cs;
    if (t == 0) break;
    const REAL* prev = rows + (int64_t)(t - 1) * N;
    const REAL* ac = args.at + (size_t)cs * N;
    const int o = obs[t];
    const REAL e = (unsigned)o < (unsigned)args.nobs ? args.et[(size_t)o * N + cs] : ninf;
    double v = (double)ninf;
    int a = 0x7fffffff;
    if (dp) {
      if (e > ninf)
        for (int i = lane; i < N; i += 64) {
          const double c = (double)((ac[i] + e) + prev[i]);
          if (c > v) {
            v = c;
            a = i;
          }
        }
    } else {
      for (int i = lane; i < N; i += 64) {
        const double x = (double)(prev[i] + ac[i]);
        if (a == 0x7fffffff || x > v) {
          v = x;
          a = i;
        }
      }
    }
    wave_argmax_first_d(v, a);
    if (a == 0x7fffffff || (dec && !(e > ninf))) a = 0;
    cs = a;
  }
  if (!feasible) {  // viterbi::decode's infeasible walk (viterbi.rs:19-21, 24-30)
    if (lane == 0) {
      args.score[seq] = -__builtin_inf();
      args.status[seq] = CVK_SEQ_INFEASIBLE;
    }
    return;
  }
  if (lane == 0) {
    args.status[seq] = CVK_SEQ_OK;
    if (!args.rescore_f64) args.score[seq] = bv;
  }
  if (args.rescore_f64) {
    const double d = rescore_path_f64(path, args.obs + e0, T, args.pi64, args.a64, args.et64, N, lane);
    if (lane == 0) args.score[seq] = d;
  }
}

// ---------------------------------------------------------------------------------
// Max-marginal at one constrained position (constrained decode):
//   beta[i] = max_j(g[j] + a[i,j])   (g = last row of the reversed pass; 0 if no suffix)
//   mu[i]   = delta_tk[i] + beta[i]
// One workgroup of NP threads per constrained sequence; thread i reads at[j*NP + i] =
// a[i][j], coalesced across i.
template <int NP>
__global__ __launch_bounds__(NP) void max_marginal_f32(MaxMarginalArgs args) {
  __shared__ float g[NP];
  const int i = threadIdx.x;
  const int64_t c = blockIdx.x;
  const bool suffix = args.ranges_suffix[2 * c + 1] > args.ranges_suffix[2 * c];
  g[i] = suffix ? args.g[c * NP + i] : 0.f;
  __syncthreads();
  float beta = 0.f;
  if (suffix) {
    beta = ninf_f();
#pragma unroll 8
    for (int j = 0; j < NP; ++j) beta = fmaxf(beta, g[j] + args.at[(size_t)j * NP + i]);
  }
  args.mu[c * NP + i] = args.delta[c * NP + i] + beta;
}

template <int NP>
static hipError_t mm_np(const MaxMarginalArgs& a, int64_t ncon, hipStream_t stream) {
  hipLaunchKernelGGL(max_marginal_f32<NP>, dim3((unsigned)ncon), dim3(NP), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_max_marginal(int np, const MaxMarginalArgs& a, int64_t ncon, hipStream_t stream) {
  if (ncon <= 0) return hipSuccess;
#define CVK_MM(NP) mm_np<NP>(a, ncon, stream)
  switch (np) {
    case 32: return CVK_MM(32);
    case 64: return CVK_MM(64);
    case 96: return CVK_MM(96);
    case 128: return CVK_MM(128);
    case 160: return CVK_MM(160);
    case 192: return CVK_MM(192);
    case 224: return CVK_MM(224);
    case 256: return CVK_MM(256);
    default: return hipErrorInvalidValue;
  }
#undef CVK_MM
}

// ---------------------------------------------------------------------------------
// Host-side launchers (called from the C-ABI layer).  Forward and backtrack are launched
// separately so the host can run chunk k's backtrack beside chunk k+1's forward pass.
static bool ext_args(const TrellisFwdArgs& fa) {
  return fa.forced || fa.ranges || fa.reverse || fa.last_row || fa.start || !fa.delta || fa.split || fa.slot_order;
}

template <int NP>
static hipError_t trellis_fwd_np(const TrellisFwdArgs& fa, int64_t nseq, hipStream_t stream) {
  if (ext_args(fa))
    hipLaunchKernelGGL((trellis_fwd_f32<NP, true>), dim3((unsigned)nseq), dim3(NP * 4), 0, stream, fa);
  else
    hipLaunchKernelGGL((trellis_fwd_f32<NP, false>), dim3((unsigned)nseq), dim3(NP * 4), 0, stream, fa);
  return hipGetLastError();
}
// lds_reserve > 0: dynamic LDS the backtrack workgroup reserves but does not use, to cap how
// many of them share a CU with the forward kernel of the next chunk (overlap mode): a
// forward workgroup must always find its VGPRs free, or the pipeline stalls the forward.
template <int NP>
static hipError_t trellis_bt_np(const BacktrackArgs& ba, int64_t nseq, hipStream_t stream, int lds_reserve) {
  if (lds_reserve > 0) {
    static bool attr = false;  // allow the large dynamic-LDS reservation
    if (!attr) {
      if constexpr (NP % 64 == 0)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&backtrack_v_f32<NP>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      else
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&backtrack_f32<NP>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
  }
  if constexpr (NP % 64 == 0)
    hipLaunchKernelGGL(backtrack_v_f32<NP>, dim3((unsigned)((nseq + 3) / 4)), dim3(256), (size_t)lds_reserve, stream,
                       ba);
  else
    hipLaunchKernelGGL(backtrack_f32<NP>, dim3((unsigned)((nseq + 3) / 4)), dim3(256), (size_t)lds_reserve, stream,
                       ba);
  return hipGetLastError();
}

__global__ void scatter_forced(const int64_t* elems, const int32_t* states, int64_t n, int32_t* forced) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) forced[elems[k]] = states[k];
}

hipError_t launch_scatter_forced(const int64_t* elems, const int32_t* states, int64_t n, int32_t* forced,
                                 hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_forced, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, elems, states, n, forced);
  return hipGetLastError();
}

// First out-of-range observation in [lo, hi) (device API of the constrained decode, which
// must reject a bad batch before any term is computed, like the host API does): grid-stride
// scan, one u64 atomicMin per wave that saw one; *first stays INT64_MAX when all are valid.
__global__ void obs_first_bad(const int32_t* obs, int64_t lo, int64_t hi, uint32_t V,
                              unsigned long long* first) {
  unsigned long long mine = ~0ull;
  for (int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (int64_t)gridDim.x * blockDim.x)
    if ((uint32_t)obs[i] >= V && (unsigned long long)i < mine) mine = (unsigned long long)i;
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(mine, o);
    mine = other < mine ? other : mine;
  }
  if ((threadIdx.x & 63) == 0 && mine != ~0ull) atomicMin(first, mine);
}

hipError_t launch_obs_first_bad(const int32_t* obs, int64_t lo, int64_t hi, int64_t V, unsigned long long* first,
                                hipStream_t stream) {
  hipError_t e = hipMemsetAsync(first, 0xFF, sizeof(unsigned long long), stream);
  if (e != hipSuccess || hi <= lo) return e;
  const int64_t want = (hi - lo + 255) / 256, blocks = want < 4096 ? want : 4096;
  hipLaunchKernelGGL(obs_first_bad, dim3((unsigned)blocks), dim3(256), 0, stream, obs, lo, hi, (uint32_t)V, first);
  return hipGetLastError();
}

// ---- constrained decode, resume flow (cviterbi.cpp forced_decode_resume) ----------------
// The forced decode of a constrained sequence repeats, up to its first constrained element
// t_1, exactly the rows the terms pass's prefix computed (same adds, same max).  The terms
// pass stores those rows; the final decode then runs only [t_1, end) of such a sequence,
// starting from the stored row t_1 with the chosen state forced, and the prefix of the path
// is backtracked through the stored rows from that state.  Bit-identical to the full forced
// decode by construction (tests: CV_NO_RESUME A/B).
__global__ void resume_rows_build(const float* last, const int32_t* state, int np, float* out) {
  const int64_t i = blockIdx.x;
  const int j = threadIdx.x;
  if (j < np) out[i * np + j] = (j == state[i]) ? last[i * np + j] : ninf_f();
}

hipError_t launch_resume_rows(const float* last, const int32_t* state, int64_t n, int np, float* out,
                              hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (np <= 0 || np > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(resume_rows_build, dim3((unsigned)n), dim3(256), 0, stream, last, state, np, out);
  return hipGetLastError();
}

__global__ void compact_suffix(const int64_t* cstart, const int64_t* off2, const int32_t* obs, const int32_t* forced,
                               const int32_t* ridx, int32_t* obs2, int32_t* forced2) {
  const int64_t k = blockIdx.x;
  const int64_t e0 = cstart[k], o2 = off2[k], n = off2[k + 1] - o2;
  // forced2 == nullptr: observations only (the constrained decode's unconstrained sequences)
  const int r = ridx ? ridx[k] : -1;
  for (int64_t q = threadIdx.x; q < n; q += blockDim.x) {
    obs2[o2 + q] = obs[e0 + q];
    if (forced2) forced2[o2 + q] = (q == 0 && r >= 0) ? -2 - r : forced[e0 + q];
  }
}

hipError_t launch_compact_suffix(const int64_t* cstart, const int64_t* off2, const int32_t* obs, const int32_t* forced,
                                 const int32_t* ridx, int32_t* obs2, int32_t* forced2, int64_t nseq,
                                 hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(compact_suffix, dim3((unsigned)nseq), dim3(256), 0, stream, cstart, off2, obs, forced, ridx, obs2,
                     forced2);
  return hipGetLastError();
}

__global__ void scatter_suffix(const int64_t* cstart, const int64_t* off2, const int64_t* perm, const int32_t* path2,
                               const double* score2, const uint8_t* status2, int32_t* path, double* score,
                               uint8_t* status) {
  const int64_t k = blockIdx.x;
  const int64_t e0 = cstart[k], o2 = off2[k], n = off2[k + 1] - o2;
  for (int64_t q = threadIdx.x; q < n; q += blockDim.x) path[e0 + q] = path2[o2 + q];
  if (threadIdx.x == 0) {
    score[perm[k]] = score2[k];
    status[perm[k]] = status2[k];
  }
}

hipError_t launch_scatter_suffix(const int64_t* cstart, const int64_t* off2, const int64_t* perm,
                                 const int32_t* path2, const double* score2, const uint8_t* status2, int32_t* path,
                                 double* score, uint8_t* status, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(scatter_suffix, dim3((unsigned)nseq), dim3(256), 0, stream, cstart, off2, perm, path2, score2,
                     status2, path, score, status);
  return hipGetLastError();
}

// infeasible sequences: their whole path is 0 (backtrack_one's rule), prefix included
__global__ void zero_infeasible_prefix(PrefixBtArgs a, int64_t n) {
  const int64_t i = blockIdx.x;
  const int64_t seq = a.seq[i];
  if (a.status[seq] == CVK_SEQ_OK) return;
  const int64_t e0 = a.offsets[seq], e1 = a.t1[i];
  for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) a.path[e] = 0;
}

hipError_t launch_zero_infeasible_prefix(const PrefixBtArgs& a, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(zero_infeasible_prefix, dim3((unsigned)n), dim3(64), 0, stream, a, n);
  return hipGetLastError();
}

template <int NP>
__global__ __launch_bounds__(256) void prefix_backtrack(PrefixBtArgs a, int64_t n) {
  constexpr int VL = NP / 64;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t seq = a.seq[i];
  const int64_t e0 = a.offsets[seq];
  const int T = (int)(a.t1[i] - e0 + 1);
  // an infeasible forced row (-inf at the state) backtracks garbage: zero_infeasible_prefix
  // overwrites it once the suffix decode has told which sequences are infeasible
  BacktrackArgs b{};
  b.path = a.path;
  backtrack_one<VL, NP>(b, seq, e0, T, lane, a.rows + a.row_base[i] * NP + VL * lane, a.at + VL * lane, false,
                        a.state[i], false);
}

template <int NP>
static hipError_t prefix_bt_np(const PrefixBtArgs& a, int64_t n, hipStream_t stream, int lds_reserve) {
  static bool attr = false;  // allow the large dynamic-LDS reservation (see trellis_bt_np)
  if (lds_reserve > 0 && !attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&prefix_backtrack<NP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(prefix_backtrack<NP>, dim3((unsigned)((n + 3) / 4)), dim3(256), (size_t)lds_reserve, stream, a,
                     n);
  return hipGetLastError();
}

hipError_t launch_prefix_backtrack(int np, const PrefixBtArgs& a, int64_t n, hipStream_t stream, int lds_reserve) {
  if (n <= 0) return hipSuccess;
  switch (np) {
    case 128: return prefix_bt_np<128>(a, n, stream, lds_reserve);
    case 192: return prefix_bt_np<192>(a, n, stream, lds_reserve);
    case 256: return prefix_bt_np<256>(a, n, stream, lds_reserve);
    default: return hipErrorInvalidValue;
  }
}

int trellis_padded_states(int n) {
  if (n <= 0 || n > 256) return 0;
  return ((n + 31) / 32) * 32;
}

#define CVK_NP_SWITCH(np, CALL)     \
  switch (np) {                     \
    case 32: return CALL(32);       \
    case 64: return CALL(64);       \
    case 96: return CALL(96);       \
    case 128: return CALL(128);     \
    case 160: return CALL(160);     \
    case 192: return CALL(192);     \
    case 224: return CALL(224);     \
    case 256: return CALL(256);     \
    default: return hipErrorInvalidValue; \
  }

// one barrier per step: 79.5-80.8 vs 81.8-82.4 ms forward at config 4 f32, three interleaved
// rounds on one box (profiles/r05_ab_f32_onebar.txt)
constexpr bool kF32OneBarDefault = true;

template <int NP>
static hipError_t trellis_fwd2_np(const TrellisFwdArgs& fa, int64_t npairs, hipStream_t stream) {
  if constexpr (NP % 64 != 0) {
    return hipErrorInvalidValue;
  } else {
    if (fa.ranges || fa.reverse || fa.last_row || fa.start || !fa.delta) return hipErrorInvalidValue;
    // tuning key f32_onebar = 0 / 1 (bit-identical)
    const bool onebar = kF32OneBarDefault && tuning().f32_onebar != 0;
    const dim3 grid((unsigned)npairs), block(NP * 4);
    if (fa.forced && onebar)
      hipLaunchKernelGGL((trellis_fwd2_f32<NP, true, true>), grid, block, 0, stream, fa);
    else if (fa.forced)
      hipLaunchKernelGGL((trellis_fwd2_f32<NP, true, false>), grid, block, 0, stream, fa);
    else if (onebar)
      hipLaunchKernelGGL((trellis_fwd2_f32<NP, false, true>), grid, block, 0, stream, fa);
    else
      hipLaunchKernelGGL((trellis_fwd2_f32<NP, false, false>), grid, block, 0, stream, fa);
    return hipGetLastError();
  }
}

bool trellis_pair_supported(int np) { return np >= 64 && np <= 256 && np % 64 == 0; }

hipError_t launch_trellis_fwd2(int np, const TrellisFwdArgs& fa, int64_t npairs, hipStream_t stream) {
  if (npairs <= 0) return hipSuccess;
#define CVK_FWD2(NP) trellis_fwd2_np<NP>(fa, npairs, stream)
  CVK_NP_SWITCH(np, CVK_FWD2)
#undef CVK_FWD2
}

int trellis_wave_states(int n) { return (n >= 1 && n <= 64) ? (n + 15) / 16 * 16 : 0; }

hipError_t launch_trellis_wave(int npw, const TrellisFwdArgs& fa, const BacktrackArgs& ba, int64_t nseq,
                               hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  if (fa.ranges || fa.reverse || fa.last_row || fa.start || !fa.delta || fa.split || fa.slot_order)
    return hipErrorInvalidValue;
  const dim3 grid((unsigned)((nseq + 3) / 4));
#define CVK_WAVE(NPW)                                                                        \
  do {                                                                                       \
    if (fa.forced)                                                                           \
      hipLaunchKernelGGL((trellis_wave_f32<NPW, true>), grid, dim3(256), 0, stream, fa, ba); \
    else                                                                                     \
      hipLaunchKernelGGL((trellis_wave_f32<NPW, false>), grid, dim3(256), 0, stream, fa, ba); \
  } while (0)
  switch (npw) {
    case 16: CVK_WAVE(16); break;
    case 32: CVK_WAVE(32); break;
    case 48: CVK_WAVE(48); break;
    case 64: CVK_WAVE(64); break;
    default: return hipErrorInvalidValue;
  }
#undef CVK_WAVE
  return hipGetLastError();
}

hipError_t launch_trellis_fwd(int np, const TrellisFwdArgs& fa, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
#define CVK_FWD(NP) trellis_fwd_np<NP>(fa, nseq, stream)
  CVK_NP_SWITCH(np, CVK_FWD)
#undef CVK_FWD
}

hipError_t launch_trellis_bt(int np, const BacktrackArgs& ba, int64_t nseq, hipStream_t stream, int lds_reserve) {
  if (nseq <= 0) return hipSuccess;
#define CVK_BT(NP) trellis_bt_np<NP>(ba, nseq, stream, lds_reserve)
  CVK_NP_SWITCH(np, CVK_BT)
#undef CVK_BT
}

// sequences per workgroup of generic_fwd_ms: 4 while their rows fit the LDS and the launch
// keeps >= 2 workgroups per CU (256 CUs), else fewer; 1 = generic_fwd.  Tuning key generic_s = k
// sets it (1, 2 or 4 where the rows fit; A/B and tests, bit-identical)
template <typename REAL>
int generic_seqs_per_wg(int n, int64_t nseq) {
  auto fits = [&](int s) { return 2 * (size_t)s * n * sizeof(REAL) <= 160 * 1024; };
  if (const int k = tuning().generic_s; k > 0) {
    int s = k >= 4 ? 4 : k >= 2 ? 2 : 1;
    while (s > 1 && !fits(s)) s /= 2;
    return s;
  }
  int s = 4;
  while (s > 1 && (!fits(s) || nseq < (int64_t)s * 512)) s /= 2;
  return s;
}

template <typename REAL, int S, bool ROWS>
hipError_t launch_generic_ms(const GenericFwdArgs<REAL>& fa, int64_t nseq, hipStream_t stream) {
  const size_t lds = sizeof(REAL) * 2 * S * (size_t)fa.nstates;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&generic_fwd_ms<REAL, S, ROWS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  const unsigned threads = (unsigned)std::min(1024, (fa.nstates + 63) / 64 * 64);
  hipLaunchKernelGGL((generic_fwd_ms<REAL, S, ROWS>), dim3((unsigned)((nseq + S - 1) / S)), dim3(threads), lds,
                     stream, fa, nseq);
  return hipGetLastError();
}

template <typename REAL>
hipError_t launch_generic_fwd(const GenericFwdArgs<REAL>& fa_in, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  GenericFwdArgs<REAL> fa = fa_in;
  fa.prio = tuning().generic_prio == 1 ? 1 : 0;  // tuning key (issue priority only: bit-identical)
  if (fa.grows) return launch_generic_wide<REAL>(fa, nseq, stream);
  if (fa.rows) {  // rows mode: the maximum only (VITERBI / DECODE / DP)
    if (fa.assoc == CVK_ASSOC_CP || fa.nstates > generic_max_states((int)sizeof(REAL))) return hipErrorInvalidValue;
    switch (generic_seqs_per_wg<REAL>(fa.nstates, nseq)) {
      case 4: return launch_generic_ms<REAL, 4, true>(fa, nseq, stream);
      case 2: return launch_generic_ms<REAL, 2, true>(fa, nseq, stream);
      default: return launch_generic_ms<REAL, 1, true>(fa, nseq, stream);
    }
  }
  int s = generic_seqs_per_wg<REAL>(fa.nstates, nseq);
  // CP psi mode from 256 sequences on: two per workgroup (each A load serves both, the walk
  // unrolled) -- the chain's speculative batch (~620 sequences at N = 256) 11.9 -> 8.5 ms
  // (profiles/r05_ab_spec_s2.txt); below, one per workgroup keeps more of them in flight.  The
  // CP association only: the case that was measured
  if (s == 1 && nseq >= 256 && fa.assoc == CVK_ASSOC_CP && tuning().generic_s == 0 &&
      4 * (size_t)fa.nstates * sizeof(REAL) <= 160 * 1024)
    s = 2;
  switch (s) {
    case 4: return launch_generic_ms<REAL, 4, false>(fa, nseq, stream);
    case 2: return launch_generic_ms<REAL, 2, false>(fa, nseq, stream);
    default: break;
  }
  // one sequence per workgroup: one thread per state up to N = 1,024 (64 ceil(N / 64) threads;
  // generic_fwd's 256 threads walk 4 states each at N = 1,024 -- a handful of sequences, e.g.
  // the parallel chain's speculative re-decodes, then ran latency-bound on a few CUs).
  // tuning key generic_split = 1 (A/B and tests, bit-identical): K threads per state split
  // each state's candidates (generic_fwd_split) -- measured neutral on the chain's speculative
  // batch (12.4 vs 12.2 ms, profiles/r05_ab_spec_s.txt), so off by default
  {
    const int nt = (fa.nstates + 63) / 64 * 64;
    const bool split = tuning().generic_split == 1;
    // K: at most 512 threads per workgroup, so four workgroups fit a CU and a batch of ~1,000
    // sequences runs in one round (1,024-thread workgroups: two per CU, a second round at 620
    // sequences); tuning key generic_split_k = 2 / 4 / 8 sets it
    int K = tuning().generic_split_k > 0 ? tuning().generic_split_k : 512 / nt;
    K = K >= 8 ? 8 : K >= 4 ? 4 : K >= 2 ? 2 : 1;
    while (K > 1 && nt * K > 1024) K /= 2;
    if (split && K >= 2 && fa.nstates <= 512) {
      const size_t lds = sizeof(REAL) * 2 * (size_t)fa.nstates + (sizeof(REAL) + 4) * (size_t)(K - 1) * nt;
      auto go = [&](auto kern) {
        if (lds > 64 * 1024)
          (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)nseq), dim3((unsigned)(nt * K)), lds, stream, fa, nseq);
        return hipGetLastError();
      };
      if (K >= 8) return go(generic_fwd_split<REAL, 8>);
      if (K >= 4) return go(generic_fwd_split<REAL, 4>);
      return go(generic_fwd_split<REAL, 2>);
    }
  }
  if (fa.nstates <= 1024) return launch_generic_ms<REAL, 1, false>(fa, nseq, stream);
  const size_t lds = sizeof(REAL) * 2 * (size_t)fa.nstates;
  if (lds > 64 * 1024)  // N > 4096 (f64) / 8192 (f32): the two rows in up to 160 KiB of LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&generic_fwd<REAL>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(generic_fwd<REAL>, dim3((unsigned)nseq), dim3(256), lds, stream, fa);
  return hipGetLastError();
}
template <typename REAL>
hipError_t launch_generic_bt(const GenericBtArgs<REAL>& ba, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(generic_backtrack<REAL>, dim3((unsigned)((nseq + 3) / 4)), dim3(256), 0, stream, ba);
  return hipGetLastError();
}
template <typename REAL>
hipError_t launch_generic_bt_rows(const GenericBtArgs<REAL>& ba, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(generic_bt_rows<REAL>, dim3((unsigned)((nseq + 3) / 4)), dim3(256), 0, stream, ba);
  return hipGetLastError();
}
template hipError_t launch_generic_bt_rows<float>(const GenericBtArgs<float>&, int64_t, hipStream_t);
template hipError_t launch_generic_bt_rows<double>(const GenericBtArgs<double>&, int64_t, hipStream_t);
template hipError_t launch_generic_fwd<float>(const GenericFwdArgs<float>&, int64_t, hipStream_t);
template hipError_t launch_generic_fwd<double>(const GenericFwdArgs<double>&, int64_t, hipStream_t);
template hipError_t launch_generic_bt<float>(const GenericBtArgs<float>&, int64_t, hipStream_t);
template hipError_t launch_generic_bt<double>(const GenericBtArgs<double>&, int64_t, hipStream_t);

// Generic kernel keeps 2*N REAL delta values in LDS.
// generic_ext<S> (trellis.h): S consecutive slots per workgroup (a segment table's N slots
// share one range; the terms passes' slots are ragged and finish at their own lengths), each A
// element loaded once for the S slots, 64 * ceil(N / 64) threads (<= 1,024), the rows in LDS;
// an empty range writes nothing (the host never builds one).
template <int S>
__global__ __launch_bounds__(1024) void generic_ext(GenericExtArgs g, int64_t nslots) {
  extern __shared__ __attribute__((aligned(16))) double rows[];  // [2][S][N]
  const int N = g.nstates;
  const double ninf = -__builtin_inf();
  int64_t b0[S];
  int T[S];
  int Tmax = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int64_t slot = (int64_t)blockIdx.x * S + s;
    b0[s] = 0;
    T[s] = 0;
    if (slot < nslots) {
      b0[s] = g.ranges[2 * slot];
      T[s] = (int)(g.ranges[2 * slot + 1] - b0[s]);
    }
    Tmax = T[s] > Tmax ? T[s] : Tmax;
  }
  if (Tmax <= 0) return;
  auto row = [&](int buf, int s) -> double* { return rows + ((size_t)buf * S + s) * N; };
  auto elem = [&](int s, int t) -> int64_t { return g.reverse ? b0[s] + T[s] - 1 - t : b0[s] + t; };
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (T[s] <= 0) continue;
    const double* e = g.et + (size_t)g.obs[elem(s, 0)] * N;
    const int st = g.start ? g.start[(int64_t)blockIdx.x * S + s] : -1;
    const bool emit = !(g.noemit_last && T[s] == 1);
    for (int j = threadIdx.x; j < N; j += blockDim.x)
      row(0, s)[j] = st >= 0 ? (j == st ? 0.0 : ninf) : emit ? g.pi[j] + e[j] : g.pi[j];
  }
  __syncthreads();
  for (int t = 1; t < Tmax; ++t) {
    const int pb = (t - 1) & 1, cb = t & 1;
    const double* e[S];
    bool act[S], emit[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      act[s] = t < T[s];
      e[s] = act[s] ? g.et + (size_t)g.obs[elem(s, t)] * N : g.et;
      emit[s] = !(g.noemit_last && t == T[s] - 1);
    }
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      const double* col = g.tab + j;
      double m[S];
#pragma unroll
      for (int s = 0; s < S; ++s) m[s] = ninf;
      for (int i = 0; i < N; ++i) {
        const double aij = col[(size_t)i * N];
#pragma unroll
        for (int s = 0; s < S; ++s) m[s] = fmax(m[s], row(pb, s)[i] + aij);
      }
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (act[s]) row(cb, s)[j] = emit[s] ? m[s] + e[s][j] : m[s];
    }
    __syncthreads();
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (T[s] <= 0) continue;
    const double* last = row((T[s] - 1) & 1, s);
    double* out = g.last_row + ((int64_t)blockIdx.x * S + s) * N;
    for (int j = threadIdx.x; j < N; j += blockDim.x) out[j] = last[j];
  }
}

template <int S>
hipError_t launch_generic_ext_s(const GenericExtArgs& g, int64_t nslots, hipStream_t stream) {
  const size_t lds = 2 * (size_t)S * g.nstates * sizeof(double);
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&generic_ext<S>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  const unsigned threads = (unsigned)std::min(1024, (g.nstates + 63) / 64 * 64);
  hipLaunchKernelGGL((generic_ext<S>), dim3((unsigned)((nslots + S - 1) / S)), dim3(threads), lds, stream, g, nslots);
  return hipGetLastError();
}

// generic_ext wide: step t of every slot, the slot's states over nblk workgroups (block = slot
// x nblk + column block), its two rows in g.grows -- the constrained decode's terms passes and
// segment tables above N = 10,240.  Values only (an order-free maximum): generic_ext's rows bit
// for bit.
__global__ __launch_bounds__(256) void generic_ext_wide_step(GenericExtArgs g, int t, int nblk, int64_t nslots) {
  const int N = g.nstates;
  const int64_t slot = (int64_t)(blockIdx.x / (unsigned)nblk);
  const int j = (int)(blockIdx.x % (unsigned)nblk) * 256 + (int)threadIdx.x;
  if (slot >= nslots || j >= N) return;
  const int64_t b0 = g.ranges[2 * slot];
  const int T = (int)(g.ranges[2 * slot + 1] - b0);
  if (t >= T) return;
  const double ninf = -__builtin_inf();
  const int64_t el = g.reverse ? b0 + T - 1 - t : b0 + t;
  const double e = g.et[(size_t)g.obs[el] * N + j];
  const bool emit = !(g.noemit_last && t == T - 1);
  double* cur = g.grows + slot * 2 * N + (t & 1) * N;
  double v;
  if (t == 0) {
    const int st = g.start ? g.start[slot] : -1;
    v = st >= 0 ? (j == st ? 0.0 : ninf) : emit ? g.pi[j] + e : g.pi[j];
  } else {
    const double* prev = g.grows + slot * 2 * N + ((t & 1) ^ 1) * N;
    const double* col = g.tab + j;
    double m = ninf;
#pragma unroll 8
    for (int i = 0; i < N; ++i) m = fmax(m, prev[i] + col[(size_t)i * N]);
    v = emit ? m + e : m;
  }
  cur[j] = v;
  if (t == T - 1) g.last_row[slot * N + j] = v;
}

bool generic_ext_wide(int n) {
  if (n > generic_max_states(8)) return true;
  const int m = tuning().ext_wide_min;  // tuning key (A/B and tests)
  return m > 0 && n >= m;
}

hipError_t launch_generic_ext(const GenericExtArgs& g, int64_t nslots, hipStream_t stream) {
  if (nslots <= 0) return hipSuccess;
  if (g.grows) {
    if (g.nstates <= 0 || g.nstates > kGenericGlobalMaxStates) return hipErrorInvalidValue;
    const int nblk = (g.nstates + 255) / 256;
    if (nslots * nblk > (int64_t)INT32_MAX) return hipErrorInvalidValue;
    for (int64_t t = 0; t < g.wide_steps; ++t) {
      hipLaunchKernelGGL(generic_ext_wide_step, dim3((unsigned)(nslots * nblk)), dim3(256), 0, stream, g, (int)t, nblk,
                         nslots);
      const hipError_t err = hipGetLastError();
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  if (g.nstates <= 0 || g.nstates > generic_max_states(8)) return hipErrorInvalidValue;
  // as generic_fwd_ms: 4 slots while their rows fit and the launch keeps >= 2 workgroups per
  // CU, CV_GENERIC_S=k sets it
  switch (generic_seqs_per_wg<double>(g.nstates, nslots)) {
    case 4: return launch_generic_ext_s<4>(g, nslots, stream);
    case 2: return launch_generic_ext_s<2>(g, nslots, stream);
    default: return launch_generic_ext_s<1>(g, nslots, stream);
  }
}

int generic_max_states(int real_bytes) { return (int)(160 * 1024 / (2 * real_bytes)); }

}  // namespace cvk
