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

#include <algorithm>
#include <cstdlib>

#include "trellis.h"
#include "trellis64.h"
#include "wave64.h"
#include "wide.h"
#include "../tuning.h"

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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
// constant address space: wave-uniform loads through these become s_load (SMEM), off the
// in-order vmcnt queue that the A-row ring lives in
template <typename T>
using sptr = const __attribute__((address_space(4))) T*;
template <typename T>
__device__ __forceinline__ sptr<T> scalar_view(const T* p) {
  return (sptr<T>)p;
}


// C f64 as two planes of C words each (dwordx4 / dwordx2 stores), non-temporal
template <int C>
__device__ __forceinline__ void store_split(uint32_t* hi, uint32_t* lo, const double (&v)[C]) {
  if constexpr (C % 4 == 0) {
#pragma unroll
    for (int c = 0; c < C; c += 4) {
      u32x4 h = {hi_word(v[c]), hi_word(v[c + 1]), hi_word(v[c + 2]), hi_word(v[c + 3])};
      u32x4 l = {lo_word(v[c]), lo_word(v[c + 1]), lo_word(v[c + 2]), lo_word(v[c + 3])};
      __builtin_nontemporal_store(h, reinterpret_cast<u32x4*>(hi + c));
      __builtin_nontemporal_store(l, reinterpret_cast<u32x4*>(lo + c));
    }
  } else if constexpr (C % 2 == 0) {
#pragma unroll
    for (int c = 0; c < C; c += 2) {
      u32x2 h = {hi_word(v[c]), hi_word(v[c + 1])};
      u32x2 l = {lo_word(v[c]), lo_word(v[c + 1])};
      __builtin_nontemporal_store(h, reinterpret_cast<u32x2*>(hi + c));
      __builtin_nontemporal_store(l, reinterpret_cast<u32x2*>(lo + c));
    }
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      __builtin_nontemporal_store(hi_word(v[c]), hi + c);
      __builtin_nontemporal_store(lo_word(v[c]), lo + c);
    }
  }
}

// The lane's C consecutive f64 of table row `row` through a buffer descriptor: the row offset
// is a scalar (soffset), the lane offset a constant VGPR, so the ring refills cost no VALU
// address arithmetic (64-bit flat addresses cost 2 VALU per load).
template <int C>
__device__ __forceinline__ void load_row_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double (&a)[C]) {
  if constexpr (C % 2 == 0) {
#pragma unroll
    for (int c = 0; c < C / 2; ++c) {
      const f64x2 v = __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16 * c, soff, 0));
      a[2 * c] = v.x;
      a[2 * c + 1] = v.y;
    }
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c)
      a[c] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff + 8 * c, soff, 0));
  }
}

// trellis_fwd_f64<C, S, PF, DPA, EXT>: S sequences per wave in lock step (see the file
// header).  The A-row ring is CONTINUOUS across time steps: the refill after row i loads row
// (i + PF) mod NP, so the first PF rows of step t+1 are in flight during the last rows of
// step t (A is the same matrix every step) and no step starts on an empty pipeline.
// Observations (and forced states) are scalar loads issued one step ahead; the step's
// emission rows are loaded together in the epilogue (one exposed L2 round trip per step).
// Built with -fno-honor-nans (no NaN can occur: NaN / +inf inputs are rejected), so fmax is
// a bare v_max_f64 (IEEE-mode maxnum would otherwise canonicalise loop-carried operands).
//
// DPA: DPSolver's association (dp.rs:147-177): d'[j] = max_i ((a[i,j] + b[j,o]) + d[i]); the
// emission enters every candidate, so it is loaded before the row loop (S <= 4: registers).
// EXT: the constrained decode's passes -- forced states, explicit element ranges (sequence id
// = slot), reversed traversal (the suffix pass runs on a^T with pi = 0), final-row output,
// per-slot start state (segment tables), compact delta rows (row_base), resume rows and a
// longest-first slot order.
// W: waves per workgroup splitting the NP = 64*C*W columns.  W = 2 (C = 2 at N = 256) is the
// small-batch layout: when S = 8 sequences per wave cannot give every SIMD two waves, S = 8
// sequences per PAIR of waves keeps the wave count of S = 4 with twice its A-row reuse (8,192
// sequences, 8-GPU strong scaling: profiles/r02_t64_small_batch.txt).  The W waves run the
// same S sequences, share delta_{t-1} in LDS and meet at two barriers per step (before
// overwriting delta_{t-1}, after writing delta_t).  At full batches W = 1 is faster (the VALU
// is saturated either way and W = 2 runs at a lower clock, profiles/r02_ab_fwd_w2.txt).
// per-SIMD progress table of trellis_fwd_f64's balancing: [XCC][SE][SH][CU][SIMD][wave slot]
// remaining steps (0 = empty); zero-initialised with the code object, every wave clears its slot
__device__ int g_t64_simd[16 * 8 * 2 * 16 * 4 * 16];

// SIMD balancing (T64FwdArgs::balance).  The arbiter issues the OLDEST of equal-priority waves
// first, so of a SIMD's waves one finishes far ahead and the last one then runs alone at the
// much lower one-wave issue rate (one round of 2,048 waves at 8,192 sequences: wave durations
// 12.9 .. 20.9 ms; balanced 18.3 .. 19.5 ms, tools/debug/t64_probe.py).  Each wave publishes
// its remaining steps in g_t64_simd[its SIMD][its wave slot] (HW_ID / XCC_ID) and runs at
// priority 3 only while no other wave of its SIMD has more work left, else 1: the waves of a
// SIMD finish together.  The words go through L2 (agent-scope relaxed atomics: vector memory
// operations that bypass the CU's L1); a slot is 0 when empty, so a stale word only mis-sets a
// priority, never a result.
struct SimdBalance {
  int* tab = nullptr;
  int slot = 0;
  __device__ void init(int enabled, int lane, int remaining) {
    if (!enabled) return;
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    const unsigned key = ((((xc & 15) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15)) * 4 +
                         ((hw >> 4) & 3);
    tab = g_t64_simd + (size_t)key * 16;
    slot = (int)(hw & 15);
    publish(lane, remaining);
  }
  __device__ void publish(int lane, int remaining) const {
    if (lane == 0) __hip_atomic_store(tab + slot, remaining, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // lane k < 16: the remaining steps of wave slot k of this SIMD (0 for this wave's own slot)
  __device__ int others(int lane) const {
    return (lane < 16 && lane != slot) ? __hip_atomic_load(tab + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  }
  __device__ void decide(int other, int remaining) const {
    int m = other;
#pragma unroll
    for (int k = 0; k < 16; ++k) m = max(m, __builtin_amdgcn_readlane(other, k));
    if (remaining >= m)
      __builtin_amdgcn_s_setprio(3);
    else
      __builtin_amdgcn_s_setprio(1);
  }
  __device__ void finish(int lane) const {
    if (tab) publish(lane, 0);
  }
};
#ifdef CV_T64_PROBE
// debug build only: per wave {real-time start, end, s_memtime start, end, HW_ID, XCC_ID}
__device__ uint64_t g_t64_probe[1 << 17][6];
#endif
// MINW: waves per SIMD the register allocation must allow (3: <= 168 VGPRs)
// WG: independent units per workgroup, each of W waves with its own S sequences and LDS slice
// (W * WG = 8: the CU's whole complement, two waves per SIMD).  SYNC bit 1: a workgroup barrier
// per step; bit 2: the two waves of a SIMD (waves i and i ^ 4 of the workgroup) trade issue
// priority every PF rows so that the one behind leads.  Together they keep the CU's waves on
// the same A rows, so 8 waves share each row through the L1 (L1 -> L2 read requests per L1
// access 0.44 -> 0.09 at config 4; profiles/r03_ab_wg.txt).  W > 1 units meet at workgroup
// barriers anyway (their pair rendezvous), so they take bit 2 only.
template <int C, int S, int PF, bool DPA, bool EXT, int W = 1, bool CAP2 = (W > 1), int GRP = 2, int MINW = 1,
          bool LDSFIRST = true, int WG = 1, int SYNC = 0, bool DEFST = false, bool PERSIST = false>
__global__ __launch_bounds__(64 * W * WG) __attribute__((amdgpu_waves_per_eu(MINW))) void trellis_fwd_f64(T64FwdArgs g) {
#ifdef CV_T64_PROBE
  const uint64_t pr_rt0 = __builtin_amdgcn_s_memrealtime(), pr_c0 = __builtin_amdgcn_s_memtime();
  struct ProbeEnd {
    uint64_t rt0, c0;
    __device__ ~ProbeEnd() {
      const unsigned idx = (blockIdx.x * W * WG + (threadIdx.x >> 6)) & ((1u << 17) - 1);
      if ((threadIdx.x & 63) == 0) {
        uint64_t* p = g_t64_probe[idx];
        p[0] = rt0;
        p[1] = __builtin_amdgcn_s_memrealtime();
        p[2] = c0;
        p[3] = __builtin_amdgcn_s_memtime();
        p[4] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        p[5] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
      }
    }
  } pr_end{pr_rt0, pr_c0};
#endif
  constexpr int NP = 64 * C * W;
  static_assert(S % 2 == 0, "S sequences are read from LDS two at a time");
  static_assert(NP % PF == 0, "the ring wraps around at row NP");
  // delta rows in flight ahead of their use: 1 (W = 1: 212 VGPRs already) or 3 (W = 2, the
  // small-batch layout: 32 VALU per row leave too little time for one LDS round trip)
  constexpr int DV = W > 1 ? 4 : 2;
  static_assert(PF % DV == 0, "the delta-row ring must wrap with the A-row ring");
  // delta_{t-1}: [row][S]; rows NP .. NP+DV-2 are padding, read (and ignored) by the prefetch
  static_assert(WG == 1 || W * WG == 8, "units per workgroup: the CU's eight waves");
  // DEFST: delta row t-1 is stored during step t, one sequence pair per quarter of the row loop,
  // read back from the LDS slice (spreads the 2S stores of a step over it)
  static_assert(!DEFST || (W == 1 && !EXT), "deferred stores: batch decode, one-wave units");
  // each lane's C rows are followed by 16 bytes of padding (C a power of two): the lane stride
  // C*S*8 + 16 B puts the 16 lanes of an epilogue ds_write_b128 on distinct banks (without it
  // every lane of the wave hit the same four banks); broadcast reads are unaffected
  constexpr bool PADL = (C & (C - 1)) == 0;
  constexpr int kPadGroups = PADL ? (NP + DV - 1 + C - 1) / C : 0;
  __shared__ __attribute__((aligned(16))) double dl_all[WG][(NP + DV - 1) * S + 2 * kPadGroups];
  __shared__ int wg_prog[W * WG];  // each wave's Tmax, then its progress (step * NP + row block)
  const int lane = threadIdx.x & 63;
  const int wid = (W * WG > 1) ? __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) : 0;
  const int wv = W > 1 ? wid % W : 0;
  const int wgi = WG > 1 ? wid / W : 0;
  double* const dl = dl_all[wgi];
  auto rowp = [&](int i) -> double* { return dl + i * S + (PADL ? (i / C) * 2 : 0); };
  const int j0 = (wv * 64 + lane) * C;
  const double ninf = ninf_d();
  // workgroup rendezvous without the global-memory drain of __syncthreads (the A-row ring and
  // the delta stores stay in flight): only this wave's LDS operations are waited for
  auto wg_sync = [&]() {
#ifndef CVK_ABL_NOBAR  // ablation build (timing only): no pair rendezvous
    if constexpr (W > 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
    if constexpr (W > 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
  };
  // W > 1 runs single-round small batches: reserve > 170 VGPRs so a SIMD holds at most two of
  // these waves and every SIMD gets two (at ~150 VGPRs three fit, and a round that puts three
  // on some SIMDs and one on others takes 1.5x as long)
  if constexpr (CAP2) asm volatile("" ::: "v180");

  static_assert(!PERSIST || (W == 1 && WG == 1 && EXT), "work queue: one-wave EXT units");
  // one unit = S consecutive slots; PERSIST: the wave runs units taken from a queue (below)
  auto run_unit = [&](const int64_t unit) {
  // Per-sequence bookkeeping lives in LANE s of a few VGPRs (lanes >= S idle) rather than in
  // S-element scalar arrays (those exceed the 102 SGPRs at S = 8 and spill): each step lane s
  // loads the observation (and forced state) of sequence s one step ahead, and the values a
  // step needs uniformly are read back with v_readlane.
  const int ls = lane < S ? lane : S - 1;
  const int64_t my_k = (unit * WG + wgi) * S + ls;
  int my_T = 0;
  int64_t my_seq = -1, my_eb = 0, my_rb = 0;
  if (my_k < g.nslots && lane < S) {
    const int64_t sl = (EXT && g.slot_order) ? (int64_t)g.slot_order[my_k] : g.seq_begin + my_k;
    int64_t e0;
    if (EXT && g.ranges) {
      my_seq = sl;
      e0 = g.ranges[2 * sl];
      my_T = (int)(g.ranges[2 * sl + 1] - e0);
    } else {
      my_seq = g.order ? (int64_t)g.order[sl] : sl;
      e0 = g.offsets[my_seq];
      my_T = (int)(g.offsets[my_seq + 1] - e0);
    }
    my_eb = (EXT && g.reverse) ? e0 + my_T - 1 : e0;
    my_rb = (EXT && g.row_base) ? g.row_base[sl] : e0 - g.delta_elem_base;
  }
  const int64_t my_slot = (EXT && g.slot_order && my_k < g.nslots) ? (int64_t)g.slot_order[my_k] : g.seq_begin + my_k;
  int T[S];
  int Tmax = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    T[s] = __builtin_amdgcn_readlane(my_T, s);
    Tmax = T[s] > Tmax ? T[s] : Tmax;
  }
  // Barriers are workgroup-wide once a workgroup holds several units: every wave then takes
  // part in the workgroup's barriers up to the longest unit's last step (a wave with less work
  // idles at them), so no barrier waits on a finished wave
  constexpr bool kWgBar = WG > 1 && ((SYNC & 1) || W > 1);
  // barriers per step: the pair rendezvous (W > 1: 2) or the step barrier (SYNC & 1)
  constexpr int kStepBarriers = W > 1 ? 2 : ((SYNC & 1) ? 1 : 0);
  int Twg = Tmax;
  if constexpr (kWgBar) {
    if (lane == 0) wg_prog[wid] = Tmax;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < W * WG; ++k) Twg = max(Twg, wg_prog[k]);
    __syncthreads();
  }
  if constexpr (WG > 1 && (SYNC & 2)) {
    if (lane == 0) wg_prog[wid] = 0;
  }
  if (Tmax <= 0) {
    if constexpr (kWgBar) {
      if (Twg > 0) {
        if constexpr (W > 1) asm volatile("s_barrier" ::: "memory");  // delta_0's rendezvous
        for (int t = 1; t < Twg; ++t)
          for (int k = 0; k < kStepBarriers; ++k) asm volatile("s_barrier" ::: "memory");
      }
    }
    return;
  }
  const int dir = (EXT && g.reverse) ? -1 : 1;
  const unsigned V = (unsigned)g.nobs;
  // lanes without a sequence read the first element of some sequence of the wave, so every
  // per-step load is unconditional (a load under an exec mask, waited for at once, would
  // drain the A-row ring: vmcnt is in order)
  {
    const unsigned long long live = __ballot(my_T > 0);
    const int l0 = __builtin_ctzll(live);  // Tmax > 0: some lane is live
    const int64_t eb0 = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my_eb, l0) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(my_eb >> 32), l0) << 32));
    if (my_T <= 0) my_eb = eb0;
  }
  const int my_Tc = my_T > 0 ? my_T : 1;
  bool my_bad = false;  // lane s: sequence s saw an out-of-range observation
  // lane s: raw observation of step t of sequence s (index clamped into the sequence); the
  // range check happens when the value is used, one step later (obs_use)
  auto obs_lane = [&](int t) -> unsigned {
    return (unsigned)g.obs[my_eb + (int64_t)dir * (t < my_Tc ? t : my_Tc - 1)];
  };
  auto obs_use = [&](unsigned o, int t) -> unsigned {
    my_bad = my_bad || (t < my_T && o >= V);
    return o < V ? o : 0u;
  };
  const int32_t* fsrc = (EXT && g.forced) ? g.forced : g.obs;
  auto frc_lane = [&](int t) -> int {
    if constexpr (!EXT) return -1;
    return fsrc[my_eb + (int64_t)dir * (t < my_Tc ? t : my_Tc - 1)];
  };
  auto frc_use = [&](int f) -> int { return (EXT && g.forced && my_T > 0) ? f : -1; };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g.a), 0, NP * NP * 8, 0x00020000);
  const uint32_t voff = (uint32_t)j0 * 8;
  constexpr uint32_t RB = NP * 8;  // bytes per table row
  // emission row of observation o (wave-uniform; the padded columns of the table are -inf)
  auto emis = [&](unsigned o, double (&e)[C]) {
    const double* row = g.et + (size_t)o * NP + j0;
    load_a<C>(row, e);
  };
  auto store_row = [&](int s, int t, const double (&v)[C]) {
    const int64_t r = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my_rb, s) |
                                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(my_rb >> 32), s) << 32));
#ifdef CVK_ABL_NOSTORE  // ablation build (timing only): no delta-row stores
    if (false) {
#else
    // EXT: a negative row base keeps no rows for that slot (wave-uniform)
    if (g.delta && t < T[s] && (!EXT || r >= 0)) {
#endif
      // split-plane row (see T64 row layout in trellis64.h): hi words [0, NP), lo words
      // [NP, 2 NP); streaming stores (read once, by the backtrack)
#ifndef CVK_ABL_STORE_L2
      uint32_t* dst = reinterpret_cast<uint32_t*>(g.delta) + (r + t) * (2 * NP) + j0;
#else  // ablation build (timing only): every step of a sequence overwrites its first row (L2-resident)
      uint32_t* dst = reinterpret_cast<uint32_t*>(g.delta) + r * (2 * NP) + j0;
#endif
      store_split<C>(dst, dst + NP, v);
    }
    if (EXT && g.last_row && t == T[s] - 1) {
      const int64_t k = (int64_t)__builtin_amdgcn_readlane((int)(uint32_t)(my_slot - g.seq_begin), s);
      double* dst = g.last_row + k * NP + j0;
#pragma unroll
      for (int c = 0; c < C; ++c) dst[c] = v[c];
    }
  };
  // DEFST: rows r of sequences 2 s2, 2 s2 + 1 from the LDS slice (which holds delta_r)
  auto deferred_store = [&](int s2, int r) {
    double v0[C], v1[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const f64x2 w = *reinterpret_cast<const f64x2*>(rowp(j0 + c) + 2 * s2);
      v0[c] = w.x;
      v1[c] = w.y;
    }
    store_row(2 * s2, r, v0);
    store_row(2 * s2 + 1, r, v1);
  };
  // forced state f >= 0: every other state of that element is impossible
  auto force = [&](double (&v)[C], int f) {
    if (EXT && f >= 0) {
#pragma unroll
      for (int c = 0; c < C; ++c) v[c] = (j0 + c == f) ? v[c] : ninf;
    }
  };

  // ---- t = 0: d0 = pi + b[:, o0] (hmm.rs:215-218, cp.rs:66-68) ----
  unsigned onext_l;  // lane s: observation of the next step
  int fnext_l;
  {
    const unsigned o0 = obs_use(obs_lane(0), 0);
    const int f0l = frc_use(frc_lane(0));
    const int st_l = (EXT && g.start && my_T > 0) ? g.start[my_slot - g.seq_begin] : -1;
    double e[S][C];
#pragma unroll
    for (int s = 0; s < S; ++s) emis((unsigned)__builtin_amdgcn_readlane((int)o0, s), e[s]);
#pragma unroll
    for (int s = 0; s < S; ++s) {
      double v[C];
#pragma unroll
      for (int c = 0; c < C; ++c)
        v[c] = g.zero_init ? 0.0 : (EXT && g.noemit_last && T[s] == 1) ? g.pi[j0 + c] : g.pi[j0 + c] + e[s][c];
      if (EXT && g.start) {  // segment table: start in state st with score 0 (cfn.rs:11-34 pattern)
        const int st = __builtin_amdgcn_readlane(st_l, s);
        if (st >= 0) {
#pragma unroll
          for (int c = 0; c < C; ++c) v[c] = (j0 + c == st) ? 0.0 : ninf;
        }
      }
      int f0 = __builtin_amdgcn_readlane(f0l, s);
      if (EXT && f0 <= -2) {  // resume: row t_1 of the prefix pass, already forced
        const double* rr = g.resume_rows + (size_t)(-2 - f0) * NP + j0;
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = rr[c];
        f0 = -1;
      }
      force(v, f0);
#pragma unroll
      for (int c = 0; c < C; ++c) rowp(j0 + c)[s] = v[c];
      if constexpr (!DEFST) store_row(s, 0, v);
    }
    onext_l = obs_lane(1);
    fnext_l = frc_lane(1);
  }
  wg_sync();  // every wave's columns of delta_0 are in LDS

  // forward waves win issue arbitration over co-resident backtrack waves of the previous
  // chunk (overlap mode), as in trellis_fwd2_f32
  __builtin_amdgcn_s_setprio(3);
  double ar[PF][C];  // the A-row ring: ar[u] holds row i0 + u
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    load_row_buf<C>(ra, voff, u * RB, ar[u]);
    // keep the priming loads in ring order: the waitcnt pass then counts row u as 2(PF-u)-1
    // loads old at the loop head (scheduled out of order it fell back to vmcnt(0) there)
    __builtin_amdgcn_sched_barrier(0);
  }
  double acc[C][S];
  // SIMD balancing (SimdBalance): every g.balance steps
  const int bal = g.balance;
  SimdBalance sb;
  sb.init(bal > 0, lane, Tmax - 1);
  for (int t = 1; t < Tmax; ++t) {
    const unsigned ocur_l = obs_use(onext_l, t);
    const int fcur_l = frc_use(fnext_l);
    double ecur[DPA ? S : 1][C];
    if constexpr (DPA) {
#pragma unroll
      for (int s = 0; s < S; ++s) emis((unsigned)__builtin_amdgcn_readlane((int)ocur_l, s), ecur[s]);
    }
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int s = 0; s < S; ++s) acc[c][s] = ninf;
    // delta rows in a DV-slot register ring (dv[u % DV] = row i): the broadcast reads of rows
    // i+1 .. i+DV-1 are in flight while row i computes
    f64x2 dv[DV][S / 2];
#pragma unroll
    for (int r = 0; r < DV - 1; ++r)
#pragma unroll
      for (int s2 = 0; s2 < S / 2; ++s2) dv[r][s2] = *reinterpret_cast<const f64x2*>(rowp(r) + 2 * s2);
    auto row_block = [&](const int i0) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = i0 + u;
        {
          const f64x2* nrow = reinterpret_cast<const f64x2*>(rowp(i + DV - 1));
#ifndef CVK_ABL_NOLDS  // ablation build (timing only): delta rows never re-read from LDS
#pragma unroll
          for (int s2 = 0; s2 < S / 2; ++s2) dv[(u + DV - 1) % DV][s2] = nrow[s2];
#else
          (void)nrow;
#pragma unroll
          for (int s2 = 0; s2 < S / 2; ++s2) asm volatile("" : "+v"(dv[(u + DV - 1) % DV][s2].x), "+v"(dv[(u + DV - 1) % DV][s2].y));
#endif
        }
        // the broadcast reads of row i + DV - 1 issue BEFORE row i's adds (left alone, the
        // scheduler sank them to just before their use: ~16 maxima of cover for an LDS round
        // trip); nothing crosses this barrier
        if constexpr (DV > 1 && LDSFIRST) __builtin_amdgcn_sched_barrier(0);
        // the candidates of G sequence pairs are added before their maxima are taken, so each
        // v_max_f64 issues ~2*C*G instructions after the v_add_f64 it reads (adjacent dependent
        // f64 ops cost issue slots: profiles/r02_ab_fwd_group.txt)
        constexpr int G = (S / 2) % GRP == 0 ? GRP : 1;
#pragma unroll
        for (int s0 = 0; s0 < S / 2; s0 += G) {
          double x[G][2][C];
#pragma unroll
          for (int gg = 0; gg < G; ++gg) {
            const f64x2 d = dv[u % DV][s0 + gg];
#pragma unroll
            for (int c = 0; c < C; ++c) {
              if constexpr (DPA) {
                x[gg][0][c] = (ar[u][c] + ecur[2 * (s0 + gg)][c]) + d.x;
                x[gg][1][c] = (ar[u][c] + ecur[2 * (s0 + gg) + 1][c]) + d.y;
              } else {
                x[gg][0][c] = d.x + ar[u][c];
                x[gg][1][c] = d.y + ar[u][c];
              }
            }
          }
          __builtin_amdgcn_sched_group_barrier(0x002, 2 * C * G, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 2 * C * G, 0);
#pragma unroll
          for (int gg = 0; gg < G; ++gg)
#pragma unroll
            for (int c = 0; c < C; ++c) {
              acc[c][2 * (s0 + gg)] = __builtin_fmax(acc[c][2 * (s0 + gg)], x[gg][0][c]);
              acc[c][2 * (s0 + gg) + 1] = __builtin_fmax(acc[c][2 * (s0 + gg) + 1], x[gg][1][c]);
            }
        }
        // refill this ring slot with row (i + PF) mod NP -- the wrap-around rows are the next
        // step's first rows -- only after its last use, into the same registers: no copies,
        // and the in-flight loads cross the loop back-edge without a vmcnt(0) drain
#ifndef CVK_ABL_LOADHOT
        const int nr = i + PF < NP ? i + PF : i + PF - NP;
#else  // ablation build (timing only): the ring reloads rows 0 .. PF-1 only (L1/L2-hot, same addresses in every wave)
        const int nr = u;
#endif
#ifndef CVK_ABL_NOLOAD  // ablation build (timing only): the A-row ring is never refilled
        load_row_buf<C>(ra, voff, (uint32_t)nr * RB, ar[u]);
#else
        (void)nr;
#pragma unroll
        for (int c = 0; c < C; ++c) asm volatile("" : "+v"(ar[u][c]));
#endif
      }
      if constexpr (WG > 1 && (SYNC & 2)) {
        // the wave behind its SIMD partner (or level with it) takes the higher priority; the
        // partner's word is at most a block old (LDS, no barrier: a stale word only mis-sets a
        // priority).  No C++ branch here (a divergent or scalar branch split the unrolled loop
        // body and the ring registers spilled): every lane writes the same word, and the
        // compare and branch are one asm block.
        const int me = t * NP + i0;
        wg_prog[wid] = me;
        const int other = __builtin_amdgcn_readfirstlane(wg_prog[wid ^ 4]);
        asm volatile(
            "s_cmp_le_i32 %0, %1\n\t"
            "s_cbranch_scc0 1f\n\t"
            "s_setprio 3\n\t"
            "s_branch 2f\n"
            "1:\n\t"
            "s_setprio 2\n"
            "2:" ::"s"(me), "s"(other) : "scc");
      }
        };
    // the row loop in quarters (DEFST: one sequence pair's deferred stores before each; the
    // same structure without them -- a single loop over row_block spilled ~113 VGPRs once the
    // priority-trade asm block was in it)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (DEFST) {
        if (q < S / 2) deferred_store(q, t - 1);
      }
#pragma nounroll
      for (int i0 = q * (NP / 4); i0 < (q + 1) * (NP / 4); i0 += PF) row_block(i0);
    }
    // W = 1: LDS operations of the wave execute in order, so the reads of delta_{t-1} above
    // complete before the writes below; only the compiler must not reorder.  W > 1: every
    // wave has finished reading delta_{t-1} before any wave overwrites it
    asm volatile("" ::: "memory");
    wg_sync();
    // epilogue: d_t = m + b[:, o_t] (viterbi.rs:17), emission rows of all S sequences in flight
    // together; then the next step's observations (scalar loads)
    // balancing: publish this wave's remaining steps, read the other slots of its SIMD (the
    // loads complete with the emission loads below, which the epilogue waits for anyway)
    const bool bal_step = sb.tab && (t % bal == 0);
    int other = 0;
    if (bal_step) {
      sb.publish(lane, Tmax - t);
      other = sb.others(lane);
    }
    double e[DPA ? 1 : S][C];
    if constexpr (!DPA) {
#pragma unroll
      for (int s = 0; s < S; ++s) emis((unsigned)__builtin_amdgcn_readlane((int)ocur_l, s), e[s]);
    }
    onext_l = obs_lane(t + 1);
    fnext_l = frc_lane(t + 1);
#pragma unroll
    for (int s2 = 0; s2 < S / 2; ++s2) {
      double v0[C], v1[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        v0[c] = DPA ? acc[c][2 * s2] : acc[c][2 * s2] + e[DPA ? 0 : 2 * s2][c];
        v1[c] = DPA ? acc[c][2 * s2 + 1] : acc[c][2 * s2 + 1] + e[DPA ? 0 : 2 * s2 + 1][c];
      }
      if constexpr (EXT && !DPA) {  // noemit_last: the range's last step is the bare max-plus step
        if (g.noemit_last) {
          const bool l0 = t == T[2 * s2] - 1, l1 = t == T[2 * s2 + 1] - 1;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            v0[c] = l0 ? acc[c][2 * s2] : v0[c];
            v1[c] = l1 ? acc[c][2 * s2 + 1] : v1[c];
          }
        }
      }
      force(v0, __builtin_amdgcn_readlane(fcur_l, 2 * s2));
      force(v1, __builtin_amdgcn_readlane(fcur_l, 2 * s2 + 1));
#pragma unroll
      for (int c = 0; c < C; ++c) {
        f64x2 w;
        w.x = v0[c];
        w.y = v1[c];
        *reinterpret_cast<f64x2*>(rowp(j0 + c) + 2 * s2) = w;
      }
      if constexpr (!DEFST) {
        store_row(2 * s2, t, v0);
        store_row(2 * s2 + 1, t, v1);
      }
    }
    asm volatile("" ::: "memory");
    wg_sync();  // delta_t complete in LDS before the next step reads it
    if (bal_step) sb.decide(other, Tmax - t);
    if constexpr (WG > 1 && W == 1 && (SYNC & 1)) asm volatile("s_barrier" ::: "memory");
  }
  if constexpr (DEFST) {  // the last row (the LDS slice holds delta_{Tmax-1})
#pragma unroll
    for (int s2 = 0; s2 < S / 2; ++s2) deferred_store(s2, Tmax - 1);
  }
  if constexpr (kWgBar)
    for (int t = Tmax; t < Twg; ++t)
      for (int k = 0; k < kStepBarriers; ++k) asm volatile("s_barrier" ::: "memory");
  sb.finish(lane);
  if (wv == 0 && lane < S && my_bad) g.status[my_seq] = CVK_SEQ_BADOBS;
  };
  if constexpr (PERSIST) {
    // work queue over the longest-first units: a wave takes the next unit when it finishes one,
    // so the ragged passes end together instead of on the dispatch order's starved waves
    // (oldest-first issue lets the first wave of a SIMD run ahead of its partner).  One
    // lane's vector atomic, read back uniform; every wave exits once the units are taken.
    for (;;) {
      int u = 0;
      if (lane == 0) u = atomicAdd(g.queue, 1);
      u = __builtin_amdgcn_readfirstlane(u);
      if ((int64_t)u * S >= g.nslots) break;
      run_unit(u);
    }
  } else {
    run_unit((int64_t)blockIdx.x);
  }
}

// trellis_fwd_f64_rs<PF> -- the small-batch layout with a ROW split (round 3, N = 256): a PAIR
// of waves decodes S = 8 sequences, both waves over all NP = 256 columns (C = 4 per lane), wave
// wv over the candidate rows [wv*NP/2, wv*NP/2 + NP/2).  Per row each wave keeps the full-batch
// kernel's ratios -- 2 A-row loads and 4 delta broadcasts per 64 VALU; the column split
// (trellis_fwd_f64<2, 8, .., W = 2>) needs twice the broadcasts per VALU, which cost 6.7% at
// 8,192 sequences (timing-only build without them, profiles/r03_ablate_fwd_f64.txt).  At the
// step's end each wave writes its partial maxima of the partner's 4 sequences to LDS and, after
// the rendezvous, finalises its own 4: the max of the two partials (max is exact in any order)
// plus the emission -- the same f64 value as the one-wave kernel -- into the delta slice and
// HBM (split planes).  Four pairs per workgroup (the CU's eight waves, two per SIMD); the SIMD
// partners (waves i and i ^ 4: the same row half) trade issue priority as in trellis_fwd_f64.
// Row-A0 batch decode only (no EXT, no DPSolver association).
template <int PF>
__global__ __launch_bounds__(512) void trellis_fwd_f64_rs(T64FwdArgs g) {
  constexpr int C = 4, S = 8, NP = 256, H = NP / 2, HS = S / 2, NPAIR = 4, DV = 2;
  static_assert(H % PF == 0 && (H / 2) % PF == 0, "the ring wraps inside the row half");
  constexpr int kPadGroups = (NP + DV - 1 + C - 1) / C;
  __shared__ __attribute__((aligned(16))) double dl_all[NPAIR][(NP + DV - 1) * S + 2 * kPadGroups];
  // partial maxima of the partner's sequences: [pair][writer wave][chunk k = 2c + pair][lane]
  __shared__ __attribute__((aligned(16))) f64x2 xb_all[NPAIR][2][8][64];
  __shared__ int wg_prog[8];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wv = wid & 1, pr = wid >> 1;
  double* const dl = dl_all[pr];
  // 16 bytes of padding after each lane's C rows: conflict-free epilogue writes (as trellis_fwd_f64)
  auto rowp = [&](int i) -> double* { return dl + i * S + (i / C) * 2; };
  const int j0 = lane * C;
  const int rbase = wv * H;      // this wave's candidate rows
  const int sown = wv * HS;      // this wave's sequences [sown, sown + HS)
  const double ninf = ninf_d();
  auto rendezvous = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  // per-sequence bookkeeping in lane s (s < 8), as trellis_fwd_f64 (both waves of the pair)
  const int ls = lane < S ? lane : S - 1;
  const int64_t my_k = ((int64_t)blockIdx.x * NPAIR + pr) * S + ls;
  int my_T = 0;
  int64_t my_seq = -1, my_eb = 0, my_rb = 0;
  if (my_k < g.nslots && lane < S) {
    const int64_t sl = g.seq_begin + my_k;
    my_seq = g.order ? (int64_t)g.order[sl] : sl;
    my_eb = g.offsets[my_seq];
    my_T = (int)(g.offsets[my_seq + 1] - my_eb);
    my_rb = my_eb - g.delta_elem_base;
  }
  int Tmax = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) Tmax = max(Tmax, __builtin_amdgcn_readlane(my_T, s));
  // workgroup-wide barriers (1 after row 0, 2 per step): every wave takes part up to the
  // longest pair's last step
  int Twg = Tmax;
  if (lane == 0) wg_prog[wid] = Tmax;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 8; ++k) Twg = max(Twg, wg_prog[k]);
  __syncthreads();
  if (lane == 0) wg_prog[wid] = 0;
  if (Tmax <= 0) {
    if (Twg > 0) {
      asm volatile("s_barrier" ::: "memory");
      for (int t = 1; t < Twg; ++t) {
        asm volatile("s_barrier" ::: "memory");
        asm volatile("s_barrier" ::: "memory");
      }
    }
    return;
  }
  const unsigned V = (unsigned)g.nobs;
  {
    const unsigned long long live = __ballot(my_T > 0);
    const int l0 = __builtin_ctzll(live);
    const int64_t eb0 = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my_eb, l0) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(my_eb >> 32), l0) << 32));
    if (my_T <= 0) my_eb = eb0;
  }
  const int my_Tc = my_T > 0 ? my_T : 1;
  bool my_bad = false;
  auto obs_lane = [&](int t) -> unsigned { return (unsigned)g.obs[my_eb + (t < my_Tc ? t : my_Tc - 1)]; };
  auto obs_use = [&](unsigned o, int t) -> unsigned {
    my_bad = my_bad || (t < my_T && o >= V);
    return o < V ? o : 0u;
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g.a), 0, NP * NP * 8, 0x00020000);
  const uint32_t voff = (uint32_t)j0 * 8;
  constexpr uint32_t RB = NP * 8;
  auto emis = [&](unsigned o, double (&e)[C]) { load_a<C>(g.et + (size_t)o * NP + j0, e); };
  // own sequence sown + q (q < HS): length, delta row base (uniform, from its lane)
  auto seq_T = [&](int q) { return __builtin_amdgcn_readlane(my_T, sown + q); };
  auto store_row = [&](int q, int t, const double (&v)[C]) {
    if (g.delta && t < seq_T(q)) {
      const int64_t r = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my_rb, sown + q) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(my_rb >> 32), sown + q) << 32));
      uint32_t* dst = reinterpret_cast<uint32_t*>(g.delta) + (r + t) * (2 * NP) + j0;
      store_split<C>(dst, dst + NP, v);
    }
  };
  // acc of own (partner = false) or partner sequence q of this wave (selects: no runtime
  // register indexing)
  double acc[C][S];
  auto acc_of = [&](int c, int q, bool partner) -> double {
    return ((wv == 0) != partner) ? acc[c][q] : acc[c][q + HS];
  };

  // ---- t = 0: d0 = pi + b[:, o0] for the own sequences ----
  unsigned onext_l;
  {
    const unsigned o0 = obs_use(obs_lane(0), 0);
#pragma unroll
    for (int q = 0; q < HS; ++q) {
      double e[C], v[C];
      emis((unsigned)__builtin_amdgcn_readlane((int)o0, sown + q), e);
#pragma unroll
      for (int c = 0; c < C; ++c) v[c] = g.zero_init ? 0.0 : g.pi[j0 + c] + e[c];
#pragma unroll
      for (int c = 0; c < C; ++c) rowp(j0 + c)[sown + q] = v[c];
      store_row(q, 0, v);
    }
    onext_l = obs_lane(1);
  }
  rendezvous();  // delta_0 of all 8 sequences in the slice

  __builtin_amdgcn_s_setprio(3);
  double ar[PF][C];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    load_row_buf<C>(ra, voff, (uint32_t)(rbase + u) * RB, ar[u]);
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int t = 1; t < Tmax; ++t) {
    const unsigned ocur_l = obs_use(onext_l, t);
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int s = 0; s < S; ++s) acc[c][s] = ninf;
    f64x2 dv[DV][S / 2];
#pragma unroll
    for (int s2 = 0; s2 < S / 2; ++s2) dv[0][s2] = *reinterpret_cast<const f64x2*>(rowp(rbase) + 2 * s2);
    auto row_block = [&](const int i0) __attribute__((always_inline)) {  // rows rbase + i0 .. + PF - 1
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = rbase + i0 + u;
        {
          const f64x2* nrow = reinterpret_cast<const f64x2*>(rowp(i + 1));
#pragma unroll
          for (int s2 = 0; s2 < S / 2; ++s2) dv[(u + 1) % DV][s2] = nrow[s2];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s0 = 0; s0 < S / 2; s0 += 2) {
          double x[2][2][C];
#pragma unroll
          for (int gg = 0; gg < 2; ++gg) {
            const f64x2 d = dv[u % DV][s0 + gg];
#pragma unroll
            for (int c = 0; c < C; ++c) {
              x[gg][0][c] = d.x + ar[u][c];
              x[gg][1][c] = d.y + ar[u][c];
            }
          }
          __builtin_amdgcn_sched_group_barrier(0x002, 4 * C, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4 * C, 0);
#pragma unroll
          for (int gg = 0; gg < 2; ++gg)
#pragma unroll
            for (int c = 0; c < C; ++c) {
              acc[c][2 * (s0 + gg)] = __builtin_fmax(acc[c][2 * (s0 + gg)], x[gg][0][c]);
              acc[c][2 * (s0 + gg) + 1] = __builtin_fmax(acc[c][2 * (s0 + gg) + 1], x[gg][1][c]);
            }
        }
        // refill with the half's row (i0 + u + PF) mod H: the next step's first rows wrap in
        const int rel = i0 + u + PF;
        load_row_buf<C>(ra, voff, (uint32_t)(rbase + (rel < H ? rel : rel - H)) * RB, ar[u]);
      }
      {  // SIMD partners (same row half) trade priority, as trellis_fwd_f64 (one asm block)
        const int me = t * H + i0;
        wg_prog[wid] = me;
        const int other = __builtin_amdgcn_readfirstlane(wg_prog[wid ^ 4]);
        asm volatile(
            "s_cmp_le_i32 %0, %1\n\t"
            "s_cbranch_scc0 1f\n\t"
            "s_setprio 3\n\t"
            "s_branch 2f\n"
            "1:\n\t"
            "s_setprio 2\n"
            "2:" ::"s"(me), "s"(other) : "scc");
      }
    };
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma nounroll
      for (int i0 = q * (H / 2); i0 < (q + 1) * (H / 2); i0 += PF) row_block(i0);
    }
    asm volatile("" ::: "memory");
    // epilogue: own emissions in flight, partials of the partner's sequences to LDS
    double e[HS][C];
#pragma unroll
    for (int q = 0; q < HS; ++q) emis((unsigned)__builtin_amdgcn_readlane((int)ocur_l, sown + q), e[q]);
    onext_l = obs_lane(t + 1);
    f64x2(*xw)[64] = xb_all[pr][wv];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = k >> 1, q = 2 * (k & 1);
      f64x2 w;
      w.x = acc_of(c, q, true);
      w.y = acc_of(c, q + 1, true);
      xw[k][lane] = w;
    }
    rendezvous();  // partials written; every wave is done reading delta_{t-1}
    const f64x2(*xr)[64] = xb_all[pr][wv ^ 1];
#pragma unroll
    for (int qp = 0; qp < HS / 2; ++qp) {
      double v0[C], v1[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const f64x2 p = xr[2 * c + qp][lane];
        v0[c] = __builtin_fmax(acc_of(c, 2 * qp, false), p.x) + e[2 * qp][c];       // viterbi.rs:15-17
        v1[c] = __builtin_fmax(acc_of(c, 2 * qp + 1, false), p.y) + e[2 * qp + 1][c];
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        f64x2 w;
        w.x = v0[c];
        w.y = v1[c];
        *reinterpret_cast<f64x2*>(rowp(j0 + c) + sown + 2 * qp) = w;
      }
      store_row(2 * qp, t, v0);
      store_row(2 * qp + 1, t, v1);
    }
    asm volatile("" ::: "memory");
    rendezvous();  // delta_t of all 8 sequences in the slice
  }
  for (int t = Tmax; t < Twg; ++t) {
    asm volatile("s_barrier" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
  }
  if (lane >= sown && lane < sown + HS && my_bad) g.status[my_seq] = CVK_SEQ_BADOBS;
}

// CP association (CPSolver, cp.rs:70-79 via utils.rs:24-38, hmm.rs:220-222):
//   psi = first argmax_i (d[i] + a[i,j]);  d'[j] = d[psi] + (a[psi,j] + b[j,o])
// The value depends on psi, so the forward pass tracks the first argmax: per pair one add,
// one compare, one max and one index select (4 VALU vs 2 for row A0), then per column one
// LDS gather of d[psi] and one L2 gather of a[psi,j].  psi (u16) and the last row go out in
// generic_fwd's layout; generic_backtrack<double> follows them (cp.rs:85-93).  Same wave
// layout as trellis_fwd_f64 (S sequences per wave, A rows streamed through a register ring).
// S = 1 (round 5): one sequence per wave for small batches (the parallel chain's speculative
// re-decodes, ~620 sequences at config-4 size), so every sequence has a SIMD of its own.
// W > 1 (round 6): the workgroup's W waves split the columns (C per lane, NP = 64 C W) of the
// same S sequences, delta_{t-1} shared in LDS behind the step's two workgroup barriers: each
// A element streamed from L2 serves S sequences while a wave's per-step walk (256 rows x C
// columns x S sequences x 4 VALU) stays short -- the chain's speculative batch is a few
// hundred sequences, each step of which every sequence must finish before its next.
template <int C, int S, int PF, int W = 1>
__global__ __launch_bounds__(64 * W) void trellis_cp_f64(T64FwdArgs g) {
  constexpr int NP = 64 * C * W;
  static_assert((S == 1 || S % 2 == 0) && PF % 2 == 0, "one sequence or pairs of sequences / rows");
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
        if (t == T[s] - 1) {
          g.last_row[(slot0 + s - g.seq_begin) * (int64_t)N + j0 + c] = v[c];
          if (g.cp_last) g.cp_last[seq[s] * (int64_t)N + j0 + c] = v[c];
        }
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
      // cp_init (the parallel chain's speculative re-runs): the chain's start value
      // fl(M + fl(pi + b)) of a sequence entered with running maximum M (utils.rs:32-38)
      v[c] = g.cp_init ? g.cp_init[seq[s] >= 0 ? seq[s] : 0] + (g.pi[j0 + c] + e[c]) : g.pi[j0 + c] + e[c];
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
    constexpr int S2 = S / 2 > 0 ? S / 2 : 1;
    double2 dv[2][S2];
    double d1[2];  // S = 1: delta_{t-1}[i] and the next row's
    if constexpr (S == 1) {
      d1[0] = dl[0];
    } else {
#pragma unroll
      for (int s2 = 0; s2 < S / 2; ++s2) dv[0][s2] = reinterpret_cast<const double2*>(dl)[s2];
    }
#pragma nounroll
    for (int i0 = 0; i0 < NP; i0 += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int i = i0 + u;
        if constexpr (S == 1) {
          d1[(u + 1) & 1] = dl[min(i + 1, NP - 1)];
          const double d = d1[u & 1];
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const double x = d + ar[u][c];
            idx[c][0] = x > acc[c][0] ? i : idx[c][0];
            acc[c][0] = fmax(acc[c][0], x);
          }
          const int nr = min(i + PF, NP - 1);
          load_a(arow + (size_t)nr * NP, ar[u]);
          continue;
        }
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

// wave-wide f32 max through DPP (no LDS round trips): within each row of 16 lanes by quad
// permutes and mirrors, then rows combined by the gfx9 row broadcasts; lane 63 holds the
// maximum of all 64 lanes.  -fno-honor-nans: callers pass no NaN.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float max_dpp(float v) {
  const int o = __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xF, false);
  return __builtin_fmaxf(v, __builtin_bit_cast(float, o));
}
__device__ __forceinline__ float wave_max_f32(float v) {
  v = max_dpp<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = max_dpp<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = max_dpp<0x141, 0xF>(v);  // row_half_mirror
  v = max_dpp<0x140, 0xF>(v);  // row_mirror: every lane of a row holds the row max
  v = max_dpp<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v = max_dpp<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// first index of the wave-wide maximum of s (candidate i = lane + 64k; invalid k excluded)
template <int KP>
__device__ __forceinline__ int first_argmax_d(const double (&s)[KP], const bool (&valid)[KP], double& M) {
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
}

// PF: rows in flight per wave (hi planes, 1 KiB each at NP = 256); at NP >= 192 occupancy
// hides the HBM latency better than a deeper ring (profiles/r01_t64_bt_pf.txt, 2-KiB rows).
//
// Rows come in the split-plane layout of the forward pass.  Each step first reads only the
// HI words (the f64 with its mantissa truncated to 20 bits, error < |hi| * 2^-20): every
// candidate s_i = d_{t-1}[i] + a[i, cur] gets an interval [L_i, U_i] around the f64 sum of
// the truncated value (the truncation bound plus one rounding of the add, monotone f64
// addition).  When exactly one candidate has U_i >= max_k L_k it is the unique -- hence
// first -- argmax of the exact f64 sums; otherwise (near ties, ~1% of steps at config 4) the
// LO words of that row are read too and the exact sums decide with the first-index rule.
// Half the HBM bytes of a full-row backtrack, same path bit for bit.
// One backtrack chain: path[T-1] = cur, then for t = T-1..1 the first argmax of
// d_{t-1}[i] + a[i, path[t]] (DPSolver: (a[i, path[t]] + b[path[t], o_t]) + d_{t-1}[i])
// through the split-plane rows rows[0 .. T-1] (row t = element t of the chain).
// DEC (viterbi::decode, infeasible sequences only): bt = 0 where the emission of the current
// state is -inf (viterbi.rs:19-21); on a feasible path every emission is finite, so the rule
// never changes a feasible decode.
//
// NONPOS (models whose finite log-probabilities are all in [-2^80, 0], the bench path; row A0
// and DPSolver's association): every candidate is <= 0, so the error of its estimate is
// RELATIVE to the estimate itself and the interval test collapses to one threshold on f32
// estimates
//   x_i = f32(hi_i) + at32[cur][i]      (f32 a^T table, round to nearest; DPSolver: f32 of the
//                                        f64 sum a[i,cur] + b[cur,o_t] the forward pass used)
//   |s_i - x_i| <= c |x_i|,  c = 1.25 * 2^-20:  hi truncation |h| 2^-20, the f32 roundings of
//   h, a and their sum (2^-24 each), the f64 rounding of s (2^-53); |h|, |a| <= |x| as all
//   three are <= 0; f32 flushes of subnormals stay below the 2^-100 floor
//   survivors: x_i >= M (1 + 3 * 2^-20) - 2^-100, M = max_k x_k
// since s_i* >= s_k >= M (1 + c) and s_i* <= x_i* (1 - c) give x_i* >= M (1 + c) / (1 - c),
// with (1 + c) / (1 - c) < 1 + 2.6 * 2^-20 and the f32 rounding of the threshold (2^-24 |M|)
// inside the remaining slack.  Half the L2 bytes of the f64 a^T column, a DPP wave max in
// place of six ds_bpermute rounds, and no per-candidate bound arithmetic.  |x| < 2^112 for
// T < 2^31, so no estimate overflows f32.
//
// CERT (NONPOS row A0 only, the parallel CPSolver chain): the backtrack also reduces the path's
// gaps to the chain certificate rho of cp_cert_f64 (kernels/chain.hip), so no second pass
// re-reads every row.  gap_t = s_path - max_{i != path} s_i is bounded BELOW from the step's f32
// estimates -- s_path >= x_path (1 + c') and s_i <= x_i (1 - c') with c' = 1.5 * 2^-20 > c, both
// <= 0 -- and the step's term r_t = (gap_t - (4t + 1) u0) / (3t + 1) taken from that bound when
// it already reaches rho_cap; below it the lo plane is read and the exact f64 gap used, as
// cp_cert_f64 does.  So the returned rho equals cp_cert_f64's exact rho whenever that is below
// rho_cap, and is >= rho_cap otherwise: the host's tests rho > U agree with the exact
// certificate for every U <= rho_cap (the host sizes rho_cap above the largest U it can test).
#ifndef CVK_BT_ROLL
#define CVK_BT_ROLL 0
#endif
template <int KP, int PF, bool DEC = false, bool NONPOS = false, bool CERT = false>
__device__ __forceinline__ void bt_chain_f64(const uint32_t* __restrict__ rows, int T, int cur, int32_t* __restrict__ path,
                                             const double* __restrict__ at, const double* __restrict__ et,
                                             const int32_t* __restrict__ obs, int dp_assoc, int N, int lane,
                                             const float* __restrict__ at32 = nullptr, double* rho_io = nullptr,
                                             double u0 = 0.0, double rho_cap = 0.0) {
  static_assert(!CERT || (NONPOS && !DEC), "certificates: the NONPOS row-A0 chain");
  double rho = CERT ? *rho_io : 0.0;
  constexpr int NP = 64 * KP;
  constexpr uint32_t NINF_HI = 0xFFF00000u;  // hi word of -inf (lo word 0)
  bool valid[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) valid[k] = (lane + 64 * k) < N;
  auto load_hi = [&](int r, uint32_t (&dst)[KP]) {
#pragma unroll
    for (int k = 0; k < KP; ++k)
      dst[k] = (r >= 0 && valid[k]) ? __builtin_nontemporal_load(rows + (size_t)r * (2 * NP) + lane + 64 * k) : NINF_HI;
  };
  auto load_lo = [&](int r, uint32_t (&dst)[KP]) {
#pragma unroll
    for (int k = 0; k < KP; ++k)
      dst[k] = (r >= 0 && valid[k]) ? __builtin_nontemporal_load(rows + (size_t)r * (2 * NP) + NP + lane + 64 * k) : 0u;
  };
  int pathreg = 0;
  if (lane == ((T - 1) & 63)) pathreg = cur;
  if (((T - 1) & 63) == 0 && lane == 0) path[T - 1] = cur;
  uint32_t ring[PF][KP];
#pragma unroll
  for (int u = 0; u < PF; ++u) load_hi(T - 2 - u, ring[u]);
  for (int base = T - 1; base >= 1; base -= PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int t = base - u;
      if (DEC && t >= 1 && !(et[(size_t)obs[t] * NP + cur] > ninf_d())) {
        cur = 0;
        const int tp = t - 1;
        if (lane == (tp & 63)) pathreg = cur;
        if ((tp & 63) == 0 && tp + lane < T) path[tp + lane] = pathreg;
      } else if (NONPOS && t >= 1) {
        // row A0: f32(a) from the f32 table; DPSolver (dp_assoc): f32 of the forward pass's own
        // f64 sum a + b[cur, o_t] (all terms <= 0 either way: the same bound c)
        float av32[KP];
        double edp = 0.0;
        if (dp_assoc) {
          edp = et[(size_t)obs[t] * NP + cur];
          const double* acol = at + (size_t)cur * NP + lane;
#pragma unroll
          for (int k = 0; k < KP; ++k) av32[k] = (float)(acol[64 * k] + edp);
        } else {
          const float* acol32 = at32 + (size_t)cur * NP + lane;
#pragma unroll
          for (int k = 0; k < KP; ++k) av32[k] = acol32[64 * k];
        }
        float x[KP];
        float lm = -__builtin_inff();
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          // padded candidates: hi word -inf, at32 -inf
          x[k] = (float)from_words(ring[u][k], 0u) + av32[k];
          lm = __builtin_fmaxf(lm, x[k]);
        }
        const float M = wave_max_f32(lm);
        const float thr = M * (1.0f + 0x3p-20f) - 0x1p-100f;
        int cnt = 0, idx = 0;
#pragma unroll
        for (int k = KP - 1; k >= 0; --k) {
          const unsigned long long mask = __ballot(x[k] >= thr);
          cnt += __builtin_popcountll(mask);
          if (mask) idx = 64 * k + __builtin_ctzll(mask);
        }
        bool exact = cnt != 1;
        if constexpr (CERT) {
          if (!exact) {
            // the gap's lower bound from the estimates (x_path = M: the unique survivor), O = the
            // best other estimate: lb = M (1 + 3 2^-21) - O (1 - 3 2^-21) - |M| 2^-50 - 2^-99, and
            // the step's term r = (lb - (4t + 1) u0) / (3t + 1) reaches rho_cap iff
            // O <= theta = (M (1 + 3 2^-21) - |M| 2^-50 - 2^-99 - rho_cap (3t + 1) - (4t + 1) u0)
            //              / (1 - 3 2^-21)
            // (theta <= 0: times 1 + 2^-19 > 1 / (1 - 3 2^-21), less |theta| 2^-48 for its own
            // roundings, only makes the test stricter).  So one ballot per candidate block
            // replaces the wave maximum of O; a step that reaches the cap leaves rho alone (the
            // returned rho is then >= rho_cap, which is all the host's tests need), one below
            // takes the exact gap
            const double Md = (double)M;
            const double need = rho_cap * (double)(3 * t + 1) + (double)(4 * t + 1) * u0;
            double th = (Md * (1.0 + 0x3p-21) - __builtin_fabs(Md) * 0x1p-50 - 0x1p-99 - need) * (1.0 + 0x1p-19);
            th -= __builtin_fabs(th) * 0x1p-48;
            bool over = false;
#pragma unroll
            for (int k = 0; k < KP; ++k) over |= __ballot((double)x[k] > th && 64 * k + lane != idx) != 0;
            exact = over;
          }
        }
        if (!exact) {
          cur = idx;
        } else {  // near tie (or a certificate step below rho_cap): the exact f64 sums decide (first index)
          const double* acol = at + (size_t)cur * NP + lane;
          uint32_t lw[KP];
          load_lo(t - 1, lw);
          double sx[KP];
#pragma unroll
          for (int k = 0; k < KP; ++k)
            sx[k] = valid[k] ? (dp_assoc ? (acol[64 * k] + edp) + from_words(ring[u][k], lw[k])
                                         : from_words(ring[u][k], lw[k]) + acol[64 * k])
                             : ninf_d();
          double Md;
          cur = first_argmax_d<KP>(sx, valid, Md);
          if constexpr (CERT) {  // the exact gap: the path's candidate minus the best other one
            double o = ninf_d();
#pragma unroll
            for (int k = 0; k < KP; ++k) o = fmax(o, (64 * k + lane == cur) ? ninf_d() : sx[k]);
            const double m2 = wave_max_d(o);
            rho = fmin(rho, (Md - m2 - (double)(4 * t + 1) * u0) / (double)(3 * t + 1));
            if (!(Md > ninf_d())) rho = -1.0;
          }
        }
        const int tp = t - 1;
        if (lane == (tp & 63)) pathreg = cur;
        if ((tp & 63) == 0 && tp + lane < T) path[tp + lane] = pathreg;
      } else if (t >= 1) {
        const double* acol = at + (size_t)cur * NP + lane;
        double e = 0.0;
        if (dp_assoc) e = et[(size_t)obs[t] * NP + cur];
        double av[KP];
#pragma unroll
        for (int k = 0; k < KP; ++k) av[k] = dp_assoc ? acol[64 * k] + e : acol[64 * k];
        // candidates from the truncated values: s~ = h + a (DPSolver: (a + b) + h)
        double st[KP], up[KP];
        double lmax = ninf_d();
#pragma unroll
        for (int k = 0; k < KP; ++k) {
          const double h = from_words(ring[u][k], 0u);
          const double x = valid[k] ? (dp_assoc ? av[k] + h : h + av[k]) : ninf_d();
          const bool fin = x > ninf_d();
          // |d - h| < |h| 2^-20, plus one f64 rounding of the add (< |x| 2^-52; 2^-51 kept),
          // plus an absolute floor for subnormal truncations
          const double err = __builtin_fabs(h) * 0x1p-20 + __builtin_fabs(x) * 0x1p-51 + 0x1p-1000;
          st[k] = x;
          up[k] = fin ? x + err : ninf_d();
          lmax = fmax(lmax, fin ? x - err : ninf_d());
        }
        lmax = wave_max_d(lmax);
        int cnt = 0, idx = 0;
#pragma unroll
        for (int k = KP - 1; k >= 0; --k) {
          const unsigned long long mask = __ballot(valid[k] && st[k] > ninf_d() && up[k] >= lmax);
          cnt += __builtin_popcountll(mask);
          if (mask) idx = 64 * k + __builtin_ctzll(mask);
        }
        if (cnt == 1) {
          cur = idx;
        } else {  // near tie (or all -inf): the exact f64 sums of this row decide
          uint32_t lw[KP];
          load_lo(t - 1, lw);
          double s[KP];
#pragma unroll
          for (int k = 0; k < KP; ++k) {
            const double d = from_words(ring[u][k], lw[k]);
            s[k] = valid[k] ? (dp_assoc ? av[k] + d : d + av[k]) : ninf_d();
          }
          double M;
          cur = first_argmax_d<KP>(s, valid, M);
        }
        const int tp = t - 1;
        if (lane == (tp & 63)) pathreg = cur;
        if ((tp & 63) == 0 && tp + lane < T) path[tp + lane] = pathreg;
      }
#if CVK_BT_ROLL
      load_hi(t - PF - 1, ring[u]);  // the row of step t - PF, PF steps ahead
#endif
    }
#if !CVK_BT_ROLL
#pragma unroll
    for (int u = 0; u < PF; ++u) load_hi(base - PF - 1 - u, ring[u]);
#endif
  }
  if constexpr (CERT) *rho_io = rho;
}

// NONPOS: the kernel holds only the NONPOS chain (fewer VGPRs, more waves per SIMD); the
// host launches it for row-A0 decodes without the viterbi::decode infeasible rule when
// g.at32 is set.
// prior_in >= 0: the sequence's status as its forward pass left it, passed in registers (the
// fused N <= 64 kernel: a uniform load of g.status could come from a stale scalar-cache line)
// CERT: the chain certificate (rho, gF) of cp_cert_f64 into g.cert[2 seq], computed along the way
// (bt_chain_f64 CERT); -1 for sequences that are not OK.
template <int KP, int PF, bool NONPOS, bool CERT = false>
__device__ __forceinline__ void backtrack_one_f64(const T64BtArgs& g, int64_t slot, int lane, int prior_in = -1) {
  constexpr int NP = 64 * KP;
  const int64_t seq = g.order ? (int64_t)g.order[slot] : slot;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  const int N = g.nstates;
  if (T <= 0) {
    if (lane == 0) {
      g.score[seq] = 0.0;
      g.status[seq] = CVK_SEQ_EMPTY;
      if constexpr (CERT) g.cert[2 * seq] = -1.0, g.cert[2 * seq + 1] = -1.0;
    }
    return;
  }
  int32_t* __restrict__ path = g.path + e0;
  const uint32_t* __restrict__ rows = reinterpret_cast<const uint32_t*>(g.delta) + (e0 - g.delta_elem_base) * (2 * NP);
  bool valid[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) valid[k] = (lane + 64 * k) < N;
  double bv;
  int cur;
  double gF = -1.0, rho = -1.0, u0 = 0.0;
  {
    double last[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const size_t q = (size_t)(T - 1) * (2 * NP) + lane + 64 * k;
      last[k] = valid[k] ? from_words(__builtin_nontemporal_load(rows + q), __builtin_nontemporal_load(rows + q + NP))
                         : ninf_d();
    }
    cur = first_argmax_d<KP>(last, valid, bv);  // cp.rs:86
    if constexpr (CERT) {  // the last row's top-2 gap (cp_cert_f64's gapF)
      double o = ninf_d();
#pragma unroll
      for (int k = 0; k < KP; ++k) o = fmax(o, (64 * k + lane == cur) ? ninf_d() : last[k]);
      const double m2 = wave_max_d(o);
      u0 = (__builtin_fabs(bv) + 16.0) * 0x1p-51;
      gF = bv - m2 - 4.0 * (double)T * u0;  // +inf when the row has one finite entry
      rho = gF / (double)(3 * T + 2);
    }
  }
  const uint8_t prior = prior_in >= 0 ? (uint8_t)prior_in : g.status[seq];
  if (!(bv > ninf_d()) || prior == CVK_SEQ_BADOBS) {
    if (g.decode_bt && prior != CVK_SEQ_BADOBS) {  // viterbi.rs:24-30: from argmax 0 (= cur) through bt
      // the NONPOS kernel leaves the DEC chain (more VGPRs) to the general kernel's
      // only_infeasible pass that launch_t64_bt queues after it
      if constexpr (!NONPOS) bt_chain_f64<KP, PF, true>(rows, T, cur, path, g.at, g.et, g.obs + e0, 0, N, lane);
    } else {
      for (int t = lane; t < T; t += 64) path[t] = 0;
    }
    if (lane == 0) {
      g.score[seq] = ninf_d();
      g.status[seq] = prior == CVK_SEQ_BADOBS ? CVK_SEQ_BADOBS : CVK_SEQ_INFEASIBLE;
      if constexpr (CERT) g.cert[2 * seq] = -1.0, g.cert[2 * seq + 1] = -1.0;
    }
    return;
  }
  if (!NONPOS && g.only_infeasible) return;  // feasible: done by the NONPOS kernel
  if constexpr (CERT)
    bt_chain_f64<KP, PF, false, true, true>(rows, T, cur, path, g.at, g.et, g.obs + e0, g.dp_assoc, N, lane, g.at32,
                                            &rho, u0, g.rho_cap);
  else if constexpr (NONPOS)
    bt_chain_f64<KP, PF, false, true>(rows, T, cur, path, g.at, g.et, g.obs + e0, g.dp_assoc, N, lane, g.at32);
  else
    bt_chain_f64<KP, PF>(rows, T, cur, path, g.at, g.et, g.obs + e0, g.dp_assoc, N, lane);
  if (lane == 0) {
    g.score[seq] = bv;
    g.status[seq] = CVK_SEQ_OK;
    if constexpr (CERT) {
      // the divisions and subtractions round: a relative 2^-50 covers them (as cp_cert_f64)
      const bool pass = rho > 0.0;
      g.cert[2 * seq] = pass ? rho * (1.0 - 0x1p-50) : -1.0;
      g.cert[2 * seq + 1] = pass ? gF * (1.0 - 0x1p-50) : -1.0;
    }
  }
}

// One wave per sequence; a grid smaller than the batch makes the kernel persistent (wave w of
// workgroup b takes slots b*4 + w, then strides by the grid): the overlap schedule launches one
// workgroup per CU (one wave per SIMD), which always fits beside two forward waves.
// NONPOS at NP = 64: the f32 a^T (16 KiB) is staged in LDS, so the one dependent read of each
// chain step is an LDS round trip instead of an L2 one (the longest chains set the makespan
// of ragged batches, config 3).
template <int KP, int PF, bool NONPOS = false, bool CERT = false>
__global__ __launch_bounds__(256) void backtrack_f64(T64BtArgs g) {
  constexpr bool LDS_AT = NONPOS && KP == 1;
  __shared__ float at_lds[LDS_AT ? 64 * 64 : 1];
  if constexpr (LDS_AT) {
    for (int k = threadIdx.x; k < 64 * 64; k += 256) at_lds[k] = g.at32[k];
    __syncthreads();
    g.at32 = at_lds;
  }
  const int lane = threadIdx.x & 63;
  const int64_t slot0 = g.seq_begin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (slot0 < g.seq_end) backtrack_one_f64<KP, PF, NONPOS, CERT>(g, slot0, lane);
}

// Resume flow (f64): the prefix [offsets[seq], t1] of every constrained sequence backtracked
// from its forced state through the rows the terms pass stored (split-plane, compact per slot).
template <int KP, bool NONPOS>
__global__ __launch_bounds__(256) void prefix_backtrack_f64(PrefixBt64Args a, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t seq = a.seq[i];
  const int64_t e0 = a.offsets[seq];
  const int T = (int)(a.t1[i] - e0 + 1);
  constexpr int NP = 64 * KP;
  // an infeasible forced row backtracks garbage: zero_infeasible_prefix overwrites it once the
  // suffix decode has told which sequences are infeasible
  bt_chain_f64<KP, 2, false, NONPOS>(reinterpret_cast<const uint32_t*>(a.rows) + a.row_base[i] * (2 * NP), T,
                                     a.state[i], a.path + e0, a.at, nullptr, nullptr, 0, a.nstates, lane, a.at32);
}

// Resume flow, certified suffix trace (f64; one constrained element t1; models whose finite
// entries all lie in [-2^80, 0]).  The forced decode from state s* at t1 maximises, over the
// paths P of [t1, end), the forward fold F(P) = ((D + a) + b) + ... from D = delta_{t1}(s*)
// (viterbi.rs:15-17 order).  The reversed suffix pass stored r_x(j) = b_j(o_x) + beta_x(j) for
// every element x > t1, so the path can be read FORWARD: from cur = P_x the candidates are
// w_j = r_{x+1}(j) + a[cur][j] and P_{x+1} = their first argmax.  That path is the forced
// decode's exactly when no other path's fold can reach it.  All terms are <= 0, so an fp sum
// of k terms is within ~k 2^-53 relative of its real value; a path Q leaving P at x+1 for j
// scores at most C + W_j (real) against P's C + W_P, C the common real prefix
// (|C| <= |d_x|(1 + rho), d_x = P's fold so far).  With rho = (4L + 8) 2^-52 (L = end-1-t1
// steps: 2L roundings forward, 2L + 1 in r and w, doubled for slack) the test
//     w2 (1 - rho) + 2 rho |d_x|  <  w_P (1 + rho)      (w2 = best candidate other than P_{x+1})
// at every step gives F(Q) < F(P) for every Q != P: the forced forward decode then ends in
// P's last state (unique maximum), every backtrack step's first argmax is P's predecessor (a
// tie or a larger value there would make some Q reach F(P)), and its score is F(P), the fold
// computed here in the forward order -- bit-identical.  A failed step (near tie, -inf, no
// state) leaves the slot to the fallback forced decode: cert = 0.
// CVK_TRACE_WAVES: minimum waves per SIMD the register budget must allow (A/B: 8 = at most 64
// VGPRs, so a trace wave fits beside the two 224-VGPR waves of a forward workgroup)
#ifndef CVK_TRACE_WAVES
#define CVK_TRACE_WAVES 1
#endif
template <int KP>
__global__ __launch_bounds__(256, CVK_TRACE_WAVES) void suffix_trace_f64(SuffixTrace64Args g, int64_t n) {
  constexpr int NP = 64 * KP;
  constexpr uint32_t NINF_HI = 0xFFF00000u;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int64_t seq = g.seq[i];
  const int64_t x0 = g.t1[i];
  const int64_t end = g.offsets[seq + 1];
  const int L = (int)(end - 1 - x0);
  int cur = g.state[i];
  double d = cur >= 0 ? g.dlast[(size_t)i * NP + cur] : ninf_d();
  bool ok = d > ninf_d();
  bool valid[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) valid[k] = (lane + 64 * k) < g.nstates;
  const double rho = (double)(4 * L + 8) * 0x1p-52;
  const uint32_t* rows = reinterpret_cast<const uint32_t*>(g.rows) + g.srow_base[i] * (2 * NP);
  auto readlane_d = [](double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return from_words(hi, lo);
  };
  // the next step's operands, loaded a step ahead: its row (both planes) and emission row
  uint32_t nh[KP], nl[KP];
  double ne[KP];
  auto prefetch = [&](int s) {  // step s: element x0 + s + 1 = row L - 1 - s
    const uint32_t* r = rows + (size_t)(L - 1 - s) * (2 * NP) + lane;
    const double* e = g.et + (size_t)g.obs[x0 + s + 1] * NP + lane;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      nh[k] = valid[k] ? __builtin_nontemporal_load(r + 64 * k) : NINF_HI;
      nl[k] = valid[k] ? __builtin_nontemporal_load(r + NP + 64 * k) : 0u;
      ne[k] = e[64 * k];
    }
  };
  if (ok && L > 0) prefetch(0);
  int pathreg = 0;
  for (int s = 0; ok && s < L; ++s) {
    uint32_t ch[KP], cl[KP];
    double ce[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) ch[k] = nh[k], cl[k] = nl[k], ce[k] = ne[k];
    if (s + 1 < L) prefetch(s + 1);
    const double* arow = g.a + (size_t)cur * NP + lane;
    double av[KP], w[KP];
    double m = ninf_d();
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      av[k] = arow[64 * k];
      w[k] = valid[k] ? from_words(ch[k], cl[k]) + av[k] : ninf_d();
      m = fmax(m, w[k]);
    }
    const double M = wave_max_d_dpp(m);  // DPP: no LDS round trips on the chain
    int idx = 0;
#pragma unroll
    for (int k = KP - 1; k >= 0; --k) {
      const unsigned long long mask = __ballot(valid[k] && w[k] == M);
      if (mask) idx = 64 * k + __builtin_ctzll(mask);
    }
    double m2 = ninf_d();
#pragma unroll
    for (int k = 0; k < KP; ++k) m2 = fmax(m2, (64 * k + lane == idx) ? ninf_d() : w[k]);
    const double M2 = wave_max_d_dpp(m2);
    ok = M > ninf_d() && M2 * (1.0 - rho) + 2.0 * rho * __builtin_fabs(d) < M * (1.0 + rho);
    if (!ok) break;  // wave-uniform
    // the fold's a[cur][idx] and b_idx(o): lane idx & 63 holds them in slot idx >> 6
    double asel = av[0], esel = ce[0];
#pragma unroll
    for (int k = 1; k < KP; ++k)
      if ((idx >> 6) == k) asel = av[k], esel = ce[k];
    d = (d + readlane_d(asel, idx & 63)) + readlane_d(esel, idx & 63);
    cur = idx;
    const int64_t p = x0 + s + 1;
    if (lane == (int)(p & 63)) pathreg = cur;
    if ((p & 63) == 63 || p == end - 1) {
      const int64_t q = (p & ~(int64_t)63) + lane;
      if (q > x0 && q <= p) g.path[q] = pathreg;
    }
  }
  if (lane == 0) {
    g.cert[i] = ok ? 1 : 0;
    if (ok) {
      g.score[seq] = d;
      g.status[seq] = CVK_SEQ_OK;
    }
  }
}

// Max-marginal at one constrained position (f64; max_marginal_f32 in trellis.hip):
//   beta[i] = max_j(g[j] + a[i,j])  (g = last row of the reversed pass; 0 if no suffix)
//   mu[i]   = delta_tk[i] + beta[i]
template <int NP>
__global__ __launch_bounds__(NP) void max_marginal_f64(MaxMarginal64Args args) {
  __shared__ double g[NP];
  const int i = threadIdx.x;
  const int64_t c = blockIdx.x;
  const bool suffix = args.ranges_suffix[2 * c + 1] > args.ranges_suffix[2 * c];
  g[i] = suffix ? args.g[c * NP + i] : 0.0;
  __syncthreads();
  double beta = 0.0;
  if (suffix) {
    beta = ninf_d();
#pragma unroll 8
    for (int j = 0; j < NP; ++j) beta = fmax(beta, g[j] + args.at[(size_t)j * NP + i]);
  }
  args.mu[c * NP + i] = args.delta[c * NP + i] + beta;
}

__global__ void mu_add_f64(const double* delta, const double* beta, double* mu, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) mu[k] = delta[k] + beta[k];  // max_marginal_f64's delta + beta, the same f64 add
}

__global__ void resume_rows_f64(const double* last, const int32_t* state, int np, double* out) {
  const int64_t i = blockIdx.x;
  const int j = threadIdx.x;
  if (j < np) out[i * np + j] = (j == state[i]) ? last[i * np + j] : ninf_d();
}

// tuning key t64_wg_force = 1 takes the eight-wave layout whatever the batch (T64FwdArgs::wg_ok)
bool wg_force() { return tuning().t64_wg_force != 0; }

// S sequences over a PAIR of waves (C = 2 each, N = 256): the small-batch layout
template <int S>
hipError_t fwd_w2(const T64FwdArgs& fa, int64_t nseq, bool ext, hipStream_t stream) {
  const dim3 grid((unsigned)((nseq + S - 1) / S)), block(128);
  // tuning keys (bit-identical): t64_rs = 0 keeps the column split, t64_wg = 0 one pair per
  // workgroup
  const bool rs_mode = tuning().t64_rs != 0;
  const bool wg_mode = tuning().t64_wg != 0;
  if (ext) {
    hipLaunchKernelGGL((trellis_fwd_f64<2, S, 8, false, true, 2>), grid, block, 0, stream, fa);
    return hipGetLastError();
  }
  if constexpr (S == 8) {
    if (rs_mode && !fa.dp_assoc && (fa.wg_ok || wg_force())) {  // the row split (trellis_fwd_f64_rs)
      T64FwdArgs f4 = fa;
      f4.balance = 0;
      hipLaunchKernelGGL((trellis_fwd_f64_rs<8>), dim3((unsigned)((nseq + 4 * S - 1) / (4 * S))), dim3(512), 0,
                         stream, f4);
      return hipGetLastError();
    }
  }
  if (wg_mode && (fa.wg_ok || wg_force())) {
    // four pairs per workgroup (the CU's eight waves), SIMD partners trade priority
    T64FwdArgs f4 = fa;
    f4.balance = 0;
    hipLaunchKernelGGL((trellis_fwd_f64<2, S, 8, false, false, 2, true, 2, 1, true, 4, 2>),
                       dim3((unsigned)((nseq + 4 * S - 1) / (4 * S))), dim3(512), 0, stream, f4);
  } else {
    hipLaunchKernelGGL((trellis_fwd_f64<2, S, 8, false, false, 2>), grid, block, 0, stream, fa);
  }
  return hipGetLastError();
}

// (Round 4 also ran the constrained passes from a work queue of persistent waves, CV_T64_PERSIST:
// config 5 160.5 vs 154.9 ms, profiles/r04_ab_c5_persist.txt -- 4,096 units over 2,048 waves is
// two units a wave, so the queue cannot even out the ragged tail.  Removed in round 6, with the
// deferred delta stores (DEFST, +1.4%), the compiler-placed delta reads (LDSFIRST = false), the
// 4-row A ring and the partial eight-wave mechanisms (CV_T64_WG = 1..3).)

template <int C, int S>
hipError_t fwd_cs(const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  const int64_t blocks = (nseq + S - 1) / S;
  // tuning key t64_wg (bit-identical): 1 runs the batch decode as eight independent waves per
  // workgroup with a barrier per step and the SIMD-pair priority trade (default), 0 = one wave
  // per workgroup with the global SIMD balancing (round-2 layout).  Config 4 forward 136.4 ->
  // 131.4 ms, 8,192 sequences 18.6 -> 17.7 ms (profiles/r03_ab_wg.txt)
  const bool wg_mode = tuning().t64_wg != 0;
  const bool w2 = tuning().t64_w2 != 0;  // tuning key t64_w2 = 0 keeps one wave per group
  const bool ext = fa.forced || fa.ranges || fa.reverse || fa.start || fa.row_base || fa.resume_rows ||
                   fa.slot_order || fa.last_row;
  // S = 6: three waves per SIMD (<= 168 VGPRs, 12.3 KiB of LDS each), batch decode only
  if constexpr (S == 6) {
    if (ext || fa.dp_assoc) return fwd_cs<C, 4>(fa, nseq, stream);
    // 4 A rows in flight: 157 VGPRs (8 rows spill at 168)
    hipLaunchKernelGGL((trellis_fwd_f64<C, 6, 4, false, false, 1, false, 2, 3>), dim3((unsigned)blocks), dim3(64), 0,
                       stream, fa);
    return hipGetLastError();
  } else {
  // N = 256 and fewer than 8 sequences per wave (small batch): 2S sequences over two waves --
  // the same number of waves, twice the A-row reuse
  if constexpr (C == 4 && S <= 4) {
    if (w2 && !fa.dp_assoc) return fwd_w2<2 * S>(fa, nseq, ext, stream);
  }
  const dim3 grid((unsigned)blocks), block(64);
  // C >= 3 only: at C <= 2 the one-wave workgroups fit three or more waves per SIMD, which beat
  // two aligned ones (N = 128: 37.7 vs 38.1 ms; N = 192: 84.4 -> 81.1 ms; profiles/r03_ab_wg.txt)
  if constexpr (S == 8 && C >= 3) {
    // the constrained passes (EXT) take it too from two rounds of workgroups on (fa.wg_ok)
    if (wg_mode && !fa.dp_assoc && (fa.wg_ok != 0 || wg_force())) {
      // eight independent waves per workgroup (two per SIMD), A-row reads kept together
      const dim3 g8((unsigned)((nseq + 8 * S - 1) / (8 * S))), b8(512);
      T64FwdArgs f8 = fa;
      f8.balance = 0;
      if (ext)
        hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8, false, true, 1, false, 2, 1, true, 8, 3>), g8, b8, 0, stream, f8);
      else
        hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8, false, false, 1, false, 2, 1, true, 8, 3>), g8, b8, 0, stream, f8);
      return hipGetLastError();
    }
  }
  if (fa.dp_assoc) {
    if (ext) return hipErrorInvalidValue;
    if constexpr (S <= 4)
      hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8, true, false>), grid, block, 0, stream, fa);
    else
      return hipErrorInvalidValue;
  } else if (ext) {
    hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8, false, true>), grid, block, 0, stream, fa);
  } else {
    hipLaunchKernelGGL((trellis_fwd_f64<C, S, 8, false, false>), grid, block, 0, stream, fa);
  }
  return hipGetLastError();
  }
}


// trellis_wave_f64<ZI>: N <= 64 (NP = 64) -- ONE WAVE per sequence, A register-resident.
// The lock-step layouts (S sequences per wave) run one round of waves at configs 2/3, so the
// waves holding the longest sequences set the makespan; one sequence per wave gives many
// rounds that the longest-first order balances.  Lane = 4cq + rg holds rows [16 rg, 16 rg + 16)
// of the columns 4cq .. 4cq+3 (64 doubles); delta_{t-1} comes from the wave's own LDS row
// (8 ds_read_b128; row-group stride 18 doubles puts the 4 addresses of an instruction on
// disjoint banks); per pair one v_add_f64 + one v_max_f64; the 4 row-group partials are folded
// across the lane quad by DPP (xor1 keeps a column pair, xor2 one column: lane jw =
// 4cq + 2p + q), then d_t[jw] = m + b (viterbi.rs:15-17).  Rows go to HBM split-plane for
// backtrack_f64.  Emissions are loaded 4 steps ahead with clamped indices, observations by
// scalar loads (as trellis_wave_f32).  ZI: viterbi::decode's row 0 = 0.0.
__device__ __forceinline__ double dpp_f64(double v, int ctrl_is_xor2) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  int lo = (int)(uint32_t)b, hi = (int)(uint32_t)(b >> 32);
  if (ctrl_is_xor2) {
    lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false);
  } else {
    lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  }
  return from_words((uint32_t)hi, (uint32_t)lo);
}

// (Round 3 also had a FUSE variant whose wave backtracked its own sequence right after the
// forward pass: slower -- config 3 3.46 vs 3.22 ms -- and removed in round 6.)
template <bool ZI>
__global__ __launch_bounds__(256) void trellis_wave_f64(T64FwdArgs g) {
  constexpr int NPW = 64, C = 4, R = 16, LS = R + 2;
  __shared__ __attribute__((aligned(16))) double lds_all[4][2][4 * LS];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int rg = lane & 3, cq = lane >> 2;
  const int p = rg & 1, q = rg >> 1;
  const int jw = 4 * cq + 2 * p + q;  // this lane's column after the fold
  const int64_t slot = g.seq_begin + 4 * (int64_t)blockIdx.x + wv;
  if (slot >= g.seq_begin + g.nslots) return;
  const int64_t seq = g.order ? (int64_t)g.order[slot] : slot;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  if (T <= 0) return;  // the backtrack reports empty sequences
  double(*lds)[4 * LS] = lds_all[wv];
  const sptr<int32_t> obs = scalar_view(g.obs + e0);
  uint32_t* __restrict__ rows = reinterpret_cast<uint32_t*>(g.delta) + (e0 - g.delta_elem_base) * (2 * NPW);
  const unsigned V = (unsigned)g.nobs;
  double a_reg[R * C];  // a_reg[C r + k] = A[R rg + r][C cq + k]
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const f64x2* src = reinterpret_cast<const f64x2*>(g.a + (size_t)(R * rg + r) * NPW + C * cq);
    const f64x2 v0 = src[0], v1 = src[1];
    a_reg[C * r + 0] = v0.x;
    a_reg[C * r + 1] = v0.y;
    a_reg[C * r + 2] = v1.x;
    a_reg[C * r + 3] = v1.y;
  }
  unsigned bad = 0;
  auto obs_s = [&](int t) -> unsigned {
    const unsigned o = (unsigned)obs[t];
    bad |= (o >= V);
    return o < V ? o : 0u;
  };
  auto put = [&](int t, double v) {
    uint32_t* r = rows + (size_t)t * (2 * NPW) + jw;
    __builtin_nontemporal_store(hi_word(v), r);
    __builtin_nontemporal_store(lo_word(v), r + NPW);
  };
  const int wofs = (jw / R) * LS + (jw % R);  // where this lane's column lives in an LDS row
  {
    const double d0 = ZI ? 0.0 : g.pi[jw] + g.et[(size_t)obs_s(0) * NPW + jw];  // cp.rs:66-68
    lds[0][wofs] = d0;
    put(0, d0);
  }
  const int Tm1 = T - 1;
  unsigned so[4];
  double pe[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    pe[k] = g.et[(size_t)obs_s(min(1 + k, Tm1)) * NPW + jw];  // steps 1..4
    so[k] = obs_s(min(5 + k, Tm1));                           // observations of steps 5..8
  }
  for (int t0 = 1; t0 < T; t0 += 4) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = t0 + k;
      if (t >= T) break;
      const double* src = &lds[(t - 1) & 1][rg * LS];
      f64x2 d[R / 2];
#pragma unroll
      for (int b = 0; b < R / 2; ++b) d[b] = *reinterpret_cast<const f64x2*>(src + 2 * b);
      double c[C];
#pragma unroll
      for (int kc = 0; kc < C; ++kc) {
        double m = d[0].x + a_reg[kc];  // s_i = d[i] + a[i,j]  (viterbi.rs:15)
        m = __builtin_fmax(m, d[0].y + a_reg[C + kc]);
#pragma unroll
        for (int b = 1; b < R / 2; ++b) {
          m = __builtin_fmax(m, d[b].x + a_reg[(2 * b) * C + kc]);
          m = __builtin_fmax(m, d[b].y + a_reg[(2 * b + 1) * C + kc]);
        }
        c[kc] = m;
      }
      // fold the 4 row groups of the quad: xor1 keeps columns {2p, 2p+1}, xor2 keeps 2p+q
      double k0 = p ? c[2] : c[0], k1 = p ? c[3] : c[1];
      const double g0 = p ? c[0] : c[2], g1 = p ? c[1] : c[3];
      k0 = __builtin_fmax(k0, dpp_f64(g0, 0));
      k1 = __builtin_fmax(k1, dpp_f64(g1, 0));
      double kk = q ? k1 : k0;
      const double gg = q ? k0 : k1;
      kk = __builtin_fmax(kk, dpp_f64(gg, 1));
      const double dn = kk + pe[k];  // (d + a) + b -- viterbi.rs:15-17
      lds[t & 1][wofs] = dn;
      put(t, dn);
      pe[k] = g.et[(size_t)so[k] * NPW + jw];  // step t+4
      so[k] = obs_s(min(t + 8, Tm1));          // observation of step t+8
    }
  }
  if (bad && lane == 0) g.status[seq] = CVK_SEQ_BADOBS;
}

// trellis_wave48_f64<ZI>: N <= 48 (config 2's N = 45) -- one wave per sequence like
// trellis_wave_f64, on the 48 states that exist instead of 64 padded ones (1.8x fewer pairs),
// in at most 128 VGPRs so FOUR waves share a SIMD (one round of 4,096 sequences on the chip,
// workgroups of the longest-first order spread one per quartile onto every CU).  Lane
// l = 4 cq + rg holds A[12 rg + r][3 cq + k] (r < 12, k < 3: 72 VGPRs) and walks its 12 rows for
// its 3 columns (36 pairs, one v_add_f64 + one v_max_f64 each); the 4 row groups' partial
// maxima meet in LDS (part[col][rg], written and read back by the same wave: LDS executes a
// wave's operations in order), lane j < 48 takes the max of its column's 4 partials and adds
// the emission.  Max is exact and order-free, so values, rows and results are those of
// trellis_wave_f64 bit for bit.  Rows go to HBM split-plane, 64 wide, for backtrack_f64
// (columns >= N are never read: the backtrack masks candidates >= N).
// Workgroups go to the CUs round-robin (block b and b + 256 share a CU), so a grid of four
// rounds puts one workgroup of each quarter of the longest-first order on every CU; the odd
// quarters run reversed (the block of rank r takes slots of rank 255 - r there), so every CU
// and SIMD gets long with short sequences: equal sums instead of the longest of each quarter.
#ifndef CVK_W48_PD
#define CVK_W48_PD 4  // emission rows prefetched this many steps ahead (A/B builds: -DCVK_W48_PD=n)
#endif
#ifdef CVK_W48_PROBE
// Probe build only (tools/w48_probe.py): per sequence s_memrealtime (100 MHz) after the
// sequence's offsets, at the end, at entry, after delta_0, after the first PD-step block (0 if
// none), HW_ID, XCC_ID, T -- written by lanes 0..7 with vector stores.
__device__ unsigned long long cvk_w48_probe[8192][8];
#endif
template <bool ZI, int PD = CVK_W48_PD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void trellis_wave48_f64(T64FwdArgs g) {
  constexpr int NPW = 64, C = 3, R = 12, LS = NPW + 4, P = 256;
  __shared__ __attribute__((aligned(16))) double dl_all[4][2][LS];     // delta_{t-1} / delta_t per wave
  __shared__ __attribute__((aligned(16))) double part_all[4][NPW][4];  // [col][rg] partial maxima
  const int lane = threadIdx.x & 63;
#ifdef CVK_W48_PROBE
  const unsigned long long pre = __builtin_amdgcn_s_memrealtime();
#endif
  const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int rg = lane & 3, cq = lane >> 2;
  int blk = (int)blockIdx.x;
  {
    const int q = blk / P, r = blk % P;
    if ((q & 1) && (q + 1) * P <= (int)gridDim.x) blk = q * P + (P - 1 - r);
  }
  const int64_t slot = g.seq_begin + 4 * (int64_t)blk + wv;
  if (slot >= g.seq_begin + g.nslots) return;
  const int64_t seq = g.order ? (int64_t)g.order[slot] : slot;
  const int64_t e0 = g.offsets[seq];
  const int T = (int)(g.offsets[seq + 1] - e0);
  if (T <= 0) return;  // the backtrack reports empty sequences
  double(*dl)[LS] = dl_all[wv];
  double(*part)[4] = part_all[wv];
#ifdef CVK_W48_PROBE
  const unsigned long long pr0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long prd0 = 0, prb1 = 0;
#endif
  // Every lane runs every instruction of a step (lanes >= 48 fold columns 48..63, which no
  // partial reaches: their rows land in the 64-wide rows' padding, which the backtrack masks),
  // so no branch splits the step's memory operations and the waits before each use count only
  // what is outstanding; observations come through per-lane (vector) loads of one uniform
  // address, so no scalar load shares the LDS reads' counter.
  int vz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));  // a per-lane zero: keeps the observation loads on the vector path
  const int32_t* __restrict__ obs = g.obs + e0 + vz;
  uint32_t* __restrict__ rows = reinterpret_cast<uint32_t*>(g.delta) + (e0 - g.delta_elem_base) * (2 * NPW);
  const unsigned V = (unsigned)g.nobs;
  const int Tm1 = T - 1;
  // Start-up: the observations of steps 0..2PD (and pi) in one batch, then A (L2), then the
  // emissions of steps 0..PD in one batch -- the chain before step 1 is offsets -> observations
  // -> emissions with the A loads beside it, not two observation -> emission round trips
  // queued behind the A loads (V = 50,000 at config 2: a 25.6 MB emission table, beyond L2)
  const unsigned ob0 = (unsigned)obs[0];
  const double pil = ZI ? 0.0 : g.pi[lane];
  unsigned sp[PD], so[PD];
#pragma unroll
  for (int k = 0; k < PD; ++k) {
    sp[k] = (unsigned)obs[min(1 + k, Tm1)];       // observations of steps 1..PD
    so[k] = (unsigned)obs[min(PD + 1 + k, Tm1)];  // observations of steps PD+1..2PD
  }
  double a_reg[R * C];  // a_reg[C r + k] = A[R rg + r][C cq + k]
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double* src = g.a + (size_t)(R * rg + r) * NPW + C * cq;
#pragma unroll
    for (int k = 0; k < C; ++k) a_reg[C * r + k] = src[k];
  }
  part[lane][0] = part[lane][1] = part[lane][2] = part[lane][3] = 0.0;  // columns 48..63 stay 0
  unsigned bad = 0;
  auto eaddr = [&](unsigned o) -> const double* {
    bad |= (o >= V);
    return g.et + (size_t)(o < V ? o : 0u) * NPW + lane;
  };
  auto put = [&](int t, double v) {
    uint32_t* r = rows + (size_t)t * (2 * NPW) + lane;
    __builtin_nontemporal_store(hi_word(v), r);
    __builtin_nontemporal_store(lo_word(v), r + NPW);
  };
  const double e0v = ZI ? 0.0 : *eaddr(ob0);
  double pe[PD];  // emissions PD steps ahead
#pragma unroll
  for (int k = 0; k < PD; ++k) pe[k] = *eaddr(sp[k]);  // steps 1..PD
  {
    const double d0 = ZI ? 0.0 : pil + e0v;  // cp.rs:66-68
    dl[0][lane] = d0;
    __builtin_amdgcn_wave_barrier();
    put(0, d0);
#ifdef CVK_W48_PROBE
    prd0 = __builtin_amdgcn_s_memrealtime() + (unsigned long long)(d0 == 12345.0);  // after delta_0
#endif
  }
  auto step = [&](int t, int k) {
    const double* src = &dl[(t - 1) & 1][R * rg];
    // row-major: each pair of delta rows is consumed by the 3 columns as it arrives, so few
    // delta VGPRs are live beside A's 72 (four waves per SIMD leave 128)
    double m[C];
#pragma unroll
    for (int b = 0; b < R / 2; ++b) {
      const f64x2 d = *reinterpret_cast<const f64x2*>(src + 2 * b);
#pragma unroll
      for (int kc = 0; kc < C; ++kc) {
        const double x = d.x + a_reg[2 * b * C + kc];  // s_i = d[i] + a[i,j]  (viterbi.rs:15)
        m[kc] = b == 0 ? x : __builtin_fmax(m[kc], x);
        m[kc] = __builtin_fmax(m[kc], d.y + a_reg[(2 * b + 1) * C + kc]);
      }
    }
#pragma unroll
    for (int kc = 0; kc < C; ++kc) part[C * cq + kc][rg] = m[kc];
    __builtin_amdgcn_wave_barrier();  // the partials are other lanes' (LDS: in wave order)
    const f64x2 p01 = *reinterpret_cast<const f64x2*>(&part[lane][0]);
    const f64x2 p23 = *reinterpret_cast<const f64x2*>(&part[lane][2]);
    const double mx = __builtin_fmax(__builtin_fmax(p01.x, p01.y), __builtin_fmax(p23.x, p23.y));
    const double dn = mx + pe[k];  // (d + a) + b -- viterbi.rs:15-17
    dl[t & 1][lane] = dn;
    __builtin_amdgcn_wave_barrier();  // delta_t before the next step's reads
    put(t, dn);
    pe[k] = *eaddr(so[k]);                        // step t+PD
    so[k] = (unsigned)obs[min(t + 2 * PD, Tm1)];  // observation of step t+2PD
  };
  // whole blocks of PD steps with no exit inside, so the loop's back edge carries one count of
  // outstanding loads and the wait for a step's emission covers only loads issued PD steps ago
  int t0 = 1;
  for (; t0 + PD <= T; t0 += PD) {
#pragma unroll
    for (int k = 0; k < PD; ++k) step(t0 + k, k);
#ifdef CVK_W48_PROBE
    if (t0 == 1) prb1 = __builtin_amdgcn_s_memrealtime();
#endif
  }
#pragma unroll
  for (int k = 0; k < PD - 1; ++k)
    if (t0 + k < T) step(t0 + k, k);
  if (bad) g.status[seq] = CVK_SEQ_BADOBS;
#ifdef CVK_W48_PROBE
  {
    const unsigned long long pr1 = __builtin_amdgcn_s_memrealtime();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4), xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    if (lane < 8 && seq < 8192) {  // lane-indexed: a vector store per lane
      const unsigned long long v[8] = {pr0, pr1, pre, prd0, hw, xcc, (unsigned long long)T, prb1};
      unsigned long long x = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) x = lane == i ? v[i] : x;
      cvk_w48_probe[seq][lane] = x;
    }
  }
#endif
}

#ifdef CVK_W48_PROBE
}  // namespace
}  // namespace cvk
extern "C" int cvk_w48_probe_read(void* dst, size_t bytes) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(cvk::cvk_w48_probe), bytes, 0, hipMemcpyDeviceToHost);
}
namespace cvk {
namespace {
#endif
hipError_t launch_t64_wave(const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  // (a two-sequences-per-wave variant, three waves per SIMD, measured 0.153 vs 0.070 ms at
  // config 2 and was removed)
  const dim3 grid((unsigned)((nseq + 3) / 4)), block(256);
  // N <= 48: the 48-state layout at four waves per SIMD (tuning key t64_wave = 2: always the
  // 64-state one)
  const bool w48 = fa.nstates > 0 && fa.nstates <= 48 && tuning().t64_wave != 2;
  if (w48 && fa.zero_init)
    hipLaunchKernelGGL(trellis_wave48_f64<true>, grid, block, 0, stream, fa);
  else if (w48)
    hipLaunchKernelGGL(trellis_wave48_f64<false>, grid, block, 0, stream, fa);
  else if (fa.zero_init)
    hipLaunchKernelGGL(trellis_wave_f64<true>, grid, block, 0, stream, fa);
  else
    hipLaunchKernelGGL(trellis_wave_f64<false>, grid, block, 0, stream, fa);
  return hipGetLastError();
}

template <int C>
hipError_t fwd_c(const T64FwdArgs& fa, int s, int64_t nseq, hipStream_t stream) {
  switch (s) {
    case 2: return fwd_cs<C, 2>(fa, nseq, stream);
    case 4: return fwd_cs<C, 4>(fa, nseq, stream);
    case 6: return fwd_cs<C, 6>(fa, nseq, stream);
    case 8: return fwd_cs<C, 8>(fa, nseq, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// PF: A rows in flight per wave.  Split columns (W > 1, C = 1): a wave's step is 256 dependent
// row loads of 8 B per lane from L2, so the ring must cover the L2 latency (PF = 32: 64 VGPRs)
template <int C, int W = 1, int PF = 4>
hipError_t cp_c(const T64FwdArgs& fa, int s, int64_t nseq, hipStream_t stream) {
  const dim3 block(64 * W);
  switch (s) {
    case 1: hipLaunchKernelGGL((trellis_cp_f64<C, 1, PF, W>), dim3((unsigned)nseq), block, 0, stream, fa); break;
    case 2: hipLaunchKernelGGL((trellis_cp_f64<C, 2, PF, W>), dim3((unsigned)((nseq + 1) / 2)), block, 0, stream, fa); break;
    case 4: hipLaunchKernelGGL((trellis_cp_f64<C, 4, PF, W>), dim3((unsigned)((nseq + 3) / 4)), block, 0, stream, fa); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// waves per workgroup splitting the columns (trellis_cp_f64's W): NP / 64 for the batches of at
// most 4,096 sequences (the parallel chain's speculative re-decodes), else 1; tuning key
// t64_cp_w = 1 keeps one wave per workgroup, > 1 forces the split
int t64_cp_waves(int np, int64_t nseq) {
  const int k = tuning().t64_cp_w;
  if (k == 1 || np < 128) return 1;
  return (k > 1 || nseq <= 4096) ? np / 64 : 1;
}

int t64_cp_seqs_per_wave(int s, int64_t nseq, int w) {
  s = s > 4 ? 4 : s;  // the argmax state (idx) costs registers: at most 4 sequences per wave
  // a batch that leaves SIMDs idle at two sequences per wave: one per wave (the sequences are
  // independent, so the results are the same); tuning key t64_cp_s = 1 / 2 / 4 sets it; split
  // columns (w > 1): 4 sequences share each A element
  if (const int k = tuning().t64_cp_s; k > 0) return k >= 4 ? 4 : k >= 2 ? 2 : 1;
  if (w > 1) return 4;
  return nseq <= 1024 ? 1 : s;
}

hipError_t launch_t64_cp_fwd(int np, int s, const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  const int w = t64_cp_waves(np, nseq);
  s = t64_cp_seqs_per_wave(s, nseq, w);
  if (w > 1) {
    const bool pf16 = tuning().t64_cp_pf == 16;  // A/B: 16 rows in flight instead of 32
    switch (np) {
      case 128: return pf16 ? cp_c<1, 2, 16>(fa, s, nseq, stream) : cp_c<1, 2, 32>(fa, s, nseq, stream);
      case 192: return pf16 ? cp_c<1, 3, 16>(fa, s, nseq, stream) : cp_c<1, 3, 32>(fa, s, nseq, stream);
      case 256: return pf16 ? cp_c<1, 4, 16>(fa, s, nseq, stream) : cp_c<1, 4, 32>(fa, s, nseq, stream);
      default: return hipErrorInvalidValue;
    }
  }
  switch (np) {
    case 64: return cp_c<1>(fa, s, nseq, stream);
    case 128: return cp_c<2>(fa, s, nseq, stream);
    case 192: return cp_c<3>(fa, s, nseq, stream);
    case 256: return cp_c<4>(fa, s, nseq, stream);
    default: return hipErrorInvalidValue;
  }
}

#ifdef CV_T64_PROBE
extern "C" __attribute__((visibility("default"))) int cv_debug_t64_probe(uint64_t* out, int nwaves) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t64_probe), sizeof(uint64_t) * 6 * (size_t)nwaves, 0,
                                  hipMemcpyDeviceToHost);
}
#endif

int t64_padded_states(int n) { return (n >= 1 && n <= 256) ? 64 * ((n + 63) / 64) : 0; }

// The batch decode's f64 trellis (VITERBI / DECODE rows, no forced states) also covers
// 256 < N <= 512: NP = 512 as PAIRS of C = 4 waves splitting the columns (the W = 2 layout of
// the small-batch kernel with the full batch's C), four pairs per workgroup, and backtrack_f64
// at KP = 8.  Tuning key t64_512 = 0: the generic kernels (bit-identical).
int t64_batch_states(int n) {
  if (n <= 256) return t64_padded_states(n);
  if (n <= 512) return tuning().t64_512 != 0 ? 512 : 0;
  // 512 < N <= 1,024: QUADS of C = 4 waves, where A (N^2 f64) outgrows an XCD's 4 MiB L2
  // (N > 724) and the generic kernels turn HBM-bound: 16,384 x 128 at N = 800 188 vs 455 ms,
  // N = 1,024 191 vs 552 ms; at N = 600 the padding loses (179 vs 139 ms;
  // profiles/r04_large_n.txt).  Tuning key t64_1024 = 0 / 1: never / always
  if (n > 1024) return 0;
  if (const int k = tuning().t64_1024; k == 0 || k == 1) return k == 1 ? 1024 : 0;
  return n > 724 ? 1024 : 0;
}

// every NP the f64 trellis kernels support at this N (an explicit CV_KERNEL_TRELLIS_F64
// request, and the handle's padded tables): 64 * ceil(N / 64) up to 256, then 512 and 1,024
int t64_support_states(int n) {
  if (n <= 256) return t64_padded_states(n);
  return n <= 512 ? 512 : n <= 1024 ? 1024 : 0;
}

template <int S>
hipError_t fwd_1024(const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  const dim3 grid((unsigned)((nseq + S - 1) / S)), block(256);
  if (fa.forced)
    hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, false, true, 4>), grid, block, 0, stream, fa);
  else if (fa.dp_assoc) {
    if constexpr (S <= 4)
      hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, true, false, 4>), grid, block, 0, stream, fa);
    else
      return hipErrorInvalidValue;
  } else
    hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, false, false, 4>), grid, block, 0, stream, fa);
  return hipGetLastError();
}

template <int S>
hipError_t fwd_512(const T64FwdArgs& fa, int64_t nseq, hipStream_t stream) {
  if (fa.forced) {  // forced states (EXT), one pair per workgroup
    hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, false, true, 2>), dim3((unsigned)((nseq + S - 1) / S)), dim3(128), 0,
                       stream, fa);
    return hipGetLastError();
  }
  if (fa.dp_assoc) {  // DPSolver's (a + b) + d, one pair per workgroup (S <= 4: the emissions in registers)
    if constexpr (S <= 4) {
      hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, true, false, 2>), dim3((unsigned)((nseq + S - 1) / S)), dim3(128), 0,
                         stream, fa);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (fa.wg_ok || wg_force()) {  // four pairs per workgroup, SIMD partners trade priority
    T64FwdArgs f4 = fa;
    f4.balance = 0;
    hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, false, false, 2, true, 2, 1, true, 4, 2>),
                       dim3((unsigned)((nseq + 4 * S - 1) / (4 * S))), dim3(512), 0, stream, f4);
  } else {
    hipLaunchKernelGGL((trellis_fwd_f64<4, S, 8, false, false, 2>), dim3((unsigned)((nseq + S - 1) / S)), dim3(128), 0,
                       stream, fa);
  }
  return hipGetLastError();
}

int t64_seqs_per_wave(int64_t nseq, int cus, int np) {
  // fill at least two waves per SIMD (4 SIMDs per CU), then prefer the larger S: each A row
  // streamed from L2 serves S sequences.  NP = 512 / 1,024 units are pairs / quads of waves
  // over the same S sequences (W = NP / 256 waves each), so W times fewer sequences fill the
  // chip: at NP = 1,024, where A (8 MiB) streams from beyond an XCD's L2 every step, S = 2
  // doubled that stream (4,096 x 512 at N = 1,024: ~0.8 s forward at S = 2)
  if (const int s = tuning().t64_s; s == 2 || s == 4 || s == 6 || s == 8) return s;  // tuning key (bit-identical)
  const int64_t w = np >= 512 ? np / 256 : 1;
  const int64_t simd_waves = 2 * 4 * (int64_t)(cus > 0 ? cus : 256);
  if (nseq * w >= 8 * simd_waves) return 8;
  if (nseq * w >= 4 * simd_waves) return 4;
  return 2;
}

hipError_t launch_t64_fwd(int np, int s, const T64FwdArgs& fa_in, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  const int balance = tuning().t64_bal;  // tuning key (bit-identical): steps between SIMD balancing, 0 = off
  T64FwdArgs fa = fa_in;
  // the batch decode only: the constrained decode's passes (EXT, 2 sequences per wave, two
  // streams) ran ~2% slower balanced (profiles/r02_t64_simd_balance.txt)
  fa.balance = (fa.forced || fa.ranges || fa.reverse || fa.start || fa.row_base || fa.resume_rows ||
                fa.slot_order || fa.last_row) ? 0 : balance;
  const bool wave = tuning().t64_wave != 0;  // tuning key t64_wave = 0 keeps the lock-step layout
  const bool ext = fa.forced || fa.ranges || fa.reverse || fa.start || fa.row_base || fa.resume_rows ||
                   fa.slot_order || fa.last_row;
  if (np == 64 && wave && !fa.dp_assoc && !ext) return launch_t64_wave(fa, nseq, stream);
  if (np == 512 || np == 1024) {  // batch decode only (t64_batch_states), forced states allowed
    if (fa.ranges || fa.reverse || fa.start || fa.row_base || fa.resume_rows || fa.slot_order || fa.last_row ||
        (fa.dp_assoc && fa.forced))
      return hipErrorInvalidValue;
    if ((fa.forced || fa.dp_assoc) && s > 4) s = 4;  // EXT at S = 8: 275 VGPRs + 19 AGPRs, one wave per SIMD
    if (np == 1024) {
      if (s > 4) s = 4;  // the quad's LDS slice: (NP + 3) x S doubles
      return s == 4 ? fwd_1024<4>(fa, nseq, stream) : fwd_1024<2>(fa, nseq, stream);
    }
    switch (s) {
      case 8: return fwd_512<8>(fa, nseq, stream);
      case 4: return fwd_512<4>(fa, nseq, stream);
      default: return fwd_512<2>(fa, nseq, stream);
    }
  }
  if (fa.dp_assoc && s > 4) s = 4;  // the emissions of every sequence stay in registers
  switch (np) {
    case 64: return fwd_c<1>(fa, s, nseq, stream);
    case 128: return fwd_c<2>(fa, s, nseq, stream);
    case 192: return fwd_c<3>(fa, s, nseq, stream);
    case 256: return fwd_c<4>(fa, s, nseq, stream);
    default: return hipErrorInvalidValue;
  }
}

template <int PF, bool NONPOS>
hipError_t bt_pf_np(int np, const T64BtArgs& ba, dim3 grid, dim3 block, hipStream_t stream) {
  if constexpr (PF == 32) {  // NP = 64 only (launch_t64_bt)
    if (np != 64) return hipErrorInvalidValue;
    hipLaunchKernelGGL((backtrack_f64<1, PF, NONPOS>), grid, block, 0, stream, ba);
  } else {
    switch (np) {
      case 64: hipLaunchKernelGGL((backtrack_f64<1, PF, NONPOS>), grid, block, 0, stream, ba); break;
      case 128: hipLaunchKernelGGL((backtrack_f64<2, PF, NONPOS>), grid, block, 0, stream, ba); break;
      case 192: hipLaunchKernelGGL((backtrack_f64<3, PF, NONPOS>), grid, block, 0, stream, ba); break;
      case 256: hipLaunchKernelGGL((backtrack_f64<4, PF, NONPOS>), grid, block, 0, stream, ba); break;
      case 512:
        if constexpr (PF <= 8) {
          hipLaunchKernelGGL((backtrack_f64<8, PF, NONPOS>), grid, block, 0, stream, ba);
          break;
        }
        return hipErrorInvalidValue;
      case 1024:
        if constexpr (PF <= 4) {
          hipLaunchKernelGGL((backtrack_f64<16, PF, NONPOS>), grid, block, 0, stream, ba);
          break;
        }
        return hipErrorInvalidValue;
      default: return hipErrorInvalidValue;
    }
  }
  return hipGetLastError();
}

template <int PF>
hipError_t bt_pf(int np, const T64BtArgs& ba, dim3 grid, dim3 block, hipStream_t stream) {
  if (ba.cert) {  // the parallel chain's certified backtrack (NONPOS row A0, N <= 256)
    if (!ba.at32 || ba.dp_assoc || ba.decode_bt) return hipErrorInvalidValue;
    switch (np) {
      case 64: hipLaunchKernelGGL((backtrack_f64<1, PF, true, true>), grid, block, 0, stream, ba); break;
      case 128: hipLaunchKernelGGL((backtrack_f64<2, PF, true, true>), grid, block, 0, stream, ba); break;
      case 192: hipLaunchKernelGGL((backtrack_f64<3, PF, true, true>), grid, block, 0, stream, ba); break;
      case 256: hipLaunchKernelGGL((backtrack_f64<4, PF, true, true>), grid, block, 0, stream, ba); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (ba.at32) {
    hipError_t e = bt_pf_np<PF, true>(np, ba, grid, block, stream);
    if (e == hipSuccess && ba.decode_bt) {  // viterbi::decode: the infeasible sequences' DEC chains
      T64BtArgs b2 = ba;
      b2.only_infeasible = 1;
      e = bt_pf_np<PF, false>(np, b2, grid, block, stream);
    }
    return e;
  }
  return bt_pf_np<PF, false>(np, ba, grid, block, stream);
}

hipError_t launch_t64_bt(int np, const T64BtArgs& ba, int64_t nseq, hipStream_t stream) {
  if (nseq <= 0) return hipSuccess;
  const dim3 grid((unsigned)((nseq + 3) / 4)), block(256);
  // NP = 64 (configs 2/3): the longest chains set the makespan and each step's hi row (256 B)
  // comes from HBM: 32 rows in flight, config 3 backtrack 0.615 -> 0.51 ms (16: 0.54)
  // (profiles/r02_ab_bt_pf_c3.txt); N = 256: occupancy matters more (2 rows, 8 waves/SIMD);
  // tuning key t64_bt_pf (bit-identical) sets 2, 4, 8, 16 or 32
  const int pf_key = tuning().t64_bt_pf;
  const int pf = pf_key ? pf_key : np >= 192 ? 2 : np == 64 ? 32 : 8;
  switch (pf) {
    case 2: return bt_pf<2>(np, ba, grid, block, stream);
    case 4: return bt_pf<4>(np, ba, grid, block, stream);
    case 16: return bt_pf<16>(np, ba, grid, block, stream);
    case 32: return np == 64 ? bt_pf<32>(np, ba, grid, block, stream) : hipErrorInvalidValue;
    default: return bt_pf<8>(np, ba, grid, block, stream);
  }
}

hipError_t launch_t64_prefix_bt(int np, const PrefixBt64Args& a, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 3) / 4)), block(256);
#define CVK_PBT(KP)                                                                   \
  do {                                                                                \
    if (a.at32)                                                                       \
      hipLaunchKernelGGL((prefix_backtrack_f64<KP, true>), grid, block, 0, stream, a, n); \
    else                                                                              \
      hipLaunchKernelGGL((prefix_backtrack_f64<KP, false>), grid, block, 0, stream, a, n); \
  } while (0)
  switch (np) {
    case 64: CVK_PBT(1); break;
    case 128: CVK_PBT(2); break;
    case 192: CVK_PBT(3); break;
    case 256: CVK_PBT(4); break;
    default: return hipErrorInvalidValue;
  }
#undef CVK_PBT
  return hipGetLastError();
}

hipError_t launch_t64_max_marginal(int np, const MaxMarginal64Args& a, int64_t ncon, hipStream_t stream) {
  if (ncon <= 0) return hipSuccess;
  const dim3 grid((unsigned)ncon);
  switch (np) {
    case 64: hipLaunchKernelGGL(max_marginal_f64<64>, grid, dim3(64), 0, stream, a); break;
    case 128: hipLaunchKernelGGL(max_marginal_f64<128>, grid, dim3(128), 0, stream, a); break;
    case 192: hipLaunchKernelGGL(max_marginal_f64<192>, grid, dim3(192), 0, stream, a); break;
    case 256: hipLaunchKernelGGL(max_marginal_f64<256>, grid, dim3(256), 0, stream, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_t64_mu_add(const double* delta, const double* beta, double* mu, int64_t n1, int np,
                             hipStream_t stream) {
  const int64_t n = n1 * np;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mu_add_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, delta, beta, mu, n);
  return hipGetLastError();
}

hipError_t launch_t64_resume_rows(const double* last, const int32_t* state, int64_t n, int np, double* out,
                                  hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (np <= 0 || np > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(resume_rows_f64, dim3((unsigned)n), dim3(256), 0, stream, last, state, np, out);
  return hipGetLastError();
}

hipError_t launch_t64_suffix_trace(int np, const SuffixTrace64Args& a, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 3) / 4)), block(256);
  switch (np) {
    case 64: hipLaunchKernelGGL(suffix_trace_f64<1>, grid, block, 0, stream, a, n); break;
    case 128: hipLaunchKernelGGL(suffix_trace_f64<2>, grid, block, 0, stream, a, n); break;
    case 192: hipLaunchKernelGGL(suffix_trace_f64<3>, grid, block, 0, stream, a, n); break;
    case 256: hipLaunchKernelGGL(suffix_trace_f64<4>, grid, block, 0, stream, a, n); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---- CPSolver's super-sequence decode, chained exactly (cp.rs:63-93 over utils.rs:62-103) ----
// The reference decodes the whole batch as ONE super-sequence: at a sequence start the
// predecessor term is the constant pi[j] (utils.rs:32-38), so every value of sequence k
// carries the running total of sequences 0..k-1 and rounds accordingly.  A per-sequence
// decode is the same up to those roundings; this kernel reproduces them: one workgroup walks
// the elements in order, thread j = state j (states strided over 1,024 threads above that): first argmax over i of prev[i] + trans(i, j)
// (strict '>' from i = 0), value prev[psi] + (trans(psi, j) + b[j, o]) (cp.rs:70-79), psi
// stored as u16; then the first argmax of the last row and the backtrack (cp.rs:85-93).
// Serial over elements (as the reference is): for the main.rs workflow, not the batch path.
// A is staged in LDS when it fits (N <= 126: N^2 + 2N doubles <= 160 KiB), otherwise read
// from L2 with the candidate loop unrolled so the loads overlap.  Above N = 1,024 (states
// strided over the workgroup's threads) the wide kernels below run instead (cp_chain_wide).
template <bool LDS_A>
__global__ __launch_bounds__(1024) void cp_superseq_chain(CpChainArgs g) {
  extern __shared__ double rowbuf[];  // [2][N] (+ [N][N] A when LDS_A)
  const int N = g.nstates;
  const int64_t L = g.len;
  double* prev = rowbuf;
  double* cur = rowbuf + N;
  const double* A = g.a;
  if constexpr (LDS_A) {
    double* la = rowbuf + 2 * N;
    for (int k = threadIdx.x; k < N * N; k += blockDim.x) la[k] = g.a[k];
    A = la;
  }
  // N > 1024: thread j owns states j, j + 1024, ... (each state's candidate loop is its own)
  for (int j = threadIdx.x; j < N; j += blockDim.x)  // cp.rs:66-68, or the row before this part
    prev[j] = g.init_row ? g.init_row[j] : g.pi[j] + g.et[(size_t)g.obs[0] * N + j];
  __syncthreads();
  for (int64_t t = g.init_row ? 0 : 1; t < L; ++t) {
    const int o = g.obs[t];
    const bool first = g.first[t] != 0;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      const double pj = g.pi[j];
      double m = prev[0] + (first ? pj : A[j]);
      int arg = 0;
#pragma unroll 8
      for (int i = 1; i < N; ++i) {
        const double x = prev[i] + (first ? pj : A[(size_t)i * N + j]);
        if (x > m) {
          m = x;
          arg = i;
        }
      }
      const double tr = first ? pj : A[(size_t)arg * N + j];
      cur[j] = prev[arg] + (tr + g.et[(size_t)o * N + j]);
      g.psi[t * N + j] = (uint16_t)arg;
    }
    __syncthreads();
    double* tmp = prev;
    prev = cur;
    cur = tmp;
  }
  if (g.final_row)
    for (int j = threadIdx.x; j < N; j += blockDim.x) g.final_row[j] = prev[j];
  if (threadIdx.x == 0) {
    int cs = 0;
    double obj = prev[0];
    for (int i = 1; i < N; ++i)
      if (prev[i] > obj) {
        obj = prev[i];
        cs = i;
      }
    *g.objective = obj;
    if (g.final_state) *g.final_state = cs;
    if (g.path)
      for (int64_t t = L - 1; t >= 0; --t) {
        g.path[t] = cs;
        cs = g.psi[t * N + cs];
      }
  }
}

// The chain wide: element t's states over ceil(N / 256) workgroups, one launch per element, the
// two rows in g.grows ([2][N], row t & 1 is element t's) -- one workgroup would stream the
// N x N table (>= 800 MB above N = 10,240) through a single CU per element.  Same candidates,
// order and roundings as cp_superseq_chain (cp.rs:70-79 over utils.rs:24-38).  Element 0
// without init_row seeds pi + b (cp.rs:66-68); with it, the host has put init_row in row 1.
__global__ __launch_bounds__(256) void cp_chain_wide_step(CpChainArgs g, int64_t t) {
  __shared__ double tile[256];
  const int N = g.nstates;
  const int j = (int)blockIdx.x * 256 + (int)threadIdx.x;
  const bool jv = j < N;  // threads past N stay for the tile barriers
  const int jc = jv ? j : N - 1;
  double* cur = g.grows + (t & 1) * N;
  const double* prev[1] = {g.grows + ((t & 1) ^ 1) * N};
  const int o = g.obs[t];
  if (t == 0 && !g.init_row) {  // workgroup-uniform
    if (jv) cur[j] = g.pi[j] + g.et[(size_t)o * N + j];
    return;
  }
  const bool first = g.first[t] != 0;
  const double pj = g.pi[jc];
  const double* __restrict__ col = g.a + jc;
  const double e[1] = {0.0};
  double m[1];
  int arg[1];
  // the first index of the maximum of prev[i] + (first ? pi[j] : a[i][j]) (strict '>' from -inf:
  // i = 0 seeds it whenever it is above -inf, as cp_superseq_chain's m = prev[0] + ...)
  wide_candidates<double, 1, false>(first ? nullptr : col, N, prev, e, m, arg, tile, pj);
  if (!jv) return;
  const double tr = first ? pj : col[(size_t)arg[0] * N];
  cur[j] = prev[0][arg[0]] + (tr + g.et[(size_t)o * N + j]);
  g.psi[t * N + j] = (uint16_t)arg[0];
}

// the last row's first argmax (cp.rs:85-87), final_row, and the single-thread backtrack when
// g.path is set (cp.rs:88-93)
__global__ __launch_bounds__(1024) void cp_chain_wide_finish(CpChainArgs g) {
  const int N = g.nstates;
  const double* last = g.grows + ((g.len - 1) & 1) * N;
  if (g.final_row)
    for (int j = threadIdx.x; j < N; j += blockDim.x) g.final_row[j] = last[j];
  if (threadIdx.x != 0) return;
  int cs = 0;
  double obj = last[0];
  for (int i = 1; i < N; ++i)
    if (last[i] > obj) {
      obj = last[i];
      cs = i;
    }
  *g.objective = obj;
  if (g.final_state) *g.final_state = cs;
  if (g.path)
    for (int64_t t = g.len - 1; t >= 0; --t) {
      g.path[t] = cs;
      cs = g.psi[t * N + cs];
    }
}

bool cp_chain_wide(int n) {
  if (n > kChainLdsMaxStates) return true;
  if (const int m = tuning().chain_wide_min; m > 0) return n >= m;
  if (tuning().chain_wide == 0) return false;
  return n > 1024;
}

hipError_t launch_cp_superseq_chain(const CpChainArgs& g, hipStream_t stream) {
  if (g.len <= 0) return hipSuccess;
  if (g.nstates <= 0 || g.nstates > kChainMaxStates) return hipErrorInvalidValue;
  const size_t n = (size_t)g.nstates;
  if (cp_chain_wide(g.nstates)) {
    if (!g.grows) return hipErrorInvalidValue;
    if (g.init_row) {
      const hipError_t err = hipMemcpyAsync(g.grows + n, g.init_row, n * 8, hipMemcpyDeviceToDevice, stream);
      if (err != hipSuccess) return err;
    }
    const unsigned nblk = (unsigned)((n + 255) / 256);
    for (int64_t t = 0; t < g.len; ++t) {
      hipLaunchKernelGGL(cp_chain_wide_step, dim3(nblk), dim3(256), 0, stream, g, t);
      const hipError_t err = hipGetLastError();
      if (err != hipSuccess) return err;
    }
    hipLaunchKernelGGL(cp_chain_wide_finish, dim3(1), dim3(1024), 0, stream, g);
    return hipGetLastError();
  }
  const int threads = std::min(1024, ((g.nstates + 63) / 64) * 64);
  const size_t lds_a = (n * n + 2 * n) * sizeof(double);
  if (lds_a <= 160 * 1024) {
    if (lds_a > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cp_superseq_chain<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a);
    hipLaunchKernelGGL(cp_superseq_chain<true>, dim3(1), dim3(threads), lds_a, stream, g);
  } else {
    const size_t lds = 2 * n * sizeof(double);
    if (lds > 64 * 1024)
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&cp_superseq_chain<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(cp_superseq_chain<false>, dim3(1), dim3(threads), lds, stream, g);
  }
  return hipGetLastError();
}

}  // namespace cvk
