// trellis.hip -- MI355X (gfx950) Viterbi trellis kernels.
//
// Hot path of the reference's viterbi_solver forward pass:
//   d0[j] = pi[j] + b[j,o0]                            (hmm/hmm.rs:415-418, cp.rs:98-100)
//   s_i   = d[i] + a[i,j];  m = max_i s_i                (viterbi.rs:13-16, cp.rs:103-106)
//   psi   = first i with s_i == m                       (ndarray-stats argmax)
//   d'[j] = m + b[j,o]                                  (viterbi.rs:17)
// followed by the backtrack of cp.rs:117-125 / viterbi.rs:24-31.
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
//                         (VITERBI row A0, CP cp.rs:102-110, DP dp.rs:127-177, DECODE
//                         viterbi.rs:5-32) with inline first-argmax; writes u16 psi.
//   generic_backtrack<REAL>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "trellis.h"

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

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also emits the workgroup
// release fence, which waits (vmcnt) for this wave's outstanding GLOBAL stores -- the
// delta row just written for the backtrack -- adding a store round trip to every step.
// Nothing in the kernel reads those stores back, so only the LDS writes are drained.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

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

template <int NP>
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

  const int64_t slot = args.seq_begin + blockIdx.x;
  const int64_t seq = args.order ? (int64_t)args.order[slot] : slot;
  const int64_t e0 = args.offsets[seq];
  const int T = (int)(args.offsets[seq + 1] - e0);
  if (T <= 0) return;
  // constant address space: uniform loads become s_load (SMEM), off the vmcnt queue.
  const __attribute__((address_space(4))) int32_t* obs =
      (const __attribute__((address_space(4))) int32_t*)(args.obs + e0);
  float* __restrict__ drow = args.delta + (e0 - args.delta_elem_base) * NP + j0;
  const float* __restrict__ etj = args.et + j0;
  const unsigned V = (unsigned)args.nobs;

  // A register image: float4 q of a lane = (A[rg*R+2q][j0], A[rg*R+2q][j0+1],
  // A[rg*R+2q+1][j0], A[rg*R+2q+1][j0+1]); each wave-instruction reads 1 KiB contiguous.
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

  // Observations are read with uniform (scalar) loads one step ahead of the emission
  // row they select; an out-of-range index flags the sequence and is clamped so no
  // load leaves the table.
  unsigned bad = 0;
  auto obs_s = [&](int t) -> unsigned {
    const unsigned o = (unsigned)obs[t];
    bad |= (o >= V);
    return o < V ? o : 0u;
  };
  auto et_row = [&](unsigned o) -> float2 { return *reinterpret_cast<const float2*>(etj + (size_t)o * NP); };

  const int lds_w = (j0 / R) * S + (j0 % R);
  // ---- t = 0: d0 = pi + b[:,o0]  (hmm.rs:415-418, cp.rs:98-100) ----
  {
    const float2 e = et_row(obs_s(0));
    float2 d0;
    d0.x = args.pi[j0] + e.x;
    d0.y = args.pi[j0 + 1] + e.y;
    if (rg == 0) {
      *reinterpret_cast<float2*>(&lds_delta[0][lds_w]) = d0;
      *reinterpret_cast<float2*>(drow) = d0;
    }
  }
  unsigned o_next = obs_s(T > 1 ? 1 : 0);
  float2 eA = et_row(o_next);  // emission row of t = 1
  o_next = obs_s(T > 2 ? 2 : T - 1);
  float2 eB;
  lds_barrier();

  // One trellis step t: consumes e_use (row of o_t, loaded one step earlier), issues the
  // load of the row of o_{t+1} into e_pref and the scalar load of o_{t+2}.
  auto step = [&](int t, const float2& e_use, float2& e_pref) {
    e_pref = et_row(o_next);
    const int cur = (t - 1) & 1;
    const float* dsrc = &lds_delta[cur][rg * S];
    float m0a = ninf_f(), m0b = ninf_f(), m1a = ninf_f(), m1b = ninf_f();
#pragma unroll
    for (int q4 = 0; q4 < R / 4; ++q4) {
      const float4 d = *reinterpret_cast<const float4*>(dsrc + 4 * q4);
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
    }
    o_next = obs_s(t + 2 < T ? t + 2 : T - 1);
    float m0 = fmaxf(m0a, m0b);
    float m1 = fmaxf(m1a, m1b);
    m0 = octet_max(m0);  // fold the 8 row groups of column j0
    m1 = octet_max(m1);
    float2 dn;
    dn.x = m0 + e_use.x;  // (d + a) + b -- viterbi.rs:15-17 association
    dn.y = m1 + e_use.y;
    if (rg == 0) {
      *reinterpret_cast<float2*>(&lds_delta[cur ^ 1][lds_w]) = dn;
      *reinterpret_cast<float2*>(drow + (size_t)t * NP) = dn;
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
      const double ak = __shfl(av, k);
      const double bk = __shfl(bv, k);
      if (base + k == 0)
        d = ak + bk;  // pi[p0] + b[p0,o0]
      else
        d = (d + ak) + bk;  // (d + a) + b
    }
  }
  return d;
}

template <int NP>
__global__ __launch_bounds__(256) void backtrack_f32(BacktrackArgs args) {
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
  constexpr int KP = (NP + 63) / 64;

  // first argmax of the last row (cp.rs:117-118)
  float bv = ninf_f();
  int bi = 0x7fffffff;
  {
    const float* last = drow + (size_t)(T - 1) * NP;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int i = lane + 64 * k;
      if (i < N) {
        const float v = last[i];
        if (bi == 0x7fffffff || v > bv) {  // ascending i: keeps the first maximum
          bv = v;
          bi = i;
        }
      }
    }
  }
  wave_argmax_first(bv, bi);
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
  int cur = bi;
  int pathreg = 0;
  if (lane == ((T - 1) & 63)) pathreg = cur;
  if (((T - 1) & 63) == 0) {
    if (lane == 0) path[T - 1] = cur;
  }
  const float* __restrict__ at = args.at;
  for (int t = T - 1; t >= 1; --t) {
    // s_i = d_{t-1}[i] + a[i, cur]  -- the forward pass's exact f32 add
    const float* prow = drow + (size_t)(t - 1) * NP;
    const float* acol = at + (size_t)cur * NP;
    float v = ninf_f();
    int vi = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int i = lane + 64 * k;
      if (i < N) {
        const float s = prow[i] + acol[i];
        if (vi == 0x7fffffff || s > v) {
          v = s;
          vi = i;
        }
      }
    }
    wave_argmax_first(v, vi);
    cur = vi;
    const int tp = t - 1;
    if (lane == (tp & 63)) pathreg = cur;
    if ((tp & 63) == 0) {
      // flush the block [tp, min(tp+64, T)) written in pathreg
      if (tp + lane < T) path[tp + lane] = pathreg;
    }
  }
  // Every 64-entry block is flushed when tp reaches its start (tp = 0 closes the last
  // one); a top block starting exactly at T-1 was written before the loop.
  if (lane == 0) {
    args.status[seq] = CVK_SEQ_OK;
    if (!args.rescore_f64) args.score[seq] = (double)score32;
  }
  if (args.rescore_f64) {
    const double d = rescore_path_f64(path, args.obs + e0, T, args.pi64, args.a64, args.et64, N, lane);
    if (lane == 0) args.score[seq] = d;
  }
  if (args.score32 && lane == 0) args.score32[seq] = score32;
}

// ---------------------------------------------------------------------------------
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
        d = args.pi[j] + e;
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
      psi[(size_t)t * N + j] = (uint16_t)arg;
    }
    __syncthreads();
  }
  const REAL* last = dbuf + ((T - 1) & 1) * N;
  REAL* lastout = args.last_row + (slot - args.seq_begin) * (int64_t)N;
  for (int j = threadIdx.x; j < N; j += blockDim.x) lastout[j] = last[j];
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
    for (int t = lane; t < T; t += 64) path[t] = 0;
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

// ---------------------------------------------------------------------------------
// Host-side launchers (called from the C-ABI layer).
template <int NP>
static hipError_t launch_trellis_np(const TrellisFwdArgs& fa, const BacktrackArgs& ba, int64_t nseq,
                                    hipStream_t stream, hipEvent_t ev_mid) {
  if (nseq <= 0) return hipSuccess;
  hipLaunchKernelGGL(trellis_fwd_f32<NP>, dim3((unsigned)nseq), dim3(NP * 4), 0, stream, fa);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  if (ev_mid) (void)hipEventRecord(ev_mid, stream);
  hipLaunchKernelGGL(backtrack_f32<NP>, dim3((unsigned)((nseq + 3) / 4)), dim3(256), 0, stream, ba);
  return hipGetLastError();
}

int trellis_padded_states(int n) {
  if (n <= 0 || n > 256) return 0;
  return ((n + 31) / 32) * 32;
}

hipError_t launch_trellis(int np, const TrellisFwdArgs& fa, const BacktrackArgs& ba, int64_t nseq,
                          hipStream_t stream, hipEvent_t ev_mid) {
  switch (np) {
    case 32: return launch_trellis_np<32>(fa, ba, nseq, stream, ev_mid);
    case 64: return launch_trellis_np<64>(fa, ba, nseq, stream, ev_mid);
    case 96: return launch_trellis_np<96>(fa, ba, nseq, stream, ev_mid);
    case 128: return launch_trellis_np<128>(fa, ba, nseq, stream, ev_mid);
    case 160: return launch_trellis_np<160>(fa, ba, nseq, stream, ev_mid);
    case 192: return launch_trellis_np<192>(fa, ba, nseq, stream, ev_mid);
    case 224: return launch_trellis_np<224>(fa, ba, nseq, stream, ev_mid);
    case 256: return launch_trellis_np<256>(fa, ba, nseq, stream, ev_mid);
    default: return hipErrorInvalidValue;
  }
}

template <typename REAL>
hipError_t launch_generic(const GenericFwdArgs<REAL>& fa, const GenericBtArgs<REAL>& ba, int64_t nseq,
                          hipStream_t stream, hipEvent_t ev_mid) {
  if (nseq <= 0) return hipSuccess;
  const size_t lds = sizeof(REAL) * 2 * (size_t)fa.nstates;
  hipLaunchKernelGGL(generic_fwd<REAL>, dim3((unsigned)nseq), dim3(256), lds, stream, fa);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) return err;
  if (ev_mid) (void)hipEventRecord(ev_mid, stream);
  hipLaunchKernelGGL(generic_backtrack<REAL>, dim3((unsigned)((nseq + 3) / 4)), dim3(256), 0, stream, ba);
  return hipGetLastError();
}

template hipError_t launch_generic<float>(const GenericFwdArgs<float>&, const GenericBtArgs<float>&, int64_t,
                                          hipStream_t, hipEvent_t);
template hipError_t launch_generic<double>(const GenericFwdArgs<double>&, const GenericBtArgs<double>&, int64_t,
                                           hipStream_t, hipEvent_t);

// Generic kernel keeps 2*N REAL delta values in LDS.
int generic_max_states(int real_bytes) { return (int)(65536 / (2 * real_bytes)); }

}  // namespace cvk
