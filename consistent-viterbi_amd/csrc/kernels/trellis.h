// trellis.h -- argument blocks and launchers of the HIP trellis kernels (trellis.hip).
// Internal to libcviterbi; the public boundary is include/cviterbi.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvk {

enum { CVK_SEQ_OK = 0, CVK_SEQ_INFEASIBLE = 1, CVK_SEQ_EMPTY = 2, CVK_SEQ_BADOBS = 3 };
enum { CVK_ASSOC_VITERBI = 0, CVK_ASSOC_CP = 1, CVK_ASSOC_DP = 2, CVK_ASSOC_DECODE = 3 };

struct TrellisFwdArgs {
  const float* a_img;      // register image of A, NP*NP floats (see trellis_fwd_f32)
  const float* pi;         // [NP], -inf padded
  const float* et;         // [V][NP] emission transposed, -inf padded
  const int64_t* offsets;  // [nseq_total+1] element offsets
  const int32_t* obs;      // [sum T] flattened observation indices
  const int32_t* order;    // optional schedule: slot -> sequence id
  int64_t seq_begin;       // first schedule slot of this launch
  float* delta;            // [(elements of chunk)][NP] delta rows for the backtrack
  int64_t delta_elem_base; // element offset that maps to delta row 0
  uint8_t* status;         // [nseq_total] per-sequence status (pre-zeroed)
  int nobs;                // V
  // optional features (all null/0 on the plain decode path)
  const int32_t* forced;   // [sum T] -1 free, else the state forced at that element
  const int64_t* ranges;   // [nslot][2] explicit element ranges (begin, end); slot = sequence id
  int reverse;             // 1: traverse each range from end-1 down to begin
  float* last_row;         // [nslot][NP] final delta row of each slot (slot - seq_begin)
  const int32_t* start;    // [nslot] (slot - seq_begin): s >= 0 starts the range in state s with
                           // delta = 0 there (-inf elsewhere, no pi/emission term); -1: normal
  // two passes in one launch (constrained terms: prefixes forward, suffixes reversed):
  // ranged slots >= split use a_img2 / pi2, traverse reversed and write their final row to
  // last_row2 + (slot - split) * NP; slot_order (optional) maps blockIdx -> ranged slot
  // (longest first, so the ragged tail is short ranges)
  int64_t split;
  const float* a_img2;
  const float* pi2;
  float* last_row2;
  const int32_t* slot_order;
  // constrained decode, resume flow (cviterbi.cpp forced_decode_resume):
  const int64_t* row_base;   // EXT, ranged slots < split: delta row index of the range's first
                             // element (instead of e0 - delta_elem_base); slots >= split then
                             // write no delta rows
  const float* resume_rows;  // forced[e0] = -2 - r (r >= 0): row 0 of the sequence is
                             // resume_rows[r][:] (already forced), not pi + b
};

struct BacktrackArgs {
  const float* delta;
  int64_t delta_elem_base;
  const float* at;         // [NP][NP]: at[j*NP + i] = A[i][j]
  const int64_t* offsets;
  const int32_t* obs;
  const int32_t* order;
  int64_t seq_begin, seq_end;
  int nstates;             // real N
  int32_t* path;           // [sum T]
  double* score;           // [nseq_total]
  float* score32;          // optional [nseq_total]
  uint8_t* status;
};

// f64 re-score of decoded paths, one LANE per sequence (rescore_f64_lanes)
struct RescoreArgs {
  const int32_t* path;     // [sum T]
  const int32_t* obs;      // [sum T]
  const int64_t* offsets;
  const int32_t* order;    // optional schedule: slot -> sequence id
  int64_t seq_begin, seq_end;
  int nstates;             // real N
  const double* pi64;      // [N]
  const double* a64;       // [N*N]
  const double* et64;      // [V][N]
  const uint8_t* status;   // only CVK_SEQ_OK sequences are re-scored
  double* score;           // [nseq_total]
};
hipError_t launch_rescore_f64(const RescoreArgs& r, int64_t nseq, hipStream_t stream, int lds_reserve = 0);

template <typename REAL>
struct GenericFwdArgs {
  const int32_t* forced;   // [sum T] nullable: -1 free, else forced state
  const REAL* a;           // [N*N]
  const REAL* pi;          // [N]
  const REAL* et;          // [V][N]
  const int64_t* offsets;
  const int32_t* obs;
  const int32_t* order;
  int64_t seq_begin;
  int nstates, nobs, assoc;
  uint16_t* psi;           // [(elements of chunk)][N]
  int64_t psi_elem_base;
  REAL* last_row;          // [(seqs of chunk)][N]
  uint8_t* status;
  // rows mode (VITERBI / DECODE / DP, generic_fwd_ms<.., ROWS>): the delta rows themselves
  // [(elements of chunk)][N] (from psi_elem_base) instead of psi -- the forward pass keeps
  // only the maximum (2 VALU per pair instead of 4), generic_bt_rows recomputes the argmax
  // along the path
  REAL* rows;
  // CP only (the parallel chain's speculative re-decodes, N > 256): cp_init [nseq] = offset M
  // of each sequence (row 0 = fl(M + fl(pi + b)): a chain entered with running maximum M),
  // cp_last [nseq][N] = each sequence's last row, by sequence id (null: not used / written)
  const REAL* cp_init;
  REAL* cp_last;
  // wide mode (psi only; N > generic_max_states, where the two rows no longer fit in LDS):
  // grows = [(seqs of launch)][2][N] global rows, wide_steps = the launch's longest sequence;
  // one launch per step, each sequence's states spread over ceil(N / 256) workgroups
  REAL* grows;
  int64_t wide_steps;
  // 1: the waves run at issue priority 3 (set by launch_generic_fwd from tuning key
  // generic_prio: the parallel chain's speculative batch beside a forward pass, whose waves
  // otherwise take issue slots only where the forward's leave one)
  int prio;
};

template <typename REAL>
struct GenericBtArgs {
  const uint16_t* psi;
  int64_t psi_elem_base;
  const REAL* last_row;
  const int64_t* offsets;
  const int32_t* order;
  int64_t seq_begin, seq_end;
  int nstates;
  int32_t* path;
  double* score;
  uint8_t* status;
  const int32_t* obs;      // for the f64 re-score
  int rescore_f64;         // f32 kernels only: score = f64 VITERBI re-score of the path
  int decode_bt;           // viterbi::decode: an infeasible sequence backtracks from argmax 0
                           // through psi (viterbi.rs:24-30) instead of getting the 0 path
  const double* pi64;
  const double* a64;
  const double* et64;
  // rows mode (generic_bt_rows): the forward's delta rows, a^T and b^T in REAL, the association
  const REAL* rows;
  const REAL* at;          // [N][N] at[j][i] = a[i][j]
  const REAL* et;          // [V][N]
  int assoc, nobs;
};

struct MaxMarginalArgs {
  const float* delta;          // [ncon][NP] forward row at the constrained position
  const float* g;              // [ncon][NP] last row of the reversed suffix pass
  const int64_t* ranges_suffix;// [ncon][2] suffix element range (empty -> beta = 0)
  const float* at;             // [NP][NP] at[j*NP + i] = a[i][j]
  float* mu;                   // [ncon][NP]
};
hipError_t launch_max_marginal(int np, const MaxMarginalArgs& a, int64_t ncon, hipStream_t stream);

// forced[elems[k]] = states[k] for k < n (the constrained decode's forced-state array,
// built on the device from the compact list of constrained elements)
hipError_t launch_scatter_forced(const int64_t* elems, const int32_t* states, int64_t n, int32_t* forced,
                                 hipStream_t stream);

// *first = the first element index in [lo, hi) with obs outside [0, V), or ~0 (all valid).
hipError_t launch_obs_first_bad(const int32_t* obs, int64_t lo, int64_t hi, int64_t V, unsigned long long* first,
                                hipStream_t stream);

// Resume flow of the constrained decode (forced_decode_resume in cviterbi.cpp):
// out[i][j] = j == state[i] ? last[i][j] : -inf  (row t_1 of sequence i, forced), np <= 256
hipError_t launch_resume_rows(const float* last, const int32_t* state, int64_t n, int np, float* out,
                              hipStream_t stream);
// compact suffix batch (compact sequence k, any order): elements [cstart[k], cstart[k] +
// off2[k+1] - off2[k]) of the original batch go to off2[k]; forced2 of the first element =
// -2 - ridx[k] when ridx[k] >= 0 (resume row), else the original forced value
hipError_t launch_compact_suffix(const int64_t* cstart, const int64_t* off2, const int32_t* obs, const int32_t* forced,
                                 const int32_t* ridx, int32_t* obs2, int32_t* forced2, int64_t nseq,
                                 hipStream_t stream);
// back: path[cstart[k] + q] = path2[off2[k] + q]; score/status[perm[k]] = score2/status2[k]
hipError_t launch_scatter_suffix(const int64_t* cstart, const int64_t* off2, const int64_t* perm,
                                 const int32_t* path2, const double* score2, const uint8_t* status2, int32_t* path,
                                 double* score, uint8_t* status, int64_t nseq, hipStream_t stream);
struct PrefixBtArgs {
  const float* rows;        // compact prefix delta rows (the terms pass's first pass)
  const int64_t* row_base;  // [n] first row of slot i
  const int64_t* seq;       // [n] sequence id of slot i
  const int64_t* t1;        // [n] element index of the first constrained element
  const int32_t* state;     // [n] state forced there
  const int64_t* offsets;   // original CSR offsets
  const float* at;          // [NP][NP]
  const uint8_t* status;    // final statuses (zero_infeasible_prefix)
  int32_t* path;
};
// path[off[seq] .. t1] of every slot: backtrack from `state` at t1 through the stored prefix
// rows (statuses not read: may overlap the suffix decode; lds_reserve as launch_trellis_bt)
hipError_t launch_prefix_backtrack(int np, const PrefixBtArgs& a, int64_t n, hipStream_t stream, int lds_reserve);
// path[off[seq] .. t1) = 0 for every slot whose final status is not OK
hipError_t launch_zero_infeasible_prefix(const PrefixBtArgs& a, int64_t n, hipStream_t stream);

int trellis_padded_states(int n);  // 0 if the trellis kernel does not cover n
hipError_t launch_trellis_fwd(int np, const TrellisFwdArgs& fa, int64_t nseq, hipStream_t stream);
// Two equal-length sequences per workgroup (slots seq_begin + 2k, +2k+1), plain decode only;
// NP in {64, 128, 192, 256}.
bool trellis_pair_supported(int np);
hipError_t launch_trellis_fwd2(int np, const TrellisFwdArgs& fa, int64_t npairs, hipStream_t stream);
hipError_t launch_trellis_bt(int np, const BacktrackArgs& ba, int64_t nseq, hipStream_t stream, int lds_reserve = 0);
// N <= 64: one wave per sequence, forward + backtrack fused (trellis_wave_f32), the tables
// padded to npw = trellis_wave_states(N) (16, 32, 48 or 64; 0 = not covered).  fa.a_img = the
// ROW-MAJOR padded A table, fa.pi / fa.et / ba.at and the delta rows use the npw stride;
// fa.seq_begin .. ba.seq_end = the slots.
int trellis_wave_states(int n);
hipError_t launch_trellis_wave(int npw, const TrellisFwdArgs& fa, const BacktrackArgs& ba, int64_t nseq,
                               hipStream_t stream);
template <typename REAL>
hipError_t launch_generic_fwd(const GenericFwdArgs<REAL>& fa, int64_t nseq, hipStream_t stream);
template <typename REAL>
hipError_t launch_generic_bt(const GenericBtArgs<REAL>& ba, int64_t nseq, hipStream_t stream);
// rows mode: forward (fa.rows set, assoc != CP) and its backtrack
template <typename REAL>
hipError_t launch_generic_bt_rows(const GenericBtArgs<REAL>& ba, int64_t nseq, hipStream_t stream);
int generic_max_states(int real_bytes);
// The generic decode runs wide (GenericFwdArgs::grows, up to the u16 psi's range): always above
// generic_max_states; above N = 1,024 (one thread per state no longer fits one workgroup) also
// for CP (psi mode in one workgroup: 4x the rows mode's time), batches below 4,096 sequences or
// N > 3,072 -- everywhere the one-workgroup kernels lost (profiles/r05_wide_crossover.txt).
// Read per call (A/B knobs and tests, bit-identical): CV_GENERIC_WIDE=0 only above the LDS
// limit, CV_GENERIC_WIDE_MIN=n from n states whatever the batch.
constexpr int kGenericGlobalMaxStates = 65535;
bool generic_wide(int n, int real_bytes, int64_t nseq, bool cp);

// The constrained decode's f64 passes for N > 256 (the padded EXT kernels' range): one
// workgroup per slot over an explicit element range, row-A0 association
//   row 0 = start >= 0 ? (0 at `start`, -inf elsewhere) : pi + b(o_first)   (pi alone when
//   noemit_last and the range has one element);  row t = max_i (row_{t-1}[i] + tab[i][j]) +
//   b_j(o_t), the last step without the emission when noemit_last;
// only the range's last row is written.  reverse: the range runs from end-1 down to begin (the
// suffix pass: tab = a^T, pi = 0).  Same values as trellis_fwd_f64's EXT passes, bit for bit
// (a max is exact whatever its order).
struct GenericExtArgs {
  const double* tab;       // [N][N] tab[i][j]: predecessor i -> state j (a, or a^T for the suffix)
  const double* pi;        // [N]
  const double* et;        // [V][N]
  const int32_t* obs;      // [sum T], validated by the caller
  const int64_t* ranges;   // [slot][2] element range [begin, end)
  const int32_t* start;    // [slot] nullable: start state (segment tables)
  int reverse, noemit_last;
  int nstates;
  double* last_row;        // [slot][N]
  // wide (N > generic_max_states(8), or from CV_EXT_WIDE_MIN states: read per call, tests):
  // grows = [slot][2][N] global rows, wide_steps = the longest range; one launch per step,
  // each slot's states over ceil(N / 256) workgroups
  double* grows;
  int64_t wide_steps;
};
hipError_t launch_generic_ext(const GenericExtArgs& g, int64_t nslots, hipStream_t stream);
bool generic_ext_wide(int n);

}  // namespace cvk
