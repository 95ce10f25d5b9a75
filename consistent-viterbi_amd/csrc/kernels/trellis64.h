// trellis64.h -- exact-f64 trellis kernels for N <= 1,024 (trellis64.hip).
// Internal to libcviterbi; the public boundary is include/cviterbi.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvk {

struct T64FwdArgs {
  const double* a;         // [NP][NP] row-major a[i][j], -inf padded
  const double* pi;        // [NP], -inf padded
  const double* et;        // [V][NP] emissions transposed, -inf padded
  const int64_t* offsets;  // [nseq_total+1] element offsets
  const int32_t* obs;      // [sum T]
  const int32_t* order;    // optional schedule: slot -> sequence id
  int64_t seq_begin;       // first schedule slot of this launch
  int64_t nslots;          // slots in this launch
  double* delta;           // [(elements of chunk)][NP] f64 delta rows for the backtrack
  int64_t delta_elem_base; // element offset that maps to delta row 0
  uint8_t* status;         // [nseq_total] (pre-zeroed); forward sets BADOBS
  int nobs;                // V
  int zero_init;           // 1: row 0 = 0.0 (viterbi::decode, viterbi.rs:6,9), else pi + b
  int dp_assoc;            // 1: DPSolver's (a + b) + d association (dp.rs:147-177)
  // CP association (trellis_cp_f64 only): psi / last-row outputs in the generic kernel's
  // layout so generic_backtrack<double> finishes the decode
  int nstates;             // real N (psi row stride)
  uint16_t* psi;           // [(elements of chunk)][N]
  double* last_row;        // [(slots of launch)][N] (CP); EXT: [(slots of launch)][NP] final rows
  // CP only (the parallel chain): cp_init [nseq] = offset M of each sequence (row 0 =
  // fl(M + fl(pi + b)), a chain entered with running maximum M), null = 0; cp_last
  // [nseq][N] = each sequence's last row, indexed by sequence id (null = not written)
  const double* cp_init;
  double* cp_last;
  // EXT features of trellis_fwd_f64 (the constrained decode's passes; all null/0 otherwise)
  const int32_t* forced;       // [sum T] -1 free, >= 0 forced state, <= -2: row 0 = resume_rows[-2 - f]
  const int64_t* ranges;       // [slot][2] explicit element ranges (begin, end); sequence id = slot
  int reverse;                 // 1: traverse each range from end-1 down to begin (suffix pass on a^T)
  const int32_t* start;        // [slot - seq_begin] s >= 0: row 0 = 0 at state s, -inf elsewhere
  const int64_t* row_base;     // [slot] delta row index of the range's first element (< 0: no rows kept)
  int* queue;                  // EXT one-wave passes: work-queue counter (null: one workgroup per unit)
  const double* resume_rows;   // [r][NP] already-forced rows (resume flow)
  const int32_t* slot_order;   // [launch index] -> slot (longest first)
  // 1: a range's LAST step adds no emission, so the suffix pass extended to the constrained
  // element t_m ends on beta_{t_m}(s) = max_j (a[s][j] + g_{t_m+1}[j]) itself (its last row)
  int noemit_last;
  // set by the host: the batch suits eight-wave workgroups (equal lengths, or >= 2 rounds of
  // them); a single round of longest-first workgroups puts all the longest sequences on a few
  // CUs (ragged 16,384 sequences: 65.5 vs 56 ms), the one-wave layout spreads them
  int wg_ok;
  // SIMD balancing (trellis_fwd_f64): every `balance` steps each wave publishes its remaining
  // steps in a per-SIMD table and takes issue priority 3 if no other wave of its SIMD has more
  // work left, else 1 (the arbiter runs the oldest wave first among equals); 0 = off
  int balance;
};

struct T64BtArgs {
  const double* delta;
  int64_t delta_elem_base;
  const double* at;        // [NP][NP]: at[j*NP + i] = a[i][j]
  const int64_t* offsets;
  const int32_t* order;
  int64_t seq_begin, seq_end;
  int nstates;             // real N
  int32_t* path;           // [sum T]
  double* score;           // [nseq_total]
  uint8_t* status;
  int dp_assoc;            // 1: candidates (a[i,j] + b[j,o_t]) + d[i] (dp.rs:149)
  int decode_bt;           // viterbi::decode (zero_init): an infeasible sequence backtracks from
                           // argmax 0, bt = 0 where the emission is -inf (viterbi.rs:19-30)
  const int32_t* obs;      // dp_assoc / decode_bt: observations, emissions [V][NP]
  const double* et;
  const float* at32;       // f32(a^T) [NP][NP], set only for models whose finite entries are
                           // all in [-2^80, 0]: the NONPOS interval test (null: f64 test)
  int only_infeasible;     // set by launch_t64_bt: the general kernel's viterbi::decode pass over
                           // the infeasible sequences the NONPOS kernel left (their DEC chain)
  double* cert;            // non-null (NONPOS row A0, NP <= 256): the parallel chain's certificate
                           // (rho, gF) per sequence [2 nseq], as cp_cert_f64 computes it
  double rho_cap;          // steps whose estimated certificate term reaches it skip the exact gap
};

// Delta rows of the f64 trellis (forward -> backtrack, resume-flow prefix rows) use a
// SPLIT-PLANE layout: row r = 2*NP u32 words, [0, NP) the high words of the NP f64 values and
// [NP, 2 NP) their low words (8*NP bytes per row, like a plain f64 row).  The backtrack reads
// the high plane only (a 20-bit-mantissa truncation with a rigorous error bound) and the low
// plane only on near ties.

struct PrefixBt64Args {
  const double* rows;       // compact split-plane prefix rows (the terms pass's prefix launch)
  const int64_t* row_base;  // [n] first row of slot i
  const int64_t* seq;       // [n] sequence id of slot i
  const int64_t* t1;        // [n] element index of the first constrained element
  const int32_t* state;     // [n] state forced there
  const int64_t* offsets;   // original CSR offsets
  const double* at;         // [NP][NP] a^T (t64 tables)
  const float* at32;        // f32(a^T) for the NONPOS interval test, or null (T64BtArgs::at32)
  int nstates;
  int32_t* path;
};
hipError_t launch_t64_prefix_bt(int np, const PrefixBt64Args& a, int64_t n, hipStream_t stream);

// Certified suffix trace (resume flow, f64, one constrained element t1, NONPOS models): the
// forced decode's path after t1 read off the suffix pass's stored rows instead of a second
// forward pass.  Slot i certifies when every step's first argmax beats the runner-up by more
// than the bound on the rounding of both passes (suffix_trace_f64 in trellis64.hip); then the
// path [t1 + 1, end), the score (the forward fold (d + a) + b from delta_{t1}(state)) and
// status OK are written and cert[i] = 1.  cert[i] = 0: nothing but path garbage in
// [t1 + 1, end), which the fallback forced decode overwrites.
struct SuffixTrace64Args {
  const double* rows;        // compact split-plane rows of the reversed suffix pass
  const int64_t* srow_base;  // [n] first row of slot i (row k = element end - 1 - k)
  const int64_t* seq;        // [n] sequence id of slot i
  const int64_t* t1;         // [n] the constrained element
  const int32_t* state;      // [n] state forced there (-1: no state, not traced)
  const double* dlast;       // [n][NP] the prefix pass's row t1 (delta_{t1}, unforced)
  const int64_t* offsets;    // original CSR offsets
  const int32_t* obs;        // observations (element-indexed)
  const double* a;           // [NP][NP] a (from-major, t64 tables)
  const double* et;          // [V][NP]
  int nstates;
  int32_t* path;
  double* score;
  uint8_t* status;
  uint8_t* cert;             // [n]
};
hipError_t launch_t64_suffix_trace(int np, const SuffixTrace64Args& a, int64_t n, hipStream_t stream);

struct MaxMarginal64Args {
  const double* delta;          // [ncon][NP] forward row at the constrained position
  const double* g;              // [ncon][NP] last row of the reversed suffix pass
  const int64_t* ranges_suffix; // [ncon][2] suffix element range (empty -> beta = 0)
  const double* at;             // [NP][NP] at[j*NP + i] = a[i][j]
  double* mu;                   // [ncon][NP]
};
hipError_t launch_t64_max_marginal(int np, const MaxMarginal64Args& a, int64_t ncon, hipStream_t stream);
// mu[i][j] = delta[i][j] + beta[i][j] for the first n1 rows (single-position sequences), the
// rest left to the caller (their terms are delta and beta themselves): elementwise, so the
// kernel co-resides with a long decode on the same CUs (max_marginal_f64's per-sequence
// max-plus step is the suffix pass's extra step instead, noemit_last)
hipError_t launch_t64_mu_add(const double* delta, const double* beta, double* mu, int64_t n1, int np,
                             hipStream_t stream);
// out[i][j] = j == state[i] ? last[i][j] : -inf (row t_1 of constrained sequence i, forced)
hipError_t launch_t64_resume_rows(const double* last, const int32_t* state, int64_t n, int np, double* out,
                                  hipStream_t stream);

// Parallel CPSolver chain (cv_decode_superseq_cp, log-probability models): the
// certificate of each sequence's row-A0 path at offset 0 (cp_cert_f64) and the quantised CP
// fold of a certified path at a predicted binade (cp_quant_f64).  See trellis64.hip.
struct CpCert64Args {
  const double* delta;     // split-plane rows of the row-A0 forward (decode_device's workspace)
  int64_t delta_elem_base;
  const double* at;        // [NP][NP] a^T
  const int64_t* offsets;
  const int32_t* order;
  int64_t seq_begin, seq_end;
  int nstates;
  const int32_t* path;     // the row-A0 backtrack's paths
  const uint8_t* status;
  double* out;             // [nseq_total][2]: rho, gF (-1: not certifiable)
};
// np: the f64 trellis's NP (64..256 in registers; 512 / 1,024: the split-plane rows of the
// column-split pairs / quads of waves)
hipError_t launch_cp_cert(int np, const CpCert64Args& a, hipStream_t stream);
// the same certificate over the generic kernels' plain f64 rows [elem][N] (a.at = a^T [N][N])
hipError_t launch_cp_cert_plain(const CpCert64Args& a, hipStream_t stream);
constexpr int CVK_NO_BINADE = -0x7fffffff;
struct CpQuant64Args {
  const double* a;         // [NP][NP] (t64 tables)
  const double* pi;        // [NP]
  const double* et;        // [V][NP]
  int np;
  const int64_t* offsets;
  const int32_t* obs;
  const int32_t* path;
  const int32_t* ebin;     // [nseq] predicted binade exponent of |M| (CVK_NO_BINADE: skip)
  int64_t nseq;
  long long* q;            // [nseq] quantised arc sum in units of 2^(e-52)
  uint8_t* tie;            // [nseq] 1: a tie or out-of-range arc (fold element by element)
};
hipError_t launch_cp_quant(const CpQuant64Args& a, hipStream_t stream);
// out[k] = path[offsets[k+1] - 1] (-1 for an empty sequence), k < nseq
hipError_t launch_cp_seq_ends(const int32_t* path, const int64_t* offsets, int64_t nseq, int32_t* out,
                              hipStream_t stream);
// out[dst[i] + t] = path[offsets[ids[i]] + t], t < T(ids[i]), i < n
hipError_t launch_cp_gather_paths(const int32_t* path, const int64_t* offsets, const int64_t* ids, const int64_t* dst,
                                  int64_t n, int32_t* out, hipStream_t stream);

// CPSolver's super-sequence decode chained exactly over the whole batch (cp_superseq_chain).
struct CpChainArgs {
  const double* pi;      // [N]
  const double* a;       // [N*N] from-major
  const double* et;      // [V][N] emissions transposed
  const int32_t* obs;    // [len] super-sequence observations
  const uint8_t* first;  // [len] 1 at the first element of each sequence (MetaElements t == 0)
  int64_t len;
  int nstates, nobs;
  uint16_t* psi;         // [len][N] workspace
  int32_t* path;         // [len]; null: no in-kernel backtrack (the caller runs chain_backtrack)
  double* objective;     // [1]
  // a PART of the chain (the parallel chain's fallback runs, N > 256): init_row [N] = the
  // chain's row before element 0 (element 0 then runs like any element, psi row 0 included);
  // final_row [N] receives the last row, final_state [1] its first argmax.  All optional.
  const double* init_row;
  double* final_row;
  int32_t* final_state;
  // the wide chain (cp_chain_wide(N)): [2][N] global rows
  double* grows;
};
// the chain's two rows in LDS up to N = 10,240 (2 N doubles <= 160 KiB); above, the wide chain
// (one launch per element, states over workgroups, rows in CpChainArgs::grows); psi is u16
constexpr int kChainMaxStates = 65535;
constexpr int kChainLdsMaxStates = 10240;
// the wide chain runs above N = 1,024 (one workgroup then strides its states: 0.18 vs 0.08 ms
// per element at N = 1,100, 17 vs 1.1 ms at 10,240 -- profiles/r05_wide_crossover.txt); read
// (tuning keys, bit-identical): chain_wide = 0 only above N = 10,240, chain_wide_min = n from n
// states
bool cp_chain_wide(int n);
hipError_t launch_cp_superseq_chain(const CpChainArgs& g, hipStream_t stream);

// NP = 64 * ceil(N / 64) for 1 <= N <= 256, else 0 (no f64 trellis kernel)
int t64_padded_states(int n);
// the batch decode's NP under CV_KERNEL_AUTO: t64_padded_states, 512 for 256 < N <= 512
// (column-split pairs of waves), 1,024 for 724 < N <= 1,024 (quads; tuning keys t64_512 /
// t64_1024); 0 = the generic kernels
int t64_batch_states(int n);
// every NP the kernels support at this N (64..256 padded, 512, 1,024; 0 above): what an
// explicit CV_KERNEL_TRELLIS_F64 request gets and what the handle's t64 tables are padded to
int t64_support_states(int n);
// sequences per forward wave (2, 4 or 8) for a launch of nseq sequences on `cus` CUs
int t64_seqs_per_wave(int64_t nseq, int cus, int np = 0);
hipError_t launch_t64_fwd(int np, int s, const T64FwdArgs& fa, int64_t nseq, hipStream_t stream);
// CP association (cp.rs:70-79): psi and the CP value d[psi] + (a[psi,j] + b[j,o]) in the forward
// the CP forward's layout for a batch: waves per workgroup splitting the columns, then
// sequences per workgroup for a requested s
int t64_cp_waves(int np, int64_t nseq);
int t64_cp_seqs_per_wave(int s, int64_t nseq, int w = 1);
hipError_t launch_t64_cp_fwd(int np, int s, const T64FwdArgs& fa, int64_t nseq, hipStream_t stream);
hipError_t launch_t64_bt(int np, const T64BtArgs& ba, int64_t nseq, hipStream_t stream);

}  // namespace cvk
