// Per-handle tuning and test hooks (include/cviterbi.h "Tuning keys").
//
// Every knob that selects a kernel layout, a schedule or a code path lives here, snapshotted
// ONCE per handle: at cv_hmm_create from the environment (CV_<KEY> in upper case, the only
// environment reads of the library: tuning_from_env), then changed only through
// cv_hmm_set_tuning.  A caller's stray CV_* variable set after the handle exists changes
// nothing.  The host API copies the handle's snapshot into a thread-local (tuning_enter) for
// the duration of a call, so the kernel launchers read plain fields instead of the environment.
// Every key is bit-identical in results (layouts, schedules, A/B paths); none changes what a
// decode returns.  Handle-less entry points (cv_hmm_fit_*) snapshot the environment per call.
#pragma once

#include <cstdint>

namespace cvk {

struct Tuning {
  // ---- host API ----
  int trace = 0;               // CV_TRACE=1: host phase stamps on stderr
  int host_threads = 0;        // host worker threads (0: min(16, hardware threads))
  int t64_nonpos = 1;          // 0: the general f64 interval backtrack test (and no parallel chain)
  int generic_rows = 1;        // 0: the generic kernels in psi mode (inline argmax) instead of rows mode
  int max_chunks = 8;          // f32 trellis pipeline depth (1..64)
  int host_sums = 0;           // 1: the constrained decode's exact unary sums on the host
  int no_trace = 0;            // 1: no certified suffix trace (the resume forward instead)
  int no_resume = 0;           // 1: no resume flow (the full forced decode)
  int no_side = 0;             // 1: no side-stream decode of the unconstrained sequences
  int chain_par = 1;           // 0: the serial CPSolver chain kernel
  int chain_old = 0;           // 1: the one-thread-per-state chain kernel at any N
  int chain_par_force = 0;     // m > 0: every m-th sequence of the parallel chain taken as uncertified
  int chain_spec = 1;          // 0: no speculative re-decode (uncertified sequences run serially)
  int chain_spec_kernel = 0;   // speculation (N <= 256): 0 cp_spec_psi beside a forward pass, the batched
                               // chain kernel after the forward passes; 1 trellis_cp_f64; 2 the generic
                               // CP kernel (N > 256: always the generic kernel)
  int chain_copy_overlap = 1;  // 0: the chain's path copy after the certificate pass
  int chain_cert_fused = 1;    // 0: the chain's certificates by their own pass (cp_cert_f64), not the backtrack
  int chain_parts = 1;         // 0: the chain's decode in one part; 1: a large first part, then chain_tail
                               // parts of one forward round / chain_tail_div; 2: one forward round per part
  int chain_tail = 2;          // chain_parts = 1: the small parts after the first
  int chain_tail_div = 2;      // chain_parts = 1: a small part is one forward round / this
  int chain_spec_prio = 3;     // issue priority of the speculative batches beside a forward pass (0: default)
  int chain_pin_obs = 0;       // 1: the later parts' observations through pinned staging (measured neutral)
  int chain_pin_path = 0;      // 1: the path copy through a pinned two-chunk ring (measured neutral)
  // ---- f64 trellis (kernels/trellis64.hip) ----
  int t64_s = 0;               // sequences per wave 2 / 4 / 6 / 8 (0: by batch)
  int t64_512 = -1;            // NP = 512 batch kernel: -1 auto, 0 never, 1 whenever supported
  int t64_1024 = -1;           // NP = 1,024 batch kernel: -1 auto (N > 724), 0 never, 1 always
  int t64_wg = 1;              // 0: one wave per workgroup (SIMD balancing) instead of eight-wave units
  int t64_wg_force = 0;        // 1: the eight-wave layouts whatever the batch's lengths
  int t64_rs = 1;              // 0: small batches' column-split pairs instead of the row split
  int t64_w2 = 1;              // 0: no pair-of-waves small-batch layout
  int t64_wave = 1;            // 0: N <= 64 on the lock-step kernel instead of one wave per sequence
  int t64_bal = 8;             // steps between SIMD-balancing updates (0: off)
  int t64_cp_s = 0;            // trellis_cp_f64 sequences per wave 1 / 2 / 4 (0: by batch)
  int t64_cp_pf = 0;           // split-column trellis_cp_f64 A rows in flight: 16 (0: 32)
  int t64_cp_w = 0;            // trellis_cp_f64 waves splitting the columns: 1 never, > 1 always (0: by batch)
  int t64_bt_pf = 0;           // backtrack_f64 rows in flight (0: by NP)
  // ---- generic and wide kernels (kernels/trellis.hip) ----
  int generic_s = 0;           // sequences per workgroup 1 / 2 / 4 (0: by batch and LDS)
  int generic_split = 0;       // 1: generic_fwd_split (K threads per state)
  int generic_split_k = 0;     // its K (0: by N)
  int generic_wide = 1;        // 0: never the wide (one launch per step) decode
  int generic_wide_min = 0;    // > 0: the wide decode from this N on
  int generic_prio = 0;        // 1: generic_fwd_ms waves at issue priority 3 (the chain sets it beside a forward)
  int wide_s = 0;              // wide decode sequences per workgroup 1 / 2 / 4 (0: by batch)
  int ext_wide_min = 0;        // > 0: the constrained terms passes wide from this N on
  int chain_wide = 1;          // 0: never the wide serial chain step
  int chain_wide_min = 0;      // > 0: the wide serial chain step from this N on
  int f32_onebar = 1;          // 0: two barriers per step in trellis_fwd2_f32
  // ---- Baum-Welch (kernels/fit.hip) ----
  int bw_global = 0;           // 1: the strided kernels' vectors in global scratch from N = 257
  int bw_perseq = 0;           // 1: the per-sequence E-step kernels at 64 < N <= 256
  int bw_gemm_path = 0;        // 1: the xi GEMM path at every N
};

// the current call's tuning: the handle's snapshot inside a host API call, else the defaults
const Tuning& tuning();
// makes `t` the calling thread's current tuning until the matching tuning_leave
void tuning_enter(const Tuning& t);
void tuning_leave();
// one key of the calling thread's current tuning (inside a TuningScope) set to `value` until
// destroyed; nothing outside a scope
struct TuningOverride {
  TuningOverride(int Tuning::*field, int value);
  ~TuningOverride();
  TuningOverride(const TuningOverride&) = delete;
  TuningOverride& operator=(const TuningOverride&) = delete;

 private:
  int Tuning::*field_;
  int saved_;
  bool on_;
};
struct TuningScope {
  explicit TuningScope(const Tuning& t) { tuning_enter(t); }
  ~TuningScope() { tuning_leave(); }
  TuningScope(const TuningScope&) = delete;
  TuningScope& operator=(const TuningScope&) = delete;
};

// the environment's CV_<KEY> values over the defaults (the library's only getenv calls)
Tuning tuning_from_env();
// key (lower case, as listed above) -> value; false for an unknown key
bool tuning_set(Tuning& t, const char* key, int64_t value);
bool tuning_get(const Tuning& t, const char* key, int64_t* value);
// the i-th key name (nullptr past the end)
const char* tuning_key(int i);

}  // namespace cvk
