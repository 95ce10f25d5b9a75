/*
 * cviterbi.h -- C ABI of the MI355X-native consistent-viterbi decode path.
 *
 * This is the drop-in boundary for the reference's viterbi_solver forward pass over
 * hmm::HMM (AlexandreDubray/consistent-viterbi).  The reference is a Rust crate with
 * no FFI of its own; every entry point below names the Rust item it replaces, so a
 * Rust `extern "C"` binding can stand in for it.  Plain pointers and
 * sizes only; no torch or HIP types in the signatures (streams are opaque void*).
 *
 * Conventions
 *  - Probabilities are log10 doubles, -inf for zero (src/hmm/hmm.rs:192-205); JSON
 *    `null` reads as -inf (hmm.rs:248-264).
 *  - a[from*N + to] (hmm.rs:220-226), b[state*V + obs] with obs flattened row-major
 *    over bdims exactly as ndarray indexes `b[state][&obs[..]]` (hmm.rs:228-230).
 *  - Sequences are CSR: offsets[nseq+1] (int64, element offsets), obs[offsets[nseq]]
 *    (int32 flattened observation indices).  Paths are int32 per element.
 *  - Functions return cv_status; cv_last_error() has a message for the calling thread.
 *    Nothing aborts (the reference panics: cp.rs:87, dp.rs:184-186, unwraps).
 */
#ifndef CVITERBI_H
#define CVITERBI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CV_API __attribute__((visibility("default")))
#define CV_ABI_VERSION 1

typedef enum cv_status {
  CV_OK = 0,
  CV_EINVAL = 1,        /* bad argument (shape, range, NaN/+inf log-prob, obs out of range) */
  CV_EDEVICE = 2,       /* HIP runtime error or no usable gfx950 device */
  CV_ENOMEM = 3,        /* host or device allocation failed */
  CV_EINFEASIBLE = 4,   /* at least one sequence has no finite-probability path */
  CV_EIO = 5,           /* file could not be read / written */
  CV_EPARSE = 6,        /* malformed hmm.json */
  CV_EUNSUPPORTED = 7,  /* valid request this build does not implement */
  CV_EINTERNAL = 8,
  CV_ELIMIT = 9         /* search limit reached (constrained decode: branch-and-bound nodes) */
} cv_status;

/* per-sequence status_out values */
enum { CV_SEQ_OK = 0, CV_SEQ_INFEASIBLE = 1, CV_SEQ_EMPTY = 2, CV_SEQ_BADOBS = 3 };

/* arithmetic type of the trellis recurrence */
enum { CV_DTYPE_F32 = 0, CV_DTYPE_F64 = 1 };

/* association of the recurrence:
 *  VITERBI  d' = max_i(d[i] + a[i,j]) + b[j,o]      viterbi.rs:13-18 order, pi init cp.rs:66-68
 *  CP       d' = d[psi] + (a[psi,j] + b[j,o])       CPSolver::init_viterbi cp.rs:63-83
 *  DP       d' = max_i((a[i,j] + b[j,o]) + d[i])    DPSolver::solve dp.rs:127-182 (first index)
 *  DECODE   VITERBI with row 0 = 0.0                viterbi::decode viterbi.rs:5-32 */
enum { CV_ASSOC_VITERBI = 0, CV_ASSOC_CP = 1, CV_ASSOC_DP = 2, CV_ASSOC_DECODE = 3 };

/* kernel choice: AUTO picks TRELLIS (register-resident A, f32, VITERBI, N <= 256) when it
 * applies, then TRELLIS_F64 (exact f64: any association for N <= 256, forced states with
 * VITERBI only; one wave per 2/4/8 sequences, A streamed from L2.  Above 256, VITERBI /
 * DECODE / DP without forced states (VITERBI with them) as pairs of waves at NP = 512 or quads
 * at NP = 1,024; AUTO takes NP = 512 for N >= 384 or >= 8,192 sequences and NP = 1,024 for
 * N > 724, tuning keys t64_512 / t64_1024; an explicit TRELLIS_F64 gets it for any N <= 1,024),
 * else GENERIC (f32/f64, any association, N <= 65535: one workgroup per sequence with two rows
 * of N in LDS, or above N = 1024 -- always above 20480 f32 / 10240 f64 -- wide: one launch per
 * step, each sequence's states over ceil(N / 256) workgroups, rows in global memory). */
enum { CV_KERNEL_AUTO = 0, CV_KERNEL_TRELLIS = 1, CV_KERNEL_GENERIC = 2, CV_KERNEL_TRELLIS_F64 = 3 };

/* cv_opts.flags */
/* bit 0 and bits 8-15 are reserved (they selected the retired MFMA-assisted f32 trellis,
 * measured slower than the all-VALU one on gfx950; setting them is CV_EUNSUPPORTED) */
#define CV_FLAG_SERIAL 0x2u       /* one stream, fewest chunks: no forward/backtrack overlap */
#define CV_FLAG_NO_PAIR 0x4u      /* one sequence per forward workgroup (A/B knob; bit-identical) */
#define CV_FLAG_NO_WAVE 0x8u      /* N <= 64: the workgroup kernels instead of one wave per sequence
                                     with the backtrack fused (A/B knob; bit-identical) */
#define CV_FLAG_NO_T64 0x10u     /* f64: the generic kernel instead of TRELLIS_F64 (A/B knob;
                                     bit-identical) */

typedef struct cv_hmm cv_hmm;
typedef struct cv_solver cv_solver;

/* Model description; arrays are copied.  Replaces the fields of struct HMM<D>
 * (hmm.rs:10-18: a: Array2<f64>, b: Array1<ArrayD<f64>>, pi: Array1<f64>). */
typedef struct cv_hmm_desc {
  int32_t nstates;       /* N */
  int32_t ndims;         /* D (const generic of HMM<D>) */
  const int64_t* bdims;  /* [D] shape of each state's emission array (hmm.rs:225) */
  const double* pi;      /* [N]   log10 */
  const double* a;       /* [N*N] log10, from-major */
  const double* b;       /* [N*V] log10, V = prod(bdims) */
  int32_t device;        /* HIP device ordinal */
} cv_hmm_desc;

typedef struct cv_opts {
  int32_t dtype;         /* CV_DTYPE_F64 (default: the reference's arithmetic, hmm.rs:10-18;
                            paths and scores bit-identical to the f64 recurrence) or
                            CV_DTYPE_F32 (the f32 trellis, ~2x faster, paths may differ) */
  int32_t assoc;         /* CV_ASSOC_VITERBI (default) */
  int32_t kernel;        /* CV_KERNEL_AUTO (default) */
  int32_t rescore_f64;   /* 1 (default): score_out = f64 re-score of the decoded path with
                            the VITERBI association (what the f64 reference computes along
                            that path); 0: the kernel's own score (f32 widened for F32) */
  void* stream;          /* hipStream_t for the *_device entry points; NULL = handle stream */
  uint64_t workspace_bytes; /* delta/psi workspace cap; 0 = default (8 GiB; 64 GiB for TRELLIS_F64) */
  uint32_t flags;        /* CV_FLAG_* (0 = defaults) */
  const int32_t* forced; /* [sum T] nullable: -1 = free, s >= 0 = state s forced at that element
                            (host pointer for cv_decode_batch, device pointer for *_device) */
} cv_opts;

typedef struct cv_timing {
  double fwd_ms;         /* forward kernel(s), device time, last decode call */
  double bt_ms;          /* backtrack (+ f64 re-score) kernel(s) */
  double total_ms;       /* first kernel start to last kernel end (device) */
  int64_t launches;      /* forward launches (chunks) */
  int32_t kernel;        /* CV_KERNEL_TRELLIS, _TRELLIS_F64 or _GENERIC actually used */
  int32_t padded_states; /* NP of the trellis kernel (0 for generic) */
  int32_t mfma_tiles;    /* TRELLIS_F64: sequences per forward wave (last chunk); GENERIC: 0 wide
                            (each step over many workgroups, N > 10240 f64 / 20480 f32), else -1;
                            -1 otherwise (the field name is kept for ABI stability) */
} cv_timing;

typedef struct cv_superseq_desc {
  /* The super-sequence of viterbi_solver/utils.rs:49-58 in element order: sequences
   * concatenated (after reordering), each element carrying MetaElements fields. */
  int64_t nseq;
  const int64_t* offsets;    /* [nseq+1] */
  const int32_t* obs;        /* [offsets[nseq]] flattened observation index (value) */
  const int64_t* seq_id;     /* [nseq] original sequence id (MetaElements::seq) or NULL = 0..nseq-1 */
  const int32_t* component;  /* [elements] constraint_component, -1 = none; NULL = none */
  const uint8_t* active;     /* [elements] active_cstr; NULL = all inactive */
} cv_superseq_desc;

/* ---- library ---------------------------------------------------------------------- */
CV_API const char* cv_last_error(void);
CV_API const char* cv_version(void);
CV_API int32_t cv_abi_version(void);
CV_API int32_t cv_device_count(void);
/* Device memory this process's library holds (handles' tables and workspaces, call buffers):
 * now and at most since load (either pointer may be NULL). */
CV_API cv_status cv_device_memory(int64_t* current_bytes, int64_t* peak_bytes);
CV_API void cv_opts_init(cv_opts* opts);

/* ---- hmm::HMM (src/hmm/hmm.rs) ------------------------------------------------------- */
/* HMM struct construction (hmm.rs:10-18). */
CV_API cv_status cv_hmm_create(const cv_hmm_desc* desc, cv_hmm** out);
/* HMM::from_json (hmm.rs:242-245 + null->-inf parsers 248-264). */
CV_API cv_status cv_hmm_from_json(const char* path, int32_t device, cv_hmm** out);
/* HMM::write (hmm.rs:236-240): serde_json layout, -inf written as null. */
CV_API cv_status cv_hmm_write_json(const cv_hmm* h, const char* path);
CV_API void cv_hmm_destroy(cv_hmm* h);
/* HMM::nstates (hmm.rs:207-209). */
/* ---- tuning keys (per handle) ------------------------------------------------------------
 * Layout, schedule and A/B choices of the kernels, and the test hooks that force a code path.
 * None changes a result: every key is bit-identical in paths, scores and statuses.  Each handle
 * holds ONE snapshot, taken at cv_hmm_create / cv_hmm_from_json from the environment
 * (variable CV_<KEY> in upper case, e.g. CV_T64_S=4 for "t64_s"; integers) over the defaults
 * below, and changed afterwards only by cv_hmm_set_tuning: an environment variable set after
 * the handle exists changes nothing, and no kernel launch reads the environment.  The
 * handle-less cv_hmm_fit_* read the environment once per call.
 *   trace 0               1: host phase stamps on stderr
 *   host_threads 0        host worker threads (0: min(16, hardware threads))
 *   t64_nonpos 1          0: the general f64 backtrack interval test (and no parallel chain)
 *   generic_rows 1        0: generic kernels in psi mode (inline argmax) instead of rows mode
 *   max_chunks 8          f32 trellis pipeline depth (1..64)
 *   host_sums 0           1: the constrained decode's exact unary sums on the host
 *   no_trace / no_resume / no_side 0   1: no certified suffix trace / resume flow / side-stream decode
 *   chain_par 1           0: cv_decode_superseq_cp runs the serial chain kernel
 *   chain_old 0           1: the one-thread-per-state chain kernel at any N
 *   chain_par_force 0     m > 0: every m-th sequence of the parallel chain taken as uncertified
 *   chain_spec 1          0: no speculative re-decode in the parallel chain
 *   chain_spec_kernel 0   the parallel chain's speculative re-decodes where N <= 256: 0 the serial chain
 *                         kernel's layout batched (one sequence per CU) after the forward passes and
 *                         cp_spec_psi (one sequence per workgroup, ~20 KiB of LDS) beside them;
 *                         1 trellis_cp_f64; 2 the generic CP kernel (always so above N = 256)
 *   chain_copy_overlap 1  0: the parallel chain in one decode chunk, its path copy before the walk
 *   chain_cert_fused 1    0: the chain's certificates by their own pass (cp_cert_f64), not the backtrack
 *   chain_parts 1         0: the parallel chain's decode in one part; 1: where N <= 256 and the batch
 *                         spans more than a forward round, a large first part then chain_tail small
 *                         parts (each walked beside the next part's forward pass); 2: one round each
 *   chain_tail 2, chain_tail_div 2       chain_parts = 1: the number of small parts, and a small
 *                         part's size as a forward round (64 sequences per CU) / chain_tail_div
 *   chain_spec_prio 3     issue priority (s_setprio 1..3; 0 the default) of the parallel chain's
 *                         speculative batches beside a forward pass
 *   chain_pin_obs 0, chain_pin_path 0   1: the parallel chain's later parts' observations / its
 *                         path copy through pinned staging (82 MiB of pinned host memory per handle)
 *                         instead of the runtime's pageable copies (measured neutral; the pageable
 *                         default keeps a first call ~20-70 ms shorter)
 *   t64_s 0               f64 trellis sequences per wave 2 / 4 / 6 / 8 (0: by batch)
 *   t64_512 / t64_1024 -1 NP = 512 / 1,024 batch kernel: -1 auto, 0 never, 1 always
 *   t64_wg 1              0: one wave per workgroup instead of eight-wave units
 *   t64_wg_force 0        1: eight-wave units whatever the batch's lengths
 *   t64_rs 1 / t64_w2 1   0: no row-split / no pair-of-waves small-batch layout
 *   t64_wave 1            0: N <= 64 on the lock-step kernel, not one wave per sequence; 2: N <= 48
 *                         on the 64-state one-wave kernel
 *   t64_bal 8             steps between SIMD-balancing updates (0: off)
 *   t64_cp_s 0            trellis_cp_f64 sequences per wave 1 / 2 / 4 (0: by batch)
 *   t64_cp_w 0            trellis_cp_f64 waves splitting the columns: 1 never, > 1 always (0: up to
 *                         4,096 sequences, NP >= 128); t64_cp_pf 0: its A rows in flight 32 (16)
 *   t64_bt_pf 0           backtrack_f64 rows in flight 2 / 4 / 8 / 16 / 32 (0: by NP)
 *   generic_s 0           generic kernels' sequences per workgroup 1 / 2 / 4 (0: by batch)
 *   generic_split 0, generic_split_k 0   1: K threads per state (generic_fwd_split), its K
 *   generic_wide 1, generic_wide_min 0   0: never wide / > 0: wide from this N
 *   generic_prio 0        1: generic_fwd_ms waves at issue priority 3 (the parallel chain sets it
 *                         for its speculative batch beside the last part's forward pass)
 *   wide_s 0              wide decode sequences per workgroup 1 / 2 / 4 (0: by batch)
 *   ext_wide_min 0        > 0: the constrained terms passes wide from this N
 *   chain_wide 1, chain_wide_min 0       the wide serial chain step: 0 never / from this N
 *   f32_onebar 1          0: two barriers per step in the f32 pair trellis
 *   bw_global 0, bw_perseq 0, bw_gemm_path 0   Baum-Welch: global scratch from N = 257 /
 *                         per-sequence E-step kernels / the xi GEMM path at every N
 * Unknown keys and values outside int32 are CV_EINVAL.  cv_tuning_key(i) lists the keys
 * (NULL past the last). */
/* Frees the handle's decode workspaces (delta rows, the constrained decode's and the parallel
 * chain's per-call buffers, pinned staging), which are otherwise kept grow-only between calls
 * so repeated calls do not reallocate: e.g. ~1 GB of chain buffers (observations, paths, the
 * speculative batches' psi rows) and 18 MiB of pinned staging plus the 34-69 GB delta workspace
 * after a config-4-sized cv_decode_superseq_cp / cv_decode_batch.  The model tables
 * stay; the next call allocates what it needs again.  Waits for the handle's streams. */
CV_API cv_status cv_hmm_release_workspaces(cv_hmm* h);
CV_API cv_status cv_hmm_set_tuning(cv_hmm* h, const char* key, int64_t value);
CV_API cv_status cv_hmm_get_tuning(const cv_hmm* h, const char* key, int64_t* value);
CV_API const char* cv_tuning_key(int32_t i);

CV_API int32_t cv_hmm_nstates(const cv_hmm* h);
CV_API int64_t cv_hmm_nobs(const cv_hmm* h);                   /* V = prod(bdims) */
CV_API int32_t cv_hmm_ndims(const cv_hmm* h);
CV_API cv_status cv_hmm_bdims(const cv_hmm* h, int64_t* bdims_out /*[D]*/);
/* flatten one D-dim observation value ([usize; D]) to the index used everywhere else. */
CV_API cv_status cv_obs_flatten(const cv_hmm* h, const int64_t* value /*[D]*/, int64_t* flat_out);
/* HMM::init_prob (hmm.rs:211-213) */
CV_API double cv_hmm_init_prob(const cv_hmm* h, int32_t state, int64_t obs);
/* HMM::init_probs (hmm.rs:215-218) -> out[N] */
CV_API cv_status cv_hmm_init_probs(const cv_hmm* h, int64_t obs, double* out);
/* HMM::transition_prob (hmm.rs:220-222) */
CV_API double cv_hmm_transition_prob(const cv_hmm* h, int32_t from, int32_t to, int64_t obs);
/* HMM::transitions_to (hmm.rs:224-226) -> out[N] = a[:, to] */
CV_API cv_status cv_hmm_transitions_to(const cv_hmm* h, int32_t to, double* out);
/* HMM::emit_prob (hmm.rs:228-230) */
CV_API double cv_hmm_emit_prob(const cv_hmm* h, int32_t state, int64_t obs);
/* HMM::emit_probs (hmm.rs:232-234) -> out[N] */
CV_API cv_status cv_hmm_emit_probs(const cv_hmm* h, int64_t obs, double* out);

/* ---- batch decode: the trellis forward pass + backtrack -------------------------------
 * Replaces, per sequence, the dense forward of CPSolver::init_viterbi (cp.rs:63-83) /
 * viterbi::decode (viterbi.rs:9-23) / DPSolver::solve (dp.rs:127-182) plus the backtrack
 * (cp.rs:85-93, viterbi.rs:24-31, dp.rs:71-89).  Host pointers; synchronous. */
CV_API cv_status cv_decode_batch(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                 const cv_opts* opts, int32_t* path_out, double* score_out,
                                 uint8_t* status_out);
/* Same on device-resident buffers, enqueued on opts->stream (or the handle's stream);
 * returns after enqueueing (no host synchronisation, so consecutive calls queue ahead).
 * Consecutive calls on one handle may use different streams: each waits, on its own stream,
 * for the previous call's workspace.  offsets_host (nullable) is a host copy of offsets used
 * for chunking; without it the offsets are copied back once.  Observation indices are
 * range-checked on the device: a bad one sets status CV_SEQ_BADOBS. */
CV_API cv_status cv_decode_batch_device(cv_hmm* h, int64_t nseq, const int64_t* offsets_host,
                                        const int64_t* offsets_dev, const int32_t* obs_dev,
                                        const cv_opts* opts, int32_t* path_dev, double* score_dev,
                                        uint8_t* status_dev);
/* Device timings of the last decode call on this handle (synchronizes its events). */
CV_API cv_status cv_last_timing(cv_hmm* h, cv_timing* out);
/* Device timings summed over EVERY decode call on this handle from cv_timing_begin to
 * cv_timing_end (no synchronisation in between, so a timed loop can enqueue ahead; the end
 * call synchronizes the events).  launches = chunk launches in all; total_ms = first kernel
 * start to last kernel end.  CV_ELIMIT beyond 16,384 chunk launches. */
CV_API cv_status cv_timing_begin(cv_hmm* h);
CV_API cv_status cv_timing_end(cv_hmm* h, cv_timing* out);
/* Consistency-constrained decode (the intended semantics of the reference's constrained
 * solvers, opti.rs:101-111 / dp.rs:157-164 / cp.rs:95-126): every element with
 * component[e] >= 0 takes the common state of its component, and the total log-likelihood
 * is maximised.  The objective splits at the constrained positions of each sequence
 * (cfn.rs:11-34 pattern): one position gives the max-marginal mu(s) = delta + beta; several
 * give alpha(s_1) + sum_k M_k(s_k, s_k+1) + beta(s_m) with segment tables M_k (start in s at
 * t_k with score 0, run to t_k+1) -- all computed by the trellis kernels.  Summed over
 * sequences as exact integers (units of 2^-64: independent of order and sharding) this is
 * a weighted CSP with unary and pairwise terms, solved exactly per connected group of
 * components by branch and bound (ties: lexicographically smallest state vector in
 * component order); then a forced decode.  Row-A0 (VITERBI) association, every term,
 * segment table and the final decode in opts->dtype: CV_DTYPE_F64 (default; the reference's
 * precision, cp.rs:95-126 / dp.rs:147-166 compute in f64: trellis_fwd_f64 for N <= 256, the
 * generic kernels up to N = 65535, wide above 10240) or CV_DTYPE_F32 (the f32 trellis, N <= 256, scores f64
 * re-scored).  A term outside the exact unit (|score| >= 2^32) is
 * CV_EINVAL.  comp_state_out[ncomp] gets s_c (-1: no active element, or no feasible assignment
 * of its group); objective_out = sum of the per-sequence scores.  CV_ELIMIT if the search
 * exceeds its node limit.  Host pointers; synchronous. */
CV_API cv_status cv_decode_constrained(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                       const int32_t* component, int32_t ncomp, const cv_opts* opts,
                                       int32_t* path_out, double* score_out, uint8_t* status_out,
                                       int32_t* comp_state_out, double* objective_out);
/* The same on device-resident inputs/outputs (offsets_dev/obs_dev in HBM, path_dev/score_dev/
 * status_dev written there; offsets_host and component stay on the host: the search's
 * structure is host work).  Observation indices are range-checked on the device before any
 * term is computed (CV_EINVAL, as the host API).  Enqueued on opts->stream (or the handle's
 * stream); synchronous: returns after the decode has finished. */
CV_API cv_status cv_decode_constrained_device(cv_hmm* h, int64_t nseq, const int64_t* offsets_host,
                                              const int64_t* offsets_dev, const int32_t* obs_dev,
                                              const int32_t* component, int32_t ncomp, const cv_opts* opts,
                                              int32_t* path_dev, double* score_dev, uint8_t* status_dev,
                                              int32_t* comp_state_out, double* objective_out);
/* Constrained sequences whose final forced path the last constrained decode on this handle
 * took from the certified suffix trace (f64, one constrained element, log-probability models:
 * the path after t1 read off the terms pass's suffix rows, with a rounding-error margin that
 * proves it is the forced decode's own path) instead of a second forward pass; 0 when the
 * trace was off (tuning key no_trace, f32, no kept rows). */
CV_API cv_status cv_last_suffix_traced(const cv_hmm* h, int64_t* out);
/* The same decode split at its one exchange step, for a batch sharded over processes/GPUs:
 * 0. cv_constrained_pairs (host only) on the FULL batch: the sorted component pairs (c1 < c2)
 *    that are consecutive constrained elements of some sequence -- the layout every rank
 *    agrees on.  pairs_out may be null to query *npairs_out.
 * 1. cv_constrained_partials: this shard's exact terms as CV_PARTIAL_WORDS int64 words that
 *    ADD across shards (one all-reduce SUM).  Per component: 4N base-2^32 limbs (state-major)
 *    of the unary sum in units of 2^-64, N counts of -inf terms, 1 count of constrained
 *    elements; then per pair: 4N^2 limbs (entry s1*N+s2), N^2 -inf counts, 1 count.
 * 2. cv_constrained_select (host only): the exact search on the reduced partials;
 *    explored = (component, state) candidates scored.
 * 3. cv_decode_forced_components: the shard's final decode with every constrained element
 *    forced to comp_state[component[e]]; objective_out = the shard's sum of scores.
 * cv_decode_constrained == 0 + 1 + 2 + 3 on one process. */
#define CV_PARTIAL_WORDS(nstates, ncomp, npairs) \
  ((int64_t)(ncomp) * (5 * (int64_t)(nstates) + 1) + (int64_t)(npairs) * (5 * (int64_t)(nstates) * (nstates) + 1))
CV_API cv_status cv_constrained_pairs(int64_t nseq, const int64_t* offsets, const int32_t* component, int32_t ncomp,
                                      int32_t* pairs_out, int64_t cap_pairs, int64_t* npairs_out);
CV_API cv_status cv_constrained_partials(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                         const int32_t* component, int32_t ncomp, int64_t npairs,
                                         const int32_t* pairs, const cv_opts* opts, int64_t* partials_out);
CV_API cv_status cv_constrained_select(int32_t nstates, int32_t ncomp, int64_t npairs, const int32_t* pairs,
                                       const int64_t* partials, int32_t* comp_state_out, uint64_t* explored_out);
CV_API cv_status cv_decode_forced_components(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                             const int32_t* component, int32_t ncomp, const int32_t* comp_state,
                                             const cv_opts* opts, int32_t* path_out, double* score_out,
                                             uint8_t* status_out, double* objective_out);
/* Steps 1-3 in ONE call on a shard, the exchange made by the caller's callback: after this
 * shard's partials are computed, exchange(words, nwords, ctx) must replace words[0, nwords)
 * by their SUM over all shards (e.g. an all-reduce; return 0 on success) -- then the search
 * and the shard's final decode run here, which lets the decode reuse the terms pass's prefix
 * rows (the resume flow) like cv_decode_constrained.  pairs = cv_constrained_pairs of the
 * FULL batch.  Every rank must reach the callback: it is called even for an empty shard.
 * exchange == NULL: a single process (words already total).  Host pointers; synchronous.
 * objective_out = the shard's sum of scores. */
typedef int32_t (*cv_exchange_fn)(int64_t* words, int64_t nwords, void* ctx);
CV_API cv_status cv_decode_constrained_exchange(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                                const int32_t* component, int32_t ncomp, int64_t npairs,
                                                const int32_t* pairs, cv_exchange_fn exchange, void* ctx,
                                                const cv_opts* opts, int32_t* path_out, double* score_out,
                                                uint8_t* status_out, int32_t* comp_state_out,
                                                uint64_t* explored_out, double* objective_out);
/* viterbi::decode (viterbi.rs:5): one sequence, reference decode() semantics (row 0 = 0.0,
 * f64), path only. */
CV_API cv_status cv_viterbi_decode(cv_hmm* h, int64_t T, const int32_t* obs, int32_t* path_out);
/* CPSolver::solve without active constraints, exactly (cp.rs:133-143: init_viterbi cp.rs:63-83
 * + backtrack cp.rs:85-93 over the super-sequence of utils.rs:62-103): the nseq sequences are
 * decoded as ONE chain in order -- at a sequence start the predecessor term is pi[j]
 * (utils.rs:24-38), so later sequences carry the running total and round exactly as the
 * reference does (a per-sequence decode can differ from it at near ties).  f64, first-index
 * argmax, CP association.  path_out[offsets[nseq] - offsets[0]] in super-sequence order;
 * objective_out = the chain's final maximum (main.rs:129's first number).  Log-probability
 * models (finite entries in [-2^80, 0]), any N: every sequence is decoded on its own by the
 * batch path's f64 row-A0 decode in parallel and certified to be the chain's path at the chain's running
 * total (a rounding-error margin), the running total folded on the host, and only the
 * uncertified sequences (near ties at that magnitude) re-decoded from their predicted offsets
 * or re-run through the serial chain kernel -- bit-identical to the serial chain
 * (cv_last_superseq_stats).  Otherwise serial over
 * elements on the GPU (one workgroup; above N = 1024 one launch per element with the states
 * over workgroups), as the reference is on the CPU.  N <= 65535.
 * CV_EINFEASIBLE when the maximum is -inf. */
CV_API cv_status cv_decode_superseq_cp(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                       int32_t* path_out, double* objective_out);
/* How the last cv_decode_superseq_cp on this handle ran (out[9]): out[0] = 1 when the PARALLEL
 * chain ran (every finite entry of the model in [-2^80, 0], every sequence feasible:
 * each sequence decoded on its own by the f64 trellis and certified to be the chain's own path
 * at the chain's running total), 0 for the serial chain; out[1] = sequences
 * certified, out[2] = sequences the serial chain kernel re-ran, out[3] = such runs, out[4] =
 * certified sequences folded by one quantised add, out[5] = uncertified sequences settled by
 * the parallel re-decode from their exact offsets (speculation), out[6] = such batches, out[7] =
 * sequences whose paths the host walk fetched packed while the whole path copy ran beside it,
 * out[8] = walk steps that had to wait for that copy (a prediction miss; 0 when it held). */
CV_API cv_status cv_last_superseq_stats(const cv_hmm* h, int64_t* out);

/* ---- trait Solver (viterbi_solver.rs:11-16) -------------------------------------------
 * kind: "gpu"      f32 trellis kernel, VITERBI association, f64 re-scored objective
 *       "gpu-f64"  f64, VITERBI association (reference numerics, row A0)
 *       "gpu-cp"   CPSolver (cp.rs), what main.rs:120 runs: without constraints the exact
 *                  chained super-sequence decode (cv_decode_superseq_cp, objective and path
 *                  as the reference rounds them)
 *       "gpu-cp-seq" f64, CP association, every sequence decoded on its own (parallel; equal
 *                  to gpu-cp up to the chain's running-total roundings)
 *       "gpu-dp"   f64, DP association = DPSolver (dp.rs), ascending-index ties
 * Unconstrained super-sequences decode per sequence (except "gpu-cp",
 * chained): objective = sum of per-sequence scores (sequence order), solution in element order.  Active
 * constraints go through cv_decode_constrained on the row-A0 association at the kind's
 * precision (f64 for gpu-f64 / gpu-cp / gpu-dp, f32 for gpu); get_explored_nodes then
 * reports the number of (component, state) candidates scored. */
CV_API cv_status cv_solver_create(const char* kind, cv_hmm* h, const cv_superseq_desc* seq, cv_solver** out);
CV_API cv_status cv_solver_solve(cv_solver* s);                                   /* Solver::solve */
CV_API cv_status cv_solver_get_solution(const cv_solver* s, const int32_t** sol, int64_t* len); /* get_solution */
CV_API cv_status cv_solver_get_objective(const cv_solver* s, double* obj);        /* get_objective */
CV_API const char* cv_solver_get_name(const cv_solver* s);                        /* get_name */
CV_API cv_status cv_solver_get_explored_nodes(const cv_solver* s, uint64_t* n);   /* CPSolver::get_explored_nodes cp.rs:128 */
CV_API void cv_solver_destroy(cv_solver* s);
/* write_cfn (viterbi_solver/cfn.rs:82-205): the cost-function network of the solver's
 * super-sequence for toulbar2 -- one variable per active component, unary start/end costs,
 * N x N tables of segment longest paths between consecutive constraint boundaries (rows
 * computed on the GPU in f64, bit-identical to the reference loops), the lower bound, in the
 * reference's text layout and float formatting.  *compile_ms = table time (the value main.rs
 * writes when run_cfn is set, main.rs:116-118).  Cost: (boundaries x N) segment passes of
 * N^2 per element, as in the reference -- meant for the problem sizes toulbar2 takes. */
CV_API cv_status cv_solver_write_cfn(cv_solver* s, const char* path, uint64_t* compile_ms);

/* ---- HMM fitting (hmm.rs:30-190) ------------------------------------
 * pi[N], a[N*N] (from-major), b[N*V] (state-major, obs row-major over bdims): the CURRENT
 * parameters in PROBABILITY space on entry (the reference starts from HMM::new's random
 * draw, hmm.rs:22-28), the fitted parameters log-mapped on return (the reference's log():
 * 0 -> -inf, else ln(x)/ln(10), hmm.rs:192-205) -- ready for cv_hmm_desc.  f64.
 * tags[sum T]: the state of an element, -1 = unknown (None).  device: HIP device index. */
/* maximum_likelihood_estimation (hmm.rs:30-62): exact integer counts on the GPU, ADDED to
 * the current probabilities with the reference's sequential rounding; every tag >= 0. */
CV_API cv_status cv_hmm_fit_mle(int32_t nstates, int64_t nobs, int64_t nseq, const int64_t* offsets,
                                const int32_t* obs, const int32_t* tags, int32_t device, double* pi, double* a,
                                double* b);
/* train (hmm.rs:69-190): tag-clamped Baum-Welch, E- and M-step on the GPU (N <= 65535: one wave
 * per sequence up to 64 states, 32 sequences per workgroup on the f64 matrix cores up to 256,
 * strided per-sequence kernels above (their vectors in LDS to N = 4096, in global memory
 * beyond); over 64 states the xi sums run as one f64 matrix-core
 * GEMM over stored rows per chunk) with
 * the parameters resident between iterations; the convergence test (sum |new - old| <= tol,
 * checked after the update, hmm.rs:172-177) adds per-block partial sums on the host.
 * *iters_out = iterations run. */
CV_API cv_status cv_hmm_fit_train(int32_t nstates, int64_t nobs, int64_t nseq, const int64_t* offsets,
                                  const int32_t* obs, const int32_t* tags, int32_t max_iter, double tol,
                                  int32_t device, double* pi, double* a, double* b, int32_t* iters_out);

#ifdef __cplusplus
}
#endif
#endif /* CVITERBI_H */
