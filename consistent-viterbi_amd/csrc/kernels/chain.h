// chain.h -- CPSolver's super-sequence decode chained exactly (cp.rs:63-93 over
// utils.rs:24-38), N <= 256: one workgroup walks the elements, candidates split across its
// waves; then a parallel segmented backtrack over the stored psi rows.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cvk {

struct CpChainWgArgs {
  const double* pi;      // [NP] -inf padded
  const double* a;       // [NP][NP] from-major, -inf padded
  const double* et;      // [V][NP] emissions transposed, -inf padded
  const int32_t* obs;    // [len] super-sequence observations
  const uint8_t* first;  // [len] 1 at the first element of each sequence (MetaElements t == 0)
  int64_t len;
  int nstates;
  uint16_t* psi;         // [len][NP] first argmax per (element, state); row 0 unused
                         // unless init_row is set
  double* objective;     // [1] max of the last row (cp.rs:140)
  int32_t* final_state;  // [1] its first argmax (cp.rs:86)
  // a PART of the chain (the parallel chain's fallback runs): init_row [NP] = the chain's row
  // before element 0 (element 0 then runs like any element, psi row 0 included); final_row
  // [NP] receives the last row.  Both null: the whole chain (row 0 = init_probs, cp.rs:66-68).
  const double* init_row;
  double* final_row;
  // BATCH (launch_cp_chain_wg_batch, the parallel chain's speculative re-decodes after the
  // forward passes): workgroup i decodes sequence i of a packed batch on its own, elements
  // [soff[i], soff[i + 1]) of obs, row 0 = sinit[i] + (pi + b) (the chain's start value at
  // offset sinit[i] after a clean boundary, utils.rs:32-35), psi rows at psi + soff[i] * np;
  // its last row to final_row + i * nstates and its path (first argmax of the last row,
  // cp.rs:86, then psi) to path + soff[i]
  const int64_t* soff;
  const double* sinit;
  int32_t* path;
};
// forward of the whole chain on ONE workgroup; np = 64 * ceil(N / 64) <= 256
hipError_t launch_cp_chain_wg(int np, const CpChainWgArgs& g, hipStream_t stream);
// nseq such sequences at once, one workgroup (one CU) each: A on chip, ~3.5 us per element at
// N = 256, against ~17 us for the one-thread-per-state kernels that stream A from L2
hipError_t launch_cp_chain_wg_batch(int np, const CpChainWgArgs& g, int64_t nseq, hipStream_t stream);

// The parallel chain's speculative re-decodes BESIDE a forward pass (N <= 256): one sequence per
// workgroup, thread j = state j, A through buffer loads with a scalar row offset, the candidate
// walk at 4 VALU per candidate (add, compare, max, index select), row 0 = sinit + (pi + b) like
// the batched kernel; psi [soff[i] + t][np], the last row to last[i nstates ..], the path (first
// argmax of the last row, then psi through LDS-staged rows) to path + soff[i].  ~20 KiB of LDS
// and few VGPRs: it fits beside two forward waves per SIMD.
struct CpSpecArgs {
  const double* pi;    // [np] -inf padded
  const double* a;     // [np][np] from-major, -inf padded
  const double* et;    // [V][np] -inf padded
  const int32_t* obs;  // packed batch observations
  const int64_t* soff;
  const double* sinit;
  int nstates;
  int prio;            // issue priority 1..3 (0: the default)
  uint16_t* psi;
  double* last;
  int32_t* path;
};
hipError_t launch_cp_spec_psi(int np, const CpSpecArgs& g, int64_t nseq, hipStream_t stream);
// LDS bytes launch_cp_chain_wg asks for at this np (0: unsupported)
size_t cp_chain_wg_lds(int np);

struct CpChainBtArgs {
  const uint16_t* psi;       // [len][np]
  int np;
  int64_t len;
  int64_t seg;               // elements per segment
  int64_t nseg;
  uint16_t* map;             // [nseg][np]: segment k >= 1, state at its last element -> state at e0 - 1
  const int32_t* end_state;  // [nseg] state at the last element of segment k
  int32_t* path;             // [len]
};
// pass 1: every segment k >= 1 backtracks from ALL np end states at once -> map[k]
hipError_t launch_cp_chain_seg_map(const CpChainBtArgs& g, hipStream_t stream);
// pass 2 (after the host resolved end_state[] through the maps): each segment's path
hipError_t launch_cp_chain_seg_path(const CpChainBtArgs& g, hipStream_t stream);

}  // namespace cvk
