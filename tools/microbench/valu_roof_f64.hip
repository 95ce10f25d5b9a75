// The f64 VALU roof trellis_fwd_f64 is graded against, measured per SIMD.
//
// Every wave of a one-workgroup-per-CU grid (W waves per SIMD, 4W waves per workgroup) stamps
// s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop and records HW_ID /
// XCC_ID.  The host groups the waves by SIMD and takes each SIMD's span from its FIRST wave's
// start to its LAST wave's end, so waves that do not overlap cannot inflate the rate (the
// per-wave spans of round 5's mfma_f64_coissue.hip could).  The clock is
// d(memtime) / d(memrealtime) x 100 MHz over the same spans (MI355X_MICROARCH.md, DVFS item 6),
// after >= 2 s of back-to-back launches.  A kernel-wide HIP-event rate is the cross-check.
//
// Mixes (one (from, to) pair = one v_add_f64 + one v_max_f64, 16 independent accumulators):
//   0 "pairs"   : the forward's inner loop alone -- 8 adds then their 8 maxima, as
//                 trellis_fwd_f64 groups them (sched_group_barrier), delta a VGPR operand
//   1 "fwd-mix" : per A row as trellis_fwd_f64 at C = 4, S = 8 issues it: 2 global_load_dwordx4
//                 (an L1-resident row), 4 ds_read_b128 broadcasts (the S deltas), 32 pairs;
//                 loads a row ahead, waited with vmcnt / lgkmcnt like the kernel's ring
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_roof_f64 valu_roof_f64.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

struct Stamp {
  unsigned long long c0, c1, r0, r1;
  unsigned hw, xcc;
};

// KIND 0: ITERS x 64 pairs per wave
template <int KIND>
__global__ __launch_bounds__(1024) void roof_k(double* sink, Stamp* st, const double* arow, int iters, double seed) {
  __shared__ double lds[64];
  const int tid = threadIdx.x;
  if (tid < 64) lds[tid] = seed - tid;
  __syncthreads();
  if (lds[0] == 1234.5) sink[tid] = lds[1];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  // the loop in one asm block, fixed registers (no compiler moves): 2 A rows per iteration,
  // x = v[0:7] / v[8:15] (C = 4 columns), deltas v[16:31] / v[32:47] (S = 8), temporaries
  // v[64:79], accumulators v[80:111]; 64 pairs per iteration
  const double* p = arow + (tid & 63) * 4;
  const unsigned la = 0;  // every lane the same LDS address: a broadcast
  if constexpr (KIND == 0) {
    asm volatile(
        "v_mov_b32 v0, 0\n"
        "v_mov_b32 v1, 0\n"
        "v_mov_b32 v2, 0\n"
        "v_mov_b32 v3, 0\n"
        "v_mov_b32 v4, 0\n"
        "v_mov_b32 v5, 0\n"
        "v_mov_b32 v6, 0\n"
        "v_mov_b32 v7, 0\n"
        "v_mov_b32 v8, 0\n"
        "v_mov_b32 v9, 0\n"
        "v_mov_b32 v10, 0\n"
        "v_mov_b32 v11, 0\n"
        "v_mov_b32 v12, 0\n"
        "v_mov_b32 v13, 0\n"
        "v_mov_b32 v14, 0\n"
        "v_mov_b32 v15, 0\n"
        "v_mov_b32 v16, 0\n"
        "v_mov_b32 v17, 0\n"
        "v_mov_b32 v18, 0\n"
        "v_mov_b32 v19, 0\n"
        "v_mov_b32 v20, 0\n"
        "v_mov_b32 v21, 0\n"
        "v_mov_b32 v22, 0\n"
        "v_mov_b32 v23, 0\n"
        "v_mov_b32 v24, 0\n"
        "v_mov_b32 v25, 0\n"
        "v_mov_b32 v26, 0\n"
        "v_mov_b32 v27, 0\n"
        "v_mov_b32 v28, 0\n"
        "v_mov_b32 v29, 0\n"
        "v_mov_b32 v30, 0\n"
        "v_mov_b32 v31, 0\n"
        "v_mov_b32 v32, 0\n"
        "v_mov_b32 v33, 0\n"
        "v_mov_b32 v34, 0\n"
        "v_mov_b32 v35, 0\n"
        "v_mov_b32 v36, 0\n"
        "v_mov_b32 v37, 0\n"
        "v_mov_b32 v38, 0\n"
        "v_mov_b32 v39, 0\n"
        "v_mov_b32 v40, 0\n"
        "v_mov_b32 v41, 0\n"
        "v_mov_b32 v42, 0\n"
        "v_mov_b32 v43, 0\n"
        "v_mov_b32 v44, 0\n"
        "v_mov_b32 v45, 0\n"
        "v_mov_b32 v46, 0\n"
        "v_mov_b32 v47, 0\n"
        "v_mov_b32 v48, 0\n"
        "v_mov_b32 v49, 0\n"
        "v_mov_b32 v50, 0\n"
        "v_mov_b32 v51, 0\n"
        "v_mov_b32 v52, 0\n"
        "v_mov_b32 v53, 0\n"
        "v_mov_b32 v54, 0\n"
        "v_mov_b32 v55, 0\n"
        "v_mov_b32 v56, 0\n"
        "v_mov_b32 v57, 0\n"
        "v_mov_b32 v58, 0\n"
        "v_mov_b32 v59, 0\n"
        "v_mov_b32 v60, 0\n"
        "v_mov_b32 v61, 0\n"
        "v_mov_b32 v62, 0\n"
        "v_mov_b32 v63, 0\n"
        "v_mov_b32 v64, 0\n"
        "v_mov_b32 v65, 0\n"
        "v_mov_b32 v66, 0\n"
        "v_mov_b32 v67, 0\n"
        "v_mov_b32 v68, 0\n"
        "v_mov_b32 v69, 0\n"
        "v_mov_b32 v70, 0\n"
        "v_mov_b32 v71, 0\n"
        "v_mov_b32 v72, 0\n"
        "v_mov_b32 v73, 0\n"
        "v_mov_b32 v74, 0\n"
        "v_mov_b32 v75, 0\n"
        "v_mov_b32 v76, 0\n"
        "v_mov_b32 v77, 0\n"
        "v_mov_b32 v78, 0\n"
        "v_mov_b32 v79, 0\n"
        "v_mov_b32 v80, 0\n"
        "v_mov_b32 v81, 0\n"
        "v_mov_b32 v82, 0\n"
        "v_mov_b32 v83, 0\n"
        "v_mov_b32 v84, 0\n"
        "v_mov_b32 v85, 0\n"
        "v_mov_b32 v86, 0\n"
        "v_mov_b32 v87, 0\n"
        "v_mov_b32 v88, 0\n"
        "v_mov_b32 v89, 0\n"
        "v_mov_b32 v90, 0\n"
        "v_mov_b32 v91, 0\n"
        "v_mov_b32 v92, 0\n"
        "v_mov_b32 v93, 0\n"
        "v_mov_b32 v94, 0\n"
        "v_mov_b32 v95, 0\n"
        "v_mov_b32 v96, 0\n"
        "v_mov_b32 v97, 0\n"
        "v_mov_b32 v98, 0\n"
        "v_mov_b32 v99, 0\n"
        "v_mov_b32 v100, 0\n"
        "v_mov_b32 v101, 0\n"
        "v_mov_b32 v102, 0\n"
        "v_mov_b32 v103, 0\n"
        "v_mov_b32 v104, 0\n"
        "v_mov_b32 v105, 0\n"
        "v_mov_b32 v106, 0\n"
        "v_mov_b32 v107, 0\n"
        "v_mov_b32 v108, 0\n"
        "v_mov_b32 v109, 0\n"
        "v_mov_b32 v110, 0\n"
        "v_mov_b32 v111, 0\n"
        "s_mov_b32 s40, %[it]\n"
        "1:\n"
        "v_add_f64 v[64:65], v[16:17], v[0:1]\n"
        "v_add_f64 v[66:67], v[16:17], v[2:3]\n"
        "v_add_f64 v[68:69], v[16:17], v[4:5]\n"
        "v_add_f64 v[70:71], v[16:17], v[6:7]\n"
        "v_add_f64 v[72:73], v[18:19], v[0:1]\n"
        "v_add_f64 v[74:75], v[18:19], v[2:3]\n"
        "v_add_f64 v[76:77], v[18:19], v[4:5]\n"
        "v_add_f64 v[78:79], v[18:19], v[6:7]\n"
        "v_max_f64 v[80:81], v[80:81], v[64:65]\n"
        "v_max_f64 v[82:83], v[82:83], v[66:67]\n"
        "v_max_f64 v[84:85], v[84:85], v[68:69]\n"
        "v_max_f64 v[86:87], v[86:87], v[70:71]\n"
        "v_max_f64 v[88:89], v[88:89], v[72:73]\n"
        "v_max_f64 v[90:91], v[90:91], v[74:75]\n"
        "v_max_f64 v[92:93], v[92:93], v[76:77]\n"
        "v_max_f64 v[94:95], v[94:95], v[78:79]\n"
        "v_add_f64 v[64:65], v[20:21], v[0:1]\n"
        "v_add_f64 v[66:67], v[20:21], v[2:3]\n"
        "v_add_f64 v[68:69], v[20:21], v[4:5]\n"
        "v_add_f64 v[70:71], v[20:21], v[6:7]\n"
        "v_add_f64 v[72:73], v[22:23], v[0:1]\n"
        "v_add_f64 v[74:75], v[22:23], v[2:3]\n"
        "v_add_f64 v[76:77], v[22:23], v[4:5]\n"
        "v_add_f64 v[78:79], v[22:23], v[6:7]\n"
        "v_max_f64 v[96:97], v[96:97], v[64:65]\n"
        "v_max_f64 v[98:99], v[98:99], v[66:67]\n"
        "v_max_f64 v[100:101], v[100:101], v[68:69]\n"
        "v_max_f64 v[102:103], v[102:103], v[70:71]\n"
        "v_max_f64 v[104:105], v[104:105], v[72:73]\n"
        "v_max_f64 v[106:107], v[106:107], v[74:75]\n"
        "v_max_f64 v[108:109], v[108:109], v[76:77]\n"
        "v_max_f64 v[110:111], v[110:111], v[78:79]\n"
        "v_add_f64 v[64:65], v[24:25], v[0:1]\n"
        "v_add_f64 v[66:67], v[24:25], v[2:3]\n"
        "v_add_f64 v[68:69], v[24:25], v[4:5]\n"
        "v_add_f64 v[70:71], v[24:25], v[6:7]\n"
        "v_add_f64 v[72:73], v[26:27], v[0:1]\n"
        "v_add_f64 v[74:75], v[26:27], v[2:3]\n"
        "v_add_f64 v[76:77], v[26:27], v[4:5]\n"
        "v_add_f64 v[78:79], v[26:27], v[6:7]\n"
        "v_max_f64 v[112:113], v[112:113], v[64:65]\n"
        "v_max_f64 v[114:115], v[114:115], v[66:67]\n"
        "v_max_f64 v[116:117], v[116:117], v[68:69]\n"
        "v_max_f64 v[118:119], v[118:119], v[70:71]\n"
        "v_max_f64 v[120:121], v[120:121], v[72:73]\n"
        "v_max_f64 v[122:123], v[122:123], v[74:75]\n"
        "v_max_f64 v[124:125], v[124:125], v[76:77]\n"
        "v_max_f64 v[126:127], v[126:127], v[78:79]\n"
        "v_add_f64 v[64:65], v[28:29], v[0:1]\n"
        "v_add_f64 v[66:67], v[28:29], v[2:3]\n"
        "v_add_f64 v[68:69], v[28:29], v[4:5]\n"
        "v_add_f64 v[70:71], v[28:29], v[6:7]\n"
        "v_add_f64 v[72:73], v[30:31], v[0:1]\n"
        "v_add_f64 v[74:75], v[30:31], v[2:3]\n"
        "v_add_f64 v[76:77], v[30:31], v[4:5]\n"
        "v_add_f64 v[78:79], v[30:31], v[6:7]\n"
        "v_max_f64 v[128:129], v[128:129], v[64:65]\n"
        "v_max_f64 v[130:131], v[130:131], v[66:67]\n"
        "v_max_f64 v[132:133], v[132:133], v[68:69]\n"
        "v_max_f64 v[134:135], v[134:135], v[70:71]\n"
        "v_max_f64 v[136:137], v[136:137], v[72:73]\n"
        "v_max_f64 v[138:139], v[138:139], v[74:75]\n"
        "v_max_f64 v[140:141], v[140:141], v[76:77]\n"
        "v_max_f64 v[142:143], v[142:143], v[78:79]\n"
        "v_add_f64 v[64:65], v[32:33], v[8:9]\n"
        "v_add_f64 v[66:67], v[32:33], v[10:11]\n"
        "v_add_f64 v[68:69], v[32:33], v[12:13]\n"
        "v_add_f64 v[70:71], v[32:33], v[14:15]\n"
        "v_add_f64 v[72:73], v[34:35], v[8:9]\n"
        "v_add_f64 v[74:75], v[34:35], v[10:11]\n"
        "v_add_f64 v[76:77], v[34:35], v[12:13]\n"
        "v_add_f64 v[78:79], v[34:35], v[14:15]\n"
        "v_max_f64 v[80:81], v[80:81], v[64:65]\n"
        "v_max_f64 v[82:83], v[82:83], v[66:67]\n"
        "v_max_f64 v[84:85], v[84:85], v[68:69]\n"
        "v_max_f64 v[86:87], v[86:87], v[70:71]\n"
        "v_max_f64 v[88:89], v[88:89], v[72:73]\n"
        "v_max_f64 v[90:91], v[90:91], v[74:75]\n"
        "v_max_f64 v[92:93], v[92:93], v[76:77]\n"
        "v_max_f64 v[94:95], v[94:95], v[78:79]\n"
        "v_add_f64 v[64:65], v[36:37], v[8:9]\n"
        "v_add_f64 v[66:67], v[36:37], v[10:11]\n"
        "v_add_f64 v[68:69], v[36:37], v[12:13]\n"
        "v_add_f64 v[70:71], v[36:37], v[14:15]\n"
        "v_add_f64 v[72:73], v[38:39], v[8:9]\n"
        "v_add_f64 v[74:75], v[38:39], v[10:11]\n"
        "v_add_f64 v[76:77], v[38:39], v[12:13]\n"
        "v_add_f64 v[78:79], v[38:39], v[14:15]\n"
        "v_max_f64 v[96:97], v[96:97], v[64:65]\n"
        "v_max_f64 v[98:99], v[98:99], v[66:67]\n"
        "v_max_f64 v[100:101], v[100:101], v[68:69]\n"
        "v_max_f64 v[102:103], v[102:103], v[70:71]\n"
        "v_max_f64 v[104:105], v[104:105], v[72:73]\n"
        "v_max_f64 v[106:107], v[106:107], v[74:75]\n"
        "v_max_f64 v[108:109], v[108:109], v[76:77]\n"
        "v_max_f64 v[110:111], v[110:111], v[78:79]\n"
        "v_add_f64 v[64:65], v[40:41], v[8:9]\n"
        "v_add_f64 v[66:67], v[40:41], v[10:11]\n"
        "v_add_f64 v[68:69], v[40:41], v[12:13]\n"
        "v_add_f64 v[70:71], v[40:41], v[14:15]\n"
        "v_add_f64 v[72:73], v[42:43], v[8:9]\n"
        "v_add_f64 v[74:75], v[42:43], v[10:11]\n"
        "v_add_f64 v[76:77], v[42:43], v[12:13]\n"
        "v_add_f64 v[78:79], v[42:43], v[14:15]\n"
        "v_max_f64 v[112:113], v[112:113], v[64:65]\n"
        "v_max_f64 v[114:115], v[114:115], v[66:67]\n"
        "v_max_f64 v[116:117], v[116:117], v[68:69]\n"
        "v_max_f64 v[118:119], v[118:119], v[70:71]\n"
        "v_max_f64 v[120:121], v[120:121], v[72:73]\n"
        "v_max_f64 v[122:123], v[122:123], v[74:75]\n"
        "v_max_f64 v[124:125], v[124:125], v[76:77]\n"
        "v_max_f64 v[126:127], v[126:127], v[78:79]\n"
        "v_add_f64 v[64:65], v[44:45], v[8:9]\n"
        "v_add_f64 v[66:67], v[44:45], v[10:11]\n"
        "v_add_f64 v[68:69], v[44:45], v[12:13]\n"
        "v_add_f64 v[70:71], v[44:45], v[14:15]\n"
        "v_add_f64 v[72:73], v[46:47], v[8:9]\n"
        "v_add_f64 v[74:75], v[46:47], v[10:11]\n"
        "v_add_f64 v[76:77], v[46:47], v[12:13]\n"
        "v_add_f64 v[78:79], v[46:47], v[14:15]\n"
        "v_max_f64 v[128:129], v[128:129], v[64:65]\n"
        "v_max_f64 v[130:131], v[130:131], v[66:67]\n"
        "v_max_f64 v[132:133], v[132:133], v[68:69]\n"
        "v_max_f64 v[134:135], v[134:135], v[70:71]\n"
        "v_max_f64 v[136:137], v[136:137], v[72:73]\n"
        "v_max_f64 v[138:139], v[138:139], v[74:75]\n"
        "v_max_f64 v[140:141], v[140:141], v[76:77]\n"
        "v_max_f64 v[142:143], v[142:143], v[78:79]\n"
        "s_sub_u32 s40, s40, 1\n"
        "s_cmp_lg_u32 s40, 0\n"
        "s_cbranch_scc1 1b\n"
        :
        : [it] "s"(iters), [p] "v"(p), [la] "v"(la)
        : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "s40", "scc", "memory");
  } else {
    asm volatile(
        "v_mov_b32 v0, 0\n"
        "v_mov_b32 v1, 0\n"
        "v_mov_b32 v2, 0\n"
        "v_mov_b32 v3, 0\n"
        "v_mov_b32 v4, 0\n"
        "v_mov_b32 v5, 0\n"
        "v_mov_b32 v6, 0\n"
        "v_mov_b32 v7, 0\n"
        "v_mov_b32 v8, 0\n"
        "v_mov_b32 v9, 0\n"
        "v_mov_b32 v10, 0\n"
        "v_mov_b32 v11, 0\n"
        "v_mov_b32 v12, 0\n"
        "v_mov_b32 v13, 0\n"
        "v_mov_b32 v14, 0\n"
        "v_mov_b32 v15, 0\n"
        "v_mov_b32 v16, 0\n"
        "v_mov_b32 v17, 0\n"
        "v_mov_b32 v18, 0\n"
        "v_mov_b32 v19, 0\n"
        "v_mov_b32 v20, 0\n"
        "v_mov_b32 v21, 0\n"
        "v_mov_b32 v22, 0\n"
        "v_mov_b32 v23, 0\n"
        "v_mov_b32 v24, 0\n"
        "v_mov_b32 v25, 0\n"
        "v_mov_b32 v26, 0\n"
        "v_mov_b32 v27, 0\n"
        "v_mov_b32 v28, 0\n"
        "v_mov_b32 v29, 0\n"
        "v_mov_b32 v30, 0\n"
        "v_mov_b32 v31, 0\n"
        "v_mov_b32 v32, 0\n"
        "v_mov_b32 v33, 0\n"
        "v_mov_b32 v34, 0\n"
        "v_mov_b32 v35, 0\n"
        "v_mov_b32 v36, 0\n"
        "v_mov_b32 v37, 0\n"
        "v_mov_b32 v38, 0\n"
        "v_mov_b32 v39, 0\n"
        "v_mov_b32 v40, 0\n"
        "v_mov_b32 v41, 0\n"
        "v_mov_b32 v42, 0\n"
        "v_mov_b32 v43, 0\n"
        "v_mov_b32 v44, 0\n"
        "v_mov_b32 v45, 0\n"
        "v_mov_b32 v46, 0\n"
        "v_mov_b32 v47, 0\n"
        "v_mov_b32 v48, 0\n"
        "v_mov_b32 v49, 0\n"
        "v_mov_b32 v50, 0\n"
        "v_mov_b32 v51, 0\n"
        "v_mov_b32 v52, 0\n"
        "v_mov_b32 v53, 0\n"
        "v_mov_b32 v54, 0\n"
        "v_mov_b32 v55, 0\n"
        "v_mov_b32 v56, 0\n"
        "v_mov_b32 v57, 0\n"
        "v_mov_b32 v58, 0\n"
        "v_mov_b32 v59, 0\n"
        "v_mov_b32 v60, 0\n"
        "v_mov_b32 v61, 0\n"
        "v_mov_b32 v62, 0\n"
        "v_mov_b32 v63, 0\n"
        "v_mov_b32 v64, 0\n"
        "v_mov_b32 v65, 0\n"
        "v_mov_b32 v66, 0\n"
        "v_mov_b32 v67, 0\n"
        "v_mov_b32 v68, 0\n"
        "v_mov_b32 v69, 0\n"
        "v_mov_b32 v70, 0\n"
        "v_mov_b32 v71, 0\n"
        "v_mov_b32 v72, 0\n"
        "v_mov_b32 v73, 0\n"
        "v_mov_b32 v74, 0\n"
        "v_mov_b32 v75, 0\n"
        "v_mov_b32 v76, 0\n"
        "v_mov_b32 v77, 0\n"
        "v_mov_b32 v78, 0\n"
        "v_mov_b32 v79, 0\n"
        "v_mov_b32 v80, 0\n"
        "v_mov_b32 v81, 0\n"
        "v_mov_b32 v82, 0\n"
        "v_mov_b32 v83, 0\n"
        "v_mov_b32 v84, 0\n"
        "v_mov_b32 v85, 0\n"
        "v_mov_b32 v86, 0\n"
        "v_mov_b32 v87, 0\n"
        "v_mov_b32 v88, 0\n"
        "v_mov_b32 v89, 0\n"
        "v_mov_b32 v90, 0\n"
        "v_mov_b32 v91, 0\n"
        "v_mov_b32 v92, 0\n"
        "v_mov_b32 v93, 0\n"
        "v_mov_b32 v94, 0\n"
        "v_mov_b32 v95, 0\n"
        "v_mov_b32 v96, 0\n"
        "v_mov_b32 v97, 0\n"
        "v_mov_b32 v98, 0\n"
        "v_mov_b32 v99, 0\n"
        "v_mov_b32 v100, 0\n"
        "v_mov_b32 v101, 0\n"
        "v_mov_b32 v102, 0\n"
        "v_mov_b32 v103, 0\n"
        "v_mov_b32 v104, 0\n"
        "v_mov_b32 v105, 0\n"
        "v_mov_b32 v106, 0\n"
        "v_mov_b32 v107, 0\n"
        "v_mov_b32 v108, 0\n"
        "v_mov_b32 v109, 0\n"
        "v_mov_b32 v110, 0\n"
        "v_mov_b32 v111, 0\n"
        "global_load_dwordx4 v[0:3], %[p], off\n"
        "global_load_dwordx4 v[4:7], %[p], off offset:16\n"
        "ds_read_b128 v[16:19], %[la] offset:0\n"
        "ds_read_b128 v[20:23], %[la] offset:16\n"
        "ds_read_b128 v[24:27], %[la] offset:32\n"
        "ds_read_b128 v[28:31], %[la] offset:48\n"
        "s_mov_b32 s40, %[it]\n"
        "1:\n"
        "global_load_dwordx4 v[8:11], %[p], off\n"
        "global_load_dwordx4 v[12:15], %[p], off offset:16\n"
        "ds_read_b128 v[32:35], %[la] offset:0\n"
        "ds_read_b128 v[36:39], %[la] offset:16\n"
        "ds_read_b128 v[40:43], %[la] offset:32\n"
        "ds_read_b128 v[44:47], %[la] offset:48\n"
        "s_waitcnt vmcnt(2) lgkmcnt(4)\n"
        "v_add_f64 v[64:65], v[16:17], v[0:1]\n"
        "v_add_f64 v[66:67], v[16:17], v[2:3]\n"
        "v_add_f64 v[68:69], v[16:17], v[4:5]\n"
        "v_add_f64 v[70:71], v[16:17], v[6:7]\n"
        "v_add_f64 v[72:73], v[18:19], v[0:1]\n"
        "v_add_f64 v[74:75], v[18:19], v[2:3]\n"
        "v_add_f64 v[76:77], v[18:19], v[4:5]\n"
        "v_add_f64 v[78:79], v[18:19], v[6:7]\n"
        "v_max_f64 v[80:81], v[80:81], v[64:65]\n"
        "v_max_f64 v[82:83], v[82:83], v[66:67]\n"
        "v_max_f64 v[84:85], v[84:85], v[68:69]\n"
        "v_max_f64 v[86:87], v[86:87], v[70:71]\n"
        "v_max_f64 v[88:89], v[88:89], v[72:73]\n"
        "v_max_f64 v[90:91], v[90:91], v[74:75]\n"
        "v_max_f64 v[92:93], v[92:93], v[76:77]\n"
        "v_max_f64 v[94:95], v[94:95], v[78:79]\n"
        "v_add_f64 v[64:65], v[20:21], v[0:1]\n"
        "v_add_f64 v[66:67], v[20:21], v[2:3]\n"
        "v_add_f64 v[68:69], v[20:21], v[4:5]\n"
        "v_add_f64 v[70:71], v[20:21], v[6:7]\n"
        "v_add_f64 v[72:73], v[22:23], v[0:1]\n"
        "v_add_f64 v[74:75], v[22:23], v[2:3]\n"
        "v_add_f64 v[76:77], v[22:23], v[4:5]\n"
        "v_add_f64 v[78:79], v[22:23], v[6:7]\n"
        "v_max_f64 v[96:97], v[96:97], v[64:65]\n"
        "v_max_f64 v[98:99], v[98:99], v[66:67]\n"
        "v_max_f64 v[100:101], v[100:101], v[68:69]\n"
        "v_max_f64 v[102:103], v[102:103], v[70:71]\n"
        "v_max_f64 v[104:105], v[104:105], v[72:73]\n"
        "v_max_f64 v[106:107], v[106:107], v[74:75]\n"
        "v_max_f64 v[108:109], v[108:109], v[76:77]\n"
        "v_max_f64 v[110:111], v[110:111], v[78:79]\n"
        "v_add_f64 v[64:65], v[24:25], v[0:1]\n"
        "v_add_f64 v[66:67], v[24:25], v[2:3]\n"
        "v_add_f64 v[68:69], v[24:25], v[4:5]\n"
        "v_add_f64 v[70:71], v[24:25], v[6:7]\n"
        "v_add_f64 v[72:73], v[26:27], v[0:1]\n"
        "v_add_f64 v[74:75], v[26:27], v[2:3]\n"
        "v_add_f64 v[76:77], v[26:27], v[4:5]\n"
        "v_add_f64 v[78:79], v[26:27], v[6:7]\n"
        "v_max_f64 v[112:113], v[112:113], v[64:65]\n"
        "v_max_f64 v[114:115], v[114:115], v[66:67]\n"
        "v_max_f64 v[116:117], v[116:117], v[68:69]\n"
        "v_max_f64 v[118:119], v[118:119], v[70:71]\n"
        "v_max_f64 v[120:121], v[120:121], v[72:73]\n"
        "v_max_f64 v[122:123], v[122:123], v[74:75]\n"
        "v_max_f64 v[124:125], v[124:125], v[76:77]\n"
        "v_max_f64 v[126:127], v[126:127], v[78:79]\n"
        "v_add_f64 v[64:65], v[28:29], v[0:1]\n"
        "v_add_f64 v[66:67], v[28:29], v[2:3]\n"
        "v_add_f64 v[68:69], v[28:29], v[4:5]\n"
        "v_add_f64 v[70:71], v[28:29], v[6:7]\n"
        "v_add_f64 v[72:73], v[30:31], v[0:1]\n"
        "v_add_f64 v[74:75], v[30:31], v[2:3]\n"
        "v_add_f64 v[76:77], v[30:31], v[4:5]\n"
        "v_add_f64 v[78:79], v[30:31], v[6:7]\n"
        "v_max_f64 v[128:129], v[128:129], v[64:65]\n"
        "v_max_f64 v[130:131], v[130:131], v[66:67]\n"
        "v_max_f64 v[132:133], v[132:133], v[68:69]\n"
        "v_max_f64 v[134:135], v[134:135], v[70:71]\n"
        "v_max_f64 v[136:137], v[136:137], v[72:73]\n"
        "v_max_f64 v[138:139], v[138:139], v[74:75]\n"
        "v_max_f64 v[140:141], v[140:141], v[76:77]\n"
        "v_max_f64 v[142:143], v[142:143], v[78:79]\n"
        "global_load_dwordx4 v[0:3], %[p], off\n"
        "global_load_dwordx4 v[4:7], %[p], off offset:16\n"
        "ds_read_b128 v[16:19], %[la] offset:0\n"
        "ds_read_b128 v[20:23], %[la] offset:16\n"
        "ds_read_b128 v[24:27], %[la] offset:32\n"
        "ds_read_b128 v[28:31], %[la] offset:48\n"
        "s_waitcnt vmcnt(2) lgkmcnt(4)\n"
        "v_add_f64 v[64:65], v[32:33], v[8:9]\n"
        "v_add_f64 v[66:67], v[32:33], v[10:11]\n"
        "v_add_f64 v[68:69], v[32:33], v[12:13]\n"
        "v_add_f64 v[70:71], v[32:33], v[14:15]\n"
        "v_add_f64 v[72:73], v[34:35], v[8:9]\n"
        "v_add_f64 v[74:75], v[34:35], v[10:11]\n"
        "v_add_f64 v[76:77], v[34:35], v[12:13]\n"
        "v_add_f64 v[78:79], v[34:35], v[14:15]\n"
        "v_max_f64 v[80:81], v[80:81], v[64:65]\n"
        "v_max_f64 v[82:83], v[82:83], v[66:67]\n"
        "v_max_f64 v[84:85], v[84:85], v[68:69]\n"
        "v_max_f64 v[86:87], v[86:87], v[70:71]\n"
        "v_max_f64 v[88:89], v[88:89], v[72:73]\n"
        "v_max_f64 v[90:91], v[90:91], v[74:75]\n"
        "v_max_f64 v[92:93], v[92:93], v[76:77]\n"
        "v_max_f64 v[94:95], v[94:95], v[78:79]\n"
        "v_add_f64 v[64:65], v[36:37], v[8:9]\n"
        "v_add_f64 v[66:67], v[36:37], v[10:11]\n"
        "v_add_f64 v[68:69], v[36:37], v[12:13]\n"
        "v_add_f64 v[70:71], v[36:37], v[14:15]\n"
        "v_add_f64 v[72:73], v[38:39], v[8:9]\n"
        "v_add_f64 v[74:75], v[38:39], v[10:11]\n"
        "v_add_f64 v[76:77], v[38:39], v[12:13]\n"
        "v_add_f64 v[78:79], v[38:39], v[14:15]\n"
        "v_max_f64 v[96:97], v[96:97], v[64:65]\n"
        "v_max_f64 v[98:99], v[98:99], v[66:67]\n"
        "v_max_f64 v[100:101], v[100:101], v[68:69]\n"
        "v_max_f64 v[102:103], v[102:103], v[70:71]\n"
        "v_max_f64 v[104:105], v[104:105], v[72:73]\n"
        "v_max_f64 v[106:107], v[106:107], v[74:75]\n"
        "v_max_f64 v[108:109], v[108:109], v[76:77]\n"
        "v_max_f64 v[110:111], v[110:111], v[78:79]\n"
        "v_add_f64 v[64:65], v[40:41], v[8:9]\n"
        "v_add_f64 v[66:67], v[40:41], v[10:11]\n"
        "v_add_f64 v[68:69], v[40:41], v[12:13]\n"
        "v_add_f64 v[70:71], v[40:41], v[14:15]\n"
        "v_add_f64 v[72:73], v[42:43], v[8:9]\n"
        "v_add_f64 v[74:75], v[42:43], v[10:11]\n"
        "v_add_f64 v[76:77], v[42:43], v[12:13]\n"
        "v_add_f64 v[78:79], v[42:43], v[14:15]\n"
        "v_max_f64 v[112:113], v[112:113], v[64:65]\n"
        "v_max_f64 v[114:115], v[114:115], v[66:67]\n"
        "v_max_f64 v[116:117], v[116:117], v[68:69]\n"
        "v_max_f64 v[118:119], v[118:119], v[70:71]\n"
        "v_max_f64 v[120:121], v[120:121], v[72:73]\n"
        "v_max_f64 v[122:123], v[122:123], v[74:75]\n"
        "v_max_f64 v[124:125], v[124:125], v[76:77]\n"
        "v_max_f64 v[126:127], v[126:127], v[78:79]\n"
        "v_add_f64 v[64:65], v[44:45], v[8:9]\n"
        "v_add_f64 v[66:67], v[44:45], v[10:11]\n"
        "v_add_f64 v[68:69], v[44:45], v[12:13]\n"
        "v_add_f64 v[70:71], v[44:45], v[14:15]\n"
        "v_add_f64 v[72:73], v[46:47], v[8:9]\n"
        "v_add_f64 v[74:75], v[46:47], v[10:11]\n"
        "v_add_f64 v[76:77], v[46:47], v[12:13]\n"
        "v_add_f64 v[78:79], v[46:47], v[14:15]\n"
        "v_max_f64 v[128:129], v[128:129], v[64:65]\n"
        "v_max_f64 v[130:131], v[130:131], v[66:67]\n"
        "v_max_f64 v[132:133], v[132:133], v[68:69]\n"
        "v_max_f64 v[134:135], v[134:135], v[70:71]\n"
        "v_max_f64 v[136:137], v[136:137], v[72:73]\n"
        "v_max_f64 v[138:139], v[138:139], v[74:75]\n"
        "v_max_f64 v[140:141], v[140:141], v[76:77]\n"
        "v_max_f64 v[142:143], v[142:143], v[78:79]\n"
        "s_sub_u32 s40, s40, 1\n"
        "s_cmp_lg_u32 s40, 0\n"
        "s_cbranch_scc1 1b\n"
        "s_waitcnt vmcnt(0) lgkmcnt(0)\n"
        :
        : [it] "s"(iters), [p] "v"(p), [la] "v"(la)
        : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "s40", "scc", "memory");
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  (void)sink;
  if ((tid & 63) == 0) {
    Stamp x{c0, c1, r0, r1, hw, xc};
    st[(size_t)blockIdx.x * (blockDim.x >> 6) + (tid >> 6)] = x;
  }
}

struct Result {
  double simd_pairs_per_clk;   // per SIMD: pairs / (last end - first start), median over SIMDs
  double wave_pairs_per_clk;   // per wave span (the round-5 method), summed over a SIMD's waves, median
  double clock_ghz;            // median d(memtime)/d(memrealtime) x 100 MHz
  double event_pairs_per_s;    // kernel-wide: pairs / HIP-event time
  int nsimd;
};

template <int KIND>
int run(int cus, int w, int iters, double* sink, Stamp* st, const double* arow, Result* out) {
  const int threads = 256 * w, blocks = cus;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // >= 2 s of back-to-back launches first, so the clock settles under this load
  const auto warm_start = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - warm_start).count() < 2.0) {
    for (int r = 0; r < 4; ++r) roof_k<KIND><<<blocks, threads>>>(sink, st, arow, iters, 1.0);
    CHECK(hipDeviceSynchronize());
  }
  CHECK(hipEventRecord(e0));
  roof_k<KIND><<<blocks, threads>>>(sink, st, arow, iters, 1.0);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = blocks * threads / 64;
  std::vector<Stamp> h(nw);
  CHECK(hipMemcpy(h.data(), st, nw * sizeof(Stamp), hipMemcpyDeviceToHost));
  const double pairs_per_wave = 64.0 * 64.0 * iters;  // 64 lanes x 64 pairs per iteration
  // SIMD key: XCC, SE, SH, CU, SIMD
  std::map<unsigned, std::vector<const Stamp*>> by;
  for (const Stamp& s : h) {
    const unsigned key = ((((s.xcc & 15) * 8 + ((s.hw >> 13) & 7)) * 2 + ((s.hw >> 12) & 1)) * 16 + ((s.hw >> 8) & 15)) * 4 +
                         ((s.hw >> 4) & 3);
    by[key].push_back(&s);
  }
  std::vector<double> simd_rate, wave_rate, clk;
  for (auto& kv : by) {
    unsigned long long cmin = ~0ull, cmax = 0, rmin = ~0ull, rmax = 0;
    double wr = 0;
    for (const Stamp* s : kv.second) {
      cmin = std::min(cmin, s->c0);
      cmax = std::max(cmax, s->c1);
      rmin = std::min(rmin, s->r0);
      rmax = std::max(rmax, s->r1);
      wr += pairs_per_wave / (double)(s->c1 - s->c0);
    }
    simd_rate.push_back(pairs_per_wave * kv.second.size() / (double)(cmax - cmin));
    wave_rate.push_back(wr);
    clk.push_back((double)(cmax - cmin) / (double)(rmax - rmin) * 0.1);
  }
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  out->simd_pairs_per_clk = med(simd_rate);
  out->wave_pairs_per_clk = med(wave_rate);
  out->clock_ghz = med(clk);
  out->event_pairs_per_s = pairs_per_wave * nw / (ms * 1e-3);
  out->nsimd = (int)by.size();
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 1;
  const int cus = p.multiProcessorCount;
  printf("device %s CUs %d\n", p.gcnArchName, cus);
  double *sink, *arow;
  Stamp* st;
  CHECK(hipMalloc(&sink, sizeof(double) * 1024));
  CHECK(hipMalloc(&arow, sizeof(double) * 256));
  CHECK(hipMemset(arow, 0, sizeof(double) * 256));
  CHECK(hipMalloc(&st, sizeof(Stamp) * 16 * cus));
  const char* names[] = {"pairs", "fwd-mix"};
  printf("%-8s %2s %12s %12s %9s %14s %14s %9s\n", "mix", "W", "SIMDspan/clk", "waveSum/clk", "clk GHz",
         "event pairs/s", "pairs/s@clk", "of 8/clk");
  for (int kind = 0; kind < 2; ++kind) {
    for (int w = 1; w <= 4; ++w) {
      // ~30 ms per launch at the expected rate
      const int iters = 40000 / w;
      Result r{};
      int rc = kind == 0 ? run<0>(cus, w, iters, sink, st, arow, &r) : run<1>(cus, w, iters, sink, st, arow, &r);
      if (rc) return rc;
      const double simds = 4.0 * cus;
      printf("%-8s %2d %12.3f %12.3f %9.3f %14.4e %14.4e %9.3f\n", names[kind], w, r.simd_pairs_per_clk,
             r.wave_pairs_per_clk, r.clock_ghz, r.event_pairs_per_s, r.simd_pairs_per_clk * simds * r.clock_ghz * 1e9,
             r.simd_pairs_per_clk / 8.0);
      fflush(stdout);
    }
  }
  printf("nominal: 8 lane-pairs/clk/SIMD (one wave64 f64 instruction per 4 clocks, 2 per pair) = %.4e pairs/s at 2.4 GHz\n",
         8.0 * 4 * cus * 2.4e9);
  return 0;
}
