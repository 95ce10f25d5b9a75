// Microbenchmark: gfx950 issue rates of the f32 max-plus instruction mix of trellis_fwd2_f32
// (per two (from, to) pairs: 2 v_add_f32 + 1 v_max3_f32) against VGPR bank placement, and of
// the alternatives (v_max_f32, v_pk_add_f32).  Core cycles per instruction per SIMD from
// s_memtime, at 1..4 waves per SIMD (the trellis runs 4: 16 waves of 104 VGPRs per CU).
// Registers are named explicitly (clobbered) so the bank (index mod 4) of every operand is known:
//   ADD     v_add_f32 x, d, a                   d, a, x in banks 0, 1, 2
//   MAX3_D  v_max3_f32 m, m, s0, s1              m, s0, s1 in banks 3, 0, 2 (distinct)
//   MAX3_S  v_max3_f32 m, m, s0, s1              m, s0, s1 all in bank 0
//   MAX2    v_max_f32 m, m, s0                   (VOP2)
//   MIX_D   the trellis mix (2 adds + 1 max3) with distinct banks
//   MIX_S   the same with the max3's operands in one bank
//   PK      v_pk_add_f32 (2 adds per lane) + v_max3_f32, distinct banks
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITERS 4096
#define CLOB ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15", \
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31", \
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63", \
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79", \
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95", \
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111", \
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127"

// 8 independent groups per block; group g uses registers v[16 g + ...]
template <int KIND>
__global__ __launch_bounds__(1024) void k(unsigned long long* cyc, float seed) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (KIND == 0) {  // ADD: x(bank2) = d(bank0) + a(bank1); 16 adds
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+2], v[\\g*16+0], v[\\g*16+1]\n"
          "v_add_f32 v[\\g*16+6], v[\\g*16+4], v[\\g*16+5]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 1) {  // MAX3_D: m(bank3) = max3(m, s0(bank0), s1(bank2)); 16
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_max3_f32 v[\\g*16+3], v[\\g*16+3], v[\\g*16+0], v[\\g*16+2]\n"
          "v_max3_f32 v[\\g*16+7], v[\\g*16+7], v[\\g*16+4], v[\\g*16+6]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 2) {  // MAX3_S: all three operands in bank 0
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_max3_f32 v[\\g*16+0], v[\\g*16+0], v[\\g*16+4], v[\\g*16+8]\n"
          "v_max3_f32 v[\\g*16+12], v[\\g*16+12], v[\\g*16+4], v[\\g*16+8]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 3) {  // MAX2: v_max_f32 m(bank3), m, s0(bank0)
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_max_f32 v[\\g*16+3], v[\\g*16+3], v[\\g*16+0]\n"
          "v_max_f32 v[\\g*16+7], v[\\g*16+7], v[\\g*16+4]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 4) {  // MIX_D: s0(b0) = d(b1) + a0(b2); s1(b2') = d + a1(b3); m(b3') = max3(m, s0, s1)
      // group regs: d=g+1, a0=g+2, a1=g+3, s0=g+4 (b0), s1=g+6 (b2), m=g+7 (b3)
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+4], v[\\g*16+1], v[\\g*16+2]\n"
          "v_add_f32 v[\\g*16+6], v[\\g*16+1], v[\\g*16+3]\n"
          "v_max3_f32 v[\\g*16+7], v[\\g*16+7], v[\\g*16+4], v[\\g*16+6]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 5) {  // MIX_S: the max3's operands all in bank 0 (s0 = g+4, s1 = g+8, m = g+12)
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+4], v[\\g*16+1], v[\\g*16+2]\n"
          "v_add_f32 v[\\g*16+8], v[\\g*16+1], v[\\g*16+3]\n"
          "v_max3_f32 v[\\g*16+12], v[\\g*16+12], v[\\g*16+4], v[\\g*16+8]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 6) {  // PK: v_pk_add_f32 s[4:5] = d[0:1] + a[2:3]; max3(m(7), s0(4), s1(5))
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_pk_add_f32 v[\\g*16+4:\\g*16+5], v[\\g*16+0:\\g*16+1], v[\\g*16+2:\\g*16+3]\n"
          "v_max3_f32 v[\\g*16+7], v[\\g*16+7], v[\\g*16+4], v[\\g*16+5]\n"
          ".endr" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15",
          "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31",
          "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47",
          "v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63",
          "v64","v65","v66","v67","v68","v69","v70","v71","v72","v73","v74","v75","v76","v77","v78","v79",
          "v80","v81","v82","v83","v84","v85","v86","v87","v88","v89","v90","v91","v92","v93","v94","v95",
          "v96","v97","v98","v99","v100","v101","v102","v103","v104","v105","v106","v107","v108","v109","v110","v111",
          "v112","v113","v114","v115","v116","v117","v118","v119","v120","v121","v122","v123","v124","v125","v126","v127");
    } else if constexpr (KIND == 7) {  // ADD_S: x(bank0) = d(bank0) + a(bank0); 16 adds
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+8], v[\\g*16+0], v[\\g*16+4]\n"
          "v_add_f32 v[\\g*16+12], v[\\g*16+0], v[\\g*16+4]\n"
          ".endr" CLOB);
    } else if constexpr (KIND == 8) {  // MIX_SS: the adds' sources in one bank (d = g+1, a0 = g+5, a1 = g+9)
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+4], v[\\g*16+1], v[\\g*16+5]\n"
          "v_add_f32 v[\\g*16+6], v[\\g*16+1], v[\\g*16+9]\n"
          "v_max3_f32 v[\\g*16+7], v[\\g*16+7], v[\\g*16+4], v[\\g*16+6]\n"
          ".endr" CLOB);
    } else if constexpr (KIND == 9) {  // DPP: v_max_f32_dpp (quad_perm), 16 independent
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_max_f32_dpp v[\\g*16+3], v[\\g*16+0], v[\\g*16+3] quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
          "v_max_f32_dpp v[\\g*16+7], v[\\g*16+4], v[\\g*16+7] quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
          ".endr" CLOB);
    } else if constexpr (KIND == 10) {  // ADD_S2: both sources in bank 0, no register reused by the next add
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+2], v[\\g*16+0], v[\\g*16+4]\n"
          "v_add_f32 v[\\g*16+6], v[\\g*16+8], v[\\g*16+12]\n"
          ".endr" CLOB);
    } else if constexpr (KIND == 11) {  // ADD_D2: sources in banks 0 / 1, no register reused by the next add
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+2], v[\\g*16+0], v[\\g*16+5]\n"
          "v_add_f32 v[\\g*16+6], v[\\g*16+8], v[\\g*16+13]\n"
          ".endr" CLOB);
    } else if constexpr (KIND == 12) {  // MIX_K: the kernel's rows4 shape -- one d (bank 0) into 2 adds with
                                        // distinct a's (banks 1, 2), two rows, then max3 of 2 sums per column
      asm volatile(
          ".irp g, 0,1,2,3,4,5,6,7\n"
          "v_add_f32 v[\\g*16+3], v[\\g*16+0], v[\\g*16+1]\n"
          "v_add_f32 v[\\g*16+7], v[\\g*16+0], v[\\g*16+2]\n"
          "v_add_f32 v[\\g*16+11], v[\\g*16+4], v[\\g*16+5]\n"
          "v_add_f32 v[\\g*16+15], v[\\g*16+4], v[\\g*16+6]\n"
          "v_max3_f32 v[\\g*16+8], v[\\g*16+8], v[\\g*16+3], v[\\g*16+11]\n"
          "v_max3_f32 v[\\g*16+9], v[\\g*16+9], v[\\g*16+7], v[\\g*16+15]\n"
          ".endr" CLOB);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
  (void)seed;
}

// instructions per iteration and the (from, to) pairs they cover per lane
constexpr int kInsts[] = {16, 16, 16, 16, 24, 24, 16, 16, 24, 16, 16, 16, 48};
constexpr int kPairs[] = {0, 0, 0, 0, 16, 16, 16, 0, 16, 0, 0, 0, 32};

template <int KIND>
void run(const char* name, int cus) {
  for (int wps : {1, 2, 4}) {
    const int threads = 256 * wps;
    unsigned long long* d;
    (void)hipMalloc(&d, sizeof(unsigned long long) * cus * 16);
    hipLaunchKernelGGL(k<KIND>, dim3(cus), dim3(threads), 0, 0, d, 1.0f);
    hipLaunchKernelGGL(k<KIND>, dim3(cus), dim3(threads), 0, 0, d, 1.0f);
    (void)hipDeviceSynchronize();
    unsigned long long h[16 * 1024];
    (void)hipMemcpy(h, d, sizeof(unsigned long long) * cus * (threads / 64), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < cus * (threads / 64); ++i) mx = h[i] > mx ? (double)h[i] : mx;
    // cycles per instruction per SIMD: all wps waves of a SIMD issue ITERS * kInsts each
    const double cpi = mx / ((double)ITERS * kInsts[KIND] * wps);
    printf("%-8s waves/SIMD %d: %.2f cyc per wave-instruction per SIMD (%.1f lanes/clk/SIMD)", name, wps, cpi, 64 / cpi);
    if (kPairs[KIND]) printf(", %.2f pairs/clk/SIMD", 64.0 * kPairs[KIND] / kInsts[KIND] / cpi);
    printf("\n");
    (void)hipFree(d);
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("device %s CUs %d\n", p.gcnArchName, cus);
  run<0>("ADD", cus);
  run<1>("MAX3_D", cus);
  run<2>("MAX3_S", cus);
  run<3>("MAX2", cus);
  run<4>("MIX_D", cus);
  run<5>("MIX_S", cus);
  run<6>("PK", cus);
  run<7>("ADD_S", cus);
  run<8>("MIX_SS", cus);
  run<9>("DPP", cus);
  run<10>("ADD_S2", cus);
  run<11>("ADD_D2", cus);
  run<12>("MIX_K", cus);
  return 0;
}
