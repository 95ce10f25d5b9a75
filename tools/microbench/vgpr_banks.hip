// Microbenchmark: does VGPR bank placement change the issue rate of the f64 trellis inner
// loop (v_add_f64 x, d, a ; v_max_f64 acc, acc, x)?  Core cycles per VALU instruction per
// SIMD (s_memtime), 1..4 waves per SIMD, three register placements of the same 64-instruction
// row (4 columns x 8 sequences, adds of a sequence pair issued before their maxima):
//   SAME  d, a, x, acc all at register indices = 0 mod 4 (operands share banks)
//   SPLIT d at = 0 mod 4, a at = 2 mod 4; x at = 2 mod 4, acc at = 0 mod 4
//   MIXED the compiler's kind of placement (consecutive pairs)
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITERS 4096

template <int KIND>
__global__ __launch_bounds__(256) void k(unsigned long long* cyc, double seed) {
  // registers are named explicitly and clobbered: v0..v127
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (KIND == 0) {
      // SAME: d = v[0:1] / v[4:5]; a = v[8:9],v[12:13],v[16:17],v[20:21]; x = v[24..]; acc = v[56..]
      asm volatile(
          ".rept 4\n"
          "v_add_f64 v[24:25], v[0:1], v[8:9]\n v_add_f64 v[28:29], v[0:1], v[12:13]\n"
          "v_add_f64 v[32:33], v[0:1], v[16:17]\n v_add_f64 v[36:37], v[0:1], v[20:21]\n"
          "v_add_f64 v[40:41], v[4:5], v[8:9]\n v_add_f64 v[44:45], v[4:5], v[12:13]\n"
          "v_add_f64 v[48:49], v[4:5], v[16:17]\n v_add_f64 v[52:53], v[4:5], v[20:21]\n"
          "v_max_f64 v[56:57], v[56:57], v[24:25]\n v_max_f64 v[60:61], v[60:61], v[28:29]\n"
          "v_max_f64 v[64:65], v[64:65], v[32:33]\n v_max_f64 v[68:69], v[68:69], v[36:37]\n"
          "v_max_f64 v[72:73], v[72:73], v[40:41]\n v_max_f64 v[76:77], v[76:77], v[44:45]\n"
          "v_max_f64 v[80:81], v[80:81], v[48:49]\n v_max_f64 v[84:85], v[84:85], v[52:53]\n"
          ".endr\n" ::
              : "v0", "v1", "v4", "v5", "v8", "v9", "v12", "v13", "v16", "v17", "v20", "v21", "v24", "v25", "v28",
                "v29", "v32", "v33", "v36", "v37", "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56",
                "v57", "v60", "v61", "v64", "v65", "v68", "v69", "v72", "v73", "v76", "v77", "v80", "v81", "v84",
                "v85");
    } else if constexpr (KIND == 1) {
      // SPLIT: d = v[0:1] / v[4:5] (bank 0/1); a = v[10:11],v[14:15],v[18:19],v[22:23] (bank 2/3);
      // x = v[26..] (bank 2/3); acc = v[56..] (bank 0/1)
      asm volatile(
          ".rept 4\n"
          "v_add_f64 v[26:27], v[0:1], v[10:11]\n v_add_f64 v[30:31], v[0:1], v[14:15]\n"
          "v_add_f64 v[34:35], v[0:1], v[18:19]\n v_add_f64 v[38:39], v[0:1], v[22:23]\n"
          "v_add_f64 v[42:43], v[4:5], v[10:11]\n v_add_f64 v[46:47], v[4:5], v[14:15]\n"
          "v_add_f64 v[50:51], v[4:5], v[18:19]\n v_add_f64 v[54:55], v[4:5], v[22:23]\n"
          "v_max_f64 v[56:57], v[56:57], v[26:27]\n v_max_f64 v[60:61], v[60:61], v[30:31]\n"
          "v_max_f64 v[64:65], v[64:65], v[34:35]\n v_max_f64 v[68:69], v[68:69], v[38:39]\n"
          "v_max_f64 v[72:73], v[72:73], v[42:43]\n v_max_f64 v[76:77], v[76:77], v[46:47]\n"
          "v_max_f64 v[80:81], v[80:81], v[50:51]\n v_max_f64 v[84:85], v[84:85], v[54:55]\n"
          ".endr\n" ::
              : "v0", "v1", "v4", "v5", "v10", "v11", "v14", "v15", "v18", "v19", "v22", "v23", "v26", "v27",
                "v30", "v31", "v34", "v35", "v38", "v39", "v42", "v43", "v46", "v47", "v50", "v51", "v54", "v55",
                "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69", "v72", "v73", "v76", "v77", "v80", "v81",
                "v84", "v85");
    } else {
      // MIXED: consecutive pairs (d = v[0:1], v[2:3]; a = v[4..11]; x = v[12..27]; acc = v[28..43])
      asm volatile(
          ".rept 4\n"
          "v_add_f64 v[12:13], v[0:1], v[4:5]\n v_add_f64 v[14:15], v[0:1], v[6:7]\n"
          "v_add_f64 v[16:17], v[0:1], v[8:9]\n v_add_f64 v[18:19], v[0:1], v[10:11]\n"
          "v_add_f64 v[20:21], v[2:3], v[4:5]\n v_add_f64 v[22:23], v[2:3], v[6:7]\n"
          "v_add_f64 v[24:25], v[2:3], v[8:9]\n v_add_f64 v[26:27], v[2:3], v[10:11]\n"
          "v_max_f64 v[28:29], v[28:29], v[12:13]\n v_max_f64 v[30:31], v[30:31], v[14:15]\n"
          "v_max_f64 v[32:33], v[32:33], v[16:17]\n v_max_f64 v[34:35], v[34:35], v[18:19]\n"
          "v_max_f64 v[36:37], v[36:37], v[20:21]\n v_max_f64 v[38:39], v[38:39], v[22:23]\n"
          "v_max_f64 v[40:41], v[40:41], v[24:25]\n v_max_f64 v[42:43], v[42:43], v[26:27]\n"
          ".endr\n" ::
              : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14",
                "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28",
                "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42",
                "v43");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6))] = t1 - t0;
    cyc[2 * (blockIdx.x * 4 + (threadIdx.x >> 6)) + 1] = r1 - r0;  // 100 MHz ticks
  }
}

template <int KIND>
double run(unsigned long long* d, int cus, int wps) {
  // wps waves per SIMD: blocks of 256 threads (one wave per SIMD each), wps blocks per CU
  const int blocks = cus * wps;
  k<KIND><<<blocks, 256>>>(d, 1.0);
  hipDeviceSynchronize();
  k<KIND><<<blocks, 256>>>(d, 1.0);
  hipDeviceSynchronize();
  static unsigned long long h[4096 * 8];
  hipMemcpy(h, d, sizeof(unsigned long long) * blocks * 8, hipMemcpyDeviceToHost);
  double mean = 0, rt = 0;
  for (int i = 0; i < blocks * 4; ++i) mean += (double)h[2 * i], rt += (double)h[2 * i + 1];
  mean /= blocks * 4;
  rt /= blocks * 4;
  // instructions per wave: ITERS * 64; a SIMD runs wps waves over the same cycles
  printf("   (clock %.3f GHz from s_memtime / s_memrealtime at 100 MHz; wall per instr per SIMD %.3f ns) ",
         mean / (rt * 10.0), rt * 10.0 / ((double)ITERS * 64 * wps));
  return mean / ((double)ITERS * 64 * wps);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * 4096 * 8);
  const char* names[] = {"SAME (operands share banks)", "SPLIT (d/a and acc/x in different banks)",
                         "MIXED (consecutive pairs)"};
  for (int wps : {1, 2, 3, 4}) {
    const double r[3] = {run<0>(d, cus, wps), run<1>(d, cus, wps), run<2>(d, cus, wps)};
    for (int i = 0; i < 3; ++i)
      printf("waves/SIMD %d %-42s %.3f core cycles per f64 VALU instruction per SIMD\n", wps, names[i], r[i]);
  }
  return 0;
}
