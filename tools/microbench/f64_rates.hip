// Microbenchmark: gfx950 issue rates of the f64 VALU forms an exact-f64 max-plus trellis
// uses (v_add_f64, v_max_f64, and the add -> max pair of the inner loop), 1..4 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
#define REP4(X) X X X X

template <int KIND>
__global__ __launch_bounds__(1024) void k(double* out, double seed) {
  double a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
         a6 = a0 + 6, a7 = a0 + 7, b = seed * 0.5;
  double t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (KIND == 0) {  // 8 independent v_add_f64
      REP4(asm volatile("v_add_f64 %0, %1, %0\n v_add_f64 %2, %1, %2\n v_add_f64 %3, %1, %3\n v_add_f64 %4, %1, %4\n v_add_f64 %5, %1, %5\n v_add_f64 %6, %1, %6\n v_add_f64 %7, %1, %7\n v_add_f64 %8, %1, %8" : "+v"(a0), "+v"(b), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 1) {  // 8 independent v_max_f64
      REP4(asm volatile("v_max_f64 %0, %1, %0\n v_max_f64 %2, %1, %2\n v_max_f64 %3, %1, %3\n v_max_f64 %4, %1, %4\n v_max_f64 %5, %1, %5\n v_max_f64 %6, %1, %6\n v_max_f64 %7, %1, %7\n v_max_f64 %8, %1, %8" : "+v"(a0), "+v"(b), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 2) {  // inner loop: t = d + a; acc = max(acc, t), 4 chains
      REP4(asm volatile("v_add_f64 %4, %8, %9\n v_add_f64 %5, %8, %10\n v_add_f64 %6, %8, %11\n v_add_f64 %7, %8, %12\n v_max_f64 %0, %0, %4\n v_max_f64 %1, %1, %5\n v_max_f64 %2, %2, %6\n v_max_f64 %3, %3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3) : "v"(b), "v"(a4), "v"(a5), "v"(a6), "v"(a7));)
    } else if constexpr (KIND == 3) {  // same with the delta operand an SGPR pair
      double s = __builtin_amdgcn_readfirstlane((int)it) * 1.0;
      REP4(asm volatile("v_add_f64 %4, %8, %9\n v_add_f64 %5, %8, %10\n v_add_f64 %6, %8, %11\n v_add_f64 %7, %8, %12\n v_max_f64 %0, %0, %4\n v_max_f64 %1, %1, %5\n v_max_f64 %2, %2, %6\n v_max_f64 %3, %3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3) : "s"(s), "v"(a4), "v"(a5), "v"(a6), "v"(a7));)
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b + t0 + t1 + t2 + t3;
}

template <int KIND>
double run(double* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<KIND><<<blocks, threads>>>(d, 1.0);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<KIND><<<blocks, threads>>>(d, 1.0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double waveinstr = 5.0 * blocks * (threads / 64) * (double)ITERS * 32;
  return waveinstr * 64 / (ms * 1e-3);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  double* d;
  hipMalloc(&d, sizeof(double) * 1024 * cus * 4);
  const char* names[] = {"v_add_f64", "v_max_f64", "add+max (v)", "add+max (s delta)"};
  for (int wps : {1, 2, 4}) {
    int threads = 256 * wps, blocks = cus;
    double r[4] = {run<0>(d, blocks, threads), run<1>(d, blocks, threads), run<2>(d, blocks, threads),
                   run<3>(d, blocks, threads)};
    for (int i = 0; i < 4; ++i)
      printf("waves/SIMD %d %-20s %.3e lane-instr/s (%.2f lane-instr/clk/CU @2.4GHz)\n", wps, names[i], r[i],
             r[i] / cus / 2.4e9);
  }
  return 0;
}
