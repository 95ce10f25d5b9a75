// Microbenchmark: issue rates of the VALU forms the max-plus trellis can use on gfx950.
// Each kernel runs a long unrolled stream of independent instructions; we report
// wave-instructions per CU per clock-equivalent (lane-ops/s) to pick the inner-loop form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define ITERS 4096

#define REP8(X) X X X X X X X X

template <int KIND>
__global__ __launch_bounds__(1024) void k(float* out, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7, b = seed * 0.5f;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (KIND == 0) {  // v_add_f32
      REP8(asm volatile("v_add_f32 %0, %1, %0\n v_add_f32 %2, %1, %2\n v_add_f32 %3, %1, %3\n v_add_f32 %4, %1, %4\n v_add_f32 %5, %1, %5\n v_add_f32 %6, %1, %6\n v_add_f32 %7, %1, %7\n v_add_f32 %8, %1, %8" : "+v"(a0), "+v"(b), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 1) {  // v_add_f32_dpp row_newbcast
      REP8(asm volatile("v_add_f32_dpp %0, %1, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %2, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %3, %1, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %4, %1, %4 row_newbcast:4 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %5, %1, %5 row_newbcast:5 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %6, %1, %6 row_newbcast:6 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %7, %1, %7 row_newbcast:7 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %8, %1, %8 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(a0), "+v"(b), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 2) {  // v_max3_f32
      REP8(asm volatile("v_max3_f32 %0, %1, %0, %2\n v_max3_f32 %2, %1, %2, %3\n v_max3_f32 %3, %1, %3, %4\n v_max3_f32 %4, %1, %4, %5\n v_max3_f32 %5, %1, %5, %6\n v_max3_f32 %6, %1, %6, %7\n v_max3_f32 %7, %1, %7, %8\n v_max3_f32 %8, %1, %8, %0" : "+v"(a0), "+v"(b), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    } else if constexpr (KIND == 3) {  // v_pk_add_f32 (2 adds per lane)
      using f2 = __attribute__((ext_vector_type(2))) float;
      f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, q = {b, b};
      REP8(asm volatile("v_pk_add_f32 %0, %4, %0\n v_pk_add_f32 %1, %4, %1\n v_pk_add_f32 %2, %4, %2\n v_pk_add_f32 %3, %4, %3\n v_pk_add_f32 %0, %4, %0\n v_pk_add_f32 %1, %4, %1\n v_pk_add_f32 %2, %4, %2\n v_pk_add_f32 %3, %4, %3" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(q));)
      a0 = p0.x + p1.y; a1 = p2.x + p3.y; a2 = p0.y; a3 = p1.x;
    } else if constexpr (KIND == 4) {  // mixed: 2 dpp adds + 1 max3 (the trellis inner loop)
      REP8(asm volatile("v_add_f32_dpp %2, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %3, %1, %3 row_newbcast:2 row_mask:0xf bank_mask:0xf\n v_max3_f32 %0, %0, %2, %3\n v_add_f32_dpp %4, %1, %4 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %5, %1, %5 row_newbcast:4 row_mask:0xf bank_mask:0xf\n v_max3_f32 %6, %6, %4, %5\n v_add_f32_dpp %7, %1, %7 row_newbcast:5 row_mask:0xf bank_mask:0xf\n v_add_f32_dpp %8, %1, %8 row_newbcast:6 row_mask:0xf bank_mask:0xf\n v_max3_f32 %0, %0, %7, %8" : "+v"(a0), "+v"(b), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b;
}

template <int KIND>
double run(float* d, int blocks, int threads, double instr_per_iter) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k<KIND><<<blocks, threads>>>(d, 1.0f);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) k<KIND><<<blocks, threads>>>(d, 1.0f);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double waveinstr = 5.0 * blocks * (threads / 64) * (double)ITERS * instr_per_iter;
  return waveinstr * 64 / (ms * 1e-3);  // lane-instr/s
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  float* d; hipMalloc(&d, sizeof(float) * 1024 * cus * 8);
  const char* names[] = {"v_add_f32", "v_add_f32_dpp(newbcast)", "v_max3_f32", "v_pk_add_f32", "mix 2dpp+1max3"};
  double ipi[] = {64, 64, 64, 64, 72};
  for (int wpb : {256, 512, 1024}) {
    for (int bpc : {1, 2, 4}) {
      if (wpb * bpc > 2048) continue;
      int blocks = cus * bpc;
      double r[5];
      r[0] = run<0>(d, blocks, wpb, ipi[0]);
      r[1] = run<1>(d, blocks, wpb, ipi[1]);
      r[2] = run<2>(d, blocks, wpb, ipi[2]);
      r[3] = run<3>(d, blocks, wpb, ipi[3]);
      r[4] = run<4>(d, blocks, wpb, ipi[4]);
      for (int i = 0; i < 5; ++i)
        printf("threads/block %4d blocks/CU %d %-26s %.3e lane-instr/s  (%.2f lane-instr/clk/CU @2.4GHz)\n", wpb, bpc,
               names[i], r[i], r[i] / cus / 2.4e9);
    }
  }
  return 0;
}
