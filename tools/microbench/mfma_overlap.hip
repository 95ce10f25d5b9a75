// Does v_mfma_f32_32x32x2_f32 overlap with VALU max3 work on gfx950?  Each wave runs ITER
// iterations of: MT independent MFMAs (D_k = fma(d, 1, A_k)) and NV v_max3_f32 folds of
// register data.  Times are per (wave-iteration) in SIMD clocks, for 1, 2 and 4 waves/SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_overlap mfma_overlap.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MT, int NV, bool USE_D, bool PRE = false>
__global__ void k(float* out, int iters, float seed) {
  f32x16 A[6];  // chained: A_k <- fma(d, 1, A_k) each iteration (keeps every MFMA live)
  for (int t = 0; t < 6; ++t)
    for (int r = 0; r < 16; ++r) A[t][r] = seed * (t * 16 + r + threadIdx.x);
  float X[16];
  for (int i = 0; i < 16; ++i) X[i] = seed * (i + threadIdx.x);
  float acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = seed * i;
  float d = seed * threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < MT && !PRE; ++t) A[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(d, 1.0f, A[t], 0, 0, 0);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int t = v / 8, r = (v % 8) * 2;
      float x = USE_D && t < MT ? A[t][r] : X[(2 * v) & 15];
      float y = USE_D && t < MT ? A[t][r + 1] : X[(2 * v + 1) & 15];
      acc[v & 7] = fmaxf(fmaxf(acc[v & 7], x), y);
      if (PRE && v % 8 == 7 && v / 8 < MT)  // D_t (previous iteration) folded: reissue MFMA t
        A[v / 8] = __builtin_amdgcn_mfma_f32_32x32x2f32(d, 1.0f, A[v / 8], 0, 0, 0);
    }
    d = d + acc[0] * 1e-30f;
    X[0] += acc[3] * 1e-30f;
    __builtin_amdgcn_sched_barrier(0);
  }
  float s = d;
  for (int i = 0; i < 8; ++i) s += acc[i];
  for (int t = 0; t < MT; ++t) s += A[t][threadIdx.x & 15];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int MT, int NV, bool USE_D, bool PRE = false>
void run(const char* name, float* out) {
  const int iters = 2000;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const double clk = p.clockRate * 1e3;
  for (int wps : {1, 2, 4}) {
    const int blocks = p.multiProcessorCount;
    const int threads = 64 * 4 * wps;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    k<MT, NV, USE_D, PRE><<<blocks, threads>>>(out, 10, 1.0f);
    hipEventRecord(a);
    k<MT, NV, USE_D, PRE><<<blocks, threads>>>(out, iters, 1.0f);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double cyc = ms * 1e-3 * clk / iters;  // SIMD clocks per iteration (all waves of a SIMD)
    printf("%-28s waves/SIMD %d  %8.1f clk/iter/SIMD  %7.1f per wave-iter\n", name, wps, cyc, cyc / wps);
  }
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096 * 4);
  run<6, 0, false>("mfma6", out);
  run<0, 48, false>("max3x48 (no mfma)", out);
  run<6, 48, false>("mfma6 + max3x48 indep", out);
  run<6, 48, true>("mfma6 + max3x48 on D", out);
  run<4, 48, true>("mfma4 + max3x48 (32 on D)", out);
  run<2, 48, false>("mfma2 + max3x48 indep", out);
  run<6, 48, true, true>("mfma6 interleaved, D(prev)", out);
  run<4, 64, true, true>("mfma4 interleaved + 32 max3", out);
  return 0;
}
