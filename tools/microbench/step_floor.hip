// Per-step floor of a one-sequence-per-workgroup decode step at small batches (the parallel
// chain's speculative batch: ~620 sequences, N = 256, T = 512, measured at ~24 us per step
// whatever the candidate layout).  Each variant adds one piece of generic_fwd_ms<1>'s step:
//   0: two barriers + an LDS row write / read per step
//   1: + the step's observation (global) and its emission (dependent global load)
//   2: + the candidate walk: 256 A loads per thread (L2), add / compare / select
//   3: + the u16 psi store per state
//   4: variant 2's walk without the observation / emission loads
// Build: hipcc --offload-arch=gfx950 -O3 -o step_floor step_floor.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int N = 256, V = 1024, T = 512;

template <int VAR>
__global__ __launch_bounds__(256) void step_kernel(const double* __restrict__ a, const double* __restrict__ et,
                                                   const int* __restrict__ obs, unsigned short* psi, double* out) {
  __shared__ double row[2][N];
  const int j = threadIdx.x;
  const int64_t seq = blockIdx.x;
  row[0][j] = -1.0 * j;
  __syncthreads();
  double acc = 0.0;
  for (int t = 1; t < T; ++t) {
    const double* prow = row[(t - 1) & 1];
    double e = 0.0;
    if constexpr (VAR == 1 || VAR == 2 || VAR == 3) {
      const int o = obs[seq * T + t];
      e = et[(size_t)o * N + j];
    }
    double best = prow[0];
    int arg = 0;
    if constexpr (VAR >= 2) {
      const double* col = a + j;
#pragma unroll 8
      for (int i = 1; i < N; ++i) {
        const double x = prow[i] + col[(size_t)i * N];
        if (x > best) {
          best = x;
          arg = i;
        }
      }
    }
    __syncthreads();
    row[t & 1][j] = best + e;
    if constexpr (VAR == 3) psi[(seq * T + t) * N + j] = (unsigned short)arg;
    acc += (double)arg;
    __syncthreads();
  }
  out[seq * N + j] = row[(T - 1) & 1][j] + acc;
}

int main(int argc, char** argv) {
  const int nseq = argc > 1 ? atoi(argv[1]) : 620;
  std::vector<double> ha((size_t)N * N), het((size_t)V * N);
  for (size_t k = 0; k < ha.size(); ++k) ha[k] = -(double)((k * 2654435761u) % 1000) / 100.0;
  for (size_t k = 0; k < het.size(); ++k) het[k] = -(double)((k * 40503u) % 1000) / 100.0;
  std::vector<int> hobs((size_t)nseq * T);
  for (size_t k = 0; k < hobs.size(); ++k) hobs[k] = (int)((k * 2246822519u) % V);
  double *a, *et, *out;
  int* obs;
  unsigned short* psi;
  CK(hipMalloc(&a, ha.size() * 8));
  CK(hipMalloc(&et, het.size() * 8));
  CK(hipMalloc(&obs, hobs.size() * 4));
  CK(hipMalloc(&psi, (size_t)nseq * T * N * 2));
  CK(hipMalloc(&out, (size_t)nseq * N * 8));
  CK(hipMemcpy(a, ha.data(), ha.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(et, het.data(), het.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(obs, hobs.data(), hobs.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](auto kern, const char* name) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(kern, dim3(nseq), dim3(256), 0, 0, a, et, obs, psi, out);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;
    }
    printf("%-58s %8.3f ms  %6.2f us/step\n", name, best, best * 1e3 / (T - 1));
  };
  printf("nseq %d, N %d, T %d, 256 threads per workgroup\n", nseq, N, T);
  run(step_kernel<0>, "0 barriers + LDS row");
  run(step_kernel<1>, "1 + observation and emission loads");
  run(step_kernel<4>, "4 candidate walk only (256 A loads / thread)");
  run(step_kernel<2>, "2 + walk with observation / emission");
  run(step_kernel<3>, "3 + u16 psi store");
  return 0;
}
