// Which SIMD does each wave of a multi-wave workgroup land on?  Launches G workgroups of W
// waves (LDS sized so one workgroup fits per CU when LDSKB is large) and prints, per wave
// index within the workgroup, the histogram of SIMD ids relative to wave 0's SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(unsigned* out, int lds_dummy) {
  extern __shared__ int lds[];
  if (threadIdx.x == 0) lds[0] = lds_dummy;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    out[2 * w] = hw;
    out[2 * w + 1] = xc;
  }
  // keep the waves resident for a while so workgroups overlap
  for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(10);
}

int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 8, G = argc > 2 ? atoi(argv[2]) : 256, ldskb = argc > 3 ? atoi(argv[3]) : 100;
  unsigned* d;
  hipMalloc(&d, sizeof(unsigned) * 2 * W * G);
  hipLaunchKernelGGL(probe, dim3(G), dim3(64 * W), ldskb * 1024, 0, d, 1);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<unsigned> h(2 * W * G);
  hipMemcpy(h.data(), d, sizeof(unsigned) * h.size(), hipMemcpyDeviceToHost);
  std::vector<int> hist(W * 4, 0);
  int same_cu = 0;
  for (int g = 0; g < G; ++g) {
    const unsigned h0 = h[2 * (g * W)];
    const int s0 = (h0 >> 4) & 3;
    for (int w = 0; w < W; ++w) {
      const unsigned hw = h[2 * (g * W + w)];
      hist[w * 4 + ((((hw >> 4) & 3) - s0) & 3)]++;
      same_cu += ((hw >> 8) & 0xff1f) == ((h0 >> 8) & 0xff1f);
    }
  }
  printf("W=%d G=%d LDS=%d KiB: waves on the same CU as wave 0: %d of %d\n", W, G, ldskb, same_cu, W * G);
  for (int w = 0; w < W; ++w)
    printf("wave %d: SIMD offset from wave 0 histogram [%d %d %d %d]\n", w, hist[w * 4], hist[w * 4 + 1], hist[w * 4 + 2], hist[w * 4 + 3]);
  return 0;
}
