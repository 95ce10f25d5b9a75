// Checks the wave-level max helpers of trellis.hip (octet_max, swap_max, wave_max) on random
// data with -inf entries against a CPU reduction.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__device__ __forceinline__ float octet_max(float x) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf"
      : "+v"(x));
  return x;
}
__device__ __forceinline__ float swap_max(float x, bool sixteen) {
  // a = vdst, b = src, both = x.  After the swap a holds the low half's values (row pair)
  // in both halves and b the high half's, so max(a, b) = max(x[l], x[l^16|32]) in every lane.
  float a = x, b = x;
  if (sixteen)
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  else
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return fmaxf(a, b);
}
__device__ __forceinline__ float swap_pair_only(float x, bool sixteen) {  // the round-1 form
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = sixteen ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                         : __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, r[0]), __builtin_bit_cast(float, r[1]));
}
__device__ __forceinline__ float wave_max(float x) {
  x = octet_max(x);
  asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(x));
  x = swap_max(x, true);
  return swap_max(x, false);
}

__global__ void k(const float* in, float* out) {
  const int l = threadIdx.x & 63;
  const float x = in[blockIdx.x * 64 + l];
  float* o = out + (size_t)blockIdx.x * 64 * 5;
  o[l] = octet_max(x);
  o[64 + l] = swap_max(x, true);
  o[128 + l] = swap_max(x, false);
  o[192 + l] = wave_max(x);
  o[256 + l] = swap_pair_only(x, true);
}

int main() {
  const int W = 4096;
  std::vector<float> in(W * 64), out(W * 64 * 5);
  std::mt19937 g(1);
  std::uniform_real_distribution<float> u(-100.f, 0.f);
  for (auto& v : in) v = (g() % 7 == 0) ? -INFINITY : u(g);
  float *din, *dout;
  hipMalloc(&din, in.size() * 4);
  hipMalloc(&dout, out.size() * 4);
  hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice);
  k<<<W, 64>>>(din, dout);
  hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  long bad[5] = {0, 0, 0, 0, 0};
  for (int w = 0; w < W; ++w) {
    const float* x = &in[w * 64];
    const float* o = &out[(size_t)w * 64 * 5];
    float wm = -INFINITY;
    for (int l = 0; l < 64; ++l) wm = std::fmax(wm, x[l]);
    for (int l = 0; l < 64; ++l) {
      float om = -INFINITY;
      for (int q = (l & ~7); q < (l & ~7) + 8; ++q) om = std::fmax(om, x[q]);
      bad[0] += o[l] != om;
      bad[1] += o[64 + l] != std::fmax(x[l], x[l ^ 16]);
      bad[2] += o[128 + l] != std::fmax(x[l], x[l ^ 32]);
      bad[3] += o[192 + l] != wm;
      bad[4] += o[256 + l] != std::fmax(x[l], x[l ^ 16]);
    }
  }
  printf("mismatches: octet %ld swap16 %ld swap32 %ld wave %ld swap16_pair_only %ld (of %d lanes)\n", bad[0], bad[1],
         bad[2], bad[3], bad[4], W * 64);
  return (bad[0] || bad[1] || bad[2] || bad[3]) ? 1 : 0;
}
