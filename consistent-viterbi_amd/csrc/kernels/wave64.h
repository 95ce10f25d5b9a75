// wave64.h -- wave-level f64 helpers shared by the f64 trellis and chain kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvk {

// f64 -> its high / low 32-bit words (the hi word alone is the value with the mantissa
// truncated to 20 bits: same sign and exponent, |d - hi| < |hi| * 2^-20)
__device__ __forceinline__ uint32_t hi_word(double d) { return (uint32_t)(__builtin_bit_cast(uint64_t, d) >> 32); }
__device__ __forceinline__ uint32_t lo_word(double d) { return (uint32_t)__builtin_bit_cast(uint64_t, d); }
__device__ __forceinline__ double from_words(uint32_t hi, uint32_t lo) {
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// The same DPP pattern for f64 (both 32-bit halves move with one control, so a lane always
// pairs the words of one source lane); the result is uniform (lane 63's, read back).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double max_dpp_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = (int)(uint32_t)u, hi = (int)(uint32_t)(u >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWMASK, 0xF, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWMASK, 0xF, false);
  return fmax(v, from_words((uint32_t)ohi, (uint32_t)olo));
}
__device__ __forceinline__ double wave_max_d_dpp(double v) {
  v = max_dpp_d<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = max_dpp_d<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = max_dpp_d<0x141, 0xF>(v);  // row_half_mirror
  v = max_dpp_d<0x140, 0xF>(v);  // row_mirror
  v = max_dpp_d<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v = max_dpp_d<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  return from_words((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), 63),
                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, 63));
}

}  // namespace cvk
