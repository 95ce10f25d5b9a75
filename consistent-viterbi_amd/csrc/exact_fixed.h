// exact_fixed.h -- the exact accumulation unit of the constrained decode's terms, shared by
// the host (csp.cpp) and the device (kernels/exact.hip) so both add bit-identical integers.
// A finite term x (a log10 path score, f32 or f64) becomes v = nearbyint(x * 2^64) (round
// half to even), added into 4 base-2^32 limbs held in int64 words (limb 3 signed); -inf is
// counted instead.  Integer sums are order-free, so partial sums from any number of threads,
// blocks, shards or GPUs add up to the same words.
// Range: |x| < kTermMax = 2^32, so |v| < 2^96 and up to 2^31 terms sum without overflowing
// the 128-bit value the search reads back (csp.cpp limbs_value); a term outside it (a
// model whose log-probabilities are absurdly large, e.g. -1e30 written for "impossible"
// instead of null) is REJECTED by the caller (CV_EINVAL), never wrapped.
#pragma once
#include <stdint.h>
#include <string.h>

#if defined(__HIP__)
#define CVX_HD __host__ __device__
#else
#define CVX_HD
#endif

namespace cvx {

constexpr double kTermMax = 4294967296.0;  // 2^32

// finite and inside the exact unit's range (NaN never reaches here: rejected at cv_hmm_create)
CVX_HD inline bool term_in_range(double x) { return x > -kTermMax && x < kTermMax; }

// The 4 limbs of v (x finite).  Integer ops only: x = +-M * 2^(E-150), so x * 2^64 =
// +-M * 2^k with k = E - 86.
CVX_HD inline void fixed64_limbs(float x, int64_t (&l)[4]) {
  uint32_t b;
  memcpy(&b, &x, 4);
  const int E = (int)((b >> 23) & 0xFF);
  const uint64_t M = E ? ((b & 0x7FFFFFu) | 0x800000u) : (b & 0x7FFFFFu);
  const int k = (E ? E : 1) - 86;
  unsigned __int128 mag;
  if (k >= 0) {
    mag = (unsigned __int128)M << k;
  } else if (-k >= 25) {
    mag = 0;  // M * 2^k < 2^24 * 2^-25 = 1/2
  } else {
    const int s = -k;
    const uint64_t q = M >> s, r = M & ((1ull << s) - 1), half = 1ull << (s - 1);
    mag = q + ((r > half || (r == half && (q & 1))) ? 1 : 0);
  }
  const __int128 v = (b >> 31) ? -(__int128)mag : (__int128)mag;
  const unsigned __int128 u = (unsigned __int128)v;
  l[0] = (int64_t)(uint32_t)u;
  l[1] = (int64_t)(uint32_t)(u >> 32);
  l[2] = (int64_t)(uint32_t)(u >> 64);
  l[3] = (int64_t)(v >> 96);
}

// The 4 limbs of v for a finite f64 x with |x| < 2^32: x = +-M * 2^(E-1075), so
// x * 2^64 = +-M * 2^k with k = E - 1011 (M < 2^53; k <= 42 inside the range).
CVX_HD inline void fixed64_limbs(double x, int64_t (&l)[4]) {
  uint64_t b;
  memcpy(&b, &x, 8);
  const int E = (int)((b >> 52) & 0x7FF);
  const uint64_t M = E ? ((b & 0xFFFFFFFFFFFFFull) | (1ull << 52)) : (b & 0xFFFFFFFFFFFFFull);
  const int k = (E ? E : 1) - 1011;
  unsigned __int128 mag;
  if (k >= 0) {
    mag = (unsigned __int128)M << k;
  } else if (-k >= 54) {
    mag = 0;  // M * 2^k < 2^53 * 2^-54 = 1/2
  } else {
    const int s = -k;
    const uint64_t q = M >> s, r = M & ((1ull << s) - 1), half = 1ull << (s - 1);
    mag = q + ((r > half || (r == half && (q & 1))) ? 1 : 0);
  }
  const __int128 v = (b >> 63) ? -(__int128)mag : (__int128)mag;
  const unsigned __int128 u = (unsigned __int128)v;
  l[0] = (int64_t)(uint32_t)u;
  l[1] = (int64_t)(uint32_t)(u >> 32);
  l[2] = (int64_t)(uint32_t)(u >> 64);
  l[3] = (int64_t)(v >> 96);
}

}  // namespace cvx
