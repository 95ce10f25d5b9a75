// Check: the integer-only add_exact (csp.cpp) equals the original double -> __int128 form
// bit for bit (strided sweep of all floats with |x| < 2^24, every exponent, 1e7 random
// log-prob-like values) and time both.  Build: g++ -O2 -o /tmp/ae add_exact_check.cpp
#include <chrono>
#include <vector>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
static void add_ref(int64_t* l, int64_t* ni, float x) {
  if (!(x > -INFINITY)) { *ni += 1; return; }
  const __int128 v = (__int128)std::nearbyint((double)x * 18446744073709551616.0);
  const unsigned __int128 u = (unsigned __int128)v;
  l[0] += (int64_t)(uint32_t)u; l[1] += (int64_t)(uint32_t)(u >> 32); l[2] += (int64_t)(uint32_t)(u >> 64); l[3] += (int64_t)(v >> 96);
}
static void add_new(int64_t* l, int64_t* ni, float x) {
  if (!(x > -INFINITY)) { *ni += 1; return; }
  uint32_t b; std::memcpy(&b, &x, 4);
  const int E = (int)((b >> 23) & 0xFF);
  const uint64_t M = E ? ((b & 0x7FFFFFu) | 0x800000u) : (b & 0x7FFFFFu);
  const int k = (E ? E : 1) - 86;  // x * 2^64 = M * 2^k
  unsigned __int128 mag;
  if (k >= 0) {
    mag = (unsigned __int128)M << k;
  } else {
    const int s = -k;
    if (s >= 25) mag = 0;
    else {
      const uint64_t q = M >> s, r = M & ((1ull << s) - 1), half = 1ull << (s - 1);
      mag = q + ((r > half || (r == half && (q & 1))) ? 1 : 0);
    }
  }
  const __int128 v = (b >> 31) ? -(__int128)mag : (__int128)mag;
  const unsigned __int128 u = (unsigned __int128)v;
  l[0] += (int64_t)(uint32_t)u; l[1] += (int64_t)(uint32_t)(u >> 32); l[2] += (int64_t)(uint32_t)(u >> 64); l[3] += (int64_t)(v >> 96);
}
int main() {
  std::mt19937_64 g(1);
  long bad = 0, n = 0;
  auto chk = [&](float x) {
    int64_t a[4] = {0}, b2[4] = {0}, na = 0, nb = 0;
    add_ref(a, &na, x); add_new(b2, &nb, x);
    ++n;
    if (memcmp(a, b2, sizeof a) || na != nb) { if (bad < 5) printf("mismatch %a\n", x); ++bad; }
  };
  // every float with |x| < 2^24 in a strided sweep + all small exponents exhaustively
  for (uint64_t b = 0; b < (1ull << 32); b += 97) {
    uint32_t u = (uint32_t)b; float x; memcpy(&x, &u, 4);
    if (std::isnan(x) || std::fabs(x) >= 16777216.0f) continue;
    chk(x);
  }
  for (uint32_t e = 0; e < 160; ++e) for (uint32_t m = 0; m < (1u << 23); m += 4093) for (uint32_t s = 0; s < 2; ++s) {
    uint32_t u = (s << 31) | (e << 23) | m; float x; memcpy(&x, &u, 4); chk(x);
  }
  for (int i = 0; i < 10000000; ++i) { float x = (float)(-std::ldexp((double)(g() >> 11), -53) * std::ldexp(1.0, (int)(g() % 40) - 20)); chk(x); }
  chk(-INFINITY); chk(0.0f); chk(-0.0f);
  printf("checked %ld, mismatches %ld\n", n, bad);
  // timing
  std::vector<float> xs(8400000); for (auto& x : xs) x = (float)(-std::ldexp((double)(g() >> 11), -53) * 40);
  int64_t acc[4] = {0}, ni = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (float x : xs) add_ref(acc, &ni, x);
  auto t1 = std::chrono::steady_clock::now();
  for (float x : xs) add_new(acc, &ni, x);
  auto t2 = std::chrono::steady_clock::now();
  printf("ref %.1f ms new %.1f ms (%lld)\n", std::chrono::duration<double, std::milli>(t1 - t0).count(), std::chrono::duration<double, std::milli>(t2 - t1).count(), (long long)acc[0]);
}
