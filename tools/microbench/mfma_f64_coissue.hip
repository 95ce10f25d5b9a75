// Does v_mfma_f64_16x16x4_f64 run beside f64 VALU work on gfx950, and is it exact for the
// max-plus add?  (VERDICT r4 "next" #2: the last untested lever on trellis_fwd_f64.)
//
// 1. Exactness: D = A.B + C with A[i][0] = x_i, A[i][1] = 1, B[0][j] = 1, B[1][j] = y_j, the
//    other K slots 0 and C = 0 (the outer SUM d_i + a_j the forward needs), and the C form
//    (A[i][0] = x_i, B[0][j] = 1, C[i][j] = y_j): every D[i][j] compared bit for bit with
//    fl(x_i + y_j) over random log10-like values, -inf, subnormals and mixed magnitudes.
// 2. Rates (one workgroup per CU, waves i and i + 4 (i + 8) share a SIMD): per SIMD, NV waves
//    issuing only the forward's inner loop (v_add_f64 + v_max_f64 per (from, to) pair, 16
//    independent chains) beside NM waves issuing only f64 MFMAs (4 independent accumulators),
//    each role timed per wave with s_memtime; iteration counts are calibrated from the
//    alone-runs so both roles span the same time when they co-run.
// 3. In-wave mix: one wave per SIMD issuing 1 MFMA per X VALU pairs, cycles per iteration vs
//    the same VALU alone -- the MFMA's cost to its own wave's vector issue.
// Build: hipcc --offload-arch=gfx950 -O3 -o mfma_f64_coissue mfma_f64_coissue.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

// ---- 1. exactness ----------------------------------------------------------------------
// lane l: A operand row = l & 15, k = l >> 4; B operand k = l >> 4, col = l & 15;
// D: col = l & 15, row = (l >> 4) + 4 r
__global__ void exact_k(const double* x, const double* y, double* d_sum, double* d_cform, int ntile) {
  const int l = threadIdx.x, tile = blockIdx.x;
  if (tile >= ntile) return;
  const double* xt = x + tile * 16;
  const double* yt = y + tile * 16;
  const int r = l & 15, k = l >> 4;
  const double a = k == 0 ? xt[r] : k == 1 ? 1.0 : 0.0;
  const double b = k == 0 ? 1.0 : k == 1 ? yt[r] : 0.0;
  d4 c = {0.0, 0.0, 0.0, 0.0};
  d4 dd = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  // C form: C[i][j] = y_j (lane's col), A[i][0] = x_i, B[0][j] = 1
  const double a2 = k == 0 ? xt[r] : 0.0, b2 = k == 0 ? 1.0 : 0.0;
  const double yc = yt[l & 15];
  d4 c2 = {yc, yc, yc, yc};
  d4 d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, b2, c2, 0, 0, 0);
  for (int q = 0; q < 4; ++q) {
    const int row = (l >> 4) + 4 * q, col = l & 15;
    d_sum[(size_t)tile * 256 + row * 16 + col] = dd[q];
    d_cform[(size_t)tile * 256 + row * 16 + col] = d2[q];
  }
}

// ---- 2./3. rates ------------------------------------------------------------------------
#define PAIRS4(D, A0, A1, A2, A3, M0, M1, M2, M3, T0, T1, T2, T3)                                  \
  asm volatile("v_add_f64 %4, %8, %9\n v_add_f64 %5, %8, %10\n v_add_f64 %6, %8, %11\n v_add_f64 %7, %8, %12\n" \
               " v_max_f64 %0, %0, %4\n v_max_f64 %1, %1, %5\n v_max_f64 %2, %2, %6\n v_max_f64 %3, %3, %7"     \
               : "+v"(M0), "+v"(M1), "+v"(M2), "+v"(M3), "=&v"(T0), "=&v"(T1), "=&v"(T2), "=&v"(T3)             \
               : "v"(D), "v"(A0), "v"(A1), "v"(A2), "v"(A3))

// role 0: VALU (8 pairs per block of PAIRS4 x2 = 16 VALU instructions per iteration unit)
// role 1: MFMA (4 independent accumulators per iteration unit)
// MIXX > 0: every wave issues 1 MFMA per MIXX/4 PAIRS4 blocks (MIXX pairs) in one stream
template <int NV, int NM, int MIXX>
__global__ __launch_bounds__(1024) void rate_k(double* sink, unsigned long long* cyc, int itv, int itm, double seed) {
  const int w = threadIdx.x >> 6;
  const int slot = w >> 2;  // waves i, i + 4, i + 8 share a SIMD
  const bool mfma_role = MIXX == 0 && slot >= NV;
  double a0 = seed + threadIdx.x, a1 = a0 - 1, a2 = a0 - 2, a3 = a0 - 3, dl = seed * 0.5;
  double m0 = -1e300, m1 = -1e300, m2 = -1e300, m3 = -1e300, m4 = -1e300, m5 = -1e300, m6 = -1e300, m7 = -1e300;
  double t0, t1, t2, t3;
  d4 acc0 = {seed, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  const double ma = seed * (threadIdx.x & 15), mb = 1.0;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  __syncthreads();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  if (MIXX > 0) {
    for (int it = 0; it < itv; ++it) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc0, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < MIXX / 8; ++q) {
        PAIRS4(dl, a0, a1, a2, a3, m0, m1, m2, m3, t0, t1, t2, t3);
        PAIRS4(dl, a0, a1, a2, a3, m4, m5, m6, m7, t0, t1, t2, t3);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  } else if (!mfma_role) {
    for (int it = 0; it < itv; ++it) {  // 64 pairs per iteration
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        PAIRS4(dl, a0, a1, a2, a3, m0, m1, m2, m3, t0, t1, t2, t3);
        PAIRS4(dl, a0, a1, a2, a3, m4, m5, m6, m7, t0, t1, t2, t3);
      }
    }
  } else {
    for (int it = 0; it < itm; ++it) {  // 4 MFMAs per iteration
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc1, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc2, 0, 0, 0);
      acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ma, mb, acc3, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const double s = m0 + m1 + m2 + m3 + m4 + m5 + m6 + m7 + acc0[0] + acc1[1] + acc2[2] + acc3[3];
  if (s == 1234.5) sink[threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    const size_t i = (size_t)blockIdx.x * (blockDim.x >> 6) + w;
    cyc[3 * i] = c1 - c0;
    cyc[3 * i + 1] = mfma_role ? 1 : 0;
    cyc[3 * i + 2] = (hw >> 4) & 3;
  }
}

struct Res {
  double valu_cyc = 0, mfma_cyc = 0;  // mean cycles per wave of each role
  int nvw = 0, nmw = 0;
  bool simd_ok = true;
};

template <int NV, int NM, int MIXX>
Res run(int cus, int itv, int itm) {
  const int waves = 4 * (MIXX > 0 ? 1 : NV + NM);
  double* sink;
  unsigned long long* cyc;
  (void)hipMalloc(&sink, 8 * 1024);
  (void)hipMalloc(&cyc, sizeof(unsigned long long) * 3 * waves * cus);
  hipLaunchKernelGGL((rate_k<NV, NM, MIXX>), dim3(cus), dim3(64 * waves), 0, 0, sink, cyc, 4, 4, 1.0);
  hipLaunchKernelGGL((rate_k<NV, NM, MIXX>), dim3(cus), dim3(64 * waves), 0, 0, sink, cyc, itv, itm, 1.0);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("launch failed\n");
    exit(1);
  }
  std::vector<unsigned long long> h((size_t)3 * waves * cus);
  (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  Res r;
  for (int b = 0; b < cus; ++b)
    for (int w = 0; w < waves; ++w) {
      const size_t i = (size_t)b * waves + w;
      if (h[3 * i + 1]) {
        r.mfma_cyc += (double)h[3 * i];
        ++r.nmw;
      } else {
        r.valu_cyc += (double)h[3 * i];
        ++r.nvw;
      }
      // waves w and w % 4 of a workgroup on the same SIMD
      if (h[3 * i + 2] != h[3 * ((size_t)b * waves + (w & 3)) + 2]) r.simd_ok = false;
    }
  if (r.nvw) r.valu_cyc /= r.nvw;
  if (r.nmw) r.mfma_cyc /= r.nmw;
  (void)hipFree(sink);
  (void)hipFree(cyc);
  return r;
}

template <int NV, int NM>
void corun(const char* name, int cus, double v_cpi, double m_cpi) {
  // same span for both roles: ~2e6 cycles each when alone
  const int itv = (int)(2e6 / v_cpi), itm = (int)(2e6 / m_cpi);
  const Res r = run<NV, NM, 0>(cus, itv, itm);
  const double vr = itv * 64.0 * 64.0 / r.valu_cyc;  // pairs (lane-level) per clk per VALU wave
  const double mr = itm * 4.0 * 256.0 / r.mfma_cyc;   // adds per clk per MFMA wave
  printf("%-34s VALU wave %7.1f cyc/iter (%.2fx alone) = %5.2f pairs/clk  | MFMA wave %7.1f cyc/iter (%.2fx alone) = %5.2f adds/clk%s\n",
         name, r.valu_cyc / itv, r.valu_cyc / itv / v_cpi, vr, r.mfma_cyc / itm, r.mfma_cyc / itm / m_cpi, mr,
         r.simd_ok ? "" : "  [SIMD placement differs]");
  printf("  per SIMD: %.2f pairs/clk on the VALU + %.2f adds/clk on the matrix pipe\n", NV * vr, NM * mr);
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("device %s CUs %d\n", p.gcnArchName, cus);

  // ---- 1. exactness
  {
    const int ntile = 4096;
    std::mt19937_64 rng(20261018);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    std::vector<double> x(ntile * 16), y(ntile * 16);
    for (int t = 0; t < ntile * 16; ++t) {
      const int kind = (int)(u(rng) * 8);
      auto val = [&](int k) -> double {
        switch (k) {
          case 0: return -INFINITY;
          case 1: return -std::ldexp(u(rng), -1070);  // subnormal
          case 2: return -u(rng) * 1e-300;
          case 3: return -u(rng) * 1e6 - 1.0;
          case 4: return -std::ldexp(1.0 + u(rng), (int)(u(rng) * 80));
          case 5: return 0.0;
          default: return std::log10(u(rng) + 1e-300);
        }
      };
      x[t] = val(kind);
      y[t] = val((int)(u(rng) * 8));
    }
    double *dx, *dy, *ds, *dc;
    (void)hipMalloc(&dx, x.size() * 8);
    (void)hipMalloc(&dy, y.size() * 8);
    (void)hipMalloc(&ds, (size_t)ntile * 256 * 8);
    (void)hipMalloc(&dc, (size_t)ntile * 256 * 8);
    (void)hipMemcpy(dx, x.data(), x.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dy, y.data(), y.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(exact_k, dim3(ntile), dim3(64), 0, 0, dx, dy, ds, dc, ntile);
    std::vector<double> hs((size_t)ntile * 256), hc((size_t)ntile * 256);
    (void)hipMemcpy(hs.data(), ds, hs.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hc.data(), dc, hc.size() * 8, hipMemcpyDeviceToHost);
    long bad_s = 0, bad_c = 0, ninf = 0, sub = 0, zsign_s = 0, zsign_c = 0;
    for (int t = 0; t < ntile; ++t)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          volatile double xi = x[t * 16 + i], yj = y[t * 16 + j];
          const double ref = xi + yj;
          const double gs = hs[(size_t)t * 256 + i * 16 + j], gc = hc[(size_t)t * 256 + i * 16 + j];
          ninf += std::isinf(ref);
          sub += ref != 0.0 && std::fabs(ref) < 2.2250738585072014e-308;
          // -0 + -0 = -0 in IEEE; the MFMA adds its zero products / zero C (+0) too: +0.  The
          // model tables are canonicalised to +0 (cv_hmm_create), so the trellis never sees it
          if (std::memcmp(&gs, &ref, 8) != 0) {
            if (ref == 0.0 && gs == 0.0) {
              ++zsign_s;
            } else {
              if (bad_s < 5) printf("  sum form: x=%a y=%a ref=%a mfma=%a\n", (double)xi, (double)yj, ref, gs);
              ++bad_s;
            }
          }
          if (std::memcmp(&gc, &ref, 8) != 0) {
            if (ref == 0.0 && gc == 0.0) {
              ++zsign_c;
            } else {
              if (bad_c < 5) printf("  C form:   x=%a y=%a ref=%a mfma=%a\n", (double)xi, (double)yj, ref, gc);
              ++bad_c;
            }
          }
        }
    printf("exactness over %d sums (%ld -inf, %ld subnormal): sum form %ld differ (+%ld -0 vs +0), C form %ld differ "
           "(+%ld -0 vs +0)\n", ntile * 256, ninf, sub, bad_s, zsign_s, bad_c, zsign_c);
  }

  // ---- 2. rates, alone
  const int IT = 20000;
  Res v1 = run<1, 0, 0>(cus, IT, 0), v2 = run<2, 0, 0>(cus, IT, 0);
  Res m1 = run<0, 1, 0>(cus, 0, IT / 8), m2 = run<0, 2, 0>(cus, 0, IT / 8);
  const double v1c = v1.valu_cyc / IT, v2c = v2.valu_cyc / IT, m1c = m1.mfma_cyc / (IT / 8), m2c = m2.mfma_cyc / (IT / 8);
  printf("alone: 1 VALU wave/SIMD %.1f cyc per 64 pairs (%.2f pairs/clk/SIMD), 2 waves %.1f (%.2f/SIMD)\n", v1c,
         64 * 64 / v1c, v2c, 2 * 64 * 64 / v2c);
  printf("alone: 1 MFMA wave/SIMD %.1f cyc per 4 MFMA (%.1f cyc each, %.2f adds/clk/SIMD), 2 waves %.1f (%.2f/SIMD)\n",
         m1c, m1c / 4, 1024 / m1c, m2c, 2 * 1024 / m2c);
  // ---- co-running roles on separate waves of each SIMD
  corun<1, 1>("1 VALU + 1 MFMA wave per SIMD", cus, v1c, m1c);
  corun<2, 1>("2 VALU + 1 MFMA wave per SIMD", cus, v2c, m1c);
  corun<2, 2>("2 VALU + 2 MFMA waves per SIMD", cus, v2c, m2c);
  corun<1, 2>("1 VALU + 2 MFMA waves per SIMD", cus, v1c, m2c);
  // ---- 3. in-wave mix: 1 MFMA per X pairs in one wave (1 wave per SIMD)
  {
    const int it = 20000;
    const Res b8 = run<1, 0, 8>(cus, it, 0), b16 = run<1, 0, 16>(cus, it, 0), b32 = run<1, 0, 32>(cus, it, 0),
              b64 = run<1, 0, 64>(cus, it, 0);
    const double vp = v1c / 64;  // VALU-only cycles per pair (lane-level, one wave)
    printf("in-wave: 1 MFMA + 8 pairs %.1f cyc (VALU alone %.1f), +16 pairs %.1f (%.1f), +32 %.1f (%.1f), +64 %.1f (%.1f)\n",
           b8.valu_cyc / it, 8 * vp, b16.valu_cyc / it, 16 * vp, b32.valu_cyc / it, 32 * vp, b64.valu_cyc / it, 64 * vp);
  }
  return 0;
}
