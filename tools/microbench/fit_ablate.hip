// Baum-Welch E-step kernel timing at the config-2 fitting shape (N=45, V=50,000, 4,096
// sequences, T ~ U[1,128], 20% tagged), with ablation switches compiled in from fit.hip:
//   CVF_ABL_NOATOMIC  no b_num atomics in the backward kernel
//   CVF_ABL_NOMFMA    no rank-4 S updates
//   CVF_ABL_NODIV     reciprocal-free: divisions replaced by multiplications
// Usage: fit_ablate [reps]   (prints average ms of bw_fwd_wave and bw_bwd_stats_wave)
#include "../../consistent-viterbi_amd/csrc/kernels/fit.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int N = 45, V = 50000, B = 4096, TMAX = 128;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  srand(7);
  std::vector<int64_t> off(B + 1, 0);
  for (int s = 0; s < B; ++s) off[s + 1] = off[s] + 1 + rand() % TMAX;
  const int64_t E = off[B];
  std::vector<int32_t> obs(E), tags(E);
  for (int64_t e = 0; e < E; ++e) {
    obs[e] = rand() % V;
    tags[e] = (rand() % 5 == 0) ? rand() % N : -1;
  }
  std::vector<double> a((size_t)N * N), et((size_t)V * N), pi(N);
  for (int i = 0; i < N; ++i) {
    double s = 0;
    for (int j = 0; j < N; ++j) s += a[i * N + j] = 1.0 + rand() % 1000;
    for (int j = 0; j < N; ++j) a[i * N + j] /= s;
    pi[i] = 1.0 / N;
  }
  for (auto& x : et) x = (1.0 + rand() % 1000) * 1e-8;
  std::vector<int64_t> ord(B);
  for (int s = 0; s < B; ++s) ord[s] = s;
  std::stable_sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return off[x + 1] - off[x] > off[y + 1] - off[y]; });
  auto up = [](const void* h, size_t n) {
    void* d;
    (void)hipMalloc(&d, n);
    (void)hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    return d;
  };
  cvf::BwArgs g{};
  g.offsets = (const int64_t*)up(off.data(), off.size() * 8);
  g.obs = (const int32_t*)up(obs.data(), obs.size() * 4);
  g.tags = (const int32_t*)up(tags.data(), tags.size() * 4);
  g.order = (const int64_t*)up(ord.data(), ord.size() * 8);
  g.nstates = N;
  g.pi = (const double*)up(pi.data(), pi.size() * 8);
  g.a = (const double*)up(a.data(), a.size() * 8);
  g.at = g.a;
  g.et = (const double*)up(et.data(), et.size() * 8);
  const size_t nacc = 3 * (size_t)N + (size_t)V * N + (size_t)N * N + 1;
  double *alpha, *acc, *dump;
  (void)hipMalloc(&alpha, (size_t)E * N * 8);
  (void)hipMalloc(&acc, nacc * 8);
  (void)hipMalloc(&dump, (size_t)cvf::kBwDumpWaves * 64 * 8);
  (void)hipMemset(acc, 0, nacc * 8);
  g.alpha = alpha;
  g.dump = dump;
  g.pi_acc = acc;
  g.a_den = acc + N;
  g.b_den = acc + 2 * N;
  g.b_num = acc + 3 * N;
  g.xi_s = g.b_num + (size_t)V * N;
  g.xi_zero = g.xi_s + (size_t)N * N;
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int64_t nwaves = std::min<int64_t>((B + 1) / 2, (int64_t)cus * 8);
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreate(&e2);
  float tf = 0, tb = 0;
  for (int r = 0; r <= reps; ++r) {
    (void)hipEventRecord(e0, nullptr);
    hipLaunchKernelGGL((cvf::bw_fwd_wave<48>), dim3((B + 3) / 4), dim3(256), 0, nullptr, g, (int64_t)B);
    (void)hipEventRecord(e1, nullptr);
    hipLaunchKernelGGL((cvf::bw_bwd_stats_wave<48>), dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0, nullptr, g,
                       (int64_t)B, nwaves);
    (void)hipEventRecord(e2, nullptr);
    (void)hipEventSynchronize(e2);
    float a1, a2;
    (void)hipEventElapsedTime(&a1, e0, e1);
    (void)hipEventElapsedTime(&a2, e1, e2);
    if (r > 0) {
      tf += a1;
      tb += a2;
    }
  }
  const hipError_t err = hipGetLastError();
  printf("elements %lld  fwd %.1f us  bwd %.1f us  (%s)\n", (long long)E, 1e3 * tf / reps, 1e3 * tb / reps,
         hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
