// One-wave-per-sequence decode kernel (trellis_wave_f32) timing at the config-2 shape (N = 45
// padded to 48, V = 50,000, 4,096 sequences, T ~ U[1,128]); ablation switches compiled in from
// trellis.hip: CVK_ABLATE_NOBT (no fused backtrack), CVK_ABLATE_NOEMIT (no emission loads).
// Usage: wave_ablate [reps] [sequences] [max length, negative = fixed length]
#include "../../consistent-viterbi_amd/csrc/kernels/trellis.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int N = 45, NPW = 48, V = 50000;
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const int B = argc > 2 ? atoi(argv[2]) : 4096;        // sequences
  const int TMAX = argc > 3 ? atoi(argv[3]) : 128;      // lengths U[1,TMAX]; negative: all -TMAX
  srand(5);
  std::vector<int64_t> off(B + 1, 0);
  for (int s = 0; s < B; ++s) off[s + 1] = off[s] + (TMAX < 0 ? -TMAX : 1 + rand() % TMAX);
  const int64_t E = off[B];
  std::vector<int32_t> obs(E);
  for (auto& o : obs) o = rand() % V;
  const float NI = -INFINITY;
  std::vector<float> arm(NPW * NPW, NI), at(NPW * NPW, NI), pi(NPW, NI), et((size_t)V * NPW, NI);
  for (int i = 0; i < N; ++i) {
    pi[i] = -(float)(rand() % 1000) / 300.0f;
    for (int j = 0; j < N; ++j) at[j * NPW + i] = arm[i * NPW + j] = -(float)(rand() % 1000) / 300.0f;
  }
  for (int64_t o = 0; o < V; ++o)
    for (int j = 0; j < N; ++j) et[o * NPW + j] = -(float)(rand() % 1000) / 100.0f;
  std::vector<int32_t> ord(B);
  for (int s = 0; s < B; ++s) ord[s] = s;
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return off[x + 1] - off[x] > off[y + 1] - off[y]; });
  auto up = [](const void* h, size_t n) {
    void* d;
    (void)hipMalloc(&d, n);
    (void)hipMemcpy(d, h, n, hipMemcpyHostToDevice);
    return d;
  };
  cvk::TrellisFwdArgs fa{};
  fa.a_img = (const float*)up(arm.data(), arm.size() * 4);
  fa.pi = (const float*)up(pi.data(), pi.size() * 4);
  fa.et = (const float*)up(et.data(), et.size() * 4);
  fa.offsets = (const int64_t*)up(off.data(), off.size() * 8);
  fa.obs = (const int32_t*)up(obs.data(), obs.size() * 4);
  fa.order = (const int32_t*)up(ord.data(), ord.size() * 4);
  fa.nobs = V;
  float* delta;
  (void)hipMalloc(&delta, (size_t)E * NPW * 4);
  fa.delta = delta;
  uint8_t* status;
  (void)hipMalloc(&status, B);
  (void)hipMemset(status, 0, B);
  fa.status = status;
  cvk::BacktrackArgs ba{};
  ba.delta = delta;
  ba.at = (const float*)up(at.data(), at.size() * 4);
  ba.offsets = fa.offsets;
  ba.obs = fa.obs;
  ba.order = fa.order;
  ba.seq_begin = 0;
  ba.seq_end = B;
  ba.nstates = N;
  int32_t* path;
  double* score;
  (void)hipMalloc(&path, E * 4);
  (void)hipMalloc(&score, B * 8);
  ba.path = path;
  ba.score = score;
  ba.status = status;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float tot = 0;
  for (int r = 0; r <= reps; ++r) {
    (void)hipEventRecord(e0, nullptr);
    (void)cvk::launch_trellis_wave(NPW, fa, ba, B, nullptr);
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r > 0) tot += ms;
  }
  const hipError_t err = hipGetLastError();
  printf("elements %lld  wave kernel %.1f us  (%s)\n", (long long)E, 1e3 * tot / reps, hipGetErrorString(err));
  return err == hipSuccess ? 0 : 1;
}
