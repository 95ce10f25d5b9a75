// Backtrack kernel timing vs batch size at config-4 shape (N=256, T=512): separates the
// per-sequence step latency (small batches) from throughput limits (a full round of
// waves, 8,192 sequences).  Random delta rows and A^T (timing does not depend on values).
// Usage: bt_bench [rescore 0|1] [kernel: v (backtrack_v_f32, default) | s (backtrack_f32)]
#include "../../consistent-viterbi_amd/csrc/kernels/trellis.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int NP = 256, T = 512, V = 1024;
  const int rescore = argc > 1 ? atoi(argv[1]) : 1;
  const bool scalar = argc > 2 && argv[2][0] == 's';
  const int64_t maxseq = 16384;
  std::vector<float> at(NP * NP);
  srand(2);
  for (auto& x : at) x = -(float)(rand() % 100000) / 20000.0f;
  std::vector<double> a64(NP * NP), et64((size_t)V * NP), pi64(NP);
  for (auto& x : a64) x = -(double)(rand() % 100000) / 20000.0;
  for (auto& x : et64) x = -(double)(rand() % 100000) / 20000.0;
  for (auto& x : pi64) x = -(double)(rand() % 100000) / 20000.0;
  std::vector<int64_t> off(maxseq + 1);
  for (int64_t i = 0; i <= maxseq; ++i) off[i] = i * T;
  std::vector<int32_t> obs((size_t)maxseq * T);
  for (auto& o : obs) o = rand() % V;
  float *d_at, *d_delta;
  double *d_a64, *d_et64, *d_pi64, *d_score;
  int64_t* d_off;
  int32_t *d_obs, *d_path;
  uint8_t* d_status;
  (void)hipMalloc(&d_at, at.size() * 4);
  (void)hipMalloc(&d_a64, a64.size() * 8);
  (void)hipMalloc(&d_et64, et64.size() * 8);
  (void)hipMalloc(&d_pi64, pi64.size() * 8);
  (void)hipMalloc(&d_off, off.size() * 8);
  (void)hipMalloc(&d_obs, obs.size() * 4);
  (void)hipMalloc(&d_path, obs.size() * 4);
  (void)hipMalloc(&d_score, maxseq * 8);
  (void)hipMalloc(&d_status, maxseq);
  (void)hipMalloc(&d_delta, (size_t)maxseq * T * NP * 4);
  (void)hipMemcpy(d_at, at.data(), at.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_a64, a64.data(), a64.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_et64, et64.data(), et64.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_pi64, pi64.data(), pi64.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_obs, obs.data(), obs.size() * 4, hipMemcpyHostToDevice);
  {  // delta rows: random finite values
    std::vector<float> row((size_t)1 << 22);
    for (auto& x : row) x = -(float)(rand() % 100000) / 20000.0f;
    const size_t total = (size_t)maxseq * T * NP;
    for (size_t o = 0; o < total; o += row.size())
      (void)hipMemcpy(d_delta + o, row.data(), std::min(row.size(), total - o) * 4, hipMemcpyHostToDevice);
  }
  cvk::BacktrackArgs ba{};
  ba.delta = d_delta;
  ba.at = d_at;
  ba.offsets = d_off;
  ba.obs = d_obs;
  ba.nstates = NP;
  ba.path = d_path;
  ba.score = d_score;
  ba.status = d_status;
  cvk::RescoreArgs ra{};
  ra.path = d_path;
  ra.obs = d_obs;
  ra.offsets = d_off;
  ra.nstates = NP;
  ra.pi64 = d_pi64;
  ra.a64 = d_a64;
  ra.et64 = d_et64;
  ra.status = d_status;
  ra.score = d_score;
  auto launch = [&](const cvk::BacktrackArgs& b, int64_t n) {
    if (scalar)
      hipLaunchKernelGGL(cvk::backtrack_f32<256>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, 0, b);
    else
      hipLaunchKernelGGL(cvk::backtrack_v_f32<256>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, 0, b);
    if (rescore) {
      cvk::RescoreArgs r = ra;
      r.seq_begin = 0;
      r.seq_end = n;
      (void)cvk::launch_rescore_f64(r, n, 0);
    }
  };
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int64_t n : {64, 256, 1024, 2048, 4096, 8192, 16384}) {
    ba.seq_begin = 0;
    ba.seq_end = n;
    (void)hipMemset(d_status, 0, maxseq);
    launch(ba, n);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      (void)hipMemset(d_status, 0, maxseq);
      (void)hipEventRecord(e0, 0);
      launch(ba, n);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    printf("%s rescore=%d nseq %6lld: %.3f ms  (%.2f us/step per sequence chain)\n", scalar ? "backtrack_f32  " : "backtrack_v_f32", rescore, (long long)n,
           best, best * 1e3 / (T - 1));
  }
  return hipGetLastError() != hipSuccess;
}
