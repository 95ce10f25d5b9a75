// Ablation timing of the forward trellis kernels at config-4 shape (N=256, T=512): the same
// kernels built with the per-step barrier removed (-DCVK_ABLATE_NOBAR).
// Usage: fwd_ablate [nseq] [kinds, e.g. "01": 0 = 1 seq/WG, 1 = 2 seq/WG]  Results of ablated builds are wrong by construction; only
// the time matters: it bounds what hiding that part could gain.  Random tables (timing
// does not depend on the values).
#include "../../consistent-viterbi_amd/csrc/kernels/trellis.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  const int NP = 256, T = 512, V = 1024;
  const int64_t nseq = argc > 1 ? atoll(argv[1]) : 8192;
  const char* kinds = argc > 2 ? argv[2] : "01";
  std::vector<float> aimg(NP * NP), et((size_t)V * NP), pi(NP);
  srand(1);
  for (auto& x : aimg) x = -(float)(rand() % 100000) / 20000.0f;
  for (auto& x : et) x = -(float)(rand() % 100000) / 20000.0f;
  for (auto& x : pi) x = -(float)(rand() % 100000) / 20000.0f;
  std::vector<int64_t> off(nseq + 1);
  for (int64_t i = 0; i <= nseq; ++i) off[i] = i * T;
  std::vector<int32_t> obs((size_t)nseq * T);
  for (auto& o : obs) o = rand() % V;
  float *d_aimg, *d_et, *d_pi, *d_delta;
  int64_t* d_off;
  int32_t* d_obs;
  uint8_t* d_status;
  hipMalloc(&d_aimg, aimg.size() * 4);
  hipMalloc(&d_et, et.size() * 4);
  hipMalloc(&d_pi, pi.size() * 4);
  hipMalloc(&d_off, off.size() * 8);
  hipMalloc(&d_obs, obs.size() * 4);
  hipMalloc(&d_status, nseq);
  hipMalloc(&d_delta, (size_t)nseq * T * NP * 4);
  hipMemcpy(d_aimg, aimg.data(), aimg.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_et, et.data(), et.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_pi, pi.data(), pi.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(d_obs, obs.data(), obs.size() * 4, hipMemcpyHostToDevice);
  hipMemset(d_status, 0, nseq);
  cvk::TrellisFwdArgs fa{};
  fa.a_img = d_aimg;
  fa.pi = d_pi;
  fa.et = d_et;
  fa.offsets = d_off;
  fa.obs = d_obs;
  fa.delta = d_delta;
  fa.status = d_status;
  fa.nobs = V;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[2] = {"fwd (1 seq/WG)", "fwd2 (2 seq/WG)"};
  for (const char* kp = kinds; *kp; ++kp) {
    const int kind = *kp - '0';
    if (kind < 0 || kind > 1) continue;
    auto launch = [&]() {
      if (kind == 0) cvk::launch_trellis_fwd(NP, fa, nseq, 0);
      else cvk::launch_trellis_fwd2(NP, fa, nseq / 2, 0);
    };
    launch();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    printf("%s %-16s nseq %lld: %.3f ms  (x %.1f for config 4 = %.1f ms)\n", VARIANT, names[kind], (long long)nseq,
           best, 65536.0 / nseq, best * 65536.0 / nseq);
  }
  return hipGetLastError() != hipSuccess;
}
