// cviterbi.cpp -- C ABI (include/cviterbi.h) over the MI355X trellis kernels.
//
// Host side of the drop-in boundary: the HMM handle mirrors struct HMM<D> and its
// log-prob lookups (src/hmm/hmm.rs:10-18, 207-245), the batch decode replaces the
// dense forward + backtrack of viterbi_solver (cp.rs:63-93, viterbi.rs:5-32,
// dp.rs:94-209), and cv_solver_* mirrors `trait Solver` (viterbi_solver.rs:11-16).
//
// There is deliberately no CPU decode path here: every decode runs the HIP kernels
// in kernels/trellis.hip and fails with CV_EDEVICE if no gfx950 device is usable.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <functional>
#include <limits>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cviterbi.h"
#include "csp.hpp"
#include "hostscan.hpp"
#include "hmm_json.hpp"
#include "kernels/chain.h"
#include "kernels/cfn.h"
#include "kernels/exact.h"
#include "kernels/fit.h"
#include "kernels/trellis.h"
#include "kernels/trellis64.h"
#include "tuning.h"

namespace {

thread_local std::string g_err;

// the handle's lock plus its tuning snapshot as the calling thread's current tuning (tuning.h)
#define CV_LOCK(h)                             \
  std::lock_guard<std::mutex> lk((h)->mu);     \
  cvk::TuningScope tuning_scope((h)->tuning)

inline uint64_t dbits(double x) {
  uint64_t b;
  std::memcpy(&b, &x, 8);
  return b;
}
inline double from_dbits(uint64_t b) {
  double x;
  std::memcpy(&x, &b, 8);
  return x;
}

cv_status set_err(cv_status st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return st;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return set_err(CV_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                     __LINE__);                                                                \
  } while (0)

// device bytes this process's library holds now / at most (cv_device_memory)
std::atomic<int64_t> g_dev_cur{0}, g_dev_peak{0};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) {
      (void)hipFree(p);
      g_dev_cur -= (int64_t)bytes;
    }
    p = nullptr;
    bytes = 0;
  }
  cv_status ensure(size_t n) {
    if (n <= bytes && p) return CV_OK;
    release();
    if (n == 0) n = 16;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
      p = nullptr;
      (void)hipGetLastError();
      return set_err(CV_ENOMEM, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    }
    bytes = n;
    const int64_t cur = g_dev_cur += (int64_t)n;
    int64_t pk = g_dev_peak.load();
    while (cur > pk && !g_dev_peak.compare_exchange_weak(pk, cur)) {
    }
    return CV_OK;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

cv_status upload(DevBuf& buf, const void* src, size_t bytes) {
  cv_status st = buf.ensure(bytes);
  if (st != CV_OK) return st;
  HIP_TRY(hipMemcpy(buf.p, src, bytes, hipMemcpyHostToDevice));
  return CV_OK;
}

constexpr uint64_t kDefaultWorkspace = 8ull << 30;
constexpr uint64_t kDefaultWorkspaceT64 = 64ull << 30;  // config 5 resume decode in one chunk: 3% faster than 40 GiB
constexpr size_t kMaxTimedEvents = 1 << 16;  // cv_timing_begin: at most 16,384 chunk launches timed

}  // namespace

// Pinned, double-buffered host staging of a decode call's longest-first order: the call
// writes slot k only after that slot's previous copy has completed (its event), so the
// copy is truly asynchronous and the host never waits for the stream's earlier work
// A grow-only pinned host buffer (hipHostMalloc) for small device-to-host results read right
// after a synchronize (the parallel chain's scores, statuses and certificates: two direct
// copies instead of three through the runtime's pageable staging).
struct PinnedHost {
  void* p = nullptr;
  size_t cap = 0;
  PinnedHost() = default;
  PinnedHost(const PinnedHost&) = delete;
  PinnedHost& operator=(const PinnedHost&) = delete;
  ~PinnedHost() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  bool ensure(size_t bytes) {
    if (cap >= bytes && p) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes, 4096);
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    cap = want;
    return true;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(p); }
};

struct OrderStage {
  int32_t* p[2] = {nullptr, nullptr};
  size_t cap[2] = {0, 0};
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool pending[2] = {false, false};
  int slot = 0;
  OrderStage() = default;
  OrderStage(const OrderStage&) = delete;
  OrderStage& operator=(const OrderStage&) = delete;
  ~OrderStage() {
    for (int k = 0; k < 2; ++k) {
      if (pending[k]) (void)hipEventSynchronize(ev[k]);
      if (p[k]) (void)hipHostFree(p[k]);
      if (ev[k]) (void)hipEventDestroy(ev[k]);
    }
  }
  // the current slot, at least n entries, free to write (nullptr: allocation failed)
  int32_t* acquire(size_t n) {
    const int k = slot;
    if (pending[k]) {
      if (hipEventSynchronize(ev[k]) != hipSuccess) return nullptr;
      pending[k] = false;
    }
    if (!ev[k] && hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) return nullptr;
    if (cap[k] < n) {
      if (p[k]) (void)hipHostFree(p[k]);
      p[k] = nullptr;
      cap[k] = 0;
      const size_t want = std::max<size_t>(n, 4096);
      if (hipHostMalloc((void**)&p[k], want * 4, hipHostMallocDefault) != hipSuccess) return nullptr;
      cap[k] = want;
    }
    return p[k];
  }
  // after the copy out of the current slot is enqueued on `stream`
  hipError_t release(hipStream_t stream) {
    const hipError_t e = hipEventRecord(ev[slot], stream);
    pending[slot] = e == hipSuccess;
    slot ^= 1;
    return e;
  }
};

struct cv_hmm {
  int N = 0, D = 0;
  std::vector<int64_t> bdims;
  int64_t V = 0;
  std::vector<double> pi, a, b;  // host log10, canonical (-0.0 -> +0.0); b state-major [N*V]
  int device = 0;
  int cus = 0;                      // compute units of the device (workgroup rounds)
  hipStream_t stream = nullptr;     // default stream of the handle
  hipStream_t bt_stream = nullptr;  // backtrack stream (overlaps the next chunk's forward)
  std::mutex mu;
  // tuning keys and test hooks (tuning.h): the environment at cv_hmm_create, then
  // cv_hmm_set_tuning only; every locked host API call makes it the thread's current tuning
  cvk::Tuning tuning;

  // trellis kernel tables (f32, padded to NP)
  int np = 0;
  DevBuf t_aimg, t_pi, t_et, t_at, t_arm;  // t_arm: row-major A (one-wave kernel)
  // one-wave kernel (N <= 64): tables padded to npw = 16 * ceil(N / 16) states
  int npw = 0;
  DevBuf w_arm, w_pi, w_et, w_at;
  DevBuf t_aimg_T, t_pi0;  // reversed (backward) pass: VALU image of a^T, pi = 0
  // f64 tables (generic f64 kernel + re-scoring): pi[N], a[N*N], et[V][N]
  bool f64_ready = false;
  DevBuf d_pi64, d_a64, d_et64;
  DevBuf d_at64;  // [N][N] a^T, f64: the constrained decode's suffix pass for N > 256

  // exact-f64 trellis tables (trellis_fwd_f64 / backtrack_f64), padded to np64 = 64*ceil(N/64)
  int np64 = 0;
  bool t64_ready = false;
  DevBuf q_a, q_at, q_pi, q_et;
  DevBuf q_at32;            // f32(a^T), uploaded when t64_nonpos
  bool t64_nonpos = false;  // every finite pi/a/b entry in [-2^80, 0] (NONPOS backtrack test)
  int nonpos_cache = -1;    // model_nonpos(): the same predicate without the t64 tables (any N)
  double arc_max = -1.0;    // max finite |pi| or |a|, plus max finite |b| (< 0: not computed yet)
  double cert_rho_cap = 0.0;  // the parallel chain's certified backtrack (T64BtArgs::rho_cap)
  DevBuf q_pi0;  // the reversed (suffix) pass: pi = 0 for the N states, -inf padding
  // f32 generic tables
  bool g32_ready = false;
  DevBuf d_pi32, d_a32, d_et32;
  DevBuf d_at32;  // [N][N] a^T f32 (generic_bt_rows)
  // workspace
  DevBuf ws_main, ws_last, ws_order;
  // a second decode workspace + stream: the constrained decode's unconstrained sequences run
  // on it beside the terms pass (constrained decode)
  struct SideWs {
    DevBuf main, last, order, idx, obs2, path2, res2;
    std::vector<int32_t> order_host;
    OrderStage order_pin;
    hipEvent_t ws_done = nullptr;  // the last decode_device call on this workspace has finished
    bool ws_rec = false;
    std::vector<int64_t> idx_host;
    std::vector<hipEvent_t> ev;
    hipStream_t stream = nullptr;  // lowest priority: fills what the constrained work leaves idle
    hipStream_t hi = nullptr;      // highest priority: the constrained work itself
    hipEvent_t start = nullptr, done = nullptr, after = nullptr;
  } side;
  DevBuf st_off, st_obs, st_path, st_score, st_status, st_forced;
  DevBuf cs_ranges, cs_delta, cs_g, cs_mu, cs_start, cs_zero, cs_queue;  // constrained-decode scratch
  DevBuf cs_wrows;  // the wide generic_ext's rows ([slot][2][N], N > 10,240)
  DevBuf cs_comp, cs_words;  // device exact unary sums: per-sequence components, output words
  DevBuf cs_flag;            // device exact sums: out-of-range term flag
  DevBuf cs_seg;             // segment-table rows (cs_delta keeps the prefix rows t_1)
  // resume flow of the constrained decode: stored prefix rows, forced row t_1 per constrained
  // sequence, the compact suffix batch and its index arrays
  DevBuf rs_rows, rs_rowbase, rs_resume, rs_start, rs_off2, rs_ridx, rs_slot, rs_obs2, rs_frc2, rs_path2;
  // certified suffix trace (f64): the suffix pass's rows, their per-slot bases, the slot flags
  DevBuf rs_srows, rs_srowbase, rs_cert;
  hipEvent_t rs_ev = nullptr;  // prefix backtrack done / staging done
  std::vector<int32_t> order_host;
  OrderStage order_pin;
  // the last decode_device call on the main workspace has finished (recorded on its stream;
  // the next call waits for it on ITS stream, so calls on different streams never share the
  // workspace while it is in use)
  hipEvent_t ws_done = nullptr;
  bool ws_rec = false;
  std::vector<float> host_dl, host_mu;  // constrained-decode term rows (kept: no per-call page faults)
  std::vector<int64_t> sort_pos;        // counting-sort buckets of the longest-first order
  // timing events of the last call
  std::vector<hipEvent_t> ev;  // 4 per chunk: fwd start/end (main stream), bt start/end
  int64_t last_launches = 0;
  size_t last_ev_base = 0;  // first event of the last call in ev
  // cv_timing_begin/end: every decode call's events kept (appended) until cv_timing_end
  bool acc_on = false, acc_overflow = false;
  size_t acc_used = 0;
  int32_t last_kernel = 0;
  int32_t last_np = 0;
  int32_t last_mt = -1;
  uint64_t last_explored = 0;
  int64_t last_traced = 0;  // constrained sequences the last resume flow certified (suffix trace)
  // the last cv_decode_superseq_cp: parallel chain ran (1/0), sequences certified, sequences in
  // serial-chain runs, runs, certified folds done by the quantised sum, sequences taken from
  // speculative parallel re-decodes, such batches
  // speculative parallel re-decodes, such batches, candidate paths fetched packed for the walk,
  // walk steps that waited for the whole path copy
  int64_t last_chain[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  // the parallel chain's per-call device arrays, kept between calls (grow-only): a
  // config-4-sized call allocated and freed ~0.4 GB of them each time (hipFree synchronises)
  struct ChainBufs {
    DevBuf off, obs, path, res, cert, ebin, q, ends, gid, gpath;
    // serial runs and speculative batches (kept, so no hipFree -- a device-wide sync -- lands
    // while the second part's forward pass runs)
    DevBuf first, rpsi, rows, small, rpath, soff, sobs, spath, sres, sinit, slast, spsi;
  } chainb;
  // the chain's own stream (high priority: its walk-side kernels -- end states, quantised folds,
  // gathers, runs, speculative batches -- run beside the second part's forward pass) and the
  // events closing each part's decode
  hipStream_t chain_stream = nullptr;
  std::vector<hipEvent_t> part_ev;
  // the parallel chain's path copy: per decode chunk, behind that chunk's backtrack (chunk_ev),
  // on a non-blocking stream of its own, from a host thread of its own
  std::vector<hipEvent_t> chunk_ev;
  hipStream_t copy_stream = nullptr;
  PinnedHost chain_pin;  // the chain's scores, statuses and certificates on their way to the host
  PinnedHost chain_gpin;  // the chain's gathered candidate paths and speculative results (16 MiB)
  // the chain's later parts' observations and its path copy's two-chunk ring, staged through
  // pinned memory: the DMA engines move them, where a pageable copy runs blit kernels beside
  // the forward passes (tuning keys chain_pin_obs / chain_pin_path)
  PinnedHost chain_obs_pin, chain_ring[2];
  hipEvent_t ring_ev[2] = {nullptr, nullptr};

  ~cv_hmm() {
    for (auto e : ring_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : ev) (void)hipEventDestroy(e);
    for (auto e : side.ev) (void)hipEventDestroy(e);
    if (side.start) (void)hipEventDestroy(side.start);
    if (side.done) (void)hipEventDestroy(side.done);
    if (side.after) (void)hipEventDestroy(side.after);
    if (side.stream) (void)hipStreamDestroy(side.stream);
    if (side.hi) (void)hipStreamDestroy(side.hi);
    if (rs_ev) (void)hipEventDestroy(rs_ev);
    if (ws_done) (void)hipEventDestroy(ws_done);
    if (side.ws_done) (void)hipEventDestroy(side.ws_done);
    if (stream) (void)hipStreamDestroy(stream);
    if (bt_stream) (void)hipStreamDestroy(bt_stream);
    for (auto e : chunk_ev) (void)hipEventDestroy(e);
    for (auto e : part_ev) (void)hipEventDestroy(e);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    if (chain_stream) (void)hipStreamDestroy(chain_stream);
  }
};

namespace {

// Device bytes free right now plus `held` (buffers the caller is about to re-size); 0 when the
// runtime cannot tell.
uint64_t free_device_bytes(uint64_t held) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (uint64_t)fr + held;
}

// The default delta-workspace cap when the caller leaves opts.workspace_bytes at 0: `base`
// (sized for 288 GB of HBM3E), clamped to 3/4 of what the device can still give the workspace
// being sized (`held` = its current bytes, reclaimable), so a smaller or busier card chunks the
// batch instead of failing in hipMalloc.
uint64_t default_workspace_cap(uint64_t held, uint64_t base) {
  const uint64_t avail = free_device_bytes(held);
  if (avail == 0) return base;
  return std::max<uint64_t>(std::min<uint64_t>(base, avail / 4 * 3), 256ull << 20);
}

cv_status set_device(cv_hmm* h) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    return set_err(CV_EDEVICE, "no HIP device available");
  }
  if (h->device < 0 || h->device >= n) return set_err(CV_EDEVICE, "device %d out of range (%d devices)", h->device, n);
  HIP_TRY(hipSetDevice(h->device));
  if (!h->cus) HIP_TRY(hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, h->device));
  if (!h->stream) HIP_TRY(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  if (!h->bt_stream) HIP_TRY(hipStreamCreateWithFlags(&h->bt_stream, hipStreamNonBlocking));
  return CV_OK;
}

float f32(double x) { return (float)x; }

// Trellis tables.  a_img: float4 per (wave w, pair q, lane): rows r0 = rg*R + 2q, r0+1 and
// columns j0 = 16w + 2cp, j0+1 with rg = lane&7, cp = lane>>3 (trellis_fwd_f32 layout).
cv_status ensure_trellis_tables(cv_hmm* h) {
  const int np = cvk::trellis_padded_states(h->N);
  if (!np) return set_err(CV_EUNSUPPORTED, "trellis kernel covers 1 <= N <= 256 (N=%d)", h->N);
  if (h->np == np) return CV_OK;
  const int N = h->N;
  const int64_t V = h->V;
  const int R = np / 8;
  const float NI = -INFINITY;
  auto A = [&](int i, int j) -> float { return (i < N && j < N) ? f32(h->a[(size_t)i * N + j]) : NI; };
  std::vector<float> img((size_t)np * np);
  for (int w = 0; w < np / 16; ++w)
    for (int q = 0; q < R / 2; ++q)
      for (int lane = 0; lane < 64; ++lane) {
        const int rg = lane & 7, cp = lane >> 3, j0 = 16 * w + 2 * cp, r0 = rg * R + 2 * q;
        float* dst = &img[(((size_t)w * (R / 2) + q) * 64 + lane) * 4];
        dst[0] = A(r0, j0);
        dst[1] = A(r0, j0 + 1);
        dst[2] = A(r0 + 1, j0);
        dst[3] = A(r0 + 1, j0 + 1);
      }
  std::vector<float> pi(np, NI), at((size_t)np * np, NI), arm((size_t)np * np, NI), et((size_t)V * np, NI);
  for (int j = 0; j < N; ++j) pi[j] = f32(h->pi[j]);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) at[(size_t)j * np + i] = arm[(size_t)i * np + j] = f32(h->a[(size_t)i * N + j]);
  for (int j = 0; j < N; ++j)
    for (int64_t o = 0; o < V; ++o) et[(size_t)o * np + j] = f32(h->b[(size_t)j * V + o]);
  cv_status st;
  if ((st = upload(h->t_aimg, img.data(), img.size() * 4)) != CV_OK) return st;
  {  // the backward max-plus pass runs the same kernel on a^T with pi = 0
    auto AT = [&](int i, int j) -> float { return A(j, i); };
    std::vector<float> imgT((size_t)np * np);
    for (int w = 0; w < np / 16; ++w)
      for (int q = 0; q < R / 2; ++q)
        for (int lane = 0; lane < 64; ++lane) {
          const int rg = lane & 7, cp = lane >> 3, j0 = 16 * w + 2 * cp, r0 = rg * R + 2 * q;
          float* dst = &imgT[(((size_t)w * (R / 2) + q) * 64 + lane) * 4];
          dst[0] = AT(r0, j0);
          dst[1] = AT(r0, j0 + 1);
          dst[2] = AT(r0 + 1, j0);
          dst[3] = AT(r0 + 1, j0 + 1);
        }
    std::vector<float> pi0(np, NI);
    for (int j = 0; j < N; ++j) pi0[j] = 0.f;
    if ((st = upload(h->t_aimg_T, imgT.data(), imgT.size() * 4)) != CV_OK) return st;
    if ((st = upload(h->t_pi0, pi0.data(), pi0.size() * 4)) != CV_OK) return st;
  }
  if ((st = upload(h->t_pi, pi.data(), pi.size() * 4)) != CV_OK) return st;
  if ((st = upload(h->t_at, at.data(), at.size() * 4)) != CV_OK) return st;
  if ((st = upload(h->t_arm, arm.data(), arm.size() * 4)) != CV_OK) return st;
  if ((st = upload(h->t_et, et.data(), et.size() * 4)) != CV_OK) return st;
  h->npw = cvk::trellis_wave_states(N);
  if (h->npw) {  // the one-wave kernel's tables: row-major A, A^T, pi, E^T at the npw stride
    const int nw = h->npw;
    std::vector<float> wpi(nw, NI), wat((size_t)nw * nw, NI), warm((size_t)nw * nw, NI), wet((size_t)V * nw, NI);
    for (int j = 0; j < N; ++j) wpi[j] = f32(h->pi[j]);
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) wat[(size_t)j * nw + i] = warm[(size_t)i * nw + j] = f32(h->a[(size_t)i * N + j]);
    for (int j = 0; j < N; ++j)
      for (int64_t o = 0; o < V; ++o) wet[(size_t)o * nw + j] = f32(h->b[(size_t)j * V + o]);
    if ((st = upload(h->w_pi, wpi.data(), wpi.size() * 4)) != CV_OK) return st;
    if ((st = upload(h->w_at, wat.data(), wat.size() * 4)) != CV_OK) return st;
    if ((st = upload(h->w_arm, warm.data(), warm.size() * 4)) != CV_OK) return st;
    if ((st = upload(h->w_et, wet.data(), wet.size() * 4)) != CV_OK) return st;
  }
  h->np = np;
  return CV_OK;
}

cv_status ensure_f64_tables(cv_hmm* h) {
  if (h->f64_ready) return CV_OK;
  const int N = h->N;
  const int64_t V = h->V;
  std::vector<double> et((size_t)V * N);
  for (int j = 0; j < N; ++j)
    for (int64_t o = 0; o < V; ++o) et[(size_t)o * N + j] = h->b[(size_t)j * V + o];
  cv_status st;
  if ((st = upload(h->d_pi64, h->pi.data(), (size_t)N * 8)) != CV_OK) return st;
  if ((st = upload(h->d_a64, h->a.data(), (size_t)N * N * 8)) != CV_OK) return st;
  if ((st = upload(h->d_et64, et.data(), et.size() * 8)) != CV_OK) return st;
  h->f64_ready = true;
  return CV_OK;
}

// a^T [N][N] f64 (generic_ext's suffix pass, generic_bt_rows), uploaded on first use
cv_status ensure_at64(cv_hmm* h) {
  if (h->d_at64.p) return CV_OK;
  const int N = h->N;
  std::vector<double> at((size_t)N * N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) at[(size_t)j * N + i] = h->a[(size_t)i * N + j];
  return upload(h->d_at64, at.data(), at.size() * 8);
}

// a^T [N][N] f32 (generic_bt_rows), uploaded on first use
cv_status ensure_at32(cv_hmm* h) {
  if (h->d_at32.p) return CV_OK;
  const int N = h->N;
  std::vector<float> at((size_t)N * N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) at[(size_t)j * N + i] = f32(h->a[(size_t)i * N + j]);
  return upload(h->d_at32, at.data(), at.size() * 4);
}

// Every finite pi/a/b entry in [-2^80, 0] (log-probabilities): the NONPOS backtrack test and the
// parallel chain's certificates hold for such models.  Tuning key t64_nonpos = 0 forces the
// general f64 interval test (same paths, bit for bit) and turns the parallel chain off.
bool model_nonpos(cv_hmm* h) {
  if (h->nonpos_cache >= 0) return h->nonpos_cache != 0;
  const bool nonpos_knob = h->tuning.t64_nonpos != 0;
  auto nonpos = [](const std::vector<double>& v) {
    for (double x : v)
      if (std::isfinite(x) && !(x <= 0.0 && x >= -0x1p80)) return false;
    return true;
  };
  h->nonpos_cache = nonpos_knob && nonpos(h->pi) && nonpos(h->a) && nonpos(h->b) ? 1 : 0;
  return h->nonpos_cache != 0;
}

// Exact-f64 trellis tables: a [NP][NP] row-major, a^T, pi [NP], et [V][NP]; -inf padded to the
// NP every f64 trellis kernel supports at this N (cvk::t64_support_states: 512 / 1,024 above 256).
cv_status ensure_t64_tables(cv_hmm* h) {
  if (h->t64_ready) return CV_OK;
  const int N = h->N, NP = cvk::t64_support_states(N);
  if (NP == 0) return set_err(CV_EUNSUPPORTED, "f64 trellis tables need N <= 1024 (N=%d)", N);
  const int64_t V = h->V;
  const double ninf = -INFINITY;
  std::vector<double> a((size_t)NP * NP, ninf), at((size_t)NP * NP, ninf), pi(NP, ninf), et((size_t)V * NP, ninf);
  for (int i = 0; i < N; ++i) {
    pi[i] = h->pi[i];
    for (int j = 0; j < N; ++j) {
      a[(size_t)i * NP + j] = h->a[(size_t)i * N + j];
      at[(size_t)j * NP + i] = h->a[(size_t)i * N + j];
    }
  }
  for (int j = 0; j < N; ++j)
    for (int64_t o = 0; o < V; ++o) et[(size_t)o * NP + j] = h->b[(size_t)j * V + o];
  cv_status st;
  if ((st = upload(h->q_a, a.data(), a.size() * 8)) != CV_OK) return st;
  if ((st = upload(h->q_at, at.data(), at.size() * 8)) != CV_OK) return st;
  if ((st = upload(h->q_pi, pi.data(), pi.size() * 8)) != CV_OK) return st;
  if ((st = upload(h->q_et, et.data(), et.size() * 8)) != CV_OK) return st;
  std::vector<double> pi0(NP, ninf);
  for (int i = 0; i < N; ++i) pi0[i] = 0.0;
  if ((st = upload(h->q_pi0, pi0.data(), pi0.size() * 8)) != CV_OK) return st;
  // NONPOS backtrack test (trellis64.hip bt_chain_f64): log-probability models only
  h->t64_nonpos = model_nonpos(h);
  if (h->t64_nonpos) {
    std::vector<float> at32(at.size());
    for (size_t k = 0; k < at.size(); ++k) at32[k] = (float)at[k];
    if ((st = upload(h->q_at32, at32.data(), at32.size() * 4)) != CV_OK) return st;
  }
  h->np64 = NP;
  h->t64_ready = true;
  return CV_OK;
}

cv_status ensure_g32_tables(cv_hmm* h) {
  if (h->g32_ready) return CV_OK;
  const int N = h->N;
  const int64_t V = h->V;
  std::vector<float> pi(N), a((size_t)N * N), et((size_t)V * N);
  for (int j = 0; j < N; ++j) pi[j] = f32(h->pi[j]);
  for (size_t k = 0; k < a.size(); ++k) a[k] = f32(h->a[k]);
  for (int j = 0; j < N; ++j)
    for (int64_t o = 0; o < V; ++o) et[(size_t)o * N + j] = f32(h->b[(size_t)j * V + o]);
  cv_status st;
  if ((st = upload(h->d_pi32, pi.data(), pi.size() * 4)) != CV_OK) return st;
  if ((st = upload(h->d_a32, a.data(), a.size() * 4)) != CV_OK) return st;
  if ((st = upload(h->d_et32, et.data(), et.size() * 4)) != CV_OK) return st;
  h->g32_ready = true;
  return CV_OK;
}

cv_status validate_model(int N, int64_t V, const double* pi, const double* a, const double* b) {
  auto bad = [](double x) { return std::isnan(x) || x == INFINITY; };
  for (int i = 0; i < N; ++i)
    if (bad(pi[i])) return set_err(CV_EINVAL, "pi[%d] is NaN or +inf (log10 probabilities must be <= 0 or -inf)", i);
  for (int64_t k = 0; k < (int64_t)N * N; ++k)
    if (bad(a[k])) return set_err(CV_EINVAL, "a[%lld] is NaN or +inf", (long long)k);
  for (int64_t k = 0; k < (int64_t)N * V; ++k)
    if (bad(b[k])) return set_err(CV_EINVAL, "b[%lld] is NaN or +inf", (long long)k);
  return CV_OK;
}

cv_status make_hmm(int N, const std::vector<int64_t>& bdims, const double* pi, const double* a, const double* b,
                   int device, cv_hmm** out) {
  if (N <= 0) return set_err(CV_EINVAL, "nstates must be > 0");
  if (bdims.empty()) return set_err(CV_EINVAL, "ndims must be > 0");
  int64_t V = 1;
  for (auto d : bdims) {
    if (d <= 0) return set_err(CV_EINVAL, "bdims entries must be > 0");
    V *= d;
  }
  if (V > (int64_t)1 << 31) return set_err(CV_EINVAL, "observation alphabet too large (%lld)", (long long)V);
  if (!pi || !a || !b) return set_err(CV_EINVAL, "null model array");
  cv_status st = validate_model(N, V, pi, a, b);
  if (st != CV_OK) return st;
  auto h = std::make_unique<cv_hmm>();
  h->N = N;
  h->D = (int)bdims.size();
  h->bdims = bdims;
  h->V = V;
  auto canon = [](double x) { return x == 0.0 ? 0.0 : x; };  // -0.0 -> +0.0
  h->pi.resize(N);
  h->a.resize((size_t)N * N);
  h->b.resize((size_t)N * V);
  std::transform(pi, pi + N, h->pi.begin(), canon);
  std::transform(a, a + (size_t)N * N, h->a.begin(), canon);
  std::transform(b, b + (size_t)N * V, h->b.begin(), canon);
  h->device = device;
  h->tuning = cvk::tuning_from_env();  // the handle's snapshot: no later environment read
  *out = h.release();
  return CV_OK;
}

// tuning key trace (CV_TRACE=1): host-side phase timestamps on stderr (profiling aid).
bool trace_on() { return cvk::tuning().trace != 0; }
void trace_mark(const char* what) {
  if (!trace_on()) return;
  static thread_local auto last = std::chrono::steady_clock::now();
  const auto now = std::chrono::steady_clock::now();
  fprintf(stderr, "[cv] %-28s +%8.3f ms\n", what, std::chrono::duration<double, std::milli>(now - last).count());
  last = now;
}

// Host worker threads for the O(elements) loops of the host API (validation, constraint
// bookkeeping, exact accumulation): min(16, hardware threads), tuning key host_threads overrides.
int host_threads() {
  static const int hw = (int)std::thread::hardware_concurrency();
  const int v = cvk::tuning().host_threads > 0 ? cvk::tuning().host_threads : hw;
  return std::max(1, std::min(v > 0 ? v : 1, 16));
}

// f(t, lo, hi) over [0, n) split into contiguous ranges, one per worker (t = worker index).
template <typename F>
void parallel_ranges(int64_t n, F&& f, int64_t min_per_thread = 1 << 16) {
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / std::max<int64_t>(min_per_thread, 1)));
  if (nt <= 1) {
    f(0, (int64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int t = 0; t < nt; ++t) th.emplace_back([&, t] { f(t, n * t / nt, n * (t + 1) / nt); });
  for (auto& x : th) x.join();
}

// First index k in [lo, hi) with bad(k), or -1 (parallel scan; the smallest index wins).
template <typename P>
int64_t first_bad(int64_t lo, int64_t hi, P&& bad) {
  std::vector<int64_t> first((size_t)host_threads(), -1);
  parallel_ranges(hi - lo, [&](int t, int64_t a, int64_t b) {
    for (int64_t k = lo + a; k < lo + b; ++k)
      if (bad(k)) {
        first[t] = k;
        return;
      }
  });
  for (int64_t f : first)
    if (f >= 0) return f;  // workers hold ascending ranges
  return -1;
}

cv_status check_batch(const cv_hmm* h, int64_t nseq, const int64_t* offsets) {
  if (nseq < 0) return set_err(CV_EINVAL, "nseq < 0");
  if (!offsets) return set_err(CV_EINVAL, "offsets is NULL");
  if (offsets[0] < 0) return set_err(CV_EINVAL, "offsets[0] < 0");
  for (int64_t s = 0; s < nseq; ++s) {
    const int64_t T = offsets[s + 1] - offsets[s];
    if (T < 0) return set_err(CV_EINVAL, "offsets not non-decreasing at %lld", (long long)s);
    if (T > INT32_MAX) return set_err(CV_EINVAL, "sequence %lld too long", (long long)s);
  }
  (void)h;
  return CV_OK;
}

hipEvent_t get_event(std::vector<hipEvent_t>& ev, size_t i) {
  while (ev.size() <= i) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ev.push_back(e);
  }
  return ev[i];
}

cvk::BacktrackArgs make_bt_args(cv_hmm* h, unsigned char* wsb, const int64_t* offsets_host,
                                const int64_t* offsets_dev, const int32_t* obs_dev, const int32_t* order_dev,
                                const std::pair<int64_t, int64_t>& c, int32_t* path_dev, double* score_dev,
                                uint8_t* status_dev) {
  cvk::BacktrackArgs ba{};
  ba.delta = reinterpret_cast<const float*>(wsb);
  ba.delta_elem_base = offsets_host[c.first];
  ba.at = h->t_at.as<float>();
  ba.offsets = offsets_dev;
  ba.obs = obs_dev;
  ba.order = order_dev;
  ba.seq_begin = c.first;
  ba.seq_end = c.second;
  ba.nstates = h->N;
  ba.path = path_dev;
  ba.score = score_dev;
  ba.score32 = nullptr;
  ba.status = status_dev;
  return ba;
}

// Core device-side decode.  All pointers are device pointers except offsets_host.
cv_status decode_device(cv_hmm* h, int64_t nseq, const int64_t* offsets_host, const int64_t* offsets_dev,
                        const int32_t* obs_dev, const cv_opts& o, int32_t* path_dev, double* score_dev,
                        uint8_t* status_dev, hipStream_t stream, const void* resume_rows = nullptr,
                        bool side_ws = false, double* cp_cert = nullptr, const double* cp_init = nullptr,
                        double* cp_last = nullptr,
                        std::vector<std::pair<int64_t, int64_t>>* chunks_out = nullptr) {
  // cp_cert (the parallel CPSolver chain, row-A0 f64 trellis only): each chunk's backtrack
  // computes its certificates (or cp_cert_f64 reads the chunk's rows and paths) -> [nseq][2];
  // chunks_out: h->chunk_ev[i] is recorded after chunk i's backtrack (its paths written,
  // before any certificate pass) and its sequence range [s0, s1) appended
  // side_ws: the handle's second workspace (h->side), no timing / last-call bookkeeping -- a
  // decode running beside another decode_device call of the same handle on another stream
  DevBuf& w_main = side_ws ? h->side.main : h->ws_main;
  DevBuf& w_last = side_ws ? h->side.last : h->ws_last;
  DevBuf& w_order = side_ws ? h->side.order : h->ws_order;
  std::vector<int32_t>& order_host = side_ws ? h->side.order_host : h->order_host;
  OrderStage& order_pin = side_ws ? h->side.order_pin : h->order_pin;
  hipEvent_t& ws_done = side_ws ? h->side.ws_done : h->ws_done;
  bool& ws_rec = side_ws ? h->side.ws_rec : h->ws_rec;
  std::vector<hipEvent_t>& evv = side_ws ? h->side.ev : h->ev;
  int64_t launches_done = 0;
  if (o.dtype != CV_DTYPE_F32 && o.dtype != CV_DTYPE_F64) return set_err(CV_EINVAL, "bad dtype %d", o.dtype);
  if (o.assoc < CV_ASSOC_VITERBI || o.assoc > CV_ASSOC_DECODE) return set_err(CV_EINVAL, "bad assoc %d", o.assoc);
  const bool trellis_ok = o.dtype == CV_DTYPE_F32 && o.assoc == CV_ASSOC_VITERBI &&
                          cvk::trellis_padded_states(h->N) != 0;
  bool use_trellis;
  if (o.kernel == CV_KERNEL_TRELLIS) {
    if (!trellis_ok)
      return set_err(CV_EUNSUPPORTED, "trellis kernel needs dtype f32, assoc VITERBI and N <= 256");
    use_trellis = true;
  } else if (o.kernel == CV_KERNEL_GENERIC || o.kernel == CV_KERNEL_AUTO || o.kernel == CV_KERNEL_TRELLIS_F64) {
    use_trellis = o.kernel == CV_KERNEL_AUTO && trellis_ok;
  } else {
    return set_err(CV_EINVAL, "bad kernel %d", o.kernel);
  }
  // exact f64, row-A0 association, N <= 256, no forced states: trellis_fwd_f64 (one wave per
  // S sequences) unless the generic kernel is asked for
  // VITERBI (row A0), DECODE (row 0 = 0.0) and DP ((a + b) + d) share trellis_fwd_f64 +
  // backtrack_f64; CP runs
  // trellis_cp_f64 (argmax in the forward pass) + generic_backtrack<double>
  // forced states / resume rows (the constrained decode): row A0 only (trellis_fwd_f64 EXT)
  // 256 < N <= 512 (cvk::t64_batch_states): VITERBI (forced states too) / DECODE / DP, where
  // the padded NP = 512 trellis beats the generic kernels: N >= 384 or >= 8,192 sequences
  // (4,096 x 128: N = 384 15.3 vs 15.8 ms, N = 320 15.4 vs 12.3; 16,384 x 128: N = 320 34.1
  // vs 46.7 ms, N = 512 35.8 vs 84.0 -- profiles/r04_large_n.txt); CV_T64_512=1 forces it
  // What the f64 trellis SUPPORTS (an explicit CV_KERNEL_TRELLIS_F64 request gets it) is wider
  // than what AUTO picks: 256 < N <= 512 only for N >= 384 or >= 8,192 sequences, 512 < N <=
  // 1,024 only above N = 724 (cvk::t64_batch_states; the generic kernels win below)
  const bool t512_pick = h->tuning.t64_512 == 1 || h->N >= 384 || nseq >= 8192;
  const bool small_ok = (o.assoc == CV_ASSOC_VITERBI || o.assoc == CV_ASSOC_DECODE || o.assoc == CV_ASSOC_CP ||
                         o.assoc == CV_ASSOC_DP) &&
                        (!(o.forced || resume_rows) || o.assoc == CV_ASSOC_VITERBI) && cvk::t64_padded_states(h->N) != 0;
  const bool big_ok = cvk::t64_support_states(h->N) >= 512 &&
                      (o.assoc == CV_ASSOC_VITERBI || ((o.assoc == CV_ASSOC_DECODE || o.assoc == CV_ASSOC_DP) && !o.forced)) &&
                      !resume_rows && !cp_init && !cp_last;
  const bool big_pick = cvk::t64_batch_states(h->N) >= 512 && (t512_pick || h->N > 512);
  const bool t64_ok = o.dtype == CV_DTYPE_F64 && (small_ok || big_ok);
  if (o.kernel == CV_KERNEL_TRELLIS_F64 && !t64_ok)
    return set_err(CV_EUNSUPPORTED,
                   "f64 trellis kernel needs dtype f64 and N <= 1024; above N = 256 only the VITERBI, DECODE and DP "
                   "associations, forced states only with VITERBI (N=%d, assoc %d)",
                   h->N, o.assoc);
  const bool use_t64 = !use_trellis && t64_ok &&
                       (o.kernel == CV_KERNEL_TRELLIS_F64 ||
                        (o.kernel == CV_KERNEL_AUTO && !(o.flags & CV_FLAG_NO_T64) && (small_ok || big_pick)));
  // above generic_max_states (10,240 f64 / 20,480 f32) the generic decode runs wide (two rows
  // per sequence in global memory, states over many workgroups, psi mode); psi is u16
  if (!use_trellis && !use_t64 && h->N > cvk::kGenericGlobalMaxStates)
    return set_err(CV_EUNSUPPORTED, "N=%d exceeds the generic kernel's u16 back-pointer range (N <= %d)", h->N,
                   cvk::kGenericGlobalMaxStates);
  // (the chain's certificates read the rows mode's rows: no wide decode for them below the limit)
  const bool gen_global =
      !use_trellis && !use_t64 &&
      (h->N > cvk::generic_max_states(o.dtype == CV_DTYPE_F64 ? 8 : 4) ||
       (!cp_cert && cvk::generic_wide(h->N, o.dtype == CV_DTYPE_F64 ? 8 : 4, nseq, o.assoc == CV_ASSOC_CP)));

  std::vector<int64_t> off_copy;
  if (!offsets_host) {
    off_copy.resize((size_t)nseq + 1);
    HIP_TRY(hipMemcpyAsync(off_copy.data(), offsets_dev, off_copy.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    offsets_host = off_copy.data();
  }
  cv_status st = check_batch(h, nseq, offsets_host);
  if (st != CV_OK) return st;

  const bool need_f64 = (o.rescore_f64 && o.dtype == CV_DTYPE_F32) || o.dtype == CV_DTYPE_F64;
  if (use_trellis && (st = ensure_trellis_tables(h)) != CV_OK) return st;
  if (need_f64 && (st = ensure_f64_tables(h)) != CV_OK) return st;
  if (!use_trellis && o.dtype == CV_DTYPE_F32 && (st = ensure_g32_tables(h)) != CV_OK) return st;
  if (use_t64 && (st = ensure_t64_tables(h)) != CV_OK) return st;
  const bool t64cp = use_t64 && o.assoc == CV_ASSOC_CP;

  // CV_FLAG_MFMA_TRELLIS (bit 0) and the MFMA tile bits 8-15 belonged to the retired
  // MFMA-assisted f32 trellis (slower than the all-VALU one on gfx950: DESIGN.md §3)
  if ((o.flags & 0x1u) || ((o.flags >> 8) & 0xFF))
    return set_err(CV_EUNSUPPORTED, "the MFMA-assisted trellis was retired (flags 0x%x)", o.flags);
  const bool wave = use_trellis && h->npw > 0 && !(o.flags & CV_FLAG_NO_WAVE);
  if (!side_ws) {
    h->last_launches = 0;
    h->last_kernel = use_trellis ? CV_KERNEL_TRELLIS : use_t64 ? CV_KERNEL_TRELLIS_F64 : CV_KERNEL_GENERIC;
    h->last_np = use_trellis ? (wave ? h->npw : h->np) : use_t64 ? h->np64 : 0;
    h->last_mt = gen_global ? 0 : -1;  // GENERIC: 0 = wide (states over workgroups)
  }
  // N <= 64: one wave per sequence, forward and backtrack fused (trellis_wave_f32) on tables
  // padded to npw = 16 * ceil(N / 16); its chunks run back to back on one stream (nothing to
  // overlap)
  if (nseq == 0) return CV_OK;
  // the workspace of the previous call on this handle may still be in use on another stream
  if (ws_rec) HIP_TRY(hipStreamWaitEvent(stream, ws_done, 0));
  HIP_TRY(hipMemsetAsync(status_dev, 0, (size_t)nseq, stream));

  // Per-element workspace bytes: trellis keeps f32 delta rows [NP]; generic keeps u16 psi [N].
  // f64 trellis: 2 KiB of delta per element at N = 256 and >= 16,384 sequences per launch for
  // 8 sequences per wave, so its default cap is larger (HBM3E: 288 GB per GPU)
  const uint64_t cap = o.workspace_bytes ? o.workspace_bytes
                                         : default_workspace_cap(w_main.bytes, use_t64 ? kDefaultWorkspaceT64 : kDefaultWorkspace);
  // generic kernels: rows mode (the delta rows, argmax recomputed along the path) for every
  // association but CP (whose values need the argmax in the forward pass); A/B knob
  // tuning key generic_rows = 0 (psi mode, bit-identical).  4,096 x 128 sequences:
  // N = 300 14.9 -> 11.5 ms, N = 512 28.7 -> 21.5 ms, N = 1,024 163 -> 139 ms
  // (profiles/r04_large_n.txt)
  const bool gen_rows =
      !use_trellis && !use_t64 && !gen_global && o.assoc != CV_ASSOC_CP && h->tuning.generic_rows != 0;
  if (cp_cert && !use_t64 && !(gen_rows && o.dtype == CV_DTYPE_F64))
    return set_err(CV_EUNSUPPORTED, "chain certificates need the f64 trellis or the generic kernels' rows mode");
  if (gen_rows && (st = o.dtype == CV_DTYPE_F64 ? ensure_at64(h) : ensure_at32(h)) != CV_OK) return st;
  const uint64_t per_elem = use_trellis ? (uint64_t)(wave ? h->npw : h->np) * 4
                           : (use_t64 && !t64cp) ? (uint64_t)h->np64 * 8
                           : gen_rows ? (uint64_t)h->N * (o.dtype == CV_DTYPE_F64 ? 8 : 4)
                                       : (uint64_t)h->N * 2;
  const int real_bytes = o.dtype == CV_DTYPE_F64 ? 8 : 4;
  const uint64_t total_elems = (uint64_t)(offsets_host[nseq] - offsets_host[0]);
  // Chunks (contiguous in the original order) are pipelined over two streams: the forward
  // pass of chunk k+1 runs while chunk k backtracks, out of a double-buffered workspace.
  // At least ~2,048 sequences per chunk (8 per CU), at most 8 chunks unless the
  // workspace cap forces more.
  // t64 runs serial: its 212-VGPR forward waves fill each SIMD exactly twice per launch and
  // saturate the VALU; a co-running backtrack cost more than it hid (config 4: 159.8 ms with a
  // persistent one-wave-per-SIMD backtrack vs 152.4 ms serial, profiles/r02_ab_t64_overlap.txt)
  const bool serial = (o.flags & CV_FLAG_SERIAL) != 0 || wave || use_t64 || side_ws;
  // Sequences per forward workgroup: 2 (trellis_fwd2_f32, equal-length pairs; default) or 1
  // (trellis_fwd_f32: leftovers, N not a multiple of 64).
  const bool plain = use_trellis && !wave && cvk::trellis_pair_supported(h->np);
  const int group = (!plain || (o.flags & CV_FLAG_NO_PAIR)) ? 1 : 2;
  const uint64_t max_chunks = [&] {  // tuning key max_chunks (bit-identical): pipeline depth
    const int v = h->tuning.max_chunks;
    return (uint64_t)(v >= 1 && v <= 64 ? v : 8);
  }();
  const uint64_t half_cap = std::max<uint64_t>(serial ? cap : cap / 2, per_elem);
  uint64_t nchunks = std::max<uint64_t>(1, (total_elems * per_elem + half_cap - 1) / half_cap);
  if (!serial) nchunks = std::max<uint64_t>(nchunks, std::min<uint64_t>(max_chunks, (uint64_t)(nseq / 2048)));
  const uint64_t target = std::max<uint64_t>(1, (total_elems + nchunks - 1) / nchunks);
  const uint64_t elem_cap = std::max<uint64_t>(half_cap / per_elem, 1);
  std::vector<std::pair<int64_t, int64_t>> chunks;
  {
    int64_t s0 = 0;
    while (s0 < nseq) {
      int64_t s1 = s0;
      uint64_t elems = 0;
      while (s1 < nseq) {
        const uint64_t T = (uint64_t)(offsets_host[s1 + 1] - offsets_host[s1]);
        if (s1 > s0 && (elems + T > elem_cap || elems + T > target)) break;
        elems += T;
        ++s1;
        if (s1 - s0 >= (1 << 30)) break;
      }
      chunks.emplace_back(s0, s1);
      s0 = s1;
    }
  }
  {
    // Equal lengths: whole rounds of workgroups (group x CUs sequences) per chunk, so only
    // the last chunk ends on a partly filled round (a chunk's launch waits for the last).
    const int64_t T0c = offsets_host[1] - offsets_host[0];
    bool uniform = T0c > 0;
    for (int64_t s = 1; s < nseq && uniform; ++s) uniform = (offsets_host[s + 1] - offsets_host[s]) == T0c;
    const int64_t unit = (use_t64 ? 64 : group) * (int64_t)std::max(h->cus, 1);
    if (uniform && chunks.size() > 1) {
      const int64_t cap_seqs = std::max<int64_t>((int64_t)(elem_cap / (uint64_t)T0c), 1);
      int64_t per = (nseq + (int64_t)chunks.size() - 1) / (int64_t)chunks.size();
      per = ((per + unit - 1) / unit) * unit;
      if (per > cap_seqs) per = cap_seqs >= unit ? (cap_seqs / unit) * unit : cap_seqs;
      chunks.clear();
      for (int64_t s0 = 0; s0 < nseq; s0 += per) chunks.emplace_back(s0, std::min(nseq, s0 + per));
    }
  }
  uint64_t max_elems = 0;
  int64_t max_seqs = 0;
  bool varlen = false;
  for (auto& c : chunks) {
    max_elems = std::max<uint64_t>(max_elems, (uint64_t)(offsets_host[c.second] - offsets_host[c.first]));
    max_seqs = std::max<int64_t>(max_seqs, c.second - c.first);
  }
  const int nbuf = (chunks.size() > 1 && !serial) ? 2 : 1;
  const int64_t T0 = offsets_host[1] - offsets_host[0];
  for (int64_t s = 1; s < nseq && !varlen; ++s) varlen = (offsets_host[s + 1] - offsets_host[s]) != T0;
  const size_t buf_bytes = ((std::max<uint64_t>(max_elems, 1) * per_elem + 255) / 256) * 256;
  // gen_global: each sequence's two rows follow the chunk's last rows ([max_seqs][2][N])
  const size_t last_bytes = ((size_t)max_seqs * h->N * real_bytes * (gen_global ? 3 : 1) + 255) / 256 * 256;
  if ((st = w_main.ensure(buf_bytes * nbuf)) != CV_OK) return st;
  if (!use_trellis && (st = w_last.ensure(last_bytes * nbuf)) != CV_OK) return st;
  const int32_t* order_dev = nullptr;
  // group == 2: chunk slots [first, first + 2*npair) hold equal-length pairs, the rest run
  // one per workgroup.
  const bool pairing = group == 2;
  std::vector<int64_t> npair(chunks.size(), 0);
  if (varlen) {
    // longest-first schedule inside each chunk so the tail of the grid is short sequences;
    // with pairing, equal-length neighbours are paired first and leftovers go last
    order_host.resize((size_t)nseq);
    std::vector<int32_t> tail;
    for (size_t ci = 0; ci < chunks.size(); ++ci) {
      const auto& c = chunks[ci];
      auto b = order_host.begin() + c.first, e = order_host.begin() + c.second;
      auto len = [&](int32_t x) { return offsets_host[x + 1] - offsets_host[x]; };
      // stable longest-first: a counting sort on the lengths (a comparison sort of 16,384
      // sequences cost ~1 ms of host time per call), a stable sort for very long lengths
      int64_t maxlen = 0;
      for (int64_t x = c.first; x < c.second; ++x) maxlen = std::max<int64_t>(maxlen, len((int32_t)x));
      if (maxlen <= 4 * (c.second - c.first) + (1 << 16)) {
        std::vector<int64_t>& pos = h->sort_pos;
        pos.assign((size_t)maxlen + 2, 0);
        for (int64_t x = c.first; x < c.second; ++x) ++pos[(size_t)(maxlen - len((int32_t)x)) + 1];
        for (size_t k = 1; k < pos.size(); ++k) pos[k] += pos[k - 1];
        for (int64_t x = c.first; x < c.second; ++x) b[pos[(size_t)(maxlen - len((int32_t)x))]++] = (int32_t)x;
      } else {
        std::iota(b, e, (int32_t)c.first);
        std::stable_sort(b, e, [&](int32_t x, int32_t y) { return len(x) > len(y); });
      }
      if (!pairing) continue;
      tail.clear();
      auto out = b;
      for (auto it = b; it != e;) {
        if (it + 1 != e && len(*it) == len(*(it + 1))) {
          *out++ = *it++;
          *out++ = *it++;
        } else {
          tail.push_back(*it++);
        }
      }
      npair[ci] = (out - b) / 2;
      std::copy(tail.begin(), tail.end(), out);
    }
    if ((st = w_order.ensure((size_t)nseq * 4)) != CV_OK) return st;
    int32_t* pin = order_pin.acquire((size_t)nseq);
    if (!pin) return set_err(CV_ENOMEM, "pinned staging of %lld order entries failed", (long long)nseq);
    std::memcpy(pin, order_host.data(), (size_t)nseq * 4);
    HIP_TRY(hipMemcpyAsync(w_order.p, pin, (size_t)nseq * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(order_pin.release(stream));
    order_dev = w_order.as<int32_t>();
  }

  hipStream_t bts = serial ? stream : h->bt_stream;
  const size_t nev = 4 * chunks.size();
  // events of this call: from 0 (each call overwrites the last), or appended after the calls
  // already timed since cv_timing_begin
  if (!side_ws && h->acc_on && h->acc_used + nev > kMaxTimedEvents) h->acc_on = false, h->acc_overflow = true;
  const size_t eb = (!side_ws && h->acc_on) ? h->acc_used : 0;
  if (!side_ws) h->last_ev_base = eb;
  for (size_t i = 0; i < nev; ++i)
    if (!get_event(evv, eb + i)) return set_err(CV_EDEVICE, "hipEventCreate failed");
  // the f64 trellis backtrack of one chunk (backtrack_f64, or fused into the N <= 64 forward)
  auto t64_bt_args = [&](const std::pair<int64_t, int64_t>& c, unsigned char* wsb) {
    cvk::T64BtArgs ba{};
    ba.delta = reinterpret_cast<const double*>(wsb);
    ba.delta_elem_base = offsets_host[c.first];
    ba.at = h->q_at.as<double>();
    ba.offsets = offsets_dev;
    ba.order = order_dev;
    ba.seq_begin = c.first;
    ba.seq_end = c.second;
    ba.nstates = h->N;
    ba.path = path_dev;
    ba.score = score_dev;  // the f64 delta is already the reference score: no re-score
    ba.status = status_dev;
    ba.dp_assoc = o.assoc == CV_ASSOC_DP ? 1 : 0;
    ba.decode_bt = o.assoc == CV_ASSOC_DECODE ? 1 : 0;
    ba.obs = obs_dev;
    ba.et = h->q_et.as<double>();
    ba.at32 = h->t64_nonpos ? h->q_at32.as<float>() : nullptr;
    return ba;
  };
  for (size_t ci = 0; ci < chunks.size(); ++ci) {
    const auto& c = chunks[ci];
    const int64_t n = c.second - c.first;
    const int buf = nbuf == 2 ? (int)(ci % 2) : 0;
    unsigned char* wsb = w_main.as<unsigned char>() + buf * buf_bytes;
    unsigned char* lrb = w_last.as<unsigned char>() + buf * last_bytes;
    hipEvent_t f0 = evv[eb + 4 * ci], f1 = evv[eb + 4 * ci + 1], b0 = evv[eb + 4 * ci + 2], b1 = evv[eb + 4 * ci + 3];
    if (!serial && ci >= 2) HIP_TRY(hipStreamWaitEvent(stream, evv[eb + 4 * (ci - 2) + 3], 0));  // buffer reuse
    HIP_TRY(hipEventRecord(f0, stream));
    hipError_t err;
    if (use_trellis) {
      cvk::TrellisFwdArgs fa{};
      fa.a_img = h->t_aimg.as<float>();
      fa.pi = h->t_pi.as<float>();
      fa.et = h->t_et.as<float>();
      fa.offsets = offsets_dev;
      fa.obs = obs_dev;
      fa.order = order_dev;
      fa.seq_begin = c.first;
      fa.delta = reinterpret_cast<float*>(wsb);
      fa.delta_elem_base = offsets_host[c.first];
      fa.status = status_dev;
      fa.nobs = (int)h->V;
      fa.forced = o.forced;
      fa.resume_rows = static_cast<const float*>(resume_rows);
      if (wave) {
        fa.a_img = h->w_arm.as<float>();
        fa.pi = h->w_pi.as<float>();
        fa.et = h->w_et.as<float>();
        cvk::BacktrackArgs ba =
            make_bt_args(h, wsb, offsets_host, offsets_dev, obs_dev, order_dev, c, path_dev, score_dev, status_dev);
        ba.at = h->w_at.as<float>();
        err = cvk::launch_trellis_wave(h->npw, fa, ba, n, stream);
      } else {
        const int64_t np2 = pairing ? (varlen ? npair[ci] : n / 2) : 0;
        err = cvk::launch_trellis_fwd2(h->np, fa, np2, stream);
        if (err == hipSuccess && n > 2 * np2) {
          fa.seq_begin = c.first + 2 * np2;
          err = cvk::launch_trellis_fwd(h->np, fa, n - 2 * np2, stream);
        }
      }
    } else if (use_t64) {
      cvk::T64FwdArgs fa{};
      fa.a = h->q_a.as<double>();
      fa.pi = h->q_pi.as<double>();
      fa.et = h->q_et.as<double>();
      fa.offsets = offsets_dev;
      fa.obs = obs_dev;
      fa.order = order_dev;
      fa.seq_begin = c.first;
      fa.nslots = n;
      fa.delta = reinterpret_cast<double*>(wsb);
      fa.delta_elem_base = offsets_host[c.first];
      fa.status = status_dev;
      fa.nobs = (int)h->V;
      fa.zero_init = o.assoc == CV_ASSOC_DECODE ? 1 : 0;
      fa.dp_assoc = o.assoc == CV_ASSOC_DP ? 1 : 0;
      fa.forced = o.forced;
      fa.resume_rows = static_cast<const double*>(resume_rows);
      const int spw = cvk::t64_seqs_per_wave(n, h->cus, h->np64);
      // the S actually launched: CP / DP, NP = 1,024 and forced NP = 512 run S <= 4 (launch_t64_fwd)
      if (!side_ws)
        h->last_mt = t64cp ? cvk::t64_cp_seqs_per_wave(spw, n, cvk::t64_cp_waves(h->np64, n))
                           : (fa.dp_assoc || h->np64 == 1024 || (h->np64 == 512 && o.forced)) ? std::min(spw, 4) : spw;
      {  // eight-wave workgroups: equal lengths (within 1/8), or >= 2 rounds of 64 x CUs
         // (ragged T in [32, 1024], chunks of 32,768: 158 vs 168 ms; one round, 16,384: 65.5
         // vs 56 ms -- profiles/r03_ab_wg.txt)
        int64_t tmin = INT64_MAX, tmax = 0;
        for (int64_t sq = c.first; sq < c.second; ++sq) {
          const int64_t T = offsets_host[sq + 1] - offsets_host[sq];
          tmin = std::min(tmin, T);
          tmax = std::max(tmax, T);
        }
        fa.wg_ok = (8 * tmin >= 7 * tmax || n >= 2 * 64 * (int64_t)std::max(h->cus, 1)) ? 1 : 0;
      }
      if (t64cp) {
        fa.nstates = h->N;
        fa.psi = reinterpret_cast<uint16_t*>(wsb);
        fa.last_row = reinterpret_cast<double*>(lrb);
        fa.cp_init = cp_init;  // the parallel chain's speculative re-decodes (start offsets)
        fa.cp_last = cp_last;
        err = cvk::launch_t64_cp_fwd(h->np64, spw, fa, n, stream);
      } else {
        fa.nstates = h->N;  // the N <= 48 one-wave kernel
        err = cvk::launch_t64_fwd(h->np64, spw, fa, n, stream);
      }
    } else if (o.dtype == CV_DTYPE_F64) {
      cvk::GenericFwdArgs<double> fa{};
      fa.a = h->d_a64.as<double>();
      fa.pi = h->d_pi64.as<double>();
      fa.et = h->d_et64.as<double>();
      fa.offsets = offsets_dev;
      fa.obs = obs_dev;
      fa.order = order_dev;
      fa.seq_begin = c.first;
      fa.nstates = h->N;
      fa.nobs = (int)h->V;
      fa.assoc = o.assoc;
      fa.psi = reinterpret_cast<uint16_t*>(wsb);
      fa.psi_elem_base = offsets_host[c.first];
      fa.last_row = reinterpret_cast<double*>(lrb);
      fa.status = status_dev;
      fa.forced = o.forced;
      fa.cp_init = cp_init;  // the parallel chain's speculative re-decodes (N > 256)
      fa.cp_last = cp_last;
      if (gen_rows) fa.rows = reinterpret_cast<double*>(wsb);
      if (gen_global) {  // wide: the chunk's rows after its last rows, one launch per step
        fa.grows = reinterpret_cast<double*>(lrb) + (size_t)max_seqs * h->N;
        for (int64_t sq = c.first; sq < c.second; ++sq)
          fa.wide_steps = std::max<int64_t>(fa.wide_steps, offsets_host[sq + 1] - offsets_host[sq]);
      }
      err = cvk::launch_generic_fwd<double>(fa, n, stream);
    } else {
      cvk::GenericFwdArgs<float> fa{};
      fa.a = h->d_a32.as<float>();
      fa.pi = h->d_pi32.as<float>();
      fa.et = h->d_et32.as<float>();
      fa.offsets = offsets_dev;
      fa.obs = obs_dev;
      fa.order = order_dev;
      fa.seq_begin = c.first;
      fa.nstates = h->N;
      fa.nobs = (int)h->V;
      fa.assoc = o.assoc;
      fa.psi = reinterpret_cast<uint16_t*>(wsb);
      fa.psi_elem_base = offsets_host[c.first];
      fa.last_row = reinterpret_cast<float*>(lrb);
      fa.status = status_dev;
      fa.forced = o.forced;
      if (gen_rows) fa.rows = reinterpret_cast<float*>(wsb);
      if (gen_global) {  // wide: the chunk's rows after its last rows, one launch per step
        fa.grows = reinterpret_cast<float*>(lrb) + (size_t)max_seqs * h->N;
        for (int64_t sq = c.first; sq < c.second; ++sq)
          fa.wide_steps = std::max<int64_t>(fa.wide_steps, offsets_host[sq + 1] - offsets_host[sq]);
      }
      err = cvk::launch_generic_fwd<float>(fa, n, stream);
    }
    if (err != hipSuccess) return set_err(CV_EDEVICE, "forward launch failed: %s", hipGetErrorString(err));
    HIP_TRY(hipEventRecord(f1, stream));
    if (!serial) HIP_TRY(hipStreamWaitEvent(bts, f1, 0));
    HIP_TRY(hipEventRecord(b0, bts));
    if (use_trellis) {
      const cvk::BacktrackArgs ba =
          make_bt_args(h, wsb, offsets_host, offsets_dev, obs_dev, order_dev, c, path_dev, score_dev, status_dev);
      // overlap mode: at most ONE backtrack workgroup (one 64-VGPR wave per SIMD) per CU, so
      // the next forward workgroup (4 waves x 104 VGPRs per SIMD) always
      // finds its registers free: reserve 100 KiB of LDS (2 x 100 > 160 KiB)
      // the last chunk's backtrack has the device to itself: full occupancy
      const int reserve = (serial || ci + 1 == chunks.size()) ? 0 : 100 * 1024;
      err = wave ? hipSuccess : cvk::launch_trellis_bt(h->np, ba, n, bts, reserve);  // wave: fused
      if (err == hipSuccess && o.rescore_f64) {
        cvk::RescoreArgs ra{};
        ra.path = path_dev;
        ra.obs = obs_dev;
        ra.offsets = offsets_dev;
        ra.order = order_dev;
        ra.seq_begin = c.first;
        ra.seq_end = c.second;
        ra.nstates = h->N;
        ra.pi64 = h->d_pi64.as<double>();
        ra.a64 = h->d_a64.as<double>();
        ra.et64 = h->d_et64.as<double>();
        ra.status = status_dev;
        ra.score = score_dev;
        err = cvk::launch_rescore_f64(ra, n, bts, reserve);
      }
    } else if (use_t64 && !t64cp) {
      cvk::T64BtArgs ba = t64_bt_args(c, wsb);
      // the parallel chain's certificates inside the backtrack (NONPOS row A0, NP <= 256): no
      // second pass over every row (tuning key chain_cert_fused = 0: the cp_cert_f64 pass)
      const bool fused_cert = cp_cert && ba.at32 && !ba.dp_assoc && !ba.decode_bt && h->np64 <= 256 &&
                              h->tuning.chain_cert_fused != 0;
      if (fused_cert) {
        ba.cert = cp_cert;
        ba.rho_cap = h->cert_rho_cap;
      }
      err = cvk::launch_t64_bt(h->np64, ba, n, bts);
      if (err == hipSuccess && chunks_out) {
        hipEvent_t ce = get_event(h->chunk_ev, chunks_out->size());
        if (!ce) return set_err(CV_EDEVICE, "hipEventCreate failed");
        HIP_TRY(hipEventRecord(ce, bts));
        chunks_out->push_back(c);
      }
      if (err == hipSuccess && cp_cert && !fused_cert) {
        cvk::CpCert64Args ca{};
        ca.delta = reinterpret_cast<const double*>(wsb);
        ca.delta_elem_base = offsets_host[c.first];
        ca.at = h->q_at.as<double>();
        ca.offsets = offsets_dev;
        ca.order = order_dev;
        ca.seq_begin = c.first;
        ca.seq_end = c.second;
        ca.nstates = h->N;
        ca.path = path_dev;
        ca.status = status_dev;
        ca.out = cp_cert;
        err = cvk::launch_cp_cert(h->np64, ca, bts);
      }
    } else if (o.dtype == CV_DTYPE_F64) {
      cvk::GenericBtArgs<double> ba{};
      ba.psi = reinterpret_cast<const uint16_t*>(wsb);
      ba.psi_elem_base = offsets_host[c.first];
      ba.last_row = reinterpret_cast<const double*>(lrb);
      ba.offsets = offsets_dev;
      ba.order = order_dev;
      ba.seq_begin = c.first;
      ba.seq_end = c.second;
      ba.nstates = h->N;
      ba.path = path_dev;
      ba.score = score_dev;
      ba.status = status_dev;
      ba.obs = obs_dev;
      ba.rescore_f64 = 0;  // the f64 kernel's own score is already reference numerics
      ba.decode_bt = o.assoc == CV_ASSOC_DECODE ? 1 : 0;
      ba.pi64 = h->d_pi64.as<double>();
      ba.a64 = h->d_a64.as<double>();
      ba.et64 = h->d_et64.as<double>();
      if (gen_rows) {
        ba.rows = reinterpret_cast<const double*>(wsb);
        ba.at = h->d_at64.as<double>();
        ba.et = h->d_et64.as<double>();
        ba.assoc = o.assoc;
        ba.nobs = (int)h->V;
      }
      err = gen_rows ? cvk::launch_generic_bt_rows<double>(ba, n, bts) : cvk::launch_generic_bt<double>(ba, n, bts);
      if (err == hipSuccess && chunks_out) {
        hipEvent_t ce = get_event(h->chunk_ev, chunks_out->size());
        if (!ce) return set_err(CV_EDEVICE, "hipEventCreate failed");
        HIP_TRY(hipEventRecord(ce, bts));
        chunks_out->push_back(c);
      }
      if (err == hipSuccess && cp_cert) {  // the parallel chain (N > 256): certificates over the plain rows
        cvk::CpCert64Args ca{};
        ca.delta = reinterpret_cast<const double*>(wsb);
        ca.delta_elem_base = offsets_host[c.first];
        ca.at = h->d_at64.as<double>();
        ca.offsets = offsets_dev;
        ca.order = order_dev;
        ca.seq_begin = c.first;
        ca.seq_end = c.second;
        ca.nstates = h->N;
        ca.path = path_dev;
        ca.status = status_dev;
        ca.out = cp_cert;
        err = cvk::launch_cp_cert_plain(ca, bts);
      }
    } else {
      cvk::GenericBtArgs<float> ba{};
      ba.psi = reinterpret_cast<const uint16_t*>(wsb);
      ba.psi_elem_base = offsets_host[c.first];
      ba.last_row = reinterpret_cast<const float*>(lrb);
      ba.offsets = offsets_dev;
      ba.order = order_dev;
      ba.seq_begin = c.first;
      ba.seq_end = c.second;
      ba.nstates = h->N;
      ba.path = path_dev;
      ba.score = score_dev;
      ba.status = status_dev;
      ba.obs = obs_dev;
      ba.rescore_f64 = o.rescore_f64 ? 1 : 0;
      ba.decode_bt = o.assoc == CV_ASSOC_DECODE ? 1 : 0;
      ba.pi64 = h->d_pi64.as<double>();
      ba.a64 = h->d_a64.as<double>();
      ba.et64 = h->d_et64.as<double>();
      if (gen_rows) {
        ba.rows = reinterpret_cast<const float*>(wsb);
        ba.at = h->d_at32.as<float>();
        ba.et = h->d_et32.as<float>();
        ba.assoc = o.assoc;
        ba.nobs = (int)h->V;
      }
      err = gen_rows ? cvk::launch_generic_bt_rows<float>(ba, n, bts) : cvk::launch_generic_bt<float>(ba, n, bts);
    }
    if (err != hipSuccess) return set_err(CV_EDEVICE, "backtrack launch failed: %s", hipGetErrorString(err));
    HIP_TRY(hipEventRecord(b1, bts));
    ++launches_done;
    if (!side_ws) h->last_launches = launches_done;
  }
  // the caller's stream sees the whole decode complete
  if (!serial) HIP_TRY(hipStreamWaitEvent(stream, evv[eb + 4 * (chunks.size() - 1) + 3], 0));
  if (!side_ws && h->acc_on) h->acc_used += nev;
  if (!ws_done) HIP_TRY(hipEventCreateWithFlags(&ws_done, hipEventDisableTiming));
  HIP_TRY(hipEventRecord(ws_done, stream));
  ws_rec = true;
  return CV_OK;
}

cv_opts default_opts() {
  cv_opts o;
  cv_opts_init(&o);
  return o;
}

}  // namespace

// ===================================================================================
extern "C" {

CV_API const char* cv_last_error(void) { return g_err.c_str(); }
CV_API const char* cv_version(void) { return "cviterbi 0.1.0 (gfx950)"; }
CV_API int32_t cv_abi_version(void) { return CV_ABI_VERSION; }
CV_API cv_status cv_device_memory(int64_t* current_bytes, int64_t* peak_bytes) {
  if (current_bytes) *current_bytes = g_dev_cur.load();
  if (peak_bytes) *peak_bytes = g_dev_peak.load();
  return CV_OK;
}
CV_API int32_t cv_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

CV_API void cv_opts_init(cv_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof *o);
  o->dtype = CV_DTYPE_F64;  // the reference's arithmetic (hmm.rs:10-18)
  o->assoc = CV_ASSOC_VITERBI;
  o->kernel = CV_KERNEL_AUTO;
  o->rescore_f64 = 1;
}

CV_API cv_status cv_hmm_create(const cv_hmm_desc* d, cv_hmm** out) {
  if (!d || !out) return set_err(CV_EINVAL, "null argument");
  if (d->ndims <= 0 || !d->bdims) return set_err(CV_EINVAL, "ndims/bdims required");
  std::vector<int64_t> bd(d->bdims, d->bdims + d->ndims);
  return make_hmm(d->nstates, bd, d->pi, d->a, d->b, d->device, out);
}

CV_API cv_status cv_hmm_from_json(const char* path, int32_t device, cv_hmm** out) {
  if (!path || !out) return set_err(CV_EINVAL, "null argument");
  std::string text, err;
  if (!cvh::read_file(path, text)) return set_err(CV_EIO, "cannot read %s", path);
  cvh::HmmJson j;
  if (!cvh::parse_hmm_json(text, j, err)) return set_err(CV_EPARSE, "%s", err.c_str());
  return make_hmm(j.nstates, j.bdims, j.pi.data(), j.a.data(), j.b.data(), device, out);
}

CV_API cv_status cv_hmm_write_json(const cv_hmm* h, const char* path) {
  if (!h || !path) return set_err(CV_EINVAL, "null argument");
  const std::string s = cvh::format_hmm_json(h->N, h->bdims, h->pi.data(), h->a.data(), h->b.data());
  FILE* f = fopen(path, "wb");
  if (!f) return set_err(CV_EIO, "cannot write %s", path);
  const size_t n = fwrite(s.data(), 1, s.size(), f);
  fclose(f);
  if (n != s.size()) return set_err(CV_EIO, "short write to %s", path);
  return CV_OK;
}

CV_API void cv_hmm_destroy(cv_hmm* h) {
  if (!h) return;
  int n = 0;
  if (hipGetDeviceCount(&n) == hipSuccess && h->device >= 0 && h->device < n) (void)hipSetDevice(h->device);
  delete h;
}

CV_API cv_status cv_hmm_set_tuning(cv_hmm* h, const char* key, int64_t value) {
  if (!h || !key) return set_err(CV_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(h->mu);
  if (!cvk::tuning_set(h->tuning, key, value)) return set_err(CV_EINVAL, "unknown tuning key '%s' or value out of range", key);
  if (std::strcmp(key, "t64_nonpos") == 0) {  // model_nonpos reads it: rebuild the f64 trellis tables
    h->nonpos_cache = -1;
    h->t64_ready = false;
  }
  return CV_OK;
}
CV_API cv_status cv_hmm_release_workspaces(cv_hmm* h) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  // every stream the workspaces were used on has drained before the memory goes
  for (hipStream_t s : {h->stream, h->bt_stream, h->side.stream, h->side.hi, h->copy_stream, h->chain_stream})
    if (s) HIP_TRY(hipStreamSynchronize(s));
  for (DevBuf* b : {&h->ws_main, &h->ws_last, &h->ws_order, &h->side.main, &h->side.last, &h->side.order,
                    &h->side.idx, &h->side.obs2, &h->side.path2, &h->side.res2, &h->st_off, &h->st_obs, &h->st_path,
                    &h->st_score, &h->st_status, &h->st_forced, &h->cs_ranges, &h->cs_delta, &h->cs_g, &h->cs_mu,
                    &h->cs_start, &h->cs_zero, &h->cs_queue, &h->cs_wrows, &h->cs_comp, &h->cs_words, &h->cs_flag,
                    &h->cs_seg, &h->rs_rows, &h->rs_rowbase, &h->rs_resume, &h->rs_start, &h->rs_off2, &h->rs_ridx,
                    &h->rs_slot, &h->rs_obs2, &h->rs_frc2, &h->rs_path2, &h->rs_srows, &h->rs_srowbase, &h->rs_cert,
                    &h->chainb.off, &h->chainb.obs, &h->chainb.path, &h->chainb.res, &h->chainb.cert, &h->chainb.ebin,
                    &h->chainb.q, &h->chainb.ends, &h->chainb.gid, &h->chainb.gpath, &h->chainb.first,
                    &h->chainb.rpsi, &h->chainb.rows, &h->chainb.small, &h->chainb.rpath, &h->chainb.soff,
                    &h->chainb.sobs, &h->chainb.spath, &h->chainb.sres, &h->chainb.sinit, &h->chainb.slast})
    b->release();
  h->ws_rec = false;
  h->side.ws_rec = false;
  h->chain_pin.release();
  h->chain_gpin.release();
  h->chain_obs_pin.release();
  h->chain_ring[0].release();
  h->chain_ring[1].release();
  return CV_OK;
}
CV_API cv_status cv_hmm_get_tuning(const cv_hmm* h, const char* key, int64_t* value) {
  if (!h || !key || !value) return set_err(CV_EINVAL, "bad argument");
  std::lock_guard<std::mutex> lk(const_cast<cv_hmm*>(h)->mu);
  if (!cvk::tuning_get(h->tuning, key, value)) return set_err(CV_EINVAL, "unknown tuning key '%s'", key);
  return CV_OK;
}
CV_API const char* cv_tuning_key(int32_t i) { return cvk::tuning_key(i); }
CV_API int32_t cv_hmm_nstates(const cv_hmm* h) { return h ? h->N : -1; }
CV_API int64_t cv_hmm_nobs(const cv_hmm* h) { return h ? h->V : -1; }
CV_API int32_t cv_hmm_ndims(const cv_hmm* h) { return h ? h->D : -1; }
CV_API cv_status cv_hmm_bdims(const cv_hmm* h, int64_t* out) {
  if (!h || !out) return set_err(CV_EINVAL, "null argument");
  std::copy(h->bdims.begin(), h->bdims.end(), out);
  return CV_OK;
}

CV_API cv_status cv_obs_flatten(const cv_hmm* h, const int64_t* value, int64_t* flat) {
  if (!h || !value || !flat) return set_err(CV_EINVAL, "null argument");
  int64_t f = 0;
  for (int d = 0; d < h->D; ++d) {
    if (value[d] < 0 || value[d] >= h->bdims[d])
      return set_err(CV_EINVAL, "observation component %d = %lld out of range [0,%lld)", d, (long long)value[d],
                     (long long)h->bdims[d]);
    f = f * h->bdims[d] + value[d];  // row-major, ndarray default (C) order
  }
  *flat = f;
  return CV_OK;
}

static bool lookup_ok(const cv_hmm* h, int32_t s, int64_t o) {
  return h && s >= 0 && s < h->N && o >= 0 && o < h->V;
}

CV_API double cv_hmm_init_prob(const cv_hmm* h, int32_t state, int64_t obs) {
  if (!lookup_ok(h, state, obs)) return NAN;
  return h->pi[state] + h->b[(size_t)state * h->V + obs];
}
CV_API cv_status cv_hmm_init_probs(const cv_hmm* h, int64_t obs, double* out) {
  if (!lookup_ok(h, 0, obs) || !out) return set_err(CV_EINVAL, "bad argument");
  for (int s = 0; s < h->N; ++s) out[s] = h->pi[s] + h->b[(size_t)s * h->V + obs];
  return CV_OK;
}
CV_API double cv_hmm_transition_prob(const cv_hmm* h, int32_t from, int32_t to, int64_t obs) {
  if (!lookup_ok(h, to, obs) || from < 0 || from >= h->N) return NAN;
  return h->a[(size_t)from * h->N + to] + h->b[(size_t)to * h->V + obs];
}
CV_API cv_status cv_hmm_transitions_to(const cv_hmm* h, int32_t to, double* out) {
  if (!h || to < 0 || to >= h->N || !out) return set_err(CV_EINVAL, "bad argument");
  for (int s = 0; s < h->N; ++s) out[s] = h->a[(size_t)s * h->N + to];
  return CV_OK;
}
CV_API double cv_hmm_emit_prob(const cv_hmm* h, int32_t state, int64_t obs) {
  if (!lookup_ok(h, state, obs)) return NAN;
  return h->b[(size_t)state * h->V + obs];
}
CV_API cv_status cv_hmm_emit_probs(const cv_hmm* h, int64_t obs, double* out) {
  if (!lookup_ok(h, 0, obs) || !out) return set_err(CV_EINVAL, "bad argument");
  for (int s = 0; s < h->N; ++s) out[s] = h->b[(size_t)s * h->V + obs];
  return CV_OK;
}

CV_API cv_status cv_decode_batch_device(cv_hmm* h, int64_t nseq, const int64_t* offsets_host,
                                        const int64_t* offsets_dev, const int32_t* obs_dev, const cv_opts* opts,
                                        int32_t* path_dev, double* score_dev, uint8_t* status_dev) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq > 0 && (!offsets_dev || !obs_dev || !path_dev || !score_dev || !status_dev))
    return set_err(CV_EINVAL, "null device buffer");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  const cv_opts o = opts ? *opts : default_opts();
  hipStream_t stream = o.stream ? (hipStream_t)o.stream : h->stream;
  return decode_device(h, nseq, offsets_host, offsets_dev, obs_dev, o, path_dev, score_dev, status_dev, stream);
}

// Host-pointer decode; caller holds h->mu and has selected the device.
// obs_staged: h->st_obs already holds the (validated) observations of [offsets[0],
// offsets[nseq]); forced_staged: o.forced is a validated DEVICE array indexed like obs.
static cv_status decode_host_locked(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs, cv_opts o,
                                    int32_t* path_out, double* score_out, uint8_t* status_out,
                                    bool obs_staged = false, bool forced_staged = false) {
  cv_status st;
  if (nseq == 0) return CV_OK;
  if ((st = check_batch(h, nseq, offsets)) != CV_OK) return st;
  const int64_t base = offsets[0];
  const int64_t total = offsets[nseq];  // obs/path are indexed by absolute element offset
  if (!obs_staged) {
    const int64_t V = h->V;
    const int64_t k = first_bad(base, total, [&](int64_t i) { return obs[i] < 0 || obs[i] >= V; });
    if (k >= 0)
      return set_err(CV_EINVAL, "obs[%lld] = %d out of range [0,%lld)", (long long)k, obs[k], (long long)h->V);
  }
  hipStream_t stream = o.stream ? (hipStream_t)o.stream : h->stream;
  if ((st = h->st_off.ensure((size_t)(nseq + 1) * 8)) != CV_OK) return st;
  if ((st = h->st_obs.ensure((size_t)std::max<int64_t>(total, 1) * 4)) != CV_OK) return st;
  if ((st = h->st_path.ensure((size_t)std::max<int64_t>(total, 1) * 4)) != CV_OK) return st;
  if ((st = h->st_score.ensure((size_t)nseq * 8)) != CV_OK) return st;
  if ((st = h->st_status.ensure((size_t)nseq)) != CV_OK) return st;
  HIP_TRY(hipMemcpyAsync(h->st_off.p, offsets, (size_t)(nseq + 1) * 8, hipMemcpyHostToDevice, stream));
  if (total > base && !obs_staged)
    HIP_TRY(hipMemcpyAsync(h->st_obs.as<int32_t>() + base, obs + base, (size_t)(total - base) * 4,
                           hipMemcpyHostToDevice, stream));
  if (o.forced && !forced_staged) {  // host forced[] -> device staging, indexed like obs
    const int32_t N = h->N;
    const int32_t* fr = o.forced;
    const int64_t k = first_bad(base, total, [&](int64_t i) { return fr[i] < -1 || fr[i] >= N; });
    if (k >= 0) return set_err(CV_EINVAL, "forced[%lld] = %d out of range [-1,%d)", (long long)k, o.forced[k], h->N);
    if ((st = h->st_forced.ensure((size_t)std::max<int64_t>(total, 1) * 4)) != CV_OK) return st;
    if (total > base)
      HIP_TRY(hipMemcpyAsync(h->st_forced.as<int32_t>() + base, o.forced + base, (size_t)(total - base) * 4,
                             hipMemcpyHostToDevice, stream));
    o.forced = h->st_forced.as<int32_t>();
  }
  st = decode_device(h, nseq, offsets, h->st_off.as<int64_t>(), h->st_obs.as<int32_t>(), o, h->st_path.as<int32_t>(),
                     h->st_score.as<double>(), h->st_status.as<uint8_t>(), stream);
  if (st != CV_OK) {
    (void)hipStreamSynchronize(stream);
    return st;
  }
  if (total > base)
    HIP_TRY(hipMemcpyAsync(path_out + base, h->st_path.as<int32_t>() + base, (size_t)(total - base) * 4,
                           hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipMemcpyAsync(score_out, h->st_score.p, (size_t)nseq * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipMemcpyAsync(status_out, h->st_status.p, (size_t)nseq, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  return CV_OK;
}

CV_API cv_status cv_decode_batch(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                 const cv_opts* opts, int32_t* path_out, double* score_out, uint8_t* status_out) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq < 0 || (nseq > 0 && (!offsets || !obs || !path_out || !score_out || !status_out)))
    return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  return decode_host_locked(h, nseq, offsets, obs, opts ? *opts : default_opts(), path_out, score_out, status_out);
}

// ---- consistency-constrained decode --------------------------------------------------------
// Spec: oracle/np_oracle.py constrained_decode; host search: csp.hpp.
}  // extern "C"

namespace {
constexpr uint64_t kCspNodeLimit = 20000000;  // branch-and-bound nodes per call
constexpr int64_t kSegmentSlots = 65536;      // segment-table rows per launch (64 MiB of rows)

struct ConSeq {
  int64_t seq;
  std::vector<int64_t> elems;  // constrained elements, ascending
};

// Constrained sequences in sequence order (per-worker lists concatenated in order), and the
// range check of the components in the same pass: returns the first element with a component
// outside [-1, ncomp), or -1.  One vectorised min / max / AND pass per sequence
// (hostscan.cpp); the positions only for sequences with a component >= 0.
int64_t build_conseq_checked(int64_t nseq, const int64_t* offsets, const int32_t* component, int32_t ncomp,
                             std::vector<ConSeq>& cs) {
  cs.clear();
  std::vector<std::vector<ConSeq>> part((size_t)host_threads());
  std::vector<int64_t> bad((size_t)host_threads(), -1);
  parallel_ranges(nseq, [&](int t, int64_t lo, int64_t hi) {
    for (int64_t s = lo; s < hi; ++s) {
      const int64_t n = offsets[s + 1] - offsets[s];
      const cvscan::SeqScan r = cvscan::scan_sequence(component + offsets[s], n, ncomp);
      if (r.bad >= 0) {
        bad[(size_t)t] = offsets[s] + r.bad;
        return;
      }
      if (!r.constrained) continue;  // every component is -1
      ConSeq q{s, {}};
      cvscan::constrained_positions(component + offsets[s], n, offsets[s], q.elems);
      part[(size_t)t].push_back(std::move(q));
    }
  }, 1024);
  for (int64_t b : bad)
    if (b >= 0) return b;  // workers hold ascending ranges
  for (auto& p : part)
    for (auto& c : p) cs.push_back(std::move(c));
  return -1;
}

// The same list for components already range-checked.
void build_conseq(int64_t nseq, const int64_t* offsets, const int32_t* component, std::vector<ConSeq>& cs) {
  cs.clear();
  std::vector<std::vector<ConSeq>> part((size_t)host_threads());
  parallel_ranges(nseq, [&](int t, int64_t lo, int64_t hi) {
    for (int64_t s = lo; s < hi; ++s) {
      ConSeq c{s, {}};
      cvscan::constrained_positions(component + offsets[s], offsets[s + 1] - offsets[s], offsets[s], c.elems);
      if (!c.elems.empty()) part[t].push_back(std::move(c));
    }
  }, 1024);
  for (auto& p : part)
    for (auto& c : p) cs.push_back(std::move(c));
}

// Pairs (c1 < c2) of different components at consecutive constrained elements, sorted and
// unique -- cvcsp::component_pairs restricted to the constrained elements.
std::vector<int32_t> conseq_pairs(const std::vector<ConSeq>& cs, const int32_t* component) {
  std::vector<std::pair<int32_t, int32_t>> ps;
  for (const auto& c : cs)
    for (size_t k = 0; k + 1 < c.elems.size(); ++k) {
      const int32_t a = component[c.elems[k]], b = component[c.elems[k + 1]];
      if (a != b) ps.emplace_back(std::min(a, b), std::max(a, b));
    }
  std::sort(ps.begin(), ps.end());
  ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
  std::vector<int32_t> out;
  out.reserve(ps.size() * 2);
  for (auto& p : ps) out.push_back(p.first), out.push_back(p.second);
  return out;
}

// The constrained decode's arithmetic: the row-A0 association (the terms of csp.hpp are
// defined on it) in f64 -- the reference's precision: trellis_fwd_f64 for N <= 256, the
// generic kernels above (generic_ext + generic_fwd, wide above N = 10,240, N <= 65,535) -- or
// f32 (the f32 trellis, N <= 256).
bool constrained_generic(const cv_hmm* h, const cv_opts& o) {
  return o.dtype == CV_DTYPE_F64 && !cvk::t64_padded_states(h->N);
}

cv_status constrained_dtype_check(const cv_hmm* h, const cv_opts& o) {
  if (o.assoc != CV_ASSOC_VITERBI)
    return set_err(CV_EUNSUPPORTED, "constrained decode runs the row-A0 (VITERBI) association");
  if (o.dtype == CV_DTYPE_F64 && (cvk::t64_padded_states(h->N) || h->N <= cvk::kGenericGlobalMaxStates)) return CV_OK;
  if (o.dtype == CV_DTYPE_F32 && cvk::trellis_padded_states(h->N)) return CV_OK;
  return set_err(CV_EUNSUPPORTED, "constrained decode needs f64 with N <= %d, or f32 with N <= 256 (N=%d)",
                 cvk::kGenericGlobalMaxStates, h->N);
}

cv_status constrained_validate(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                               const int32_t* component, int32_t ncomp, const cv_opts& o, std::vector<ConSeq>& cs) {
  if ((cv_status)constrained_dtype_check(h, o) != CV_OK) return CV_EUNSUPPORTED;
  if (o.forced) return set_err(CV_EINVAL, "opts->forced is set by the constrained decode itself");
  cs.clear();
  if (nseq == 0) return CV_OK;
  cv_status st;
  if ((st = check_batch(h, nseq, offsets)) != CV_OK) return st;
  {
    const int64_t V = h->V;
    int64_t k = first_bad(offsets[0], offsets[nseq], [&](int64_t i) { return obs[i] < 0 || obs[i] >= V; });
    if (k >= 0)
      return set_err(CV_EINVAL, "obs[%lld] = %d out of range [0,%lld)", (long long)k, obs[k], (long long)h->V);
    k = first_bad(offsets[0], offsets[nseq], [&](int64_t i) { return component[i] < -1 || component[i] >= ncomp; });
    if (k >= 0)
      return set_err(CV_EINVAL, "component[%lld] = %d out of range [-1,%d)", (long long)k, component[k], ncomp);
  }
  build_conseq(nseq, offsets, component, cs);
  return CV_OK;
}

// Device passes of one shard + exact accumulation into its partials (csp.hpp layout;
// `part` is zeroed by the caller).  Per sequence with constrained elements t_1 < .. < t_m:
//   m == 1: mu = delta_{t_1} + beta  -> unary of c_1
//   m >= 2: alpha = delta_{t_1} -> unary c_1; beta -> unary c_m; segment tables M_k -> the
//           pair (c_k, c_{k+1}) (or the diagonal into the unary when c_k == c_{k+1}).
// `pre`: the caller's already validated constrained-sequence list (else validated here);
// on return *obs_staged tells whether h->st_obs holds the batch's observations.
// What the terms pass leaves on the device for the resume flow (forced_decode_resume): the
// delta rows of every prefix [offsets[seq], t_1] (h->rs_rows, slot i from row row_base[i]) and
// row t_1 itself (h->cs_delta row i).
struct PrefixKeep {
  bool kept = false;
  std::vector<int64_t> seq, t1, row_base;  // per terms slot i
  // f64: the suffix pass's rows are kept too (h->rs_srows, slot i from row srow_base[i]) for
  // the certified suffix trace, which reads the one-element slots [0, n1) only; the pass writes
  // every slot's rows, so the multi-element slots' rows are stored (and counted in the
  // free-memory check) as well -- few at config 5, where every sequence has one element
  bool suffix_kept = false;
  int64_t n1 = 0;
};

// The certified suffix trace (suffix_trace_f64) replaces the resume flow's second forward pass
// for one-position sequences: f64, models whose finite entries are all in [-2^80, 0].  Tuning key
// (bit-identical): no_trace = 1.
bool trace_supported(const cv_hmm* h) { return h->tuning.no_trace == 0 && h->t64_nonpos; }

// The resume flow covers f32 N > 64 with NP % 64 == 0 (pair kernel + backtrack_v) and every f64
// N <= 256; its stored rows must fit 4x the workspace cap (32 GiB by default: config 5 needs
// 8.6 GB of f32 rows; f64 rows are twice that, within the f64 trellis's 64 GiB cap x 4).
bool resume_supported(const cv_hmm* h, bool f64) {
  if (h->tuning.no_resume != 0) return false;  // tuning key (bit-identical)
  if (f64) return cvk::t64_padded_states(h->N) != 0;  // trellis_fwd_f64 EXT + prefix_backtrack_f64
  return h->N > 64 && (h->np == 128 || h->np == 192 || h->np == 256);
}

cv_status constrained_partials_locked(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                      const int32_t* component, int32_t ncomp, const int32_t* pairs, int64_t npairs,
                                      cv_opts& o, int64_t* part, const std::vector<ConSeq>* pre = nullptr,
                                      bool* obs_staged = nullptr, const int32_t* obs_dev = nullptr,
                                      PrefixKeep* keep = nullptr,
                                      const std::function<cv_status()>& after_terms = nullptr) {
  if (keep) *keep = PrefixKeep{};
  h->last_traced = 0;
  if (obs_staged) *obs_staged = false;
  std::vector<ConSeq> own;
  cv_status st = CV_OK;
  if (!pre && (st = constrained_validate(h, nseq, offsets, obs, component, ncomp, o, own)) != CV_OK) return st;
  const std::vector<ConSeq>& cs = pre ? *pre : own;
  if (cs.empty()) return CV_OK;
  const int N = (int)h->N;
  const int64_t uw = cvcsp::unary_words(N), pw = cvcsp::pair_words(N);
  int64_t* pbase = part + (int64_t)ncomp * uw;
  // pair lookups first: a missing pair is a caller error, found before any device work
  std::vector<int64_t> seg_pair;  // per segment: pair index, or -1 for a same-component segment
  for (const auto& c : cs)
    for (size_t k = 0; k + 1 < c.elems.size(); ++k) {
      const int32_t c1 = component[c.elems[k]], c2 = component[c.elems[k + 1]];
      if (c1 == c2) {
        seg_pair.push_back(-1);
        continue;
      }
      const int64_t p = cvcsp::pair_index(pairs, npairs, std::min(c1, c2), std::max(c1, c2));
      if (p < 0) return set_err(CV_EINVAL, "component pair (%d,%d) missing from the pair list", c1, c2);
      seg_pair.push_back(p);
    }
  const bool f64 = o.dtype == CV_DTYPE_F64;
  const bool gen = constrained_generic(h, o);  // f64, N > 256: generic_ext passes, rows of N
  if (!f64 && (st = ensure_trellis_tables(h)) != CV_OK) return st;
  if (f64 && !gen && (st = ensure_t64_tables(h)) != CV_OK) return st;
  if ((st = ensure_f64_tables(h)) != CV_OK) return st;
  if (gen && (st = ensure_at64(h)) != CV_OK) return st;
  const int np = gen ? N : f64 ? h->np64 : h->np;
  const size_t rb = f64 ? 8 : 4;  // bytes per term
  hipStream_t stream = o.stream ? (hipStream_t)o.stream : h->stream;
  // h->ws_order below is the main workspace's: a cv_decode_batch_device call still running on
  // another stream reads it (cviterbi.h promises cross-stream workspace ordering)
  if (h->ws_rec) HIP_TRY(hipStreamWaitEvent(stream, h->ws_done, 0));
  const int64_t base = offsets[0], total = offsets[nseq];
  // observations on the device: the caller's (device API, validated) or staged here
  const int32_t* dobs = obs_dev;
  if (!dobs) {
    if ((st = h->st_obs.ensure((size_t)std::max<int64_t>(total, 1) * 4)) != CV_OK) return st;
    HIP_TRY(hipMemcpyAsync(h->st_obs.as<int32_t>() + base, obs + base, (size_t)(total - base) * 4,
                           hipMemcpyHostToDevice, stream));
    if (obs_staged) *obs_staged = true;
    dobs = h->st_obs.as<int32_t>();
    trace_mark("obs H2D enqueued");
  }

  // ---- prefix / suffix passes for every constrained sequence (m == 1 ones first) ----
  std::vector<const ConSeq*> order;
  for (const auto& c : cs)
    if (c.elems.size() == 1) order.push_back(&c);
  const int64_t n1 = (int64_t)order.size();
  for (const auto& c : cs)
    if (c.elems.size() > 1) order.push_back(&c);
  const int64_t nc = (int64_t)order.size();
  std::vector<int64_t> rg((size_t)nc * 4);  // prefix ranges, then suffix ranges
  for (int64_t i = 0; i < nc; ++i) {
    const ConSeq& c = *order[i];
    rg[2 * i] = offsets[c.seq];
    rg[2 * i + 1] = c.elems.front() + 1;
    // f64: the suffix range starts AT t_m (one extra max-plus step without emission, the
    // kernel's noemit_last): its last row is beta_{t_m} itself; f32: after t_m (max_marginal)
    rg[2 * nc + 2 * i] = c.elems.back() + (o.dtype == CV_DTYPE_F64 ? 0 : 1);
    rg[2 * nc + 2 * i + 1] = offsets[c.seq + 1];
  }
  const int64_t nslot_max = std::max<int64_t>(nc, std::min<int64_t>(kSegmentSlots, (int64_t)seg_pair.size() * N));
  if ((st = h->cs_ranges.ensure(std::max(rg.size(), (size_t)nslot_max * 2) * 8)) != CV_OK) return st;
  if ((st = h->cs_delta.ensure((size_t)nc * np * rb)) != CV_OK) return st;
  if ((st = h->cs_g.ensure((size_t)nc * np * rb)) != CV_OK) return st;
  if ((st = h->cs_mu.ensure((size_t)nc * np * rb)) != CV_OK) return st;
  if ((st = h->cs_zero.ensure((size_t)nc * np * rb)) != CV_OK) return st;
  if ((st = h->st_status.ensure((size_t)std::max<int64_t>(nseq, std::max<int64_t>(nslot_max, 2 * nc)))) != CV_OK)
    return st;
  HIP_TRY(hipMemcpyAsync(h->cs_ranges.p, rg.data(), rg.size() * 8, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemsetAsync(h->cs_zero.p, 0, (size_t)nc * np * rb, stream));
  // prefix rows kept on the device for the resume flow's final decode
  const uint64_t row_bytes = (uint64_t)np * rb;  // f64: split-plane rows of 2 NP words
  const int64_t* row_base_d = nullptr;
  void* rows_d = nullptr;
  const int64_t* srow_base_d = nullptr;  // the suffix pass's rows (certified suffix trace)
  void* srows_d = nullptr;
  std::vector<int64_t> sbv;  // read by an async copy: lives until the slot-order sync below
  if (keep && resume_supported(h, f64)) {
    std::vector<int64_t> rbv((size_t)nc);
    int64_t rows = 0;
    for (int64_t i = 0; i < nc; ++i) rbv[(size_t)i] = rows, rows += rg[2 * i + 1] - rg[2 * i];
    // kept rows live beside the final decode's delta workspace: at most 4x the workspace cap
    // AND at most half of the device memory this handle can still get (the other half stays
    // for that workspace); too large, or a failed allocation, means the final decode runs the
    // full forced passes instead (bit-identical, DESIGN.md §3 resume flow)
    const uint64_t cap = std::min<uint64_t>(
        4 * (o.workspace_bytes ? o.workspace_bytes : f64 ? kDefaultWorkspaceT64 : kDefaultWorkspace),
        free_device_bytes(h->rs_rows.bytes) / 2);
    bool fits = (uint64_t)rows * row_bytes <= cap;
    if (fits && h->rs_rows.ensure((size_t)std::max<int64_t>(rows, 1) * row_bytes) != CV_OK) {
      fits = false;
      g_err.clear();
    }
    if (fits) {
      if ((st = h->rs_rowbase.ensure((size_t)nc * 8)) != CV_OK) return st;
      HIP_TRY(hipMemcpyAsync(h->rs_rowbase.p, rbv.data(), (size_t)nc * 8, hipMemcpyHostToDevice, stream));
      rows_d = h->rs_rows.p;
      row_base_d = h->rs_rowbase.as<int64_t>();
      keep->kept = true;
      keep->row_base = std::move(rbv);
      keep->seq.resize((size_t)nc);
      keep->t1.resize((size_t)nc);
      for (int64_t i = 0; i < nc; ++i) {
        keep->seq[(size_t)i] = order[i]->seq;
        keep->t1[(size_t)i] = order[i]->elems.front();
      }
      // f64, one-position slots present: keep the suffix pass's rows as well, within half of
      // what the device can still give (else the resume decode covers those slots)
      if (f64 && n1 > 0 && trace_supported(h)) {
        // rows only for the one-position slots [0, n1) the trace reads (row base -1: none kept)
        sbv.assign((size_t)nc, -1);
        int64_t srows = 0;
        for (int64_t i = 0; i < n1; ++i) sbv[(size_t)i] = srows, srows += rg[2 * nc + 2 * i + 1] - rg[2 * nc + 2 * i];
        bool sfits = (uint64_t)srows * row_bytes <= free_device_bytes(h->rs_srows.bytes) / 2;
        if (sfits && h->rs_srows.ensure((size_t)std::max<int64_t>(srows, 1) * row_bytes) != CV_OK) {
          sfits = false;
          g_err.clear();
        }
        if (sfits) {
          if ((st = h->rs_srowbase.ensure((size_t)nc * 8)) != CV_OK) return st;
          HIP_TRY(hipMemcpyAsync(h->rs_srowbase.p, sbv.data(), (size_t)nc * 8, hipMemcpyHostToDevice, stream));
          srows_d = h->rs_srows.p;
          srow_base_d = h->rs_srowbase.as<int64_t>();
          keep->suffix_kept = true;
          keep->n1 = n1;
        }
      }
    }
  }
  hipError_t err = hipSuccess;
  {
    // longest first, stable: counting sort on the range lengths (a comparison sort of the
    // 2nc slots cost ~4 ms of host time at config 5 with the GPU idle).  f32: the 2nc slots in
    // one launch; f64: prefixes and suffixes in two launches (a wave's S sequences share one
    // A table), each sorted on its own.
    std::vector<int32_t> so((size_t)2 * nc);
    auto sort_slots = [&](int64_t x0, int64_t x1, int32_t* out, int32_t sub) {
      int64_t maxlen = 0;
      for (int64_t x = x0; x < x1; ++x) maxlen = std::max(maxlen, rg[2 * x + 1] - rg[2 * x]);
      std::vector<int64_t> pos((size_t)maxlen + 2, 0);
      for (int64_t x = x0; x < x1; ++x) ++pos[(size_t)(maxlen - (rg[2 * x + 1] - rg[2 * x])) + 1];
      for (size_t k = 1; k < pos.size(); ++k) pos[k] += pos[k - 1];
      for (int64_t x = x0; x < x1; ++x)
        out[pos[(size_t)(maxlen - (rg[2 * x + 1] - rg[2 * x]))]++] = (int32_t)(x - sub);
    };
    if (f64) {
      sort_slots(0, nc, so.data(), 0);
      sort_slots(nc, 2 * nc, so.data() + nc, (int32_t)nc);
    } else {
      sort_slots(0, 2 * nc, so.data(), 0);
    }
    if ((st = h->ws_order.ensure(so.size() * 4)) != CV_OK) return st;
    HIP_TRY(hipMemcpyAsync(h->ws_order.p, so.data(), so.size() * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));  // `so` is a local buffer
    trace_mark("obs H2D + slot order");
  }
  if (!f64) {
    cvk::TrellisFwdArgs fa{};
    fa.a_img = h->t_aimg.as<float>();
    fa.pi = h->t_pi.as<float>();
    fa.et = h->t_et.as<float>();
    fa.obs = dobs;
    fa.status = h->st_status.as<uint8_t>();
    fa.nobs = (int)h->V;
    fa.ranges = h->cs_ranges.as<int64_t>();
    // one launch, longest range first: slots [0, nc) = prefixes, forward -> delta_{t_1};
    // slots [nc, 2nc) = suffixes, the backward pass = same kernel on a^T with pi = 0,
    // reversed -> g_{t_m+1}
    fa.last_row = h->cs_delta.as<float>();
    fa.split = nc;
    fa.a_img2 = h->t_aimg_T.as<float>();
    fa.pi2 = h->t_pi0.as<float>();
    fa.last_row2 = h->cs_g.as<float>();
    fa.delta = static_cast<float*>(rows_d);
    fa.row_base = row_base_d;
    fa.slot_order = h->ws_order.as<int32_t>();
    err = cvk::launch_trellis_fwd(np, fa, 2 * nc, stream);
    cvk::MaxMarginalArgs ma{};
    ma.g = h->cs_g.as<float>();
    ma.ranges_suffix = h->cs_ranges.as<int64_t>() + 2 * nc;
    ma.at = h->t_at.as<float>();
    ma.mu = h->cs_mu.as<float>();
    if (err == hipSuccess) {  // m == 1: mu = delta + beta
      ma.delta = h->cs_delta.as<float>();
      err = cvk::launch_max_marginal(np, ma, n1, stream);
    }
    if (err == hipSuccess && nc > n1) {  // m >= 2: beta alone (0 + beta is exact)
      ma.delta = h->cs_zero.as<float>();
      ma.g += n1 * np;
      ma.ranges_suffix += 2 * n1;
      ma.mu += n1 * np;
      err = cvk::launch_max_marginal(np, ma, nc - n1, stream);
    }
  } else if (gen) {
    // N > 256: the same passes, one workgroup per slot (generic_ext); no rows kept (the final
    // decode runs the full forced passes)
    cvk::GenericExtArgs ga{};
    ga.tab = h->d_a64.as<double>();
    ga.pi = h->d_pi64.as<double>();
    ga.et = h->d_et64.as<double>();
    ga.obs = dobs;
    ga.ranges = h->cs_ranges.as<int64_t>();
    ga.nstates = N;
    ga.last_row = h->cs_delta.as<double>();
    if (cvk::generic_ext_wide(N)) {  // the rows in global memory, one launch per step
      // sized once for the segment tables' batches too (no reallocation under running launches)
      if ((st = h->cs_wrows.ensure((size_t)nslot_max * 2 * N * 8)) != CV_OK) return st;
      ga.grows = h->cs_wrows.as<double>();
      for (int64_t i = 0; i < 2 * nc; ++i) ga.wide_steps = std::max<int64_t>(ga.wide_steps, rg[2 * i + 1] - rg[2 * i]);
    }
    err = cvk::launch_generic_ext(ga, nc, stream);
    if (err == hipSuccess) {
      ga.tab = h->d_at64.as<double>();
      ga.pi = h->cs_zero.as<double>();  // zeroed above: pi = 0 for the reversed pass
      ga.ranges = h->cs_ranges.as<int64_t>() + 2 * nc;
      ga.reverse = 1;
      ga.noemit_last = 1;
      ga.last_row = h->cs_g.as<double>();
      err = cvk::launch_generic_ext(ga, nc, stream);
    }
    if (err == hipSuccess)
      err = cvk::launch_t64_mu_add(h->cs_delta.as<double>(), h->cs_g.as<double>(), h->cs_mu.as<double>(), n1, np,
                                   stream);
    if (err == hipSuccess && nc > n1)
      err = hipMemcpyAsync(h->cs_mu.as<double>() + n1 * np, h->cs_g.as<double>() + n1 * np,
                           (size_t)(nc - n1) * np * 8, hipMemcpyDeviceToDevice, stream);
  } else {
    // prefixes: forward on a from each sequence start to t_1 (its last row = delta_{t_1})
    cvk::T64FwdArgs fa{};
    fa.a = h->q_a.as<double>();
    fa.pi = h->q_pi.as<double>();
    fa.et = h->q_et.as<double>();
    fa.obs = dobs;
    fa.status = h->st_status.as<uint8_t>();
    fa.nobs = (int)h->V;
    fa.ranges = h->cs_ranges.as<int64_t>();
    fa.nslots = nc;
    fa.last_row = h->cs_delta.as<double>();
    fa.delta = static_cast<double*>(rows_d);
    fa.row_base = row_base_d;
    fa.slot_order = h->ws_order.as<int32_t>();
    // the ragged passes take their units from a work queue (one counter, reset before each
    // launch on this stream)
    if ((st = h->cs_queue.ensure(16)) != CV_OK) return st;
    fa.queue = h->cs_queue.as<int>();
    // prefix / suffix passes: longest-first ranges; with CV_T64_WG_TERMS=1 and at least two
    // rounds of eight-wave workgroups, that layout
    // one-wave workgroups: the eight-wave layout measured neutral here (CV_T64_WG_TERMS, round 3:
    // 185.2 vs 185.9 ms -- the faster prefix/suffix passes leave the side decode less room;
    // removed in round 6)
    fa.wg_ok = 0;
    err = cvk::launch_t64_fwd(np, cvk::t64_seqs_per_wave(nc, h->cus), fa, nc, stream);
    // suffixes: the same recurrence on a^T with pi = 0, reversed (its last row = g_{t_m+1})
    if (err == hipSuccess) {
      cvk::T64FwdArgs fb = fa;
      fb.a = h->q_at.as<double>();
      fb.pi = h->q_pi0.as<double>();
      fb.ranges = h->cs_ranges.as<int64_t>() + 2 * nc;
      fb.reverse = 1;
      fb.noemit_last = 1;
      fb.last_row = h->cs_g.as<double>();  // beta_{t_m}
      fb.delta = static_cast<double*>(srows_d);  // kept for the certified suffix trace, or none
      fb.row_base = srow_base_d;
      fb.slot_order = h->ws_order.as<int32_t>() + nc;
      err = cvk::launch_t64_fwd(np, cvk::t64_seqs_per_wave(nc, h->cus), fb, nc, stream);
    }
    // m == 1: mu = delta + beta (elementwise); m >= 2: the term is beta itself (0 + beta is
    // exact), copied into place
    if (err == hipSuccess)
      err = cvk::launch_t64_mu_add(h->cs_delta.as<double>(), h->cs_g.as<double>(), h->cs_mu.as<double>(), n1, np,
                                   stream);
    if (err == hipSuccess && nc > n1)
      err = hipMemcpyAsync(h->cs_mu.as<double>() + n1 * np, h->cs_g.as<double>() + n1 * np,
                           (size_t)(nc - n1) * np * 8, hipMemcpyDeviceToDevice, stream);
  }
  if (err != hipSuccess) return set_err(CV_EDEVICE, "term launches failed: %s", hipGetErrorString(err));
  trace_mark("term launches enqueued");
  // work queued behind the term launches on another stream (the device API's side decode): it
  // takes the slots the terms pass leaves free at its tails
  if (after_terms && (st = after_terms()) != CV_OK) return st;
  for (int64_t i = 0; i < nc; ++i)
    for (int64_t e : order[i]->elems) part[(int64_t)component[e] * uw + 5 * N] += 1;
  auto range_err = [] {
    return set_err(CV_EINVAL, "a constrained-decode term is outside the exact unit's range (|score| >= 2^32): "
                              "check the model's log-probabilities (null, not a huge negative, for impossible)");
  };
  // tuning key host_sums = 1 takes the host loop (tests compare the two; same integers by construction)
  const bool host_sums = h->tuning.host_sums != 0;
  if (!host_sums && ncomp <= cvx::kUnarySumMaxComp && N <= 256) {
    // exact unary sums on the device (kernels/exact.hip): only the ncomp x uw words come back
    std::vector<int32_t> cc((size_t)2 * nc);
    for (int64_t i = 0; i < nc; ++i) {
      cc[(size_t)i] = component[order[i]->elems.front()];
      cc[(size_t)nc + i] = component[order[i]->elems.back()];
    }
    if ((st = h->cs_comp.ensure(cc.size() * 4)) != CV_OK) return st;
    if ((st = h->cs_words.ensure((size_t)ncomp * uw * 8)) != CV_OK) return st;
    if ((st = h->cs_flag.ensure(16)) != CV_OK) return st;
    HIP_TRY(hipMemcpyAsync(h->cs_comp.p, cc.data(), cc.size() * 4, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemsetAsync(h->cs_words.p, 0, (size_t)ncomp * uw * 8, stream));
    HIP_TRY(hipMemsetAsync(h->cs_flag.p, 0, 4, stream));
    cvx::UnarySumArgs us{};
    us.mu = h->cs_mu.p;
    us.dl = h->cs_delta.p;
    us.c1 = h->cs_comp.as<int32_t>();
    us.cm = h->cs_comp.as<int32_t>() + nc;
    us.nc = nc;
    us.n1 = n1;
    us.np = np;
    us.nstates = N;
    us.ncomp = ncomp;
    us.f64 = f64 ? 1 : 0;
    us.uw = uw;
    us.part = h->cs_words.as<long long>();
    us.bad = h->cs_flag.as<unsigned>();
    const int nblocks = (int)std::max<int64_t>(1, std::min<int64_t>(2 * std::max(h->cus, 1), (nc + 31) / 32));
    const hipError_t e = cvx::launch_unary_sums(us, nblocks, stream);
    if (e != hipSuccess) return set_err(CV_EDEVICE, "unary sum launch failed: %s", hipGetErrorString(e));
    std::vector<int64_t> words((size_t)ncomp * uw);
    unsigned bad = 0;
    HIP_TRY(hipMemcpyAsync(words.data(), h->cs_words.p, words.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(&bad, h->cs_flag.p, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));  // `cc` and `words` are local buffers
    trace_mark("terms + exact sums (device)");
    if (bad) return range_err();
    for (size_t q = 0; q < words.size(); ++q) part[q] += words[q];
  } else {
    std::vector<double> dl64, mu64;
    std::vector<float>& dl = h->host_dl;
    std::vector<float>& mu = h->host_mu;
    if (f64) {
      dl64.resize((size_t)nc * np);
      mu64.resize((size_t)nc * np);
    } else {
      if (dl.size() < (size_t)nc * np) dl.resize((size_t)nc * np);
      if (mu.size() < (size_t)nc * np) mu.resize((size_t)nc * np);
    }
    HIP_TRY(hipMemcpyAsync(f64 ? (void*)dl64.data() : (void*)dl.data(), h->cs_delta.p, (size_t)nc * np * rb,
                           hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(f64 ? (void*)mu64.data() : (void*)mu.data(), h->cs_mu.p, (size_t)nc * np * rb,
                           hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    trace_mark("terms device + D2H");
    // exact accumulation, parallel over states into worker-local words (the components'
    // word blocks are not cache-line aligned: writing `part` directly would false-share),
    // added into `part` at the end (integer sums: order-free)
    std::vector<uint8_t> badw((size_t)host_threads() + 1, 0);
    parallel_ranges(N, [&](int t, int64_t s0, int64_t s1) {
      const int64_t ns = s1 - s0;
      std::vector<int64_t> loc((size_t)ncomp * ns * 5, 0);  // [comp][state][4 limbs], then [comp][state] -inf counts
      int64_t* lim = loc.data();
      int64_t* cnt = loc.data() + (size_t)ncomp * ns * 4;
      bool ok = true;
      auto run = [&](const auto* mrow, const auto* drow) {
        for (int64_t i = 0; i < nc; ++i) {
          const ConSeq& c = *order[i];
          const int64_t c1 = component[c.elems.front()], cm = component[c.elems.back()];
          const auto* mr = mrow + (size_t)i * np;
          const auto* dr = drow + (size_t)i * np;
          for (int64_t s = s0; s < s1; ++s) {
            const int64_t q1 = c1 * ns + (s - s0), qm = cm * ns + (s - s0);
            if (i < n1) {
              ok &= cvcsp::add_exact(lim + 4 * q1, cnt + q1, mr[s]);
            } else {
              ok &= cvcsp::add_exact(lim + 4 * q1, cnt + q1, dr[s]);
              ok &= cvcsp::add_exact(lim + 4 * qm, cnt + qm, mr[s]);
            }
          }
        }
      };
      if (f64) run(mu64.data(), dl64.data());
      else run(mu.data(), dl.data());
      if (!ok) badw[(size_t)t] = 1;
      for (int64_t c = 0; c < ncomp; ++c)
        for (int64_t s = s0; s < s1; ++s) {
          const int64_t q = c * ns + (s - s0);
          int64_t* u = part + c * uw;
          for (int k = 0; k < 4; ++k) u[4 * s + k] += lim[4 * q + k];
          u[4 * N + s] += cnt[q];
        }
    }, 1);
    trace_mark("exact sums (host)");
    for (uint8_t b : badw)
      if (b) return range_err();
  }
  // ---- segment tables: one slot per (segment, start state), in batches ----
  struct Seg { int64_t e0, e1; int32_t c1, c2; int64_t p; };
  std::vector<Seg> segs;
  {
    size_t q = 0;  // seg_pair follows cs order, and so do the m >= 2 entries of `order`
    for (int64_t i = n1; i < nc; ++i) {
      const ConSeq& c = *order[i];
      for (size_t k = 0; k + 1 < c.elems.size(); ++k, ++q)
        segs.push_back({c.elems[k], c.elems[k + 1], component[c.elems[k]], component[c.elems[k + 1]], seg_pair[q]});
    }
  }
  const int64_t nslots = (int64_t)segs.size() * N;
  std::vector<int64_t> srg;
  std::vector<int32_t> sst;
  std::vector<float> rows;
  std::vector<double> rows64;
  bool ok = true;
  for (int64_t b0 = 0; b0 < nslots; b0 += kSegmentSlots) {
    const int64_t nb = std::min(kSegmentSlots, nslots - b0);
    srg.resize((size_t)nb * 2);
    sst.resize((size_t)nb);
    for (int64_t k = 0; k < nb; ++k) {
      const Seg& sg = segs[(b0 + k) / N];
      srg[2 * k] = sg.e0;
      srg[2 * k + 1] = sg.e1 + 1;
      sst[k] = (int32_t)((b0 + k) % N);
    }
    if ((st = h->cs_start.ensure((size_t)nb * 4)) != CV_OK) return st;
    HIP_TRY(hipMemcpyAsync(h->cs_ranges.p, srg.data(), srg.size() * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(h->cs_start.p, sst.data(), sst.size() * 4, hipMemcpyHostToDevice, stream));
    if ((st = h->cs_seg.ensure((size_t)nb * np * rb)) != CV_OK) return st;
    if (gen) {
      cvk::GenericExtArgs sa{};
      sa.tab = h->d_a64.as<double>();
      sa.pi = h->d_pi64.as<double>();
      sa.et = h->d_et64.as<double>();
      sa.obs = dobs;
      sa.ranges = h->cs_ranges.as<int64_t>();
      sa.start = h->cs_start.as<int32_t>();
      sa.nstates = N;
      sa.last_row = h->cs_seg.as<double>();
      if (cvk::generic_ext_wide(N)) {
        if ((st = h->cs_wrows.ensure((size_t)nb * 2 * N * 8)) != CV_OK) return st;
        sa.grows = h->cs_wrows.as<double>();
        for (int64_t k = 0; k < nb; ++k) sa.wide_steps = std::max<int64_t>(sa.wide_steps, srg[2 * k + 1] - srg[2 * k]);
      }
      err = cvk::launch_generic_ext(sa, nb, stream);
    } else if (!f64) {
      cvk::TrellisFwdArgs sa{};
      sa.a_img = h->t_aimg.as<float>();
      sa.pi = h->t_pi.as<float>();
      sa.et = h->t_et.as<float>();
      sa.obs = dobs;
      sa.status = h->st_status.as<uint8_t>();
      sa.nobs = (int)h->V;
      sa.ranges = h->cs_ranges.as<int64_t>();
      sa.start = h->cs_start.as<int32_t>();
      sa.last_row = h->cs_seg.as<float>();
      err = cvk::launch_trellis_fwd(np, sa, nb, stream);
    } else {
      // the N slots of a segment share its range: a wave's S sequences run equal lengths
      cvk::T64FwdArgs sa{};
      sa.a = h->q_a.as<double>();
      sa.pi = h->q_pi.as<double>();
      sa.et = h->q_et.as<double>();
      sa.obs = dobs;
      sa.status = h->st_status.as<uint8_t>();
      sa.nobs = (int)h->V;
      sa.ranges = h->cs_ranges.as<int64_t>();
      sa.nslots = nb;
      sa.start = h->cs_start.as<int32_t>();
      sa.last_row = h->cs_seg.as<double>();
      err = cvk::launch_t64_fwd(np, cvk::t64_seqs_per_wave(nb, h->cus), sa, nb, stream);
    }
    if (err != hipSuccess) return set_err(CV_EDEVICE, "segment-table launch failed: %s", hipGetErrorString(err));
    if (f64) rows64.resize((size_t)nb * np);
    else rows.resize((size_t)nb * np);
    HIP_TRY(hipMemcpyAsync(f64 ? (void*)rows64.data() : (void*)rows.data(), h->cs_seg.p, (size_t)nb * np * rb,
                           hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    auto acc = [&](const auto* all) {
      for (int64_t k = 0; k < nb; ++k) {
        const Seg& sg = segs[(b0 + k) / N];
        const int s = (int)((b0 + k) % N);
        const auto* r = all + (size_t)k * np;
        if (sg.p < 0) {  // same component at both ends: only the diagonal is consistent
          int64_t* u = part + (int64_t)sg.c1 * uw;
          ok &= cvcsp::add_exact(u + 4 * s, u + 4 * N + s, r[s]);
          continue;
        }
        int64_t* pp = pbase + sg.p * pw;
        if (s == 0) pp[5 * (int64_t)N * N] += 1;
        for (int s2 = 0; s2 < N; ++s2) {
          const int64_t e = sg.c1 < sg.c2 ? (int64_t)s * N + s2 : (int64_t)s2 * N + s;
          ok &= cvcsp::add_exact(pp + 4 * e, pp + 4 * (int64_t)N * N + e, r[s2]);
        }
      }
    };
    if (f64) acc(rows64.data());
    else acc(rows.data());
  }
  if (!ok) return range_err();
  return CV_OK;
}

// Final decode: every constrained element forced to its component's state; sequences whose
// component has no feasible state are infeasible.  objective = sum of the f64 scores.  The
// forced-state array is built on the device (fill -1, scatter the constrained elements of
// `cs`); obs_staged: h->st_obs already holds the batch's observations.
// The forced-state array of a batch on the device (h->st_forced, indexed like obs, -1 = free):
// every constrained element of `cs` takes comp_state[component[e]] (0 when the component has
// no state: such sequences are marked infeasible afterwards by mark_unassigned).
cv_status stage_forced_locked(cv_hmm* h, const int64_t* offsets, int64_t nseq, const int32_t* component,
                              const int32_t* comp_state, const std::vector<ConSeq>& cs, hipStream_t stream) {
  const int64_t base = offsets[0], total = offsets[nseq];
  std::vector<int64_t> el;
  std::vector<int32_t> sv;
  for (const auto& c : cs)
    for (int64_t e : c.elems) {
      el.push_back(e);
      sv.push_back(comp_state[component[e]] >= 0 ? comp_state[component[e]] : 0);
    }
  cv_status st;
  if ((st = h->st_forced.ensure((size_t)std::max<int64_t>(total, 1) * 4)) != CV_OK) return st;
  if ((st = h->cs_ranges.ensure(std::max<size_t>(el.size(), 1) * 8)) != CV_OK) return st;
  if ((st = h->cs_start.ensure(std::max<size_t>(sv.size(), 1) * 4)) != CV_OK) return st;
  if (total > base) HIP_TRY(hipMemsetAsync(h->st_forced.as<int32_t>() + base, 0xFF, (size_t)(total - base) * 4, stream));
  if (!el.empty()) {
    HIP_TRY(hipMemcpyAsync(h->cs_ranges.p, el.data(), el.size() * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(h->cs_start.p, sv.data(), sv.size() * 4, hipMemcpyHostToDevice, stream));
    const hipError_t err = cvk::launch_scatter_forced(h->cs_ranges.as<int64_t>(), h->cs_start.as<int32_t>(),
                                                      (int64_t)el.size(), h->st_forced.as<int32_t>(), stream);
    if (err != hipSuccess) return set_err(CV_EDEVICE, "forced-state scatter failed: %s", hipGetErrorString(err));
    // the host vectors die at return: the copies must have read them
    HIP_TRY(hipStreamSynchronize(stream));
  }
  trace_mark("forced array (device)");
  return CV_OK;
}

// Host copies of the decode's scores/statuses: sequences with an element of a component
// that got no state are infeasible; objective = the f64 sum in sequence order (that sum's
// rounding is part of the spec).
double mark_unassigned(int64_t nseq, const int32_t* component, const int32_t* comp_state,
                       const std::vector<ConSeq>& cs, double* score, uint8_t* status) {
  for (const auto& c : cs)
    for (int64_t e : c.elems)
      if (comp_state[component[e]] < 0) {
        status[c.seq] = CV_SEQ_INFEASIBLE;
        score[c.seq] = -INFINITY;
      }
  double obj = 0.0;
  for (int64_t s = 0; s < nseq; ++s) obj += status[s] == CV_SEQ_INFEASIBLE ? -INFINITY : score[s];
  return obj;
}

// Final decode with every constrained element forced (caller holds h->mu; `cs` as built by
// `constrained_validate`); obs_staged: h->st_obs already holds the batch's observations.
cv_status forced_decode_locked(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                               const int32_t* component, const int32_t* comp_state, cv_opts o,
                               const std::vector<ConSeq>& cs, bool obs_staged, int32_t* path_out,
                               double* score_out, uint8_t* status_out, double* objective_out) {
  hipStream_t stream = o.stream ? (hipStream_t)o.stream : h->stream;
  cv_status st;
  if ((st = stage_forced_locked(h, offsets, nseq, component, comp_state, cs, stream)) != CV_OK) return st;
  o.forced = h->st_forced.as<int32_t>();
  st = decode_host_locked(h, nseq, offsets, obs, o, path_out, score_out, status_out, obs_staged, true);
  if (st != CV_OK) return st;
  trace_mark("forced decode (sync)");
  const double obj = mark_unassigned(nseq, component, comp_state, cs, score_out, status_out);
  if (objective_out) *objective_out = obj;
  return CV_OK;
}

// Final decode of the resume flow (see kernels/trellis.hip "resume flow"): the terms pass
// stored every constrained sequence's prefix rows, so the decode runs [t_1, end) of those
// sequences (from row t_1 with the chosen state forced) and whole unconstrained sequences as
// one compact batch, ordered longest first (contiguous chunks of near-equal lengths pair and
// pack well); the prefix paths are backtracked from their forced states on the backtrack
// stream beside that decode; then suffix paths, scores and statuses go back to the original
// layout and every path is re-scored in f64 over its whole sequence.  Bit-identical to
// forced_decode_locked's full forced decode.  Device pointers; synchronous.
// The constrained decode's UNCONSTRAINED sequences (no constrained element) do not depend on
// the component states: they are decoded on the handle's side stream and workspace (h->side),
// launched before the terms pass, so their waves fill the terms pass's tails and the host
// phases (checks, search) that leave the GPU idle; the results are scattered into the caller's
// outputs.  f64 only (the f32 resume flow re-scores every sequence at its end).  *launched:
// h->side.done is recorded on the side stream; the caller waits for it (and synchronizes the
// side stream on any error) before the outputs are read.
cv_status side_decode_launch(cv_hmm* h, int64_t nseq, const int64_t* offsets_host, const int32_t* obs_dev,
                             const std::vector<ConSeq>& cs, const cv_opts& o, int32_t* path_dev, double* score_dev,
                             uint8_t* status_dev, hipStream_t stream, bool* launched) {
  *launched = false;
  auto& sd = h->side;
  std::vector<uint8_t> con((size_t)nseq, 0);
  for (const auto& c : cs) con[(size_t)c.seq] = 1;
  int64_t nu = 0;
  for (int64_t q = 0; q < nseq; ++q) nu += con[(size_t)q] ? 0 : 1;
  if (nu == 0) return CV_OK;
  // [cstart | seq | off2 (nu + 1)] int64, in sequence order (decode_device orders by length)
  sd.idx_host.assign((size_t)3 * nu + 1, 0);
  int64_t* cstart = sd.idx_host.data();
  int64_t* cseq = cstart + nu;
  int64_t* off2 = cseq + nu;
  for (int64_t q = 0, k = 0; q < nseq; ++q) {
    if (con[(size_t)q]) continue;
    cstart[k] = offsets_host[q];
    cseq[k] = q;
    off2[k + 1] = off2[k] + offsets_host[q + 1] - offsets_host[q];
    ++k;
  }
  const int64_t total2 = off2[nu];
  cv_status st;
  if (!sd.done && hipEventCreateWithFlags(&sd.done, hipEventDisableTiming) != hipSuccess)
    return set_err(CV_EDEVICE, "hipEventCreate failed");
  // no room for the side buffers: the final forced decode covers these sequences as well
  // (launched stays false; same results)
  if ((st = sd.idx.ensure(sd.idx_host.size() * 8)) != CV_OK || (st = sd.obs2.ensure((size_t)std::max<int64_t>(total2, 1) * 4)) != CV_OK ||
      (st = sd.path2.ensure((size_t)std::max<int64_t>(total2, 1) * 4)) != CV_OK ||
      (st = sd.res2.ensure((size_t)nu * 9)) != CV_OK) {
    if (st != CV_ENOMEM) return st;
    g_err.clear();
    return CV_OK;
  }
  // the side stream starts behind everything the caller had queued on its stream when the
  // constrained decode began (h->side.start, recorded then), not behind the term launches
  // (round 4 measured every other order slower: DESIGN.md §3, rejected variants)
  HIP_TRY(hipStreamWaitEvent(sd.stream, sd.start, 0));
  HIP_TRY(hipMemcpyAsync(sd.idx.p, sd.idx_host.data(), sd.idx_host.size() * 8, hipMemcpyHostToDevice, sd.stream));
  const int64_t* cstart_d = sd.idx.as<int64_t>();
  const int64_t* cseq_d = cstart_d + nu;
  const int64_t* off2_d = cseq_d + nu;
  double* score2 = sd.res2.as<double>();
  uint8_t* status2 = reinterpret_cast<uint8_t*>(score2 + nu);
  hipError_t err = cvk::launch_compact_suffix(cstart_d, off2_d, obs_dev, nullptr, nullptr, sd.obs2.as<int32_t>(),
                                              nullptr, nu, sd.stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "side batch staging failed: %s", hipGetErrorString(err));
  *launched = true;  // from here on the side stream holds work
  cv_opts o2 = o;
  o2.forced = nullptr;
  o2.rescore_f64 = 0;  // f64: the decode's score is the reference's
  if ((st = decode_device(h, nu, off2, off2_d, sd.obs2.as<int32_t>(), o2, sd.path2.as<int32_t>(), score2, status2,
                          sd.stream, nullptr, /*side_ws=*/true)) != CV_OK) {
    if (st != CV_ENOMEM) return st;
    // the side workspace did not fit beside the terms pass's buffers: drop the side decode (its
    // staging kernel wrote only side buffers) and let the final forced decode cover these
    // sequences -- the same results, no CV_ENOMEM for the caller
    HIP_TRY(hipStreamSynchronize(sd.stream));
    *launched = false;
    g_err.clear();
    return CV_OK;
  }
  err = cvk::launch_scatter_suffix(cstart_d, off2_d, cseq_d, sd.path2.as<int32_t>(), score2, status2, path_dev,
                                   score_dev, status_dev, nu, sd.stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "side scatter failed: %s", hipGetErrorString(err));
  HIP_TRY(hipEventRecord(sd.done, sd.stream));
  trace_mark("side decode of the unconstrained sequences enqueued");
  return CV_OK;
}

// Synchronizes the side stream at scope exit when a side decode was launched and not joined,
// and the high-priority stream when the constrained work ran on it.
struct SideJoin {
  cv_hmm* h;
  bool active = false, hi = false;
  ~SideJoin() {
    if (active) (void)hipStreamSynchronize(h->side.stream);
    if (hi) (void)hipStreamSynchronize(h->side.hi);
  }
};

// The side-decode streams (lowest / highest priority; equal priorities if CV_SIDE_PRIO=0,
// swapped if CV_SIDE_PRIO=2).
cv_status side_streams(cv_hmm* h) {
  auto& sd = h->side;
  if (!sd.stream) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
      (void)hipGetLastError();
      least = greatest = 0;
    }
    if (hipStreamCreateWithPriority(&sd.stream, hipStreamNonBlocking, least) != hipSuccess ||
        hipStreamCreateWithPriority(&sd.hi, hipStreamNonBlocking, greatest) != hipSuccess)
      return set_err(CV_EDEVICE, "hipStreamCreateWithPriority failed");
  }
  if (!sd.start && hipEventCreateWithFlags(&sd.start, hipEventDisableTiming) != hipSuccess)
    return set_err(CV_EDEVICE, "hipEventCreate failed");
  return CV_OK;
}

cv_status forced_decode_resume(cv_hmm* h, int64_t nseq, const int64_t* offsets_host, const int64_t* offsets_dev,
                               const int32_t* obs_dev, const int32_t* component, const int32_t* comp_state,
                               const std::vector<ConSeq>& cs, const PrefixKeep& keep, cv_opts o, int32_t* path_dev,
                               double* score_dev, uint8_t* status_dev, hipStream_t stream,
                               bool constrained_only = false) {
  // constrained_only: the unconstrained sequences were decoded beside the terms pass
  // (side_decode_launch); the compact batch holds the constrained sequences alone
  cv_status st;
  if ((st = stage_forced_locked(h, offsets_host, nseq, component, comp_state, cs, stream)) != CV_OK) return st;
  const int64_t nc = (int64_t)keep.seq.size();
  const bool f64 = o.dtype == CV_DTYPE_F64;
  const int np = f64 ? h->np64 : h->np;
  const size_t rb = f64 ? 8 : 4;
  std::vector<int64_t> start(offsets_host, offsets_host + nseq);
  std::vector<int32_t> ridx((size_t)nseq, -1), state((size_t)nc);
  for (int64_t i = 0; i < nc; ++i) {
    start[(size_t)keep.seq[i]] = keep.t1[i];
    ridx[(size_t)keep.seq[i]] = (int32_t)i;
    const int32_t c = comp_state[component[keep.t1[i]]];
    state[(size_t)i] = c >= 0 ? c : 0;  // no state: forced to 0 and marked infeasible (mark_unassigned)
  }
  // per-slot arrays: [seq | t1 | row_base] int64, then state int32
  std::vector<int64_t> slot64((size_t)nc * 3);
  std::copy(keep.seq.begin(), keep.seq.end(), slot64.begin());
  std::copy(keep.t1.begin(), keep.t1.end(), slot64.begin() + nc);
  std::copy(keep.row_base.begin(), keep.row_base.end(), slot64.begin() + 2 * nc);
  if ((st = h->rs_slot.ensure((size_t)std::max<int64_t>(nc, 1) * 28)) != CV_OK) return st;
  int64_t* slot_d = h->rs_slot.as<int64_t>();
  int32_t* state_d = reinterpret_cast<int32_t*>(slot_d + 3 * nc);
  HIP_TRY(hipMemcpyAsync(slot_d, slot64.data(), (size_t)nc * 24, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(state_d, state.data(), (size_t)nc * 4, hipMemcpyHostToDevice, stream));
  // certified suffix trace (f64, suffix rows kept): the one-position slots whose forced path
  // after t1 reads off the suffix pass's rows (suffix_trace_f64) need no second forward pass;
  // only the others join the compact forced decode below
  std::vector<uint8_t> cert((size_t)nc, 0);
  if (f64 && keep.suffix_kept && keep.n1 > 0) {
    const int64_t n1 = keep.n1;
    std::vector<int32_t> tstate((size_t)n1);
    for (int64_t i = 0; i < n1; ++i) tstate[(size_t)i] = comp_state[component[keep.t1[i]]] >= 0 ? state[(size_t)i] : -1;
    const size_t cert_bytes = (size_t)((n1 + 3) / 4) * 4;  // then the states, 4-byte aligned
    if ((st = h->rs_cert.ensure(cert_bytes + (size_t)n1 * 4)) != CV_OK) return st;
    uint8_t* cert_d = h->rs_cert.as<uint8_t>();
    int32_t* tstate_d = reinterpret_cast<int32_t*>(cert_d + cert_bytes);
    HIP_TRY(hipMemcpyAsync(tstate_d, tstate.data(), (size_t)n1 * 4, hipMemcpyHostToDevice, stream));
    cvk::SuffixTrace64Args ta{};
    ta.rows = h->rs_srows.as<double>();
    ta.srow_base = h->rs_srowbase.as<int64_t>();
    ta.seq = slot_d;
    ta.t1 = slot_d + nc;
    ta.state = tstate_d;
    ta.dlast = h->cs_delta.as<double>();
    ta.offsets = offsets_dev;
    ta.obs = obs_dev;
    ta.a = h->q_a.as<double>();
    ta.et = h->q_et.as<double>();
    ta.nstates = h->N;
    ta.path = path_dev;
    ta.score = score_dev;
    ta.status = status_dev;
    ta.cert = cert_d;
    const hipError_t e = cvk::launch_t64_suffix_trace(np, ta, n1, stream);
    if (e != hipSuccess) return set_err(CV_EDEVICE, "suffix trace failed: %s", hipGetErrorString(e));
    HIP_TRY(hipMemcpyAsync(cert.data(), cert_d, (size_t)n1, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    trace_mark("resume: certified suffix trace");
  }
  int64_t ncert = 0;
  for (uint8_t c : cert) ncert += c;
  h->last_traced = ncert;
  // compact order: longest first, stable (counting sort) over the member sequences
  const int64_t nm = (constrained_only ? nc : nseq) - ncert;
  std::vector<int64_t> mem;
  mem.reserve((size_t)nm);
  if (constrained_only) {  // keep.seq is in sequence order (terms-pass slot order)
    for (int64_t i = 0; i < nc; ++i)
      if (!cert[(size_t)i]) mem.push_back(keep.seq[(size_t)i]);
    std::sort(mem.begin(), mem.end());
  } else {
    for (int64_t s = 0; s < nseq; ++s)
      if (ridx[(size_t)s] < 0 || !cert[(size_t)ridx[(size_t)s]]) mem.push_back(s);
  }
  int64_t maxlen = 0;
  for (int64_t s : mem) maxlen = std::max(maxlen, offsets_host[s + 1] - start[(size_t)s]);
  std::vector<int64_t> pos((size_t)maxlen + 2, 0), perm((size_t)nm);
  for (int64_t s : mem) ++pos[(size_t)(maxlen - (offsets_host[s + 1] - start[(size_t)s])) + 1];
  for (size_t k = 1; k < pos.size(); ++k) pos[k] += pos[k - 1];
  for (int64_t s : mem) perm[(size_t)pos[(size_t)(maxlen - (offsets_host[s + 1] - start[(size_t)s]))]++] = s;
  // per compact sequence: [cstart | perm | off2 (nm+1)] int64, then ridx int32
  std::vector<int64_t> c64((size_t)3 * nm + 1);
  std::vector<int32_t> cridx((size_t)nm);
  int64_t* cstart = c64.data();
  int64_t* cperm = cstart + nm;
  int64_t* off2 = cperm + nm;
  off2[0] = 0;
  for (int64_t k = 0; k < nm; ++k) {
    const int64_t s = perm[(size_t)k];
    cstart[k] = start[(size_t)s];
    cperm[k] = s;
    cridx[(size_t)k] = ridx[(size_t)s];
    off2[k + 1] = off2[k] + offsets_host[s + 1] - start[(size_t)s];
  }
  const int64_t total2 = off2[nm];
  if ((st = h->rs_start.ensure(c64.size() * 8)) != CV_OK) return st;
  if ((st = h->rs_ridx.ensure((size_t)std::max<int64_t>(nm, 1) * 4)) != CV_OK) return st;
  if ((st = h->rs_off2.ensure((size_t)std::max<int64_t>(nm, 1) * 9)) != CV_OK) return st;  // score2 f64 + status2 u8
  if ((st = h->rs_resume.ensure((size_t)std::max<int64_t>(nc, 1) * np * rb)) != CV_OK) return st;
  if ((st = h->rs_obs2.ensure((size_t)std::max<int64_t>(total2, 1) * 4)) != CV_OK) return st;
  if ((st = h->rs_frc2.ensure((size_t)std::max<int64_t>(total2, 1) * 4)) != CV_OK) return st;
  if ((st = h->rs_path2.ensure((size_t)std::max<int64_t>(total2, 1) * 4)) != CV_OK) return st;
  if (!h->rs_ev && hipEventCreateWithFlags(&h->rs_ev, hipEventDisableTiming) != hipSuccess)
    return set_err(CV_EDEVICE, "hipEventCreate failed");
  const int64_t* cstart_d = h->rs_start.as<int64_t>();
  const int64_t* cperm_d = cstart_d + nm;
  const int64_t* off2_d = cperm_d + nm;
  double* score2 = h->rs_off2.as<double>();
  uint8_t* status2 = reinterpret_cast<uint8_t*>(score2 + nm);
  HIP_TRY(hipMemcpyAsync(h->rs_start.p, c64.data(), c64.size() * 8, hipMemcpyHostToDevice, stream));
  if (nm > 0) HIP_TRY(hipMemcpyAsync(h->rs_ridx.p, cridx.data(), (size_t)nm * 4, hipMemcpyHostToDevice, stream));
  hipError_t err = f64 ? cvk::launch_t64_resume_rows(h->cs_delta.as<double>(), state_d, nc, np,
                                                     h->rs_resume.as<double>(), stream)
                       : cvk::launch_resume_rows(h->cs_delta.as<float>(), state_d, nc, np, h->rs_resume.as<float>(),
                                                 stream);
  if (err == hipSuccess)
    err = cvk::launch_compact_suffix(cstart_d, off2_d, obs_dev, h->st_forced.as<int32_t>(), h->rs_ridx.as<int32_t>(),
                                     h->rs_obs2.as<int32_t>(), h->rs_frc2.as<int32_t>(), nm, stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "resume staging failed: %s", hipGetErrorString(err));
  // prefix paths on the backtrack stream, beside the suffix decode (one workgroup per CU at
  // most: the 100 KiB LDS reservation, as the chunk pipeline's backtracks)
  cvk::PrefixBtArgs pa{};
  pa.rows = h->rs_rows.as<float>();
  pa.seq = slot_d;
  pa.t1 = slot_d + nc;
  pa.row_base = slot_d + 2 * nc;
  pa.state = state_d;
  pa.offsets = offsets_dev;
  pa.at = h->t_at.as<float>();
  pa.status = status_dev;
  pa.path = path_dev;
  if (!f64) {
    HIP_TRY(hipEventRecord(h->rs_ev, stream));
    HIP_TRY(hipStreamWaitEvent(h->bt_stream, h->rs_ev, 0));
    err = cvk::launch_prefix_backtrack(np, pa, nc, h->bt_stream, 100 * 1024);
    if (err != hipSuccess) return set_err(CV_EDEVICE, "prefix backtrack failed: %s", hipGetErrorString(err));
    HIP_TRY(hipEventRecord(h->rs_ev, h->bt_stream));
  }
  trace_mark("resume: compact suffix batch");
  cv_opts o2 = o;
  o2.forced = h->rs_frc2.as<int32_t>();
  o2.rescore_f64 = 0;  // f32: re-scored below over the whole sequences; f64: the score is exact
  if ((st = decode_device(h, nm, off2, off2_d, h->rs_obs2.as<int32_t>(), o2, h->rs_path2.as<int32_t>(), score2,
                          status2, stream, h->rs_resume.p)) != CV_OK) {
    (void)hipStreamSynchronize(stream);
    (void)hipStreamSynchronize(h->bt_stream);
    return st;
  }
  if (f64) {
    // f64: the prefix backtrack runs after the suffix decode on the same stream (a co-running
    // backtrack slowed the 2-wave f64 forward more than it hid, profiles/r02_bench_c4_f64_overlap.log)
    cvk::PrefixBt64Args p64{};
    p64.rows = h->rs_rows.as<double>();
    p64.seq = slot_d;
    p64.t1 = slot_d + nc;
    p64.row_base = slot_d + 2 * nc;
    p64.state = state_d;
    p64.offsets = offsets_dev;
    p64.at = h->q_at.as<double>();
    p64.at32 = h->t64_nonpos ? h->q_at32.as<float>() : nullptr;
    p64.nstates = h->N;
    p64.path = path_dev;
    err = cvk::launch_t64_prefix_bt(np, p64, nc, stream);
    if (err != hipSuccess) return set_err(CV_EDEVICE, "prefix backtrack failed: %s", hipGetErrorString(err));
  } else {
    HIP_TRY(hipStreamWaitEvent(stream, h->rs_ev, 0));  // prefix paths written
  }
  err = cvk::launch_scatter_suffix(cstart_d, off2_d, cperm_d, h->rs_path2.as<int32_t>(), score2, status2, path_dev,
                                   score_dev, status_dev, nm, stream);
  if (err == hipSuccess) err = cvk::launch_zero_infeasible_prefix(pa, nc, stream);
  if (err == hipSuccess && o.rescore_f64 && !f64) {
    cvk::RescoreArgs ra{};
    ra.path = path_dev;
    ra.obs = obs_dev;
    ra.offsets = offsets_dev;
    ra.seq_begin = 0;
    ra.seq_end = nseq;
    ra.nstates = h->N;
    ra.pi64 = h->d_pi64.as<double>();
    ra.a64 = h->d_a64.as<double>();
    ra.et64 = h->d_et64.as<double>();
    ra.status = status_dev;
    ra.score = score_dev;
    err = cvk::launch_rescore_f64(ra, nseq, stream);
  }
  if (err != hipSuccess) return set_err(CV_EDEVICE, "resume finish failed: %s", hipGetErrorString(err));
  HIP_TRY(hipStreamSynchronize(stream));  // host index vectors die at return
  trace_mark("resume: decode + prefix backtrack + re-score");
  return CV_OK;
}

// Host-API tail of the constrained decode: the resume flow on the staged observations
// (h->st_obs) with results copied back, or the full forced decode.
cv_status final_decode_host(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                            const int32_t* component, const int32_t* comp_state, const cv_opts& o,
                            const std::vector<ConSeq>& cs, const PrefixKeep& keep, bool obs_staged, int32_t* path_out,
                            double* score_out, uint8_t* status_out, double* objective_out) {
  cv_status st;
  if (keep.kept && obs_staged) {
    hipStream_t stream = o.stream ? (hipStream_t)o.stream : h->stream;
    const int64_t base = offsets[0], total = offsets[nseq];
    if ((st = h->st_off.ensure((size_t)(nseq + 1) * 8)) != CV_OK) return st;
    if ((st = h->st_path.ensure((size_t)std::max<int64_t>(total, 1) * 4)) != CV_OK) return st;
    if ((st = h->st_score.ensure((size_t)nseq * 8)) != CV_OK) return st;
    if ((st = h->st_status.ensure((size_t)nseq)) != CV_OK) return st;
    HIP_TRY(hipMemcpyAsync(h->st_off.p, offsets, (size_t)(nseq + 1) * 8, hipMemcpyHostToDevice, stream));
    if ((st = forced_decode_resume(h, nseq, offsets, h->st_off.as<int64_t>(), h->st_obs.as<int32_t>(), component,
                                   comp_state, cs, keep, o, h->st_path.as<int32_t>(), h->st_score.as<double>(),
                                   h->st_status.as<uint8_t>(), stream)) != CV_OK)
      return st;
    if (total > base)
      HIP_TRY(hipMemcpyAsync(path_out + base, h->st_path.as<int32_t>() + base, (size_t)(total - base) * 4,
                             hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(score_out, h->st_score.p, (size_t)nseq * 8, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipMemcpyAsync(status_out, h->st_status.p, (size_t)nseq, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    const double obj = mark_unassigned(nseq, component, comp_state, cs, score_out, status_out);
    if (objective_out) *objective_out = obj;
    return CV_OK;
  }
  return forced_decode_locked(h, nseq, offsets, obs, component, comp_state, o, cs, obs_staged, path_out, score_out,
                              status_out, objective_out);
}

cv_status select_locked(int32_t nstates, int32_t ncomp, const int32_t* pairs, int64_t npairs,
                        const int64_t* partials, int32_t* comp_state_out, uint64_t* explored_out) {
  const cvcsp::SolveResult r = cvcsp::solve(nstates, ncomp, pairs, npairs, partials, comp_state_out, kCspNodeLimit);
  if (explored_out) *explored_out = r.explored;
  if (r.limit_hit)
    return set_err(CV_ELIMIT, "component-state search exceeded %llu nodes", (unsigned long long)kCspNodeLimit);
  return CV_OK;
}

bool pairs_sorted(const int32_t* pairs, int64_t npairs, int32_t ncomp) {
  for (int64_t p = 0; p < npairs; ++p) {
    if (pairs[2 * p] < 0 || pairs[2 * p] >= pairs[2 * p + 1] || pairs[2 * p + 1] >= ncomp) return false;
    if (p > 0 && !(pairs[2 * p - 2] < pairs[2 * p] || (pairs[2 * p - 2] == pairs[2 * p] && pairs[2 * p - 1] <
                                                                                             pairs[2 * p + 1])))
      return false;
  }
  return true;
}
}  // namespace

extern "C" {

CV_API cv_status cv_constrained_pairs(int64_t nseq, const int64_t* offsets, const int32_t* component, int32_t ncomp,
                                      int32_t* pairs_out, int64_t cap_pairs, int64_t* npairs_out) {
  if (nseq < 0 || ncomp < 0 || !npairs_out || (nseq > 0 && (!offsets || !component)))
    return set_err(CV_EINVAL, "bad argument");
  *npairs_out = 0;
  if (nseq == 0) return CV_OK;
  for (int64_t s = 0; s < nseq; ++s)
    if (offsets[s + 1] < offsets[s]) return set_err(CV_EINVAL, "offsets must be non-decreasing");
  for (int64_t k = offsets[0]; k < offsets[nseq]; ++k)
    if (component[k] < -1 || component[k] >= ncomp)
      return set_err(CV_EINVAL, "component[%lld] = %d out of range [-1,%d)", (long long)k, component[k], ncomp);
  const std::vector<int32_t> p = cvcsp::component_pairs(nseq, offsets, component);
  *npairs_out = (int64_t)p.size() / 2;
  if (pairs_out) {
    if (cap_pairs < *npairs_out) return set_err(CV_EINVAL, "pairs_out holds %lld pairs, %lld needed",
                                                (long long)cap_pairs, (long long)*npairs_out);
    std::copy(p.begin(), p.end(), pairs_out);
  }
  return CV_OK;
}

CV_API cv_status cv_constrained_partials(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                         const int32_t* component, int32_t ncomp, int64_t npairs,
                                         const int32_t* pairs, const cv_opts* opts, int64_t* partials_out) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq < 0 || ncomp < 0 || npairs < 0 || (nseq > 0 && (!offsets || !obs || !component)) ||
      (ncomp > 0 && !partials_out) || (npairs > 0 && !pairs))
    return set_err(CV_EINVAL, "null argument");
  if (!pairs_sorted(pairs, npairs, ncomp)) return set_err(CV_EINVAL, "pairs must be sorted (c1 < c2) and unique");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  cv_opts o = opts ? *opts : default_opts();
  std::memset(partials_out, 0, (size_t)cvcsp::partial_words((int)h->N, ncomp, npairs) * 8);
  return constrained_partials_locked(h, nseq, offsets, obs, component, ncomp, pairs, npairs, o, partials_out);
}

CV_API cv_status cv_constrained_select(int32_t nstates, int32_t ncomp, int64_t npairs, const int32_t* pairs,
                                       const int64_t* partials, int32_t* comp_state_out, uint64_t* explored_out) {
  if (nstates <= 0 || ncomp < 0 || npairs < 0 || (ncomp > 0 && (!partials || !comp_state_out)) ||
      (npairs > 0 && !pairs))
    return set_err(CV_EINVAL, "bad argument");
  if (!pairs_sorted(pairs, npairs, ncomp)) return set_err(CV_EINVAL, "pairs must be sorted (c1 < c2) and unique");
  return select_locked(nstates, ncomp, pairs, npairs, partials, comp_state_out, explored_out);
}

CV_API cv_status cv_decode_constrained(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                       const int32_t* component, int32_t ncomp, const cv_opts* opts,
                                       int32_t* path_out, double* score_out, uint8_t* status_out,
                                       int32_t* comp_state_out, double* objective_out) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq < 0 || ncomp < 0 || (nseq > 0 && (!offsets || !obs || !component || !path_out || !score_out ||
                                             !status_out)) || (ncomp > 0 && !comp_state_out))
    return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  cv_opts o = opts ? *opts : default_opts();
  for (int32_t c = 0; c < ncomp; ++c) comp_state_out[c] = -1;
  if (objective_out) *objective_out = 0.0;
  trace_mark("decode_constrained: start");
  std::vector<ConSeq> cs;
  if ((st = constrained_validate(h, nseq, offsets, obs, component, ncomp, o, cs)) != CV_OK) return st;
  trace_mark("validate + constrained list");
  if (nseq == 0) return CV_OK;
  const std::vector<int32_t> pairs = conseq_pairs(cs, component);
  const int64_t npairs = (int64_t)pairs.size() / 2;
  std::vector<int64_t> part((size_t)cvcsp::partial_words((int)h->N, ncomp, npairs), 0);
  bool obs_staged = false;
  PrefixKeep keep;
  if ((st = constrained_partials_locked(h, nseq, offsets, obs, component, ncomp, pairs.data(), npairs, o,
                                        part.data(), &cs, &obs_staged, nullptr, &keep)) != CV_OK)
    return st;
  trace_mark("partials (device + exact sums)");
  uint64_t explored = 0;
  if ((st = select_locked((int32_t)h->N, ncomp, pairs.data(), npairs, part.data(), comp_state_out, &explored)) !=
      CV_OK)
    return st;
  h->last_explored = explored;
  trace_mark("select");
  return final_decode_host(h, nseq, offsets, obs, component, comp_state_out, o, cs, keep, obs_staged, path_out,
                           score_out, status_out, objective_out);
}

CV_API cv_status cv_decode_forced_components(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                             const int32_t* component, int32_t ncomp, const int32_t* comp_state,
                                             const cv_opts* opts, int32_t* path_out, double* score_out,
                                             uint8_t* status_out, double* objective_out) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq < 0 || ncomp < 0 || (nseq > 0 && (!offsets || !obs || !component || !path_out || !score_out ||
                                             !status_out)) || (ncomp > 0 && !comp_state))
    return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  cv_opts o = opts ? *opts : default_opts();
  if (o.forced) return set_err(CV_EINVAL, "opts->forced is derived from component/comp_state");
  if (objective_out) *objective_out = 0.0;
  if (nseq == 0) return CV_OK;
  if ((st = check_batch(h, nseq, offsets)) != CV_OK) return st;
  {
    const int64_t k =
        first_bad(offsets[0], offsets[nseq], [&](int64_t i) { return component[i] < -1 || component[i] >= ncomp; });
    if (k >= 0)
      return set_err(CV_EINVAL, "component[%lld] = %d out of range [-1,%d)", (long long)k, component[k], ncomp);
  }
  for (int32_t c = 0; c < ncomp; ++c)
    if (comp_state[c] < -1 || comp_state[c] >= h->N)
      return set_err(CV_EINVAL, "comp_state[%d] = %d out of range [-1,%lld)", c, comp_state[c], (long long)h->N);
  std::vector<ConSeq> cs;
  build_conseq(nseq, offsets, component, cs);
  return forced_decode_locked(h, nseq, offsets, obs, component, comp_state, o, cs, false, path_out, score_out,
                              status_out, objective_out);
}

CV_API cv_status cv_decode_constrained_device(cv_hmm* h, int64_t nseq, const int64_t* offsets_host,
                                              const int64_t* offsets_dev, const int32_t* obs_dev,
                                              const int32_t* component, int32_t ncomp, const cv_opts* opts,
                                              int32_t* path_dev, double* score_dev, uint8_t* status_dev,
                                              int32_t* comp_state_out, double* objective_out) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq < 0 || ncomp < 0 || (nseq > 0 && (!offsets_host || !offsets_dev || !obs_dev || !component || !path_dev ||
                                             !score_dev || !status_dev)) || (ncomp > 0 && !comp_state_out))
    return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  cv_opts o = opts ? *opts : default_opts();
  for (int32_t c = 0; c < ncomp; ++c) comp_state_out[c] = -1;
  if (objective_out) *objective_out = 0.0;
  if (constrained_dtype_check(h, o) != CV_OK) return CV_EUNSUPPORTED;
  if (o.forced) return set_err(CV_EINVAL, "opts->forced is set by the constrained decode itself");
  if (nseq == 0) return CV_OK;
  if ((st = check_batch(h, nseq, offsets_host)) != CV_OK) return st;
  hipStream_t stream = o.stream ? (hipStream_t)o.stream : h->stream;
  // the handle's shared buffers (ws_order, cs_zero, st_status) may still be in use by a
  // cv_decode_batch_device call on another stream: wait for it on this one
  if (h->ws_rec) HIP_TRY(hipStreamWaitEvent(stream, h->ws_done, 0));
  // the host API rejects a bad observation before any term is computed: same here, on the
  // device, checked while the host builds the constrained list
  if ((st = h->cs_zero.ensure(8)) != CV_OK) return st;
  unsigned long long first_bad_obs = 0;
  {
    const hipError_t err = cvk::launch_obs_first_bad(obs_dev, offsets_host[0], offsets_host[nseq], h->V,
                                                     h->cs_zero.as<unsigned long long>(), stream);
    if (err != hipSuccess) return set_err(CV_EDEVICE, "observation check failed: %s", hipGetErrorString(err));
    HIP_TRY(hipMemcpyAsync(&first_bad_obs, h->cs_zero.p, 8, hipMemcpyDeviceToHost, stream));
  }
  trace_mark("device constrained: entry, observation check enqueued");
  // components checked and the constrained list built in one host pass
  std::vector<ConSeq> cs;
  const int64_t bad_comp = build_conseq_checked(nseq, offsets_host, component, ncomp, cs);
  trace_mark("device constrained: host scan of component");
  HIP_TRY(hipStreamSynchronize(stream));  // first_bad_obs is a local the copy writes
  if (bad_comp >= 0)
    return set_err(CV_EINVAL, "component[%lld] = %d out of range [-1,%d)", (long long)bad_comp, component[bad_comp],
                   ncomp);
  if (first_bad_obs != ~0ull)
    return set_err(CV_EINVAL, "obs[%llu] out of range [0,%lld)", first_bad_obs, (long long)h->V);
  trace_mark("device constrained: checks + constrained list");
  // the unconstrained sequences beside the terms pass (tuning key, bit-identical: no_side = 1)
  SideJoin side{h};
  const bool side_off = h->tuning.no_side != 0;
  if (!side_off && o.dtype == CV_DTYPE_F64 && resume_supported(h, true) && !cs.empty()) {
    // the constrained work moves to a highest-priority stream (behind the caller's stream), the
    // side decode gets the lowest: its waves take the slots the constrained work leaves free
    if ((st = side_streams(h)) != CV_OK) return st;
    HIP_TRY(hipEventRecord(h->side.start, stream));
    HIP_TRY(hipStreamWaitEvent(h->side.hi, h->side.start, 0));
    stream = h->side.hi;
    o.stream = stream;
    side.hi = true;
  }
  auto launch_side = [&]() -> cv_status {
    return side.hi ? side_decode_launch(h, nseq, offsets_host, obs_dev, cs, o, path_dev, score_dev, status_dev, stream,
                                        &side.active)
                   : CV_OK;
  };
  const std::vector<int32_t> pairs = conseq_pairs(cs, component);
  const int64_t npairs = (int64_t)pairs.size() / 2;
  std::vector<int64_t> part((size_t)cvcsp::partial_words((int)h->N, ncomp, npairs), 0);
  PrefixKeep keep;
  if ((st = constrained_partials_locked(h, nseq, offsets_host, nullptr, component, ncomp, pairs.data(), npairs, o,
                                        part.data(), &cs, nullptr, obs_dev, &keep, launch_side)) != CV_OK)
    return st;
  uint64_t explored = 0;
  if ((st = select_locked((int32_t)h->N, ncomp, pairs.data(), npairs, part.data(), comp_state_out, &explored)) !=
      CV_OK)
    return st;
  h->last_explored = explored;
  trace_mark("select");
  if (keep.kept) {
    if ((st = forced_decode_resume(h, nseq, offsets_host, offsets_dev, obs_dev, component, comp_state_out, cs, keep,
                                   o, path_dev, score_dev, status_dev, stream, side.active)) != CV_OK)
      return st;
  } else {
    // the full forced decode covers every sequence: the side results land first, then are
    // rewritten with the same values
    if (side.active) HIP_TRY(hipStreamWaitEvent(stream, h->side.done, 0));
    if ((st = stage_forced_locked(h, offsets_host, nseq, component, comp_state_out, cs, stream)) != CV_OK) return st;
    o.forced = h->st_forced.as<int32_t>();
    if ((st = decode_device(h, nseq, offsets_host, offsets_dev, obs_dev, o, path_dev, score_dev, status_dev,
                            stream)) != CV_OK) {
      (void)hipStreamSynchronize(stream);
      return st;
    }
  }
  if (side.active) {  // the unconstrained sequences' results are in the outputs
    HIP_TRY(hipStreamWaitEvent(stream, h->side.done, 0));
    side.active = false;
  }
  // scores/statuses to the host for the objective (9 B per sequence), fixed up, and back
  std::vector<double> sc((size_t)nseq);
  std::vector<uint8_t> ss((size_t)nseq);
  HIP_TRY(hipMemcpyAsync(sc.data(), score_dev, (size_t)nseq * 8, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipMemcpyAsync(ss.data(), status_dev, (size_t)nseq, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  const double obj = mark_unassigned(nseq, component, comp_state_out, cs, sc.data(), ss.data());
  if (objective_out) *objective_out = obj;
  bool fixed = false;
  for (const auto& c : cs)
    for (int64_t e : c.elems) fixed |= comp_state_out[component[e]] < 0;
  if (fixed) {
    HIP_TRY(hipMemcpyAsync(score_dev, sc.data(), (size_t)nseq * 8, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipMemcpyAsync(status_dev, ss.data(), (size_t)nseq, hipMemcpyHostToDevice, stream));
    HIP_TRY(hipStreamSynchronize(stream));
  }
  trace_mark("forced decode (device)");
  return CV_OK;
}

CV_API cv_status cv_decode_constrained_exchange(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                                const int32_t* component, int32_t ncomp, int64_t npairs,
                                                const int32_t* pairs, cv_exchange_fn exchange, void* ctx,
                                                const cv_opts* opts, int32_t* path_out, double* score_out,
                                                uint8_t* status_out, int32_t* comp_state_out,
                                                uint64_t* explored_out, double* objective_out) {
  if (!h) return set_err(CV_EINVAL, "null handle");
  if (nseq < 0 || ncomp < 0 || npairs < 0 ||
      (nseq > 0 && (!offsets || !obs || !component || !path_out || !score_out || !status_out)) ||
      (ncomp > 0 && !comp_state_out) || (npairs > 0 && !pairs))
    return set_err(CV_EINVAL, "null argument");
  if (!pairs_sorted(pairs, npairs, ncomp)) return set_err(CV_EINVAL, "pairs must be sorted (c1 < c2) and unique");
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  cv_opts o = opts ? *opts : default_opts();
  for (int32_t c = 0; c < ncomp; ++c) comp_state_out[c] = -1;
  if (objective_out) *objective_out = 0.0;
  if (explored_out) *explored_out = 0;
  std::vector<ConSeq> cs;
  if (nseq > 0 && (st = constrained_validate(h, nseq, offsets, obs, component, ncomp, o, cs)) != CV_OK) return st;
  std::vector<int64_t> part((size_t)std::max<int64_t>(cvcsp::partial_words((int)h->N, ncomp, npairs), 1), 0);
  bool obs_staged = false;
  PrefixKeep keep;
  if (nseq > 0 && (st = constrained_partials_locked(h, nseq, offsets, obs, component, ncomp, pairs, npairs, o,
                                                    part.data(), &cs, &obs_staged, nullptr, &keep)) != CV_OK)
    return st;
  trace_mark("exchange: shard partials");
  if (exchange && exchange(part.data(), cvcsp::partial_words((int)h->N, ncomp, npairs), ctx) != 0)
    return set_err(CV_EDEVICE, "exchange callback failed");
  trace_mark("exchange: callback");
  uint64_t explored = 0;
  if ((st = select_locked((int32_t)h->N, ncomp, pairs, npairs, part.data(), comp_state_out, &explored)) != CV_OK)
    return st;
  h->last_explored = explored;
  if (explored_out) *explored_out = explored;
  if (nseq == 0) return CV_OK;
  return final_decode_host(h, nseq, offsets, obs, component, comp_state_out, o, cs, keep, obs_staged, path_out,
                           score_out, status_out, objective_out);
}

namespace {
// Sums the forward / backtrack event pairs of `launches` chunks from event `eb` on.
cv_status sum_timing(cv_hmm* h, size_t eb, int64_t launches, cv_timing* out) {
  if (launches == 0) return CV_OK;
  HIP_TRY(hipSetDevice(h->device));
  const int64_t L = launches;
  HIP_TRY(hipEventSynchronize(h->ev[eb + 4 * (L - 1) + 3]));
  for (int64_t c = 0; c < L; ++c) {
    float f = 0, b = 0;
    HIP_TRY(hipEventElapsedTime(&f, h->ev[eb + 4 * c], h->ev[eb + 4 * c + 1]));
    HIP_TRY(hipEventElapsedTime(&b, h->ev[eb + 4 * c + 2], h->ev[eb + 4 * c + 3]));
    out->fwd_ms += f;
    out->bt_ms += b;
  }
  float tot = 0;
  HIP_TRY(hipEventElapsedTime(&tot, h->ev[eb], h->ev[eb + 4 * (L - 1) + 3]));
  out->total_ms = tot;
  return CV_OK;
}
}  // namespace

CV_API cv_status cv_last_superseq_stats(const cv_hmm* h, int64_t* out) {
  if (!h || !out) return set_err(CV_EINVAL, "null argument");
  for (int q = 0; q < 9; ++q) out[q] = h->last_chain[q];
  return CV_OK;
}

CV_API cv_status cv_last_suffix_traced(const cv_hmm* h, int64_t* out) {
  if (!h || !out) return set_err(CV_EINVAL, "null argument");
  *out = h->last_traced;
  return CV_OK;
}

CV_API cv_status cv_last_timing(cv_hmm* h, cv_timing* out) {
  if (!h || !out) return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  std::memset(out, 0, sizeof *out);
  out->launches = h->last_launches;
  out->kernel = h->last_kernel;
  out->padded_states = h->last_np;
  out->mfma_tiles = h->last_mt;
  return sum_timing(h, h->last_ev_base, h->last_launches, out);
}

CV_API cv_status cv_timing_begin(cv_hmm* h) {
  if (!h) return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  h->acc_on = true;
  h->acc_overflow = false;
  h->acc_used = 0;
  return CV_OK;
}

CV_API cv_status cv_timing_end(cv_hmm* h, cv_timing* out) {
  if (!h || !out) return set_err(CV_EINVAL, "null argument");
  CV_LOCK(h);
  std::memset(out, 0, sizeof *out);
  const bool was_on = h->acc_on, overflow = h->acc_overflow;
  const size_t used = h->acc_used;
  h->acc_on = false;
  h->acc_overflow = false;
  h->acc_used = 0;
  if (!was_on && !overflow) return set_err(CV_EINVAL, "cv_timing_end without cv_timing_begin");
  if (overflow) return set_err(CV_ELIMIT, "more than %zu chunk launches timed since cv_timing_begin", kMaxTimedEvents / 4);
  out->launches = (int64_t)(used / 4);
  out->kernel = h->last_kernel;
  out->padded_states = h->last_np;
  out->mfma_tiles = h->last_mt;
  return sum_timing(h, 0, out->launches, out);
}

CV_API cv_status cv_viterbi_decode(cv_hmm* h, int64_t T, const int32_t* obs, int32_t* path_out) {
  if (!h || T < 0 || (T > 0 && (!obs || !path_out))) return set_err(CV_EINVAL, "bad argument");
  if (T == 0) return CV_OK;
  const int64_t off[2] = {0, T};
  double score;
  uint8_t status;
  cv_opts o;
  cv_opts_init(&o);
  o.dtype = CV_DTYPE_F64;
  o.assoc = CV_ASSOC_DECODE;
  o.rescore_f64 = 0;
  return cv_decode_batch(h, 1, off, obs, &o, path_out, &score, &status);
}

}  // extern "C"

namespace {
// The chain's segmented backtrack (kernels/chain.hip) over psi [L][NP] from `end_state` at the
// last element: pass 1 maps every segment's last-element state to the state before it for all
// NP states (cp_chain_seg_map), the host follows the maps from the end state, pass 2 writes
// each segment's path into path_dev[0, L).
cv_status chain_backtrack(int NP, const uint16_t* psi, int64_t L, int32_t end_state, int32_t* path_dev,
                          hipStream_t stream) {
  // segments: ~8,192 of them (>= 256 elements each) for the parallel passes
  const int64_t seg = std::max<int64_t>(256, (L + 8191) / 8192);
  const int64_t nseg = (L + seg - 1) / seg;
  DevBuf d_map, d_end;
  cv_status st;
  if ((st = d_map.ensure((size_t)nseg * NP * 2)) != CV_OK) return st;
  if ((st = d_end.ensure((size_t)nseg * 4)) != CV_OK) return st;
  cvk::CpChainBtArgs b{};
  b.psi = psi;
  b.np = NP;
  b.len = L;
  b.seg = seg;
  b.nseg = nseg;
  b.map = d_map.as<uint16_t>();
  b.end_state = d_end.as<int32_t>();
  b.path = path_dev;
  hipError_t err = cvk::launch_cp_chain_seg_map(b, stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "chain backtrack (maps) failed: %s", hipGetErrorString(err));
  std::vector<uint16_t> map((size_t)nseg * NP);
  if (nseg > 1) {
    HIP_TRY(hipMemcpyAsync(map.data(), d_map.p, map.size() * 2, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
  }
  std::vector<int32_t> end((size_t)nseg);
  int32_t s = end_state;
  for (int64_t k = nseg - 1; k >= 0; --k) {
    end[(size_t)k] = s;
    if (k > 0) s = map[(size_t)k * NP + s];
  }
  HIP_TRY(hipMemcpyAsync(d_end.p, end.data(), (size_t)nseg * 4, hipMemcpyHostToDevice, stream));
  err = cvk::launch_cp_chain_seg_path(b, stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "chain backtrack (paths) failed: %s", hipGetErrorString(err));
  HIP_TRY(hipStreamSynchronize(stream));  // `end` is a local buffer
  return CV_OK;
}

// cv_decode_superseq_cp for N <= 256: the chain forward (cp_chain_wg) writes psi [L][NP] u16
// and the final state, then the segmented backtrack (chain_backtrack).
cv_status superseq_cp_wg(cv_hmm* h, int64_t L, const int32_t* obs, const std::vector<uint8_t>& first,
                         int32_t* path_out, double* objective_out) {
  cv_status st;
  if ((st = ensure_t64_tables(h)) != CV_OK) return st;
  const int NP = h->np64;
  const uint64_t psi_bytes = (uint64_t)L * NP * 2;
  const uint64_t avail = free_device_bytes(0);
  if (avail && psi_bytes + (uint64_t)L * 9 > avail / 10 * 9)
    return set_err(CV_ENOMEM,
                   "super-sequence of %lld elements needs %.1f GB of back-pointers (%.1f GB of device memory "
                   "free): decode it in parts or per sequence (solver kind gpu-cp-seq)",
                   (long long)L, psi_bytes / 1e9, avail / 1e9);
  hipStream_t stream = h->stream;
  DevBuf d_obs, d_first, d_psi, d_path, d_out;
  if ((st = d_obs.ensure((size_t)L * 4)) != CV_OK) return st;
  if ((st = d_first.ensure((size_t)L)) != CV_OK) return st;
  if ((st = d_psi.ensure((size_t)psi_bytes)) != CV_OK) return st;
  if ((st = d_path.ensure((size_t)L * 4)) != CV_OK) return st;
  if ((st = d_out.ensure(16)) != CV_OK) return st;
  HIP_TRY(hipMemcpyAsync(d_obs.p, obs, (size_t)L * 4, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(d_first.p, first.data(), (size_t)L, hipMemcpyHostToDevice, stream));
  cvk::CpChainWgArgs g{};
  g.pi = h->q_pi.as<double>();
  g.a = h->q_a.as<double>();
  g.et = h->q_et.as<double>();
  g.obs = d_obs.as<int32_t>();
  g.first = d_first.as<uint8_t>();
  g.len = L;
  g.nstates = h->N;
  g.psi = d_psi.as<uint16_t>();
  g.objective = d_out.as<double>();
  g.final_state = reinterpret_cast<int32_t*>(d_out.as<double>() + 1);
  hipError_t err = cvk::launch_cp_chain_wg(NP, g, stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "super-sequence chain launch failed: %s", hipGetErrorString(err));
  double out[2];
  HIP_TRY(hipMemcpyAsync(out, d_out.p, 16, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  *objective_out = out[0];
  int32_t fs;
  std::memcpy(&fs, &out[1], 4);
  if ((st = chain_backtrack(NP, d_psi.as<uint16_t>(), L, fs, d_path.as<int32_t>(), stream)) != CV_OK) return st;
  HIP_TRY(hipMemcpyAsync(path_out, d_path.p, (size_t)L * 4, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  if (!(*objective_out > -INFINITY))
    return set_err(CV_EINFEASIBLE, "no finite-probability path through the super-sequence (cp.rs:87 asserts)");
  return CV_OK;
}

// ---- the parallel chain (DESIGN.md §3 "parallel CPSolver chain") -------------------------
// The chain couples sequence k to sequences 0..k-1 only through M, the running maximum its
// start values carry (fl(M + fl(pi + b)) when the previous row's maximum is clean).  So:
//  1. every sequence is decoded ON ITS OWN by the row-A0 f64 trellis (the batch hot path, all
//     sequences in parallel) and cp_cert_f64 reduces its path's gaps to a certificate rho
//     (trellis64.h: the row-A0 path is the chain's path in sequence k at offset M whenever
//     rho > U = 2^-52 (|M| + |S_k| + 16));
//  2. the host walks the sequences in order: a certified sequence's maximum is the CP fold of
//     its path from M -- M + q 2^(e-52) with cp_quant_f64's quantised arc sum q when M and the
//     sequence's values share the binade 2^e predicted from the per-sequence optima, else
//     element by element -- and its end state is its path's; the boundary into the next
//     sequence must be clean (gF);
//  3. the uncertified sequences (near ties at the chain's magnitude, rho <= U) are re-decoded
//     IN PARALLEL by the per-sequence CP kernel from the offsets a fold along the row-A0 paths
//     predicts (speculation); a result is the chain's own when its offset was the chain's exact
//     maximum and its start and end boundaries are clean;
//  4. what speculation cannot settle runs through the serial chain kernel itself (cp_chain_wg)
//     from the exact previous row -- a synthetic one (M at the previous end state, -inf
//     elsewhere: what a clean boundary sees) or the previous sequence's exact last row -- and
//     consecutive such sequences form one run, backtracked from the state the next sequence's
//     boundary picks.
// Bit-identical to the serial chain by construction (tests: the serial chain, CV_CHAIN_PAR=0,
// and the C oracle cvo_cp_superseq_f64).  Models with entries outside [-2^80, 0] or infeasible
// sequences: *applied = false (the caller runs the serial chain).
// Any N (round 5): N <= 256 on the padded f64 trellis + trellis_cp_f64 + cp_chain_wg; above
// that, step 1 runs whatever row-A0 f64 decode the batch path picks (the NP = 512 / 1,024
// trellis or the generic kernels' rows mode, both with certificates), speculation the generic
// CP kernel, and the runs cp_superseq_chain (one thread per state) with the segmented backtrack.
// Knobs (bit-identical): CV_CHAIN_PAR=0 (serial chain), CV_CHAIN_PAR_FORCE=m (every m-th
// non-empty sequence taken as uncertified: exercises speculation and the runs), CV_CHAIN_SPEC=0
// (no speculation: every uncertified sequence through the serial chain kernel).

cv_status superseq_cp_par(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs, int32_t* path_out,
                          double* objective_out, bool* applied) {
  *applied = false;
  cv_status st;
  const int N = h->N;
  const bool small = cvk::t64_padded_states(N) != 0;  // N <= 256: padded tables, cp_chain_wg runs
  // the certificates need the generic kernels' rows mode, which keeps its rows in LDS
  // (N <= 10,240): above it the serial chain runs
  if (N > cvk::generic_max_states(8)) return CV_OK;
  if (small && (st = ensure_t64_tables(h)) != CV_OK) return st;
  if ((st = ensure_f64_tables(h)) != CV_OK) return st;
  if (!model_nonpos(h)) return CV_OK;
  const int W = small ? h->np64 : N;  // row width of the runs (psi rows, start / last rows)
  const int64_t V = h->V;
  const int64_t base = offsets[0], L = offsets[nseq] - base;
  hipStream_t stream = h->stream;
  trace_mark("chain: start");
  std::vector<int64_t> off((size_t)nseq + 1);
  int64_t maxT = 0;
  for (int64_t k = 0; k <= nseq; ++k) off[(size_t)k] = offsets[k] - base;
  for (int64_t k = 0; k < nseq; ++k) maxT = std::max(maxT, off[(size_t)k + 1] - off[(size_t)k]);
  // 1. the per-sequence row-A0 decode with certificates -- in parts where N <= 256 and the
  // batch spans more than a forward round: the walk over each part (its end states, quantised
  // folds, gathered paths, runs and speculative batches, all on the chain stream) runs while
  // the next part's forward pass holds the chip, so only the last part's share of that work
  // follows the last forward (tuning key chain_parts = 0: one part)
  DevBuf &d_off = h->chainb.off, &d_obs = h->chainb.obs, &d_path = h->chainb.path, &d_res = h->chainb.res,
         &d_cert = h->chainb.cert;
  if ((st = d_off.ensure((size_t)(nseq + 1) * 8)) != CV_OK) return st;
  if ((st = d_obs.ensure((size_t)L * 4)) != CV_OK) return st;
  if ((st = d_path.ensure((size_t)L * 4)) != CV_OK) return st;
  if ((st = d_res.ensure((size_t)nseq * 9)) != CV_OK) return st;
  if ((st = d_cert.ensure((size_t)nseq * 16)) != CV_OK) return st;
  double* d_score = d_res.as<double>();
  uint8_t* d_status = reinterpret_cast<uint8_t*>(d_score + nseq);
  // the certified backtrack's rho_cap (T64BtArgs): above every U = 2^-52 (|M| + |S_k| + 16) the
  // walk can test -- |M| and every |S_k| are at most L w, w the largest finite arc magnitude
  // |pi| or |a| plus |b| (every term <= 0) -- so its certificates decide like the exact ones
  if (h->arc_max < 0.0) {
    auto fmax_abs = [](const std::vector<double>& v) {
      double m = 0.0;
      for (double x : v)
        if (std::isfinite(x)) m = std::max(m, std::fabs(x));
      return m;
    };
    h->arc_max = std::max(fmax_abs(h->pi), fmax_abs(h->a)) + fmax_abs(h->b);
  }
  h->cert_rho_cap = 0x1p-52 * (2.0 * (double)L * h->arc_max + 16.0) * (1.0 + 0x1p-20);
  cv_opts o = default_opts();
  o.dtype = CV_DTYPE_F64;
  o.assoc = CV_ASSOC_VITERBI;
  o.kernel = small ? CV_KERNEL_TRELLIS_F64 : CV_KERNEL_AUTO;  // N > 256: the batch path's own pick
  o.rescore_f64 = 0;
  o.stream = stream;
  // The paths reach the caller's (pageable) buffer from a host thread of their own, one copy
  // per decode chunk behind that chunk's backtrack (a pageable D2H blocks its calling thread),
  // beside the later forward passes and the walk, which needs only the end states and the
  // paths of the few sequences it may fold element by element (fetched packed).  Tuning key
  // chain_copy_overlap = 0: one part, the copy before the walk.
  const bool overlap_copy = h->tuning.chain_copy_overlap != 0;
  // the parts: part p's walk runs beside part p + 1's forward pass, part p + 1's observations
  // cross during part p's.  A forward round is 64 sequences per CU (eight per wave); a launch
  // of one round pays its own fill and drain (one round alone: 36.8 ms vs 33.5 ms per round of
  // a four-round launch), while half a round runs at four per wave in half the time.  Tuning key
  // chain_parts = 1 (default): one large first part, then chain_tail parts of a round /
  // chain_tail_div each (config 4: 49,152 + 8,192 + 8,192), so only a small part's work follows
  // the last forward; 2: one round per part
  std::vector<int64_t> pb{0};
  if (small && overlap_copy && h->tuning.chain_parts != 0) {
    const int64_t unit = 64 * (int64_t)std::max(h->cus, 1);
    if (h->tuning.chain_parts == 2) {
      for (int64_t s = unit; s + unit <= nseq; s += unit) pb.push_back(s);
    } else {
      const int64_t ntail = std::max(0, h->tuning.chain_tail);
      const int64_t tsz = std::max<int64_t>(1, unit / std::max(1, h->tuning.chain_tail_div));
      if (ntail > 0 && nseq >= unit + ntail * tsz)
        for (int64_t i = ntail; i >= 1; --i) pb.push_back(nseq - i * tsz);
    }
  }
  pb.push_back(nseq);
  const int nparts = (int)pb.size() - 1;
  if (!h->chain_stream) {
    int least = 0, greatest = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIP_TRY(hipStreamCreateWithPriority(&h->chain_stream, hipStreamNonBlocking, greatest));
  }
  hipStream_t cs = h->chain_stream;
  // events: [0, nparts) each part's decode done, [nparts, 2 nparts) each part's observations in
  std::vector<hipEvent_t> part_done((size_t)nparts), obs_in((size_t)nparts);
  for (int p = 0; p < nparts; ++p) {
    part_done[(size_t)p] = get_event(h->part_ev, (size_t)p);
    obs_in[(size_t)p] = get_event(h->part_ev, (size_t)(nparts + p));
    if (!part_done[(size_t)p] || !obs_in[(size_t)p]) return set_err(CV_EDEVICE, "hipEventCreate failed");
  }
  if (!h->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
  HIP_TRY(hipMemcpyAsync(d_off.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, stream));
  // the later parts' observations through pinned memory (host threads fill it while the first
  // part's forward runs; a pageable copy would run the runtime's blit kernels beside it)
  const int64_t eo = off[(size_t)pb[std::min(1, nparts)]];
  int32_t* obs_pin = nullptr;
  if (nparts > 1 && h->tuning.chain_pin_obs != 0 && h->chain_obs_pin.ensure((size_t)(L - eo) * 4))
    obs_pin = h->chain_obs_pin.as<int32_t>();
  std::vector<std::pair<int64_t, int64_t>> dchunks;
  for (int p = 0; p < nparts; ++p) {
    const int64_t s0 = pb[p], s1 = pb[p + 1], e0 = off[(size_t)s0], e1 = off[(size_t)s1];
    // the second part's observations cross on the copy stream while the first part's forward runs
    hipStream_t hs = p == 0 ? stream : h->copy_stream;
    if (p > 0 && obs_pin) {
      int32_t* dst = obs_pin + (e0 - eo);
      const int32_t* src = obs + base + e0;
      parallel_ranges(e1 - e0, [&](int, int64_t a, int64_t b) { std::memcpy(dst + a, src + a, (size_t)(b - a) * 4); });
      HIP_TRY(hipMemcpyAsync(d_obs.as<int32_t>() + e0, dst, (size_t)(e1 - e0) * 4, hipMemcpyHostToDevice, hs));
    } else {
      HIP_TRY(hipMemcpyAsync(d_obs.as<int32_t>() + e0, obs + base + e0, (size_t)(e1 - e0) * 4, hipMemcpyHostToDevice, hs));
    }
    if (p > 0) {
      HIP_TRY(hipEventRecord(obs_in[(size_t)p], hs));
      HIP_TRY(hipStreamWaitEvent(stream, obs_in[(size_t)p], 0));
    }
    if (trace_on() && p == 0) {  // phase split (CV_TRACE only: the syncs cost overlap)
      HIP_TRY(hipStreamSynchronize(stream));
      trace_mark("chain: obs H2D (first part)");
    }
    const size_t c0 = dchunks.size();
    st = decode_device(h, s1 - s0, off.data() + s0, d_off.as<int64_t>() + s0, d_obs.as<int32_t>(), o,
                       d_path.as<int32_t>(), d_score + s0, d_status + s0, stream, nullptr, false,
                       d_cert.as<double>() + 2 * s0, nullptr, nullptr, &dchunks);
    if (st == CV_EUNSUPPORTED && !small) {  // no rows to certify (generic_rows = 0): the serial chain
      g_err.clear();                         // runs, and the public call succeeds
      return CV_OK;
    }
    if (st != CV_OK) return st;
    for (size_t i = c0; i < dchunks.size(); ++i) dchunks[i] = {dchunks[i].first + s0, dchunks[i].second + s0};
    HIP_TRY(hipEventRecord(part_done[(size_t)p], stream));
  }
  std::vector<double> score((size_t)nseq), cert((size_t)nseq * 2);
  std::vector<uint8_t> status((size_t)nseq);
  std::vector<int32_t> ends((size_t)nseq);
  // the copy thread; any return below joins it first (it writes into the caller's buffer)
  struct CopyThread {
    std::thread t;
    hipError_t err = hipSuccess;
    ~CopyThread() { join(); }
    void join() {
      if (t.joinable()) t.join();
    }
  } copy;
  {
    const int dev = h->device;
    hipStream_t cps = h->copy_stream;
    std::vector<hipEvent_t> evs(h->chunk_ev.begin(), h->chunk_ev.begin() + (ptrdiff_t)dchunks.size());
    int32_t* dp = d_path.as<int32_t>();
    // pinned two-chunk ring (tuning key chain_pin_path): chunk j's DMA into ring[j % 2] while the
    // thread moves chunk j - 1 into the caller's buffer
    static constexpr int64_t kRing = (int64_t)4 << 20;  // elements per ring chunk (16 MiB)
    int32_t* ring[2] = {nullptr, nullptr};
    if (h->tuning.chain_pin_path != 0 && h->chain_ring[0].ensure((size_t)kRing * 4) &&
        h->chain_ring[1].ensure((size_t)kRing * 4)) {
      for (int b = 0; b < 2; ++b)
        if (!h->ring_ev[b] && hipEventCreateWithFlags(&h->ring_ev[b], hipEventDisableTiming) != hipSuccess) {
          (void)hipGetLastError();
          h->ring_ev[b] = nullptr;
        }
      if (h->ring_ev[0] && h->ring_ev[1]) {
        ring[0] = h->chain_ring[0].as<int32_t>();
        ring[1] = h->chain_ring[1].as<int32_t>();
      }
    }
    hipEvent_t rev[2] = {h->ring_ev[0], h->ring_ev[1]};
    auto run_copies = [&copy, dev, cps, evs, dchunks, off, path_out, dp, ring, rev]() {
      if ((copy.err = hipSetDevice(dev)) != hipSuccess) return;
      if (!ring[0]) {
        for (size_t i = 0; i < dchunks.size(); ++i) {
          const int64_t e0 = off[(size_t)dchunks[i].first], e1 = off[(size_t)dchunks[i].second];
          if ((copy.err = hipStreamWaitEvent(cps, evs[i], 0)) != hipSuccess) return;
          if (e1 > e0 &&
              (copy.err = hipMemcpyAsync(path_out + e0, dp + e0, (size_t)(e1 - e0) * 4, hipMemcpyDeviceToHost, cps)) !=
                  hipSuccess)
            return;
        }
        copy.err = hipStreamSynchronize(cps);
        return;
      }
      int64_t pend[2][2] = {{0, 0}, {0, 0}};  // [buffer] = {first element, count} in flight
      int j = 0;
      auto drain = [&](int b) -> bool {
        if (pend[b][1] == 0) return true;
        if ((copy.err = hipEventSynchronize(rev[b])) != hipSuccess) return false;
        std::memcpy(path_out + pend[b][0], ring[b], (size_t)pend[b][1] * 4);
        pend[b][1] = 0;
        return true;
      };
      for (size_t i = 0; i < dchunks.size(); ++i) {
        const int64_t e0 = off[(size_t)dchunks[i].first], e1 = off[(size_t)dchunks[i].second];
        if ((copy.err = hipStreamWaitEvent(cps, evs[i], 0)) != hipSuccess) return;
        for (int64_t a = e0; a < e1; a += kRing, ++j) {
          const int b = j & 1;
          const int64_t n = std::min(kRing, e1 - a);
          if (!drain(b)) return;
          if ((copy.err = hipMemcpyAsync(ring[b], dp + a, (size_t)n * 4, hipMemcpyDeviceToHost, cps)) != hipSuccess ||
              (copy.err = hipEventRecord(rev[b], cps)) != hipSuccess)
            return;
          pend[b][0] = a;
          pend[b][1] = n;
        }
      }
      if (drain(j & 1)) drain((j + 1) & 1);
    };
    if (overlap_copy)
      copy.t = std::thread(run_copies);
    else
      run_copies();
  }
  if (!overlap_copy && copy.err != hipSuccess)
    return set_err(CV_EDEVICE, "chain path copy failed: %s", hipGetErrorString(copy.err));
  // every buffer the walk may need, sized now: growing one later would free the old one, a
  // device-wide synchronisation that would wait for the second part's forward pass
  constexpr int64_t kSpecMax = 16384;  // sequences per speculative batch
  constexpr int64_t kSpecBeside = 2048;  // ... beside a forward pass (cp_spec_psi's psi rows, sized up front)
  DevBuf &d_ends = h->chainb.ends, &d_ebin = h->chainb.ebin, &d_q = h->chainb.q, &d_gid = h->chainb.gid,
         &d_gpath = h->chainb.gpath;
  if ((st = d_ends.ensure((size_t)nseq * 4)) != CV_OK) return st;
  if ((st = d_ebin.ensure((size_t)nseq * 4)) != CV_OK) return st;
  if ((st = d_q.ensure((size_t)nseq * 9)) != CV_OK) return st;
  if ((st = d_gid.ensure((size_t)nseq * 16)) != CV_OK) return st;
  DevBuf &d_first = h->chainb.first, &d_rpsi = h->chainb.rpsi, &d_rows = h->chainb.rows, &d_small = h->chainb.small,
         &d_rpath = h->chainb.rpath;
  DevBuf &d_soff = h->chainb.soff, &d_sobs = h->chainb.sobs, &d_spath = h->chainb.spath, &d_sres = h->chainb.sres,
         &d_sinit = h->chainb.sinit, &d_slast = h->chainb.slast;
  if (nparts > 1) {
    const int64_t nspec = std::min<int64_t>(nseq, kSpecMax), lspec = std::min<int64_t>(L, nspec * maxT);
    if ((st = d_gpath.ensure((size_t)L * 4)) != CV_OK) return st;
    if ((st = d_soff.ensure((size_t)(nspec + 1) * 8)) != CV_OK) return st;
    if ((st = d_sobs.ensure((size_t)lspec * 4)) != CV_OK) return st;
    if ((st = d_spath.ensure((size_t)lspec * 4)) != CV_OK) return st;
    if ((st = d_sres.ensure((size_t)nspec * 9)) != CV_OK) return st;
    if ((st = d_sinit.ensure((size_t)nspec * 8)) != CV_OK) return st;
    if ((st = d_slast.ensure((size_t)nspec * N * 8)) != CV_OK) return st;
    if ((st = d_rpsi.ensure((size_t)std::max<int64_t>(4 * maxT, 1) * W * 2)) != CV_OK) return st;
    if ((st = d_rpath.ensure((size_t)std::max<int64_t>(4 * maxT, 1) * 4)) != CV_OK) return st;
    // psi rows of the speculative batches beside a forward (cp_spec_psi): up to kSpecBeside
    // sequences' worth (a batch beside a forward stops there)
    if (small && (st = h->chainb.spsi.ensure((size_t)std::min<int64_t>(L, kSpecBeside * std::max<int64_t>(maxT, 1)) * W *
                                             2)) != CV_OK)
      return st;
  }
  if (!h->chain_pin.ensure((size_t)nseq * 29)) return set_err(CV_ENOMEM, "pinned chain staging failed");
  unsigned char* pin = h->chain_pin.as<unsigned char>();
  // the walk's small D2H copies (gathered paths, speculative paths and last rows) through pinned
  // memory: a pageable copy is staged by the runtime and queued behind the path copy's
  constexpr size_t kGpin = (size_t)16 << 20;
  unsigned char* gpin = h->chain_gpin.ensure(kGpin) ? h->chain_gpin.as<unsigned char>() : nullptr;
  auto d2h_small = [&](void* dst, const void* src, size_t bytes, size_t pin_off) -> hipError_t {
    if (gpin && pin_off + bytes <= kGpin) {
      hipError_t e = hipMemcpyAsync(gpin + pin_off, src, bytes, hipMemcpyDeviceToHost, cs);
      if (e == hipSuccess) e = hipStreamSynchronize(cs);
      if (e == hipSuccess) std::memcpy(dst, gpin + pin_off, bytes);
      return e;
    }
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, cs);
    return e == hipSuccess ? hipStreamSynchronize(cs) : e;
  };
  double pimax = 0.0;
  for (double x : h->pi)
    if (std::isfinite(x)) pimax = std::max(pimax, std::fabs(x));
  const int force_m = std::max(0, h->tuning.chain_par_force);
  const bool spec_env = h->tuning.chain_spec != 0;  // 0: every uncertified sequence re-run serially
  const int32_t* ob = obs + base;
  std::vector<int32_t> ebin((size_t)nseq, cvk::CVK_NO_BINADE);
  std::vector<long long> qv((size_t)nseq);
  std::vector<uint8_t> tie((size_t)nseq);
  // The row-A0 paths the walk folds element by element: the sequences whose certificate may
  // fail at the running maximum the walk will see (predicted from the optima, with a 2x margin
  // on every bound), those without a quantised fold, and each one's successor, fetched packed
  // while the copy thread fills the caller's buffer; any other sequence the walk needs waits
  // for that copy (counted in path_waits).
  std::vector<int32_t> gpath;
  std::vector<int64_t> gpos((size_t)nseq, -1);
  bool copy_joined = !overlap_copy;
  int64_t path_waits = 0, gathered = 0, memo_hits = 0;
  std::vector<int64_t> ks;  // the non-empty sequences, in order (the walk's positions)
  // the prediction walk's certify() results, reused by the exact walk wherever it arrives at a
  // sequence after a certified one with the same running maximum, bit for bit (certify is a
  // function of the sequence, the maximum and the predecessor's kind): memo_in[x] = that
  // maximum, memo_out[x] = the fold (NaN: not certified), memo_q[x] = quantised (2 = no memo)
  std::vector<double> memo_in, memo_out;
  std::vector<uint8_t> memo_q;
  double mp_bin = 0.0, mp_cand = 0.0, smax = 0.0;  // running sums of |score| (binades, candidates)
  bool prev_cand = false, fallback = false;
  int64_t xc = 0;
  // 2. one part's end states, scores, statuses and certificates (through the pinned buffer),
  // predicted binades, quantised folds and gathered candidate paths, on the chain stream behind
  // the part's decode
  auto prep = [&](int p) -> cv_status {
    const int64_t s0 = pb[p], s1 = pb[p + 1], n = s1 - s0;
    HIP_TRY(hipStreamWaitEvent(cs, part_done[(size_t)p], 0));
    {
      const hipError_t e = cvk::launch_cp_seq_ends(d_path.as<int32_t>(), d_off.as<int64_t>() + s0, n,
                                                   d_ends.as<int32_t>() + s0, cs);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "chain end states failed: %s", hipGetErrorString(e));
    }
    HIP_TRY(hipMemcpyAsync(pin + s0 * 8, d_score + s0, (size_t)n * 8, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(pin + nseq * 8 + s0, d_status + s0, (size_t)n, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(pin + nseq * 9 + s0 * 16, d_cert.as<double>() + 2 * s0, (size_t)n * 16,
                           hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(pin + nseq * 25 + s0 * 4, d_ends.as<int32_t>() + s0, (size_t)n * 4, hipMemcpyDeviceToHost,
                           cs));
    HIP_TRY(hipStreamSynchronize(cs));
    std::memcpy(score.data() + s0, pin + s0 * 8, (size_t)n * 8);
    std::memcpy(status.data() + s0, pin + nseq * 8 + s0, (size_t)n);
    std::memcpy(cert.data() + 2 * s0, pin + nseq * 9 + s0 * 16, (size_t)n * 16);
    std::memcpy(ends.data() + s0, pin + nseq * 25 + s0 * 4, (size_t)n * 4);
    trace_mark("chain: part's scores, certificates, end states D2H");
    for (int64_t k = s0; k < s1; ++k)
      if (status[(size_t)k] == CV_SEQ_BADOBS) {  // the caller's observations were not scanned on the host
        const int64_t V = h->V;
        const int64_t e = first_bad(base, offsets[nseq], [&](int64_t i) { return obs[i] < 0 || obs[i] >= V; });
        return set_err(CV_EINVAL, "obs[%lld] = %d out of range [0,%lld)", (long long)e, e >= 0 ? obs[e] : 0,
                       (long long)V);
      }
    for (int64_t k = s0; k < s1; ++k)
      if (status[(size_t)k] != CV_SEQ_OK && status[(size_t)k] != CV_SEQ_EMPTY) {
        fallback = true;  // the serial chain
        return CV_OK;
      }
    // predicted binades and the quantised folds of every path
    for (int64_t k = s0; k < s1; ++k) {
      if (off[(size_t)k + 1] == off[(size_t)k]) continue;
      const double em = std::fabs(mp_bin), sk = std::fabs(score[(size_t)k]);
      if (em >= 0x1p12) {
        const int e = std::ilogb(em);
        // the prediction is off by far less than 2^-20 relative: both ends of the sequence's
        // value range stay in the binade with that margin
        if (std::ilogb(em * (1.0 - 0x1p-20)) == e && std::ilogb((em + sk + 16.0) * (1.0 + 0x1p-20)) == e)
          ebin[(size_t)k] = e;
      }
      mp_bin -= sk;
    }
    HIP_TRY(hipMemcpyAsync(d_ebin.as<int32_t>() + s0, ebin.data() + s0, (size_t)n * 4, hipMemcpyHostToDevice, cs));
    {
      cvk::CpQuant64Args qa{};
      qa.a = small ? h->q_a.as<double>() : h->d_a64.as<double>();
      qa.pi = small ? h->q_pi.as<double>() : h->d_pi64.as<double>();
      qa.et = small ? h->q_et.as<double>() : h->d_et64.as<double>();
      qa.np = W;
      qa.offsets = d_off.as<int64_t>() + s0;
      qa.obs = d_obs.as<int32_t>();
      qa.path = d_path.as<int32_t>();
      qa.ebin = d_ebin.as<int32_t>() + s0;
      qa.nseq = n;
      qa.q = d_q.as<long long>() + s0;
      qa.tie = reinterpret_cast<uint8_t*>(d_q.as<long long>() + nseq) + s0;
      const hipError_t err = cvk::launch_cp_quant(qa, cs);
      if (err != hipSuccess) return set_err(CV_EDEVICE, "chain quantised folds failed: %s", hipGetErrorString(err));
    }
    HIP_TRY(hipMemcpyAsync(qv.data() + s0, d_q.as<long long>() + s0, (size_t)n * 8, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(tie.data() + s0, reinterpret_cast<uint8_t*>(d_q.as<long long>() + nseq) + s0, (size_t)n,
                           hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    trace_mark("chain: quantised folds");
    const size_t x0 = ks.size();
    for (int64_t k = s0; k < s1; ++k) {
      if (off[(size_t)k + 1] > off[(size_t)k]) ks.push_back(k);
      smax = std::max(smax, std::fabs(score[(size_t)k]));
    }
    memo_in.resize(ks.size());
    memo_out.resize(ks.size());
    memo_q.resize(ks.size(), 2);
    // candidates (the successor of the part's last candidate is the next part's first sequence:
    // prev_cand carries over)
    std::vector<int64_t> gids, gdst;
    const int64_t gbase = (int64_t)gpath.size();
    int64_t tot = 0;
    for (size_t xi = x0; xi < ks.size(); ++xi) {
      const int64_t k = ks[xi];
      const int64_t T = off[(size_t)k + 1] - off[(size_t)k];
      const double S = std::fabs(score[(size_t)k]);
      const double Up = 0x1p-52 * (mp_cand * (1.0 + 0x1p-8) + S + 16.0);
      const double Up1 = 0x1p-52 * ((mp_cand + S) * (1.0 + 0x1p-8) + smax + pimax + 16.0);
      const double rho = cert[(size_t)k * 2], gF = cert[(size_t)k * 2 + 1];
      const bool cand = !(rho > 2.0 * Up) || !(gF - 6.0 * (double)T * Up > 4.0 * Up1) || tie[(size_t)k] ||
                        ebin[(size_t)k] == cvk::CVK_NO_BINADE ||
                        (force_m > 0 && (int64_t)(xc % (int64_t)force_m) == force_m - 1);
      if (cand || prev_cand) {
        gids.push_back(k);
        gdst.push_back(tot);
        gpos[(size_t)k] = gbase + tot;
        tot += T;
      }
      prev_cand = cand;
      mp_cand += S;
      ++xc;
    }
    gathered += (int64_t)gids.size();
    trace_mark("chain: candidates listed");
    if (!copy_joined && !gids.empty()) {
      const int64_t ng = (int64_t)gids.size();
      if ((st = d_gid.ensure((size_t)ng * 16)) != CV_OK || (st = d_gpath.ensure((size_t)tot * 4)) != CV_OK) return st;
      gids.insert(gids.end(), gdst.begin(), gdst.end());
      HIP_TRY(hipMemcpyAsync(d_gid.p, gids.data(), gids.size() * 8, hipMemcpyHostToDevice, cs));
      const hipError_t e = cvk::launch_cp_gather_paths(d_path.as<int32_t>(), d_off.as<int64_t>(), d_gid.as<int64_t>(),
                                                       d_gid.as<int64_t>() + ng, ng, d_gpath.as<int32_t>(), cs);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "chain path gather failed: %s", hipGetErrorString(e));
      gpath.resize((size_t)(gbase + tot));
      HIP_TRY(d2h_small(gpath.data() + gbase, d_gpath.p, (size_t)tot * 4, 0));
    }
    trace_mark("chain: candidate paths gathered");
    return CV_OK;
  };
  auto join_copy = [&]() -> cv_status {
    if (copy_joined) return CV_OK;
    copy.join();
    copy_joined = true;
    if (copy.err != hipSuccess) return set_err(CV_EDEVICE, "chain path copy failed: %s", hipGetErrorString(copy.err));
    return CV_OK;
  };
  cv_status path_st = CV_OK;
  auto seq_path = [&](int64_t k) -> const int32_t* {  // sequence k's row-A0 path
    if (!copy_joined && gpos[(size_t)k] >= 0) return gpath.data() + gpos[(size_t)k];
    if (!copy_joined) {
      ++path_waits;
      if (path_st == CV_OK) path_st = join_copy();
    }
    return path_out + off[(size_t)k];
  };
  auto fold_elems = [&](int64_t k, double M) {  // the CP fold of sequence k's path from M
    const int64_t e0 = off[(size_t)k], T = off[(size_t)k + 1] - e0;
    const int32_t* P = seq_path(k);
    int32_t p = P[0];
    double d = M + (h->pi[(size_t)p] + h->b[(size_t)p * V + ob[e0]]);
    for (int64_t t = 1; t < T; ++t) {
      const int32_t c = P[t];
      d = d + (h->a[(size_t)p * N + c] + h->b[(size_t)c * V + ob[e0 + t]]);
      p = c;
    }
    return d;
  };
  // writes into the caller's buffer that must land after the copy thread's (serial runs,
  // accepted speculative decodes): applied once it has joined
  std::vector<std::pair<int64_t, std::vector<int32_t>>> deferred;
  // the fold of a certified path: M + q 2^(e-52) when M and the sequence's values share the
  // predicted binade 2^e (cp_quant_f64), else element by element
  // the binade of a normal nonzero double from its exponent bits (std::ilogb otherwise)
  auto ilogb_fast = [](double x) {
    const uint64_t b = dbits(x);
    const int be = (int)((b >> 52) & 0x7FF);
    return (be != 0 && be != 0x7FF) ? be - 1023 : std::ilogb(x);
  };
  auto fold = [&](int64_t k, double M, bool* quant) {
    *quant = false;
    const int e = ebin[(size_t)k];
    if (e != cvk::CVK_NO_BINADE && !tie[(size_t)k] && M != 0.0 && ilogb_fast(M) == e &&
        std::fabs((double)qv[(size_t)k]) < 0x1p53 && e - 52 > -1022 && e - 52 < 1023) {
      // q 2^(e-52): |q| < 2^53 and a normal power of two, so the product is exact (= ldexp)
      const double g2 = from_dbits((uint64_t)(e - 52 + 1023) << 52);
      const double Mn = M + (double)qv[(size_t)k] * g2;
      if (ilogb_fast(Mn) == e) {
        *quant = true;
        return Mn;
      }
    }
    return fold_elems(k, M);
  };
  auto score_of = [&](size_t x) { return x < ks.size() ? std::fabs(score[(size_t)ks[x]]) : 0.0; };

  // The state of the chain before the sequence at hand: NONE (first sequence), CERT (a certified
  // sequence ended in prev_end with maximum M, a clean boundary), ROW (the exact last row is
  // known: row_host, W wide, -inf padded; on the device at row_dev when non-null).
  enum Kind { NONE, CERT, ROW };
  Kind prev = NONE;
  int32_t prev_end = 0, row_arg = 0;
  double M = 0.0;
  std::vector<double> row_host((size_t)W, -INFINITY), syn((size_t)W);
  const double* row_dev = nullptr;
  // the last row is clean for a start whose values reach magnitude `mag`: no earlier state's
  // value can round onto its maximum when pi[j] is added (utils.rs:32-35)
  auto row_clean = [&](const double* row, int32_t arg, double m1, double mag) {
    const double gap = 0x1p-51 * (std::fabs(m1) + mag);
    for (int32_t i = 0; i < arg; ++i)
      if (!(m1 - row[i] > gap)) return false;
    return true;
  };
  // sequence ks[x] certified at running maximum Mc after a predecessor of kind pk (the row test
  // against row_host when pk == ROW); *Mn = its fold.  ks[x + 1] must be known (the walk of a
  // part stops before its last sequence until the next part's scores are in).
  auto certify = [&](size_t x, double Mc, Kind pk, double* Mn, bool* quant) {
    const int64_t k = ks[x];
    const int64_t T = off[(size_t)k + 1] - off[(size_t)k];
    const double S = score_of(x), rho = cert[(size_t)k * 2], gF = cert[(size_t)k * 2 + 1];
    const double U = 0x1p-52 * (std::fabs(Mc) + S + 16.0);
    if (!(rho > U) || (force_m > 0 && (int64_t)(x % (size_t)force_m) == force_m - 1)) return false;
    if (pk == ROW && !row_clean(row_host.data(), row_arg, Mc, S + pimax + 16.0)) return false;
    *Mn = fold(k, Mc, quant);
    // the boundary into the next sequence: its start values must not merge with this
    // sequence's maximum (the exact final gap, less the chain's drift, beats 2 ulps there)
    const double U1 = 0x1p-52 * (std::fabs(*Mn) + score_of(x + 1) + pimax + 16.0);
    return x + 1 >= ks.size() || gF - 3.0 * (double)T * U > 2.0 * U1;
  };

  // ---- runs: the serial chain kernel over consecutive uncertified sequences ----
  if ((st = d_first.ensure((size_t)std::max<int64_t>(maxT, 1))) != CV_OK) return st;
  HIP_TRY(hipMemsetAsync(d_first.p, 0, (size_t)std::max<int64_t>(maxT, 1), cs));
  HIP_TRY(hipMemsetAsync(d_first.p, 1, 1, cs));  // one sequence per launch: its element 0 starts it
  if ((st = d_rows.ensure((size_t)W * 8 * 3)) != CV_OK) return st;
  // objective, final state (+ the wide chain's two rows, CV_CHAIN_WIDE_MIN)
  if ((st = d_small.ensure(16 + (!small && cvk::cp_chain_wide(N) ? (size_t)N * 16 : 0))) != CV_OK) return st;
  double* row_in = d_rows.as<double>();  // start row uploaded from the host
  double* row_a = row_in + W;            // the run's last rows (ping-pong)
  double* row_b = row_a + W;
  bool in_run = false;
  int64_t run_e0 = 0, run_len = 0, runs = 0, run_seqs = 0, ncert = 0, nquant = 0, spec_acc = 0, spec_batches = 0;
  int64_t psi_cap = (int64_t)(d_rpsi.bytes / ((size_t)W * 2));
  auto end_run = [&](int32_t end_state) -> cv_status {
    if ((st = d_rpath.ensure((size_t)run_len * 4)) != CV_OK) return st;
    if ((st = chain_backtrack(W, d_rpsi.as<uint16_t>(), run_len, end_state, d_rpath.as<int32_t>(), cs)) != CV_OK)
      return st;
    std::vector<int32_t> rp((size_t)run_len);
    HIP_TRY(hipMemcpyAsync(rp.data(), d_rpath.p, (size_t)run_len * 4, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    deferred.emplace_back(run_e0, std::move(rp));
    in_run = false;
    return CV_OK;
  };
  auto run_step = [&](int64_t k) -> cv_status {  // sequence k through the serial chain kernel
    const int64_t e0 = off[(size_t)k], T = off[(size_t)k + 1] - e0;
    const double* init = nullptr;
    if (prev == CERT) {  // what a clean boundary after a certified sequence sees
      std::fill(syn.begin(), syn.end(), -INFINITY);
      syn[(size_t)prev_end] = M;
      HIP_TRY(hipMemcpyAsync(row_in, syn.data(), (size_t)W * 8, hipMemcpyHostToDevice, cs));
      init = row_in;
    } else if (prev == ROW) {
      if (!row_dev) {  // a speculative decode's last row: the exact row, uploaded
        HIP_TRY(hipMemcpyAsync(row_in, row_host.data(), (size_t)W * 8, hipMemcpyHostToDevice, cs));
        row_dev = row_in;
      }
      init = row_dev;
    }
    if (!in_run) {
      in_run = true;
      run_e0 = e0;
      run_len = 0;
      ++runs;
    }
    if (run_len + T > psi_cap) {  // grow the run's psi rows (rare: long runs)
      const int64_t cap = std::max<int64_t>(2 * psi_cap, std::max<int64_t>(run_len + T, 4 * maxT));
      DevBuf nb;
      if ((st = nb.ensure((size_t)cap * W * 2)) != CV_OK) return st;
      if (run_len > 0)
        HIP_TRY(hipMemcpyAsync(nb.p, d_rpsi.p, (size_t)run_len * W * 2, hipMemcpyDeviceToDevice, cs));
      HIP_TRY(hipStreamSynchronize(cs));
      std::swap(nb.p, d_rpsi.p);
      std::swap(nb.bytes, d_rpsi.bytes);
      psi_cap = cap;
    }
    if (!init) HIP_TRY(hipMemsetAsync(d_rpsi.as<uint16_t>() + run_len * W, 0, (size_t)W * 2, cs));
    double* out_row = init == row_a ? row_b : row_a;
    hipError_t err;
    if (small) {
      cvk::CpChainWgArgs g{};
      g.pi = h->q_pi.as<double>();
      g.a = h->q_a.as<double>();
      g.et = h->q_et.as<double>();
      g.obs = d_obs.as<int32_t>() + e0;
      g.first = d_first.as<uint8_t>();
      g.len = T;
      g.nstates = N;
      g.psi = d_rpsi.as<uint16_t>() + run_len * W;
      g.objective = d_small.as<double>();
      g.final_state = reinterpret_cast<int32_t*>(d_small.as<double>() + 1);
      g.init_row = init;
      g.final_row = out_row;
      err = cvk::launch_cp_chain_wg(W, g, cs);
    } else {  // N > 256: one thread per state (cp_superseq_chain), the unpadded f64 tables
      cvk::CpChainArgs g{};
      g.pi = h->d_pi64.as<double>();
      g.a = h->d_a64.as<double>();
      g.et = h->d_et64.as<double>();
      g.obs = d_obs.as<int32_t>() + e0;
      g.first = d_first.as<uint8_t>();
      g.len = T;
      g.nstates = N;
      g.nobs = (int)V;
      g.psi = d_rpsi.as<uint16_t>() + run_len * W;
      g.path = nullptr;
      g.objective = d_small.as<double>();
      g.final_state = reinterpret_cast<int32_t*>(d_small.as<double>() + 1);
      g.init_row = init;
      g.final_row = out_row;
      if (cvk::cp_chain_wide(N)) g.grows = d_small.as<double>() + 2;
      err = cvk::launch_cp_superseq_chain(g, cs);
    }
    if (err != hipSuccess) return set_err(CV_EDEVICE, "chain run launch failed: %s", hipGetErrorString(err));
    double out[2];
    HIP_TRY(hipMemcpyAsync(out, d_small.p, 16, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipMemcpyAsync(row_host.data(), out_row, (size_t)W * 8, hipMemcpyDeviceToHost, cs));
    HIP_TRY(hipStreamSynchronize(cs));
    row_dev = out_row;
    M = out[0];
    std::memcpy(&row_arg, &out[1], 4);
    run_len += T;
    ++run_seqs;
    prev = ROW;
    return CV_OK;
  };

  // ---- speculation: the uncertified sequences re-decoded IN PARALLEL by the per-sequence CP
  // kernel (trellis_cp_f64) from the offsets a fold along the row-A0 paths predicts.  A
  // sequence's result is the chain's own exactly when its offset was the chain's exact running
  // maximum and its start clean; a prediction goes wrong only after an earlier uncertified
  // sequence's path changed, so one batch resolves the fallbacks up to there, and the next
  // batch (from the exact maximum) the ones after.  Batches that resolve little (tie-heavy
  // models) switch speculation off: the serial runs take over.  A batch covers positions
  // below x_lim (the walk's limit: the sequences whose successors' scores are in).
  std::vector<int64_t> spec_idx((size_t)nseq, -1);
  bool beside_fwd = false;  // the walk runs beside the last part's forward pass
  std::vector<double> spec_guess, spec_last;
  std::vector<int64_t> spec_off;
  std::vector<int32_t> spec_path;
  bool spec_on = spec_env;
  int64_t batch_acc = 0, batch_size = 0;
  size_t spec_from = SIZE_MAX;  // position a batch was last launched from
  auto speculate = [&](size_t x0, size_t x_lim) -> cv_status {
    std::vector<int64_t> F;
    std::vector<double> G;
    double Ms = M;
    Kind pk = prev;
    // beside a forward, on cp_spec_psi: as many sequences as its psi rows hold
    const bool spec_psi = small && beside_fwd && h->tuning.chain_spec_kernel == 0;
    const int64_t psi_rows = spec_psi ? (int64_t)(h->chainb.spsi.bytes / ((size_t)W * 2)) : INT64_MAX;
    int64_t rows_used = 0;
    for (size_t y = x0; y < x_lim && (int64_t)F.size() < kSpecMax; ++y) {
      double Mn;
      bool qd;
      const Kind ky = y == x0 ? pk : CERT;
      const bool ok = certify(y, Ms, ky, &Mn, &qd);
      if (ky == CERT) {
        memo_in[y] = Ms;
        memo_out[y] = ok ? Mn : std::numeric_limits<double>::quiet_NaN();
        memo_q[y] = qd ? 1 : 0;
      }
      if (ok) {
        Ms = Mn;
        continue;
      }
      if (y == x0 && pk == ROW && !row_clean(row_host.data(), row_arg, Ms, score_of(y) + pimax + 16.0)) break;
      const int64_t Ty = off[(size_t)ks[y] + 1] - off[(size_t)ks[y]];
      if (rows_used + Ty > psi_rows) break;
      rows_used += Ty;
      F.push_back(ks[y]);
      G.push_back(Ms);
      Ms = fold_elems(ks[y], Ms);  // predicted: the chain keeps the row-A0 path
    }
    trace_mark("chain: speculation predicted");
    std::fill(spec_idx.begin(), spec_idx.end(), -1);
    spec_guess.clear();
    if (F.empty()) return CV_OK;
    const int64_t nf = (int64_t)F.size();
    std::vector<int64_t> so((size_t)nf + 1, 0);
    for (int64_t i = 0; i < nf; ++i) so[(size_t)i + 1] = so[(size_t)i] + (off[(size_t)F[i] + 1] - off[(size_t)F[i]]);
    const int64_t Ls = so[(size_t)nf];
    std::vector<int32_t> sob((size_t)Ls);
    for (int64_t i = 0; i < nf; ++i)
      std::memcpy(sob.data() + so[(size_t)i], ob + off[(size_t)F[i]], (size_t)(so[(size_t)i + 1] - so[(size_t)i]) * 4);
    if ((st = d_soff.ensure((size_t)(nf + 1) * 8)) != CV_OK) return st;
    if ((st = d_sobs.ensure((size_t)Ls * 4)) != CV_OK) return st;
    if ((st = d_spath.ensure((size_t)Ls * 4)) != CV_OK) return st;
    if ((st = d_sres.ensure((size_t)nf * 9)) != CV_OK) return st;
    if ((st = d_sinit.ensure((size_t)nf * 8)) != CV_OK) return st;
    if ((st = d_slast.ensure((size_t)nf * N * 8)) != CV_OK) return st;
    HIP_TRY(hipMemcpyAsync(d_soff.p, so.data(), so.size() * 8, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipMemcpyAsync(d_sobs.p, sob.data(), sob.size() * 4, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipMemcpyAsync(d_sinit.p, G.data(), (size_t)nf * 8, hipMemcpyHostToDevice, cs));
    trace_mark("chain: speculative batch packed");
    if (spec_psi) {
      // beside a forward pass: cp_spec_psi (4 VALU per candidate, A by buffer loads, ~20 KiB of
      // LDS), its psi rows sized up front (no reallocation -- a device-wide synchronisation --
      // while the forward runs)
      cvk::CpSpecArgs g{};
      g.pi = h->q_pi.as<double>();
      g.a = h->q_a.as<double>();
      g.et = h->q_et.as<double>();
      g.obs = d_sobs.as<int32_t>();
      g.soff = d_soff.as<int64_t>();
      g.sinit = d_sinit.as<double>();
      g.nstates = N;
      g.prio = std::min(std::max(h->tuning.chain_spec_prio, 0), 3);
      g.psi = h->chainb.spsi.as<uint16_t>();
      g.last = d_slast.as<double>();
      g.path = d_spath.as<int32_t>();
      const hipError_t e = cvk::launch_cp_spec_psi(W, g, nf, cs);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "chain speculative batch failed: %s", hipGetErrorString(e));
    } else if (small && !beside_fwd && h->tuning.chain_spec_kernel == 0) {
      // N <= 256 after the last forward pass (the chip is free): the serial chain kernel's
      // layout, one sequence per workgroup and CU (A on chip, ~3.5 us per element), its path
      // backtracked in the same workgroup
      DevBuf& d_spsi = h->chainb.spsi;
      if ((st = d_spsi.ensure((size_t)Ls * W * 2)) != CV_OK) return st;
      cvk::CpChainWgArgs g{};
      g.pi = h->q_pi.as<double>();
      g.a = h->q_a.as<double>();
      g.et = h->q_et.as<double>();
      g.obs = d_sobs.as<int32_t>();
      g.nstates = N;
      g.psi = d_spsi.as<uint16_t>();
      g.final_row = d_slast.as<double>();
      g.soff = d_soff.as<int64_t>();
      g.sinit = d_sinit.as<double>();
      g.path = d_spath.as<int32_t>();
      const hipError_t e = cvk::launch_cp_chain_wg_batch(W, g, nf, cs);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "chain speculative batch failed: %s", hipGetErrorString(e));
    } else {
    cv_opts oc = default_opts();
    oc.dtype = CV_DTYPE_F64;
    oc.assoc = CV_ASSOC_CP;
    // generic_fwd_ms (psi, one state per thread, one sequence per workgroup) or, N <= 256,
    // trellis_cp_f64 by tuning key chain_spec_kernel = 1 (bit-identical): config-4 size, 620
    // sequences, the batch 15-17 vs 17-17.7 ms (profiles/r05_spec_ab.txt)
    const bool spec_generic = !small || h->tuning.chain_spec_kernel != 1;
    oc.kernel = spec_generic ? CV_KERNEL_GENERIC : CV_KERNEL_TRELLIS_F64;
    oc.rescore_f64 = 0;
    oc.stream = cs;
    double* sc = d_sres.as<double>();
    // beside the last part's forward pass (two waves of 224 VGPRs per SIMD, 31.5 KiB of LDS per
    // CU left): one sequence per workgroup, whose 58-VGPR waves fit the 64 VGPRs left, instead
    // of the two-sequence kernel's 78, which waited for the forward pass to drain
    cvk::TuningOverride one_seq(&cvk::Tuning::generic_s, beside_fwd && h->tuning.generic_s == 0 ? 1 : h->tuning.generic_s);
    // ... and at issue priority 3: a latency-bound walk that takes few issue slots, which the
    // forward's waves (priority 2-3) would otherwise leave it only when they stall
    cvk::TuningOverride prio(&cvk::Tuning::generic_prio,
                             beside_fwd && h->tuning.chain_spec_prio ? 1 : h->tuning.generic_prio);
    // the side workspace: the main one may still hold the last part's forward pass
    if ((st = decode_device(h, nf, so.data(), d_soff.as<int64_t>(), d_sobs.as<int32_t>(), oc, d_spath.as<int32_t>(), sc,
                            reinterpret_cast<uint8_t*>(sc + nf), cs, nullptr, true, nullptr, d_sinit.as<double>(),
                            d_slast.as<double>())) != CV_OK)
      return st;
    }
    spec_path.resize((size_t)Ls);
    spec_last.resize((size_t)nf * N);
    HIP_TRY(d2h_small(spec_last.data(), d_slast.p, (size_t)nf * N * 8, 0));
    HIP_TRY(d2h_small(spec_path.data(), d_spath.p, (size_t)Ls * 4, (size_t)nf * N * 8));
    trace_mark("chain: speculative batch (pack, decode, D2H)");
    spec_off = std::move(so);
    spec_guess = std::move(G);
    for (int64_t i = 0; i < nf; ++i) spec_idx[(size_t)F[i]] = i;
    ++spec_batches;
    batch_acc = 0;
    batch_size = nf;
    return CV_OK;
  };

  // 3. the walk over positions [x, x_lim)
  size_t x = 0;
  auto walk = [&](size_t x_lim) -> cv_status {
    while (x < x_lim) {
      const int64_t k = ks[x];
      const int64_t e0 = off[(size_t)k], T = off[(size_t)k + 1] - e0;
      double Mn;
      bool qd;
      bool ok;
      if (prev == CERT && memo_q[x] != 2 && dbits(memo_in[x]) == dbits(M)) {
        ok = !std::isnan(memo_out[x]);  // the prediction walk's decision at this very maximum
        Mn = memo_out[x];
        qd = memo_q[x] == 1;
        ++memo_hits;
      } else {
        ok = certify(x, M, prev, &Mn, &qd);
      }
      if (ok) {
        if (in_run && (st = end_run(row_arg)) != CV_OK) return st;  // clean: the run ends in its argmax
        M = Mn;
        prev = CERT;
        prev_end = ends[(size_t)k];
        ++ncert;
        nquant += qd ? 1 : 0;
        ++x;
        continue;
      }
      const double S = score_of(x);
      const bool start_clean = prev != ROW || row_clean(row_host.data(), row_arg, M, S + pimax + 16.0);
      const int64_t si = spec_idx[(size_t)k];
      if (si >= 0 && start_clean && spec_guess[(size_t)si] == M &&
          std::signbit(spec_guess[(size_t)si]) == std::signbit(M)) {
        // the speculative decode started from the chain's exact state: it IS the chain there
        const double* lr = spec_last.data() + (size_t)si * N;
        int32_t arg = 0;
        for (int32_t i = 1; i < N; ++i)
          if (lr[i] > lr[arg]) arg = i;
        const double m1 = lr[arg];
        if (m1 > -INFINITY && (x + 1 >= ks.size() || row_clean(lr, arg, m1, score_of(x + 1) + pimax + 16.0))) {
          if (in_run && (st = end_run(row_arg)) != CV_OK) return st;
          const int32_t* sp = spec_path.data() + spec_off[(size_t)si];
          deferred.emplace_back(e0, std::vector<int32_t>(sp, sp + T));
          std::copy(lr, lr + N, row_host.begin());
          std::fill(row_host.begin() + N, row_host.end(), -INFINITY);
          row_dev = nullptr;
          row_arg = arg;
          M = m1;
          prev = ROW;
          ++spec_acc;
          ++batch_acc;
          ++x;
          continue;
        }
        // its end state could differ from its argmax (an unclean boundary): the serial chain
      } else if (spec_on && start_clean && spec_from != x) {
        // no valid speculation for this sequence (none yet, or an earlier path changed): a new
        // batch from the exact state here, unless the last one resolved too little
        if (spec_batches > 0 && batch_acc < 4 && batch_acc * 4 < batch_size) spec_on = false;
        if (spec_on) {
          spec_from = x;
          if ((st = speculate(x, x_lim)) != CV_OK) return st;
          continue;  // retry x with the new batch
        }
      }
      if ((st = run_step(k)) != CV_OK) return st;
      ++x;
    }
    return CV_OK;
  };
  for (int p = 0; p < nparts; ++p) {
    if ((st = prep(p)) != CV_OK) return st;
    if (fallback) return CV_OK;
    // all but the part's last sequence (its boundary test needs the next part's first score)
    const size_t x_lim = p + 1 < nparts ? (ks.empty() ? 0 : ks.size() - 1) : ks.size();
    beside_fwd = p + 1 < nparts;
    if ((st = walk(x_lim)) != CV_OK) return st;
    if (p + 1 < nparts) trace_mark("chain: part walked");
  }
  if (in_run && (st = end_run(row_arg)) != CV_OK) return st;  // cp.rs:86: first argmax of the last row
  if (path_st != CV_OK) return path_st;
  if (trace_on()) {
    char msg[96];
    snprintf(msg, sizeof msg, "chain: walk + runs (%lld memo hits)", (long long)memo_hits);
    trace_mark(msg);
  }
  if ((st = join_copy()) != CV_OK) return st;
  for (const auto& d : deferred) std::memcpy(path_out + d.first, d.second.data(), d.second.size() * 4);
  trace_mark("chain: path copy joined");
  h->last_chain[7] = gathered;
  h->last_chain[8] = path_waits;
  h->last_chain[0] = 1;
  h->last_chain[1] = ncert;
  h->last_chain[2] = run_seqs;
  h->last_chain[3] = runs;
  h->last_chain[4] = nquant;
  h->last_chain[5] = spec_acc;
  h->last_chain[6] = spec_batches;
  *objective_out = M;
  *applied = true;
  if (!(M > -INFINITY))
    return set_err(CV_EINFEASIBLE, "no finite-probability path through the super-sequence (cp.rs:87 asserts)");
  return CV_OK;
}
}  // namespace

extern "C" {

CV_API cv_status cv_decode_superseq_cp(cv_hmm* h, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                                       int32_t* path_out, double* objective_out) {
  if (!h || nseq < 0 || (nseq > 0 && (!offsets || !obs || !path_out)) || !objective_out)
    return set_err(CV_EINVAL, "bad argument");
  *objective_out = 0.0;
  if (nseq == 0) return CV_OK;
  if (h->N > cvk::kChainMaxStates)
    return set_err(CV_EUNSUPPORTED, "super-sequence chain covers N <= %d (N=%d)", cvk::kChainMaxStates, h->N);
  CV_LOCK(h);
  cv_status st = set_device(h);
  if (st != CV_OK) return st;
  if ((st = check_batch(h, nseq, offsets)) != CV_OK) return st;
  const int64_t base = offsets[0], L = offsets[nseq] - base;
  if (L <= 0) return CV_OK;
  auto check_obs = [&]() -> cv_status {
    const int64_t V = h->V;
    const int64_t k = first_bad(base, offsets[nseq], [&](int64_t i) { return obs[i] < 0 || obs[i] >= V; });
    if (k >= 0) return set_err(CV_EINVAL, "obs[%lld] = %d out of range [0,%lld)", (long long)k, obs[k], (long long)V);
    return CV_OK;
  };
  // The parallel chain (any N, log-probability models); else serially: N <= 256 the
  // one-workgroup chain with the candidates split over its waves and A on chip
  // (kernels/chain.hip), N > 256 (or CV_CHAIN_OLD=1, an A/B knob, bit-identical) one thread per
  // state (cp_superseq_chain); both then the parallel segmented backtrack
  const bool chain_old = h->tuning.chain_old == 1;
  for (int q = 0; q < 9; ++q) h->last_chain[q] = 0;
  if (!chain_old && h->tuning.chain_par != 0) {
    // the parallel chain range-checks the observations on the device (its trellis statuses,
    // CV_SEQ_BADOBS -> CV_EINVAL with the host scan's message), not by a host scan first
    bool applied = false;
    st = superseq_cp_par(h, nseq, offsets, obs, path_out, objective_out, &applied);
    if (st != CV_OK || applied) return st;
  }
  if ((st = check_obs()) != CV_OK) return st;
  // the serial chain's sequence-start flags (MetaElements t == 0), built only when it runs (the
  // parallel chain never reads them: 33.5 MB zeroed and walked at config-4 size)
  std::vector<uint8_t> first((size_t)L, 0);
  for (int64_t q = 0; q < nseq; ++q)
    if (offsets[q + 1] > offsets[q]) first[(size_t)(offsets[q] - base)] = 1;
  if (cvk::t64_padded_states(h->N) && !chain_old)
    return superseq_cp_wg(h, L, obs + base, first, path_out, objective_out);
  if ((st = ensure_f64_tables(h)) != CV_OK) return st;
  hipStream_t stream = h->stream;
  DevBuf d_obs, d_first, d_psi, d_path, d_obj;
  if ((st = d_obs.ensure((size_t)L * 4)) != CV_OK) return st;
  if ((st = d_first.ensure((size_t)L)) != CV_OK) return st;
  if ((st = d_psi.ensure((size_t)L * h->N * 2)) != CV_OK) return st;
  if ((st = d_path.ensure((size_t)L * 4)) != CV_OK) return st;
  // the wide chain (N > 10,240): its two rows in global memory after the objective / final state
  const bool grows = cvk::cp_chain_wide(h->N);
  if ((st = d_obj.ensure(16 + (grows ? (size_t)h->N * 16 : 0))) != CV_OK) return st;
  HIP_TRY(hipMemcpyAsync(d_obs.p, obs + base, (size_t)L * 4, hipMemcpyHostToDevice, stream));
  HIP_TRY(hipMemcpyAsync(d_first.p, first.data(), (size_t)L, hipMemcpyHostToDevice, stream));
  cvk::CpChainArgs g{};
  g.pi = h->d_pi64.as<double>();
  g.a = h->d_a64.as<double>();
  g.et = h->d_et64.as<double>();
  g.obs = d_obs.as<int32_t>();
  g.first = d_first.as<uint8_t>();
  g.len = L;
  g.nstates = h->N;
  g.nobs = (int)h->V;
  g.psi = d_psi.as<uint16_t>();
  g.path = nullptr;  // the segmented backtrack below (a single-thread walk was one dependent load per element)
  g.objective = d_obj.as<double>();
  g.final_state = reinterpret_cast<int32_t*>(d_obj.as<double>() + 1);
  if (grows) g.grows = d_obj.as<double>() + 2;
  const hipError_t err = cvk::launch_cp_superseq_chain(g, stream);
  if (err != hipSuccess) return set_err(CV_EDEVICE, "super-sequence chain launch failed: %s", hipGetErrorString(err));
  double out[2];
  HIP_TRY(hipMemcpyAsync(out, d_obj.p, 16, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  *objective_out = out[0];
  int32_t fs;
  std::memcpy(&fs, &out[1], 4);
  if ((st = chain_backtrack(h->N, d_psi.as<uint16_t>(), L, fs, d_path.as<int32_t>(), stream)) != CV_OK) return st;
  HIP_TRY(hipMemcpyAsync(path_out, d_path.p, (size_t)L * 4, hipMemcpyDeviceToHost, stream));
  HIP_TRY(hipStreamSynchronize(stream));
  if (!(*objective_out > -INFINITY))
    return set_err(CV_EINFEASIBLE, "no finite-probability path through the super-sequence (cp.rs:87 asserts)");
  return CV_OK;
}

// ---- trait Solver ------------------------------------------------------------------
struct cv_solver {
  std::string kind;
  cv_hmm* hmm = nullptr;
  cv_opts opts{};
  int64_t nseq = 0;
  std::vector<int64_t> offsets;
  std::vector<int32_t> obs;
  bool constrained = false;
  std::vector<int32_t> comp;  // active constraint component per element, -1 = none
  int32_t ncomp = 0;
  std::vector<int32_t> solution;
  std::vector<double> scores;
  std::vector<uint8_t> status;
  double objective = -INFINITY;
  uint64_t explored = 0;
};

CV_API cv_status cv_solver_create(const char* kind, cv_hmm* h, const cv_superseq_desc* d, cv_solver** out) {
  if (!kind || !h || !d || !out) return set_err(CV_EINVAL, "null argument");
  if (d->nseq < 0 || (d->nseq > 0 && (!d->offsets || !d->obs))) return set_err(CV_EINVAL, "bad super-sequence");
  auto s = std::make_unique<cv_solver>();
  s->kind = kind;
  s->hmm = h;
  cv_opts_init(&s->opts);
  if (s->kind == "gpu") {  // the opt-in f32 trellis + f64 re-score (cviterbi.h)
    s->opts.dtype = CV_DTYPE_F32;
  } else if (s->kind == "gpu-f64") {
    s->opts.dtype = CV_DTYPE_F64;
  } else if (s->kind == "gpu-cp" || s->kind == "gpu-cp-seq") {
    s->opts.dtype = CV_DTYPE_F64;
    s->opts.assoc = CV_ASSOC_CP;
    s->opts.rescore_f64 = 0;
  } else if (s->kind == "gpu-dp") {
    s->opts.dtype = CV_DTYPE_F64;
    s->opts.assoc = CV_ASSOC_DP;
    s->opts.rescore_f64 = 0;
  } else {
    return set_err(CV_EINVAL, "unknown solver kind '%s' (gpu, gpu-f64, gpu-cp, gpu-cp-seq, gpu-dp)", kind);
  }
  s->nseq = d->nseq;
  s->offsets.assign(d->offsets, d->offsets + d->nseq + 1);
  if (s->offsets.empty()) s->offsets.push_back(0);
  cv_status st = check_batch(h, s->nseq, s->offsets.data());
  if (st != CV_OK) return st;
  if (s->offsets[0] != 0) return set_err(CV_EINVAL, "super-sequence offsets must start at 0");
  const int64_t total = s->offsets.back();
  s->obs.assign(d->obs, d->obs + total);
  s->comp.assign((size_t)total, -1);
  if (d->active && d->component)
    for (int64_t k = 0; k < total; ++k)
      if (d->active[k] && d->component[k] >= 0) {
        s->constrained = true;
        s->comp[k] = d->component[k];
        s->ncomp = std::max(s->ncomp, d->component[k] + 1);
      }
  *out = s.release();
  return CV_OK;
}

CV_API cv_status cv_solver_solve(cv_solver* s) {
  if (!s) return set_err(CV_EINVAL, "null solver");
  if (s->constrained) {
    // every kind: the consistency-constrained decode on the row-A0 association (the terms of
    // csp.hpp are defined on it) at the kind's precision -- f64 for gpu-f64 / gpu-cp / gpu-dp
    // (the reference's arithmetic, cp.rs:95-126 / dp.rs:147-166 in f64), f32 for "gpu"
    cv_opts co = s->opts;
    co.assoc = CV_ASSOC_VITERBI;
    co.rescore_f64 = co.dtype == CV_DTYPE_F32 ? 1 : 0;
    const int64_t total = s->offsets.back();
    s->solution.assign((size_t)total, 0);
    s->scores.assign((size_t)s->nseq, 0.0);
    s->status.assign((size_t)s->nseq, 0);
    std::vector<int32_t> states((size_t)s->ncomp, -1);
    double obj = 0;
    cv_status st = cv_decode_constrained(s->hmm, s->nseq, s->offsets.data(), s->obs.data(), s->comp.data(), s->ncomp,
                                         &co, s->solution.data(), s->scores.data(), s->status.data(),
                                         states.data(), &obj);
    if (st != CV_OK) return st;
    s->objective = obj;
    s->explored = s->hmm->last_explored;
    if (!(obj > -INFINITY)) return set_err(CV_EINFEASIBLE, "no assignment satisfies the constraints");
    return CV_OK;
  }
  const int64_t total = s->offsets.back();
  s->solution.assign((size_t)total, 0);
  s->scores.assign((size_t)s->nseq, 0.0);
  s->status.assign((size_t)s->nseq, 0);
  if (s->kind == "gpu-cp") {  // CPSolver::solve exactly: the chained super-sequence decode
    double obj = -INFINITY;
    cv_status st = cv_decode_superseq_cp(s->hmm, s->nseq, s->offsets.data(), s->obs.data(), s->solution.data(), &obj);
    s->objective = st == CV_OK ? obj : -INFINITY;
    s->explored = 0;  // no B&B node without constraints (cp.rs:137-142)
    return st;
  }
  cv_status st = cv_decode_batch(s->hmm, s->nseq, s->offsets.data(), s->obs.data(), &s->opts, s->solution.data(),
                                 s->scores.data(), s->status.data());
  if (st != CV_OK) return st;
  // objective of an unconstrained super-sequence = sum of per-sequence optima (row A6)
  double obj = 0.0;
  for (int64_t k = 0; k < s->nseq; ++k) {
    if (s->status[k] == CV_SEQ_INFEASIBLE) {
      s->objective = -INFINITY;
      return set_err(CV_EINFEASIBLE, "sequence %lld has no finite-probability path", (long long)k);
    }
    obj += s->scores[k];
  }
  s->objective = obj;
  s->explored = 0;  // CPSolver explores no B&B node without constraints (cp.rs:137-142)
  return CV_OK;
}

CV_API cv_status cv_solver_get_solution(const cv_solver* s, const int32_t** sol, int64_t* len) {
  if (!s || !sol || !len) return set_err(CV_EINVAL, "null argument");
  *sol = s->solution.data();
  *len = (int64_t)s->solution.size();
  return CV_OK;
}
CV_API cv_status cv_solver_get_objective(const cv_solver* s, double* obj) {
  if (!s || !obj) return set_err(CV_EINVAL, "null argument");
  *obj = s->objective;
  return CV_OK;
}
CV_API const char* cv_solver_get_name(const cv_solver* s) { return s ? s->kind.c_str() : ""; }
CV_API cv_status cv_solver_get_explored_nodes(const cv_solver* s, uint64_t* n) {
  if (!s || !n) return set_err(CV_EINVAL, "null argument");
  *n = s->explored;
  return CV_OK;
}
CV_API void cv_solver_destroy(cv_solver* s) { delete s; }

}  // extern "C"

namespace {

// Rust's Display for f64 (what cfn.rs writes with format!("{}")): the shortest decimal that
// reads back to the same double, in positional notation (never an exponent); inf / -inf / NaN.
void append_rust_f64(std::string& out, double x) {
  if (std::isnan(x)) {
    out += "NaN";
    return;
  }
  if (std::isinf(x)) {
    out += x < 0 ? "-inf" : "inf";
    return;
  }
  // shortest round-trip digits (scientific to_chars), then laid out positionally with zeros:
  // Rust prints 2^60 as 1152921504606847000, not the exact 1152921504606846976
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  const std::string sci(buf, r.ptr);
  const size_t epos = sci.find('e');
  std::string mant = sci.substr(0, epos);
  const int exp10 = std::atoi(sci.c_str() + epos + 1);
  const bool neg = mant[0] == '-';
  if (neg) mant.erase(0, 1);
  std::string digits;
  for (char c : mant)
    if (c != '.') digits += c;
  // value = 0.d1d2...dn x 10^(exp10 + 1)
  const int point = exp10 + 1;  // digits before the decimal point
  std::string s;
  if (point <= 0) {
    s = "0." + std::string((size_t)(-point), '0') + digits;
  } else if ((size_t)point >= digits.size()) {
    s = digits + std::string((size_t)point - digits.size(), '0');
  } else {
    s = digits.substr(0, (size_t)point) + "." + digits.substr((size_t)point);
  }
  if (s.find('.') != std::string::npos) {  // "1.0" style trailing zeros never come from to_chars, but be safe
    while (s.back() == '0') s.pop_back();
    if (s.back() == '.') s.pop_back();
  }
  if (neg) out += '-';
  out += s;
}

}  // namespace

extern "C" {

// write_cfn (viterbi_solver/cfn.rs:82-205) over the solver's super-sequence: constraint
// boundaries where the active component changes, an N x N table per ordered component pair
// of segment longest paths (accumulated over all boundaries between the two components, both
// orientations), start/end unary costs, the lower bound, and the text file toulbar2 reads.
// The segment rows run on the GPU (kernels/cfn.hip, bit-identical f64); the tables, bound and
// formatting are the reference's host loops.
CV_API cv_status cv_solver_write_cfn(cv_solver* s, const char* path, uint64_t* compile_ms) {
  if (!s || !path) return set_err(CV_EINVAL, "null argument");
  const auto t0 = std::chrono::steady_clock::now();
  cv_hmm* h = s->hmm;
  const int N = h->N;
  const int64_t len = s->offsets.back();
  if (len <= 0) return set_err(CV_EINVAL, "empty super-sequence");
  // constraint boundaries (cfn.rs:88-110)
  std::vector<std::pair<int64_t, int32_t>> bnd;
  int32_t last = -1;
  for (int64_t t = 0; t < len; ++t) {
    const int32_t c = s->comp[(size_t)t];
    if (c < 0) continue;
    if (last < 0 || c != last) bnd.emplace_back(t, c);
    last = c;
  }
  if (bnd.empty()) return set_err(CV_EINVAL, "no active constraint: cfn.rs:106 unwraps an empty boundary list");
  // k = number of components with an active element (SuperSequence::number_constraints,
  // utils.rs:200-202); the tables are indexed by component id (cfn.rs:115-118)
  std::vector<uint8_t> seen((size_t)s->ncomp, 0);
  int32_t k = 0;
  for (int64_t t = 0; t < len; ++t)
    if (s->comp[(size_t)t] >= 0 && !seen[(size_t)s->comp[(size_t)t]]) {
      seen[(size_t)s->comp[(size_t)t]] = 1;
      ++k;
    }
  if (s->ncomp > k)
    return set_err(CV_EUNSUPPORTED, "component %d >= %d active components: cfn.rs:118 indexes out of bounds",
                   s->ncomp - 1, k);
  // jobs: every boundary pair x start state, the end cost per state, the start cost
  std::vector<cvcfn::CfnJob> jobs;
  const int64_t nb = (int64_t)bnd.size();
  for (int64_t b = 0; b + 1 < nb; ++b)
    for (int n1 = 0; n1 < N; ++n1) jobs.push_back({bnd[(size_t)b].first, bnd[(size_t)b + 1].first, n1, cvcfn::kCfnSegment});
  const int64_t f_time = bnd.front().first, l_time = bnd.back().first;
  const int32_t f_cid = bnd.front().second, l_cid = bnd.back().second;
  const int64_t end_jobs = (int64_t)jobs.size();
  if (l_time != len - 1)
    for (int n = 0; n < N; ++n) jobs.push_back({l_time, len - 1, n, cvcfn::kCfnEnd});
  const int64_t start_job = (int64_t)jobs.size();
  jobs.push_back({0, f_time, 0, cvcfn::kCfnStart});
  std::vector<double> rows(jobs.size() * (size_t)N);
  {
    CV_LOCK(h);
    cv_status st = set_device(h);
    if (st != CV_OK) return st;
    if ((st = ensure_f64_tables(h)) != CV_OK) return st;
    std::vector<uint8_t> first((size_t)len, 0);
    for (int64_t q = 0; q < s->nseq; ++q)
      if (s->offsets[(size_t)q] < len) first[(size_t)s->offsets[(size_t)q]] = 1;
    DevBuf d_obs, d_comp, d_first, d_jobs, d_out;
    if ((st = upload(d_obs, s->obs.data(), (size_t)len * 4)) != CV_OK) return st;
    if ((st = upload(d_comp, s->comp.data(), (size_t)len * 4)) != CV_OK) return st;
    if ((st = upload(d_first, first.data(), (size_t)len)) != CV_OK) return st;
    // jobs in slices of <= 256 MiB of output rows
    const int64_t per = std::max<int64_t>(1, (256ll << 20) / (8ll * N));
    if ((st = d_out.ensure((size_t)std::min<int64_t>(per, (int64_t)jobs.size()) * N * 8)) != CV_OK) return st;
    for (int64_t j0 = 0; j0 < (int64_t)jobs.size(); j0 += per) {
      const int64_t nj = std::min<int64_t>(per, (int64_t)jobs.size() - j0);
      if ((st = upload(d_jobs, jobs.data() + j0, (size_t)nj * sizeof(cvcfn::CfnJob))) != CV_OK) return st;
      cvcfn::CfnArgs g{};
      g.jobs = d_jobs.as<cvcfn::CfnJob>();
      g.obs = d_obs.as<int32_t>();
      g.comp = d_comp.as<int32_t>();
      g.seq_start = d_first.as<uint8_t>();
      g.a = h->d_a64.as<double>();
      g.et = h->d_et64.as<double>();
      g.pi = h->d_pi64.as<double>();
      g.nstates = N;
      g.out = d_out.as<double>();
      const hipError_t e = cvcfn::launch_cfn_rows(g, nj, nullptr);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "cfn launch failed: %s", hipGetErrorString(e));
      HIP_TRY(hipMemcpy(rows.data() + (size_t)j0 * N, d_out.p, (size_t)nj * N * 8, hipMemcpyDeviceToHost));
    }
  }
  // cost tables (cfn.rs:117-140): [cid_from][cid_to][n1][n2], both orientations, -inf dropped
  const size_t NN = (size_t)N * N;
  std::vector<double> tab((size_t)k * k * NN, 0.0);
  auto acc = [](double& x, double c) {
    if (x == 0.0) x = c;
    else x += c;
  };
  for (int64_t b = 0; b + 1 < nb; ++b) {
    const int32_t cf = bnd[(size_t)b].second, ct = bnd[(size_t)b + 1].second;
    double* tf = tab.data() + ((size_t)cf * k + ct) * NN;
    double* tt = tab.data() + ((size_t)ct * k + cf) * NN;
    for (int n1 = 0; n1 < N; ++n1) {
      const double* row = rows.data() + ((size_t)b * N + n1) * N;
      for (int n2 = 0; n2 < N; ++n2) {
        // the row at t_to holds only n_to finite (the boundary element is constrained), so
        // longest_path's final max is row[n2]
        const double cost = row[n2];
        if (cost == -INFINITY) continue;
        acc(tf[(size_t)n1 * N + n2], cost);
        acc(tt[(size_t)n2 * N + n1], cost);
      }
    }
  }
  // unary costs (cfn.rs:142-147)
  std::vector<double> unary((size_t)k * N, 0.0);
  for (int n = 0; n < N; ++n) unary[(size_t)f_cid * N + n] += rows[(size_t)start_job * N + n];
  for (int n = 0; n < N; ++n) {
    double e = 0.0;
    if (l_time != len - 1) {
      const double* row = rows.data() + ((size_t)end_jobs + n) * N;
      e = -INFINITY;
      for (int j = 0; j < N; ++j) e = row[j] > e ? row[j] : e;
    }
    unary[(size_t)l_cid * N + n] += e;
  }
  const uint64_t ms = (uint64_t)std::chrono::duration_cast<std::chrono::milliseconds>(
                          std::chrono::steady_clock::now() - t0).count();
  // lower bound (cfn.rs:151-158) and -inf unary entries (cfn.rs:160-166)
  double lb = -1.0;
  for (int32_t k1 = 0; k1 < k; ++k1)
    for (int32_t k2 = k1 + 1; k2 < k; ++k2) {
      const double* t = tab.data() + ((size_t)k1 * k + k2) * NN;
      double m = t[0];
      for (size_t q = 1; q < NN; ++q) m = t[q] < m ? t[q] : m;
      lb += m;
    }
  for (auto& u : unary)
    if (u == -INFINITY) u = lb;
  // the file (cfn.rs:169-201)
  std::string out;
  out += "{\n\tproblem: { name: consistent_viterbi, mustbe: >";
  append_rust_f64(out, lb);
  out += "},\n\tvariables: {";
  std::string dom = "[";
  for (int i = 0; i < N; ++i) dom += "s" + std::to_string(i) + (i == N - 1 ? "]" : ",");
  for (int32_t i = 0; i < k; ++i) out += "n" + std::to_string(i) + ": " + dom + (i != k - 1 ? "," : "},\n");
  out += "\tfunctions: {\n";
  auto vec_text = [&](const double* v, size_t n) {
    out += "[";
    for (size_t q = 0; q < n; ++q) {
      append_rust_f64(out, v[q]);
      out += q == n - 1 ? "] " : ", ";
    }
  };
  for (int32_t i = 0; i < k; ++i) {
    out += "\t\tf" + std::to_string(i) + ": { scope: [n" + std::to_string(i) + "], costs: ";
    vec_text(unary.data() + (size_t)i * N, (size_t)N);
    out += "}, \n";
    for (int32_t j = i + 1; j < k; ++j) {
      const double* t = tab.data() + ((size_t)i * k + j) * NN;
      bool nonzero = false;
      for (size_t q = 0; q < NN && !nonzero; ++q) nonzero = t[q] != 0.0;  // tcost.sum() != 0.0 (costs <= 0)
      if (!nonzero) continue;
      out += "\t\tf" + std::to_string(i) + "_" + std::to_string(j) + ": { scope: [n" + std::to_string(i) + ", n" +
             std::to_string(j) + "], costs: ";
      vec_text(t, NN);
      out += "},\n";
    }
  }
  out += "\t}\n}";
  FILE* f = std::fopen(path, "wb");
  if (!f) return set_err(CV_EIO, "cannot open %s for writing", path);
  const size_t wr = std::fwrite(out.data(), 1, out.size(), f);
  const int cl = std::fclose(f);
  if (wr != out.size() || cl != 0) return set_err(CV_EIO, "short write to %s", path);
  if (compile_ms) *compile_ms = ms;
  return CV_OK;
}

}  // extern "C"

// ---- HMM fitting (hmm.rs:30-190) --------------------------------------
namespace {

// hmm.rs:192-205 `log()`: 0 -> -inf, else x.log(10.0), which Rust evaluates as ln(x) / ln(10)
double ref_log(double x) { return x == 0.0 ? -INFINITY : std::log(x) / std::log(10.0); }

cv_status fit_validate(int32_t N, int64_t V, int64_t nseq, const int64_t* offsets, const int32_t* obs,
                       const int32_t* tags, bool all_tagged, double* pi, double* a, double* b) {
  if (N <= 0 || V <= 0 || nseq <= 0) return set_err(CV_EINVAL, "nstates, nobs and nseq must be > 0");
  if (!offsets || !obs || !tags || !pi || !a || !b) return set_err(CV_EINVAL, "null argument");
  if (offsets[0] < 0) return set_err(CV_EINVAL, "offsets[0] < 0");
  for (int64_t s = 0; s < nseq; ++s)
    if (offsets[s + 1] <= offsets[s]) return set_err(CV_EINVAL, "sequence %lld is empty or offsets decrease", (long long)s);
  const int64_t lo = offsets[0], hi = offsets[nseq];
  int64_t k = first_bad(lo, hi, [&](int64_t i) { return obs[i] < 0 || obs[i] >= V; });
  if (k >= 0) return set_err(CV_EINVAL, "obs[%lld] = %d out of range [0,%lld)", (long long)k, obs[k], (long long)V);
  k = first_bad(lo, hi, [&](int64_t i) { return tags[i] < (all_tagged ? 0 : -1) || tags[i] >= N; });
  if (k >= 0) return set_err(CV_EINVAL, "tags[%lld] = %d out of range [%d,%d)", (long long)k, tags[k], all_tagged ? 0 : -1, N);
  return CV_OK;
}

struct FitDev {
  DevBuf off, obs, tags, pi, a, at, et, alpha, beta, rscale, acc, cnt, ord, dump, gscratch;
  DevBuf amin, a2, at2;  // tiny arcs: A's smallest positive entry, A 2^K and A^T 2^K
};

}  // namespace

extern "C" {

CV_API cv_status cv_hmm_fit_mle(int32_t nstates, int64_t nobs, int64_t nseq, const int64_t* offsets,
                                const int32_t* obs, const int32_t* tags, int32_t device, double* pi, double* a,
                                double* b) {
  const int32_t N = nstates;
  const int64_t V = nobs;
  cv_status st = fit_validate(N, V, nseq, offsets, obs, tags, true, pi, a, b);
  if (st != CV_OK) return st;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    (void)hipGetLastError();
    return set_err(CV_EDEVICE, "device %d not available", device);
  }
  HIP_TRY(hipSetDevice(device));
  const int64_t lo = offsets[0], total = offsets[nseq] - lo;
  FitDev d;
  std::vector<int64_t> off0((size_t)nseq + 1);
  for (int64_t s = 0; s <= nseq; ++s) off0[s] = offsets[s] - lo;
  const size_t ncnt = (size_t)N + (size_t)N * N + (size_t)N * V + 2 * (size_t)N;
  if ((st = upload(d.off, off0.data(), off0.size() * 8)) != CV_OK) return st;
  if ((st = upload(d.obs, obs + lo, (size_t)total * 4)) != CV_OK) return st;
  if ((st = upload(d.tags, tags + lo, (size_t)total * 4)) != CV_OK) return st;
  if ((st = d.cnt.ensure(ncnt * 8)) != CV_OK) return st;
  HIP_TRY(hipMemset(d.cnt.p, 0, ncnt * 8));
  cvf::MleArgs g{};
  g.offsets = d.off.as<int64_t>();
  g.obs = d.obs.as<int32_t>();
  g.tags = d.tags.as<int32_t>();
  g.nstates = N;
  g.nobs = V;
  uint64_t* c = d.cnt.as<uint64_t>();
  g.pi_cnt = c;
  g.a_cnt = c + N;
  g.b_cnt = c + N + (size_t)N * N;
  g.seen = g.b_cnt + (size_t)N * V;
  g.end = g.seen + N;
  hipError_t e = cvf::launch_mle_counts(g, nseq, nullptr);
  if (e != hipSuccess) return set_err(CV_EDEVICE, "mle launch failed: %s", hipGetErrorString(e));
  std::vector<uint64_t> cnt(ncnt);
  HIP_TRY(hipMemcpy(cnt.data(), d.cnt.p, ncnt * 8, hipMemcpyDeviceToHost));
  const uint64_t* pc = cnt.data();
  const uint64_t* ac = pc + N;
  const uint64_t* bc = ac + (size_t)N * N;
  const uint64_t* seen = bc + (size_t)N * V;
  const uint64_t* end = seen + N;
  // The reference adds 1.0 per occurrence to the current probability (hmm.rs:39-48); all
  // addends are 1.0, so the order is immaterial, but each add rounds: replay them.
  auto add_ones = [](double x, uint64_t k) {
    for (uint64_t i = 0; i < k; ++i) x += 1.0;
    return x;
  };
  parallel_ranges((int64_t)N, [&](int, int64_t s0, int64_t s1) {
    for (int64_t s = s0; s < s1; ++s) {
      const double sn = add_ones(0.0, seen[s]), en = add_ones(0.0, end[s]);
      for (int32_t j = 0; j < N; ++j) {
        double& x = a[(size_t)s * N + j];
        x = add_ones(x, ac[(size_t)s * N + j]);
        x = sn != en ? x / (sn - en) : 0.0;  // hmm.rs:52-57
      }
      pi[s] = add_ones(pi[s], pc[s]) / (double)nseq;
      for (int64_t o = 0; o < V; ++o) {
        double& x = b[(size_t)s * V + o];
        x = add_ones(x, bc[(size_t)s * V + o]) / sn;
      }
      pi[s] = ref_log(pi[s]);
      for (int32_t j = 0; j < N; ++j) a[(size_t)s * N + j] = ref_log(a[(size_t)s * N + j]);
      for (int64_t o = 0; o < V; ++o) b[(size_t)s * V + o] = ref_log(b[(size_t)s * V + o]);
    }
  }, 1);
  return CV_OK;
}

CV_API cv_status cv_hmm_fit_train(int32_t nstates, int64_t nobs, int64_t nseq, const int64_t* offsets,
                                  const int32_t* obs, const int32_t* tags, int32_t max_iter, double tol,
                                  int32_t device, double* pi, double* a, double* b, int32_t* iters_out) {
  const int32_t N = nstates;
  const int64_t V = nobs;
  cv_status st = fit_validate(N, V, nseq, offsets, obs, tags, false, pi, a, b);
  if (st != CV_OK) return st;
  if (N > cvf::kBwMaxStates) return set_err(CV_EUNSUPPORTED, "Baum-Welch covers N <= %d (N=%d)", cvf::kBwMaxStates, N);
  // no handle: the environment's tuning keys for this call (tuning.h)
  const cvk::Tuning tun = cvk::tuning_from_env();
  cvk::TuningScope tuning_scope(tun);
  // the strided kernels' vectors in global scratch: above kBwLdsMaxStates, or from N = 257
  // with tuning key bw_global = 1 (A/B and tests)
  const bool bw_global = N > cvf::kBwLdsMaxStates || (N > cvf::kBwMmStates && tun.bw_global == 1);
  if (max_iter < 0) return set_err(CV_EINVAL, "max_iter < 0");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    (void)hipGetLastError();
    return set_err(CV_EDEVICE, "device %d not available", device);
  }
  HIP_TRY(hipSetDevice(device));
  const int64_t lo = offsets[0], total = offsets[nseq] - lo;
  FitDev d;
  std::vector<int64_t> off0((size_t)nseq + 1);
  for (int64_t s = 0; s <= nseq; ++s) off0[s] = offsets[s] - lo;
  if ((st = upload(d.off, off0.data(), off0.size() * 8)) != CV_OK) return st;
  if ((st = upload(d.obs, obs + lo, (size_t)total * 4)) != CV_OK) return st;
  if ((st = upload(d.tags, tags + lo, (size_t)total * 4)) != CV_OK) return st;
  // alpha / beta rows for a chunk of sequences at a time: at least 2 GiB each, and up to half
  // of the free device memory for both (N > 64: a launch of 64-sequence workgroups fills the
  // chip only with >= 16,384 sequences; config 4's corpus is one 137 GB chunk)
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    free_b = 0;
  }
  const int64_t cap_elems = std::max<int64_t>(
      std::max<int64_t>((2ll << 30) / (8 * N), 1),
      N > cvf::kBwWaveStates ? (int64_t)(free_b / 2 / (16 * (size_t)N)) : 0);
  int64_t max_chunk = 0;
  std::vector<std::pair<int64_t, int64_t>> chunks;
  for (int64_t s0 = 0; s0 < nseq;) {
    int64_t s1 = s0 + 1;
    while (s1 < nseq && off0[s1 + 1] - off0[s0] <= cap_elems) ++s1;
    chunks.emplace_back(s0, s1);
    max_chunk = std::max(max_chunk, off0[s1] - off0[s0]);
    s0 = s1;
  }
  if ((st = d.alpha.ensure((size_t)max_chunk * N * 8)) != CV_OK) return st;
  // beta rows only for the workgroup kernels (N > 64, or CV_BW_GEMM_PATH=1); the one-wave
  // backward never stores beta
  if ((N > cvf::kBwWaveStates || cvf::bw_gemm_path()) && (st = d.beta.ensure((size_t)max_chunk * N * 8)) != CV_OK)
    return st;
  if (N > cvf::kBwWaveStates && N <= cvf::kBwMmStates && (st = d.rscale.ensure((size_t)max_chunk * 8)) != CV_OK)
    return st;
  const size_t nacc = 3 * (size_t)N + (size_t)V * N + (size_t)N * N + 1;
  constexpr int kPartsB = 1024;  // blocks of the b M-step = partial convergence sums
  const int parts_a = N > cvf::kBwLdsMaxStates ? 1024 : 1;  // blocks of the pi / a M-step
  if ((st = d.acc.ensure(nacc * 8)) != CV_OK) return st;
  if ((st = d.pi.ensure((size_t)N * 8)) != CV_OK) return st;
  if ((st = d.a.ensure((size_t)N * N * 8)) != CV_OK) return st;
  if ((st = d.at.ensure((size_t)N * N * 8)) != CV_OK) return st;
  if ((st = d.et.ensure((size_t)V * N * 8)) != CV_OK) return st;
  if ((st = d.cnt.ensure((size_t)(parts_a + kPartsB) * 8)) != CV_OK) return st;
  if (bw_global && (st = d.gscratch.ensure((size_t)cvf::kBwScratchSeqs * 4 * N * 8)) != CV_OK) return st;
  if ((st = d.dump.ensure((size_t)cvf::kBwDumpWaves * 64 * 8)) != CV_OK) return st;
  int cus = 0;
  HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  const int64_t max_waves = (int64_t)std::max(cus, 1) * 8;  // backward waves resident at 2 per SIMD
  {
    // parameters go to the device once and stay there (M-step on the device)
    std::vector<double> at((size_t)N * N), et((size_t)V * N);
    for (int32_t i = 0; i < N; ++i)
      for (int32_t j = 0; j < N; ++j) at[(size_t)j * N + i] = a[(size_t)i * N + j];
    parallel_ranges((int64_t)V, [&](int, int64_t o0, int64_t o1) {
      for (int64_t o = o0; o < o1; ++o)
        for (int32_t i = 0; i < N; ++i) et[(size_t)o * N + i] = b[(size_t)i * V + o];
    }, 4096);
    HIP_TRY(hipMemcpy(d.pi.p, pi, (size_t)N * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d.a.p, a, (size_t)N * N * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d.at.p, at.data(), at.size() * 8, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(d.et.p, et.data(), et.size() * 8, hipMemcpyHostToDevice));
  }
  cvf::MstepArgs m{};
  m.acc = d.acc.as<double>();
  m.nstates = N;
  m.nobs = V;
  m.nseq = nseq;
  m.pi = d.pi.as<double>();
  m.a = d.a.as<double>();
  m.at = d.at.as<double>();
  m.et = d.et.as<double>();
  m.part = d.cnt.as<double>();
  m.parts_a = parts_a;
  std::vector<double> part((size_t)(parts_a + kPartsB));
  // (Round 5 measured an E-step pipeline -- each chunk in P parts on P streams so one part's
  // backward and xi GEMM run beside the next part's forward -- and rejected it: the iteration got
  // longer, 262.5 ms at P = 1 vs 285.3 at P = 4, profiles/r05_ab_bw_pipe.txt; removed in round 6.)
  // parts: one per chunk
  std::vector<std::vector<std::pair<int64_t, int64_t>>> parts(chunks.size());
  for (size_t ci = 0; ci < chunks.size(); ++ci) parts[ci].emplace_back(chunks[ci].first, chunks[ci].second);
  {
    // longest sequences first within each part (indices relative to the part)
    std::vector<int64_t> ord((size_t)nseq);
    for (const auto& pc : parts)
      for (const auto& c : pc) {
        int64_t* o = ord.data() + c.first;
        for (int64_t k = 0; k < c.second - c.first; ++k) o[k] = k;
        std::stable_sort(o, o + (c.second - c.first), [&](int64_t x, int64_t y) {
          return off0[c.first + x + 1] - off0[c.first + x] > off0[c.first + y + 1] - off0[c.first + y];
        });
      }
    if ((st = upload(d.ord, ord.data(), ord.size() * 8)) != CV_OK) return st;
  }
  // Arcs below cvf::kBwTinyArc (A's smallest positive entry, checked on the device before every
  // E-step): the E-step then runs on A 2^K and A^T 2^K, K the least that lifts every arc to
  // kBwTinyArc -- its factored xi sums stay in range and no step normaliser c_t is subnormal;
  // every normalised vector is the same (the scaling is exact), and the M-step multiplies the
  // counts back by a 2^K (MstepArgs::ascale).  A model without such arcs runs unscaled.
  if ((st = d.amin.ensure(8)) != CV_OK) return st;
  static const unsigned long long kInfBits = 0x7FF0000000000000ull;
  double ascale = 0.0;
  auto scan_tiny = [&]() -> cv_status {
    HIP_TRY(hipMemcpyAsync(d.amin.p, &kInfBits, 8, hipMemcpyHostToDevice, nullptr));
    const hipError_t e = cvf::launch_bw_amin(d.a.as<double>(), (int64_t)N * N, d.amin.as<unsigned long long>(), nullptr);
    if (e != hipSuccess) return set_err(CV_EDEVICE, "arc scan launch failed: %s", hipGetErrorString(e));
    return CV_OK;
  };
  auto read_tiny = [&]() -> cv_status {
    double amin = 0.0;
    HIP_TRY(hipMemcpy(&amin, d.amin.p, 8, hipMemcpyDeviceToHost));
    ascale = 0.0;
    if (amin < cvf::kBwTinyArc) ascale = std::ldexp(1.0, std::ilogb(cvf::kBwTinyArc) - std::ilogb(amin));
    return CV_OK;
  };
  if ((st = scan_tiny()) != CV_OK || (st = read_tiny()) != CV_OK) return st;
  int32_t it = 0;
  for (it = 1; it <= max_iter; ++it) {
    HIP_TRY(hipMemsetAsync(d.acc.p, 0, nacc * 8, nullptr));
    if (ascale != 0.0) {  // this E-step's A 2^K and A^T 2^K
      if ((st = d.a2.ensure((size_t)N * N * 8)) != CV_OK || (st = d.at2.ensure((size_t)N * N * 8)) != CV_OK) return st;
      hipError_t e = cvf::launch_bw_scale(d.a.as<double>(), d.a2.as<double>(), (int64_t)N * N, ascale, nullptr);
      if (e == hipSuccess)
        e = cvf::launch_bw_scale(d.at.as<double>(), d.at2.as<double>(), (int64_t)N * N, ascale, nullptr);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "arc scaling launch failed: %s", hipGetErrorString(e));
    }
    double* A = d.acc.as<double>();
    for (size_t ci = 0; ci < chunks.size(); ++ci)
      for (size_t pi_ = 0; pi_ < parts[ci].size(); ++pi_) {
      const auto& c = parts[ci][pi_];
      // the part's rows from its first element on (a part of a chunk: rows after the chunk's
      // earlier parts, so the parts' rows never overlap)
      const int64_t row0 = off0[c.first] - off0[chunks[ci].first];
      hipStream_t ss = nullptr;
      cvf::BwArgs g{};
      g.offsets = d.off.as<int64_t>() + c.first;
      g.obs = d.obs.as<int32_t>();
      g.tags = d.tags.as<int32_t>();
      g.elem_base = off0[c.first];
      g.order = d.ord.as<int64_t>() + c.first;
      g.dump = d.dump.as<double>();
      g.gscratch = bw_global ? d.gscratch.as<double>() : nullptr;
      g.nstates = N;
      g.pi = d.pi.as<double>();
      g.a = ascale != 0.0 ? d.a2.as<double>() : d.a.as<double>();
      g.at = ascale != 0.0 ? d.at2.as<double>() : d.at.as<double>();
      g.et = d.et.as<double>();
      g.alpha = d.alpha.as<double>() + (size_t)row0 * N;
      g.beta = d.beta.p ? d.beta.as<double>() + (size_t)row0 * N : nullptr;
      g.rscale = d.rscale.p ? d.rscale.as<double>() + row0 : nullptr;  // null: R stored over alpha
      g.pi_acc = A;
      g.a_den = A + N;
      g.b_den = A + 2 * N;
      g.b_num = A + 3 * N;
      g.xi_s = g.b_num + (size_t)V * N;
      g.xi_zero = g.xi_s + (size_t)N * N;
      const hipError_t e =
          cvf::launch_bw_estep(g, c.second - c.first, max_waves, ss, off0[c.second] - off0[c.first], nullptr);
      if (e != hipSuccess) return set_err(CV_EDEVICE, "Baum-Welch launch failed: %s", hipGetErrorString(e));
    }
    // M-step (hmm.rs:145-170) on the device: new_pi = sum gamma_0 / R; new_a = sum xi / a_den
    // (row); new_b = sum gamma at o / b_den; sum_t xi_t = A o S + z / N^2 (see bw_stats);
    // d = sum |new - old| (hmm.rs:172-175) as per-block parts added here in a fixed order
    m.ascale = ascale;
    const hipError_t e = cvf::launch_bw_mstep(m, kPartsB, nullptr);
    if (e != hipSuccess) return set_err(CV_EDEVICE, "M-step launch failed: %s", hipGetErrorString(e));
    if ((st = scan_tiny()) != CV_OK) return st;  // the new A, for the next E-step
    HIP_TRY(hipMemcpy(part.data(), d.cnt.p, part.size() * 8, hipMemcpyDeviceToHost));
    if ((st = read_tiny()) != CV_OK) return st;
    double dsum = 0.0;
    for (double x : part) dsum += x;
    if (dsum <= tol) break;
  }
  if (iters_out) *iters_out = std::min(it, max_iter);
  std::vector<double> et((size_t)V * N);
  HIP_TRY(hipMemcpy(pi, d.pi.p, (size_t)N * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(a, d.a.p, (size_t)N * N * 8, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(et.data(), d.et.p, et.size() * 8, hipMemcpyDeviceToHost));
  for (int32_t i = 0; i < N; ++i) pi[i] = ref_log(pi[i]);
  for (size_t k = 0; k < (size_t)N * N; ++k) a[k] = ref_log(a[k]);
  parallel_ranges((int64_t)N, [&](int, int64_t i0, int64_t i1) {
    for (int64_t i = i0; i < i1; ++i)
      for (int64_t o = 0; o < V; ++o) b[(size_t)i * V + o] = ref_log(et[(size_t)o * N + i]);
  }, 1);
  return CV_OK;
}

}  // extern "C"
