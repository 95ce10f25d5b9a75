/*
 * cv_oracle.c -- CPU restatement of the reference Viterbi forward pass + backtrack.
 *
 * TEST INFRASTRUCTURE ONLY (see cv_oracle.h): the checker for GPU parity tests and
 * the timed CPU baseline of bench.py.  Never linked into the product library.
 * Parity status: unpinned against the (unbuildable) reference; pinned by KATs and
 * exhaustive enumeration in tests/.
 *
 * Build: see oracle/Makefile (gcc -O2 -fno-fast-math -ffp-contract=off).  All adds
 * are single IEEE adds in the declared precision; no FMA contraction, no
 * reassociation, so results are bit-reproducible across compilers.
 */
#include "cv_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/*
 * Generic body, instantiated for double and float.  Work arrays:
 *   prev/cur [N] delta rows, bt [T*N] back-pointers (int32).
 * Per-mode recurrences cite the reference lines they follow (cv_oracle.h).
 */
#define CVO_DEFINE_DECODE(NAME, REAL, NEG_INF)                                                  \
  int NAME(int N, int V, const REAL* pi, const REAL* a, const REAL* b, int T,                  \
           const int32_t* obs, const int32_t* forced, int assoc, int32_t* path, REAL* score) {  \
    (void)V;                                                                                    \
    if (T <= 0) {                                                                               \
      *score = (REAL)0;                                                                         \
      return CVO_SEQ_EMPTY;                                                                     \
    }                                                                                           \
    REAL* prev = (REAL*)malloc(sizeof(REAL) * (size_t)N);                                       \
    REAL* cur = (REAL*)malloc(sizeof(REAL) * (size_t)N);                                        \
    int32_t* bt = (int32_t*)calloc((size_t)T * (size_t)N, sizeof(int32_t));                    \
    const REAL ninf = NEG_INF;                                                                  \
    /* row 0: pi + b[:,o0] (hmm.rs:215-218, cp.rs:66-68); decode(): 0.0 (viterbi.rs:6,9) */    \
    {                                                                                           \
      const int64_t o = obs[0];                                                                 \
      for (int j = 0; j < N; ++j) {                                                             \
        if (assoc == CVO_ASSOC_DECODE)                                                          \
          prev[j] = (REAL)0;                                                                    \
        else if (assoc == CVO_ASSOC_DP) /* dp.rs:106-118: only emittable, finite states */     \
          prev[j] = (b[(int64_t)j * V + o] > ninf) ? (REAL)(pi[j] + b[(int64_t)j * V + o])      \
                                                   : ninf;                                      \
        else                                                                                    \
          prev[j] = pi[j] + b[(int64_t)j * V + o];                                              \
      }                                                                                         \
      /* forced state (consistency constraint, opti.rs:101-111): other states impossible */    \
      if (forced && forced[0] >= 0)                                                             \
        for (int j = 0; j < N; ++j)                                                             \
          if (j != forced[0]) prev[j] = ninf;                                                   \
    }                                                                                           \
    for (int t = 1; t < T; ++t) {                                                               \
      const int64_t o = obs[t];                                                                 \
      int32_t* bt_t = bt + (int64_t)t * N;                                                      \
      for (int j = 0; j < N; ++j) {                                                             \
        const REAL e = b[(int64_t)j * V + o];                                                   \
        if (assoc == CVO_ASSOC_DP) {                                                            \
          /* dp.rs:139-177: skip non-emittable targets and -inf arcs; keep strictly greater */  \
          REAL best = ninf;                                                                     \
          int arg = 0;                                                                          \
          if (e > ninf) {                                                                       \
            for (int i = 0; i < N; ++i) {                                                       \
              if (!(prev[i] > ninf)) continue;                                                  \
              const REAL arc = a[(int64_t)i * N + j] + e;                                       \
              if (!(arc > ninf)) continue;                                                      \
              const REAL c = arc + prev[i];                                                     \
              if (c > best) {                                                                   \
                best = c;                                                                       \
                arg = i;                                                                        \
              }                                                                                 \
            }                                                                                   \
          }                                                                                     \
          cur[j] = best;                                                                        \
          bt_t[j] = arg;                                                                        \
          continue;                                                                             \
        }                                                                                       \
        if (assoc == CVO_ASSOC_DECODE && !(e > ninf)) {                                         \
          /* viterbi.rs:19-21: -inf, back-pointer left at 0 */                                  \
          cur[j] = ninf;                                                                        \
          bt_t[j] = 0;                                                                          \
          continue;                                                                             \
        }                                                                                       \
        /* first argmax of prev + a[:,j] (ndarray-stats argmax = first maximal index) */        \
        REAL m = prev[0] + a[j];                                                                \
        int arg = 0;                                                                            \
        for (int i = 1; i < N; ++i) {                                                           \
          const REAL s = prev[i] + a[(int64_t)i * N + j];                                       \
          if (s > m) {                                                                          \
            m = s;                                                                              \
            arg = i;                                                                            \
          }                                                                                     \
        }                                                                                       \
        bt_t[j] = arg;                                                                          \
        if (assoc == CVO_ASSOC_CP) /* cp.rs:75-76: prev[psi] + (a[psi,j] + b[j,o]) */         \
          cur[j] = prev[arg] + (a[(int64_t)arg * N + j] + e);                                   \
        else /* viterbi.rs:15-17: (prev + a) + b */                                             \
          cur[j] = m + e;                                                                       \
      }                                                                                         \
      if (forced && forced[t] >= 0)                                                             \
        for (int j = 0; j < N; ++j)                                                             \
          if (j != forced[t]) cur[j] = ninf;                                                    \
      REAL* tmp = prev;                                                                         \
      prev = cur;                                                                               \
      cur = tmp;                                                                                \
    }                                                                                           \
    /* final: first argmax of last row (cp.rs:85-93; viterbi.rs:24) */                        \
    int end = 0;                                                                                \
    REAL best = prev[0];                                                                        \
    for (int j = 1; j < N; ++j)                                                                 \
      if (prev[j] > best) {                                                                     \
        best = prev[j];                                                                         \
        end = j;                                                                                \
      }                                                                                         \
    int status = CVO_SEQ_OK;                                                                    \
    if (!(best > ninf) && assoc != CVO_ASSOC_DECODE) {                                          \
      /* infeasible: reference panics (cp.rs:87, dp.rs:184-186); we report it */              \
      status = CVO_SEQ_INFEASIBLE;                                                              \
      for (int t = 0; t < T; ++t) path[t] = 0;                                                  \
      *score = ninf;                                                                            \
    } else if (!(best > ninf)) {                                                                \
      /* viterbi::decode: argmax 0 of the all -inf row, then bt (0 where the emission is      \
       * -inf), viterbi.rs:19-21, 24-30 */                                                     \
      status = CVO_SEQ_INFEASIBLE;                                                              \
      int cs = end;                                                                             \
      for (int t = T - 1; t >= 0; --t) {                                                        \
        path[t] = cs;                                                                           \
        cs = bt[(int64_t)t * N + cs];                                                           \
      }                                                                                         \
      *score = ninf;                                                                            \
    } else {                                                                                    \
      int cs = end;                                                                             \
      for (int t = T - 1; t >= 0; --t) {                                                        \
        path[t] = cs;                                                                           \
        cs = bt[(int64_t)t * N + cs];                                                           \
      }                                                                                         \
      *score = best;                                                                            \
    }                                                                                           \
    free(prev);                                                                                 \
    free(cur);                                                                                  \
    free(bt);                                                                                   \
    return status;                                                                              \
  }

CVO_DEFINE_DECODE(cvo_decode_forced_f64, double, -INFINITY)
CVO_DEFINE_DECODE(cvo_decode_forced_f32, float, -INFINITY)

int cvo_decode_f64(int N, int V, const double* pi, const double* a, const double* b, int T, const int32_t* obs,
                   int assoc, int32_t* path, double* score) {
  return cvo_decode_forced_f64(N, V, pi, a, b, T, obs, NULL, assoc, path, score);
}
int cvo_decode_f32(int N, int V, const float* pi, const float* a, const float* b, int T, const int32_t* obs,
                   int assoc, int32_t* path, float* score) {
  return cvo_decode_forced_f32(N, V, pi, a, b, T, obs, NULL, assoc, path, score);
}

int cvo_decode_batch_f64(int N, int V, const double* pi, const double* a, const double* b,
                         int64_t nseq, const int64_t* offsets, const int32_t* obs, int assoc,
                         int32_t* path, double* score, uint8_t* status, int nthreads) {
  return cvo_decode_batch_forced_f64(N, V, pi, a, b, nseq, offsets, obs, NULL, assoc, path, score, status,
                                     nthreads);
}

int cvo_decode_batch_forced_f64(int N, int V, const double* pi, const double* a, const double* b,
                                int64_t nseq, const int64_t* offsets, const int32_t* obs, const int32_t* forced,
                                int assoc, int32_t* path, double* score, uint8_t* status, int nthreads) {
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
  for (int64_t s = 0; s < nseq; ++s) {
    const int64_t o0 = offsets[s];
    const int T = (int)(offsets[s + 1] - o0);
    double sc;
    int st = cvo_decode_forced_f64(N, V, pi, a, b, T, obs + o0, forced ? forced + o0 : NULL, assoc, path + o0, &sc);
    score[s] = sc;
    status[s] = (uint8_t)st;
  }
  return 0;
}

int cvo_decode_batch_f32(int N, int V, const float* pi, const float* a, const float* b,
                         int64_t nseq, const int64_t* offsets, const int32_t* obs, int assoc,
                         int32_t* path, double* score, uint8_t* status, int nthreads) {
  return cvo_decode_batch_forced_f32(N, V, pi, a, b, nseq, offsets, obs, NULL, assoc, path, score, status,
                                     nthreads);
}

int cvo_decode_batch_forced_f32(int N, int V, const float* pi, const float* a, const float* b,
                                int64_t nseq, const int64_t* offsets, const int32_t* obs, const int32_t* forced,
                                int assoc, int32_t* path, double* score, uint8_t* status, int nthreads) {
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
  for (int64_t s = 0; s < nseq; ++s) {
    const int64_t o0 = offsets[s];
    const int T = (int)(offsets[s + 1] - o0);
    float sc;
    int st = cvo_decode_forced_f32(N, V, pi, a, b, T, obs + o0, forced ? forced + o0 : NULL, assoc, path + o0, &sc);
    score[s] = (double)sc;
    status[s] = (uint8_t)st;
  }
  return 0;
}

double cvo_rescore_f64(int N, int V, const double* pi, const double* a, const double* b, int T,
                       const int32_t* obs, const int32_t* path) {
  if (T <= 0) return 0.0;
  double d = pi[path[0]] + b[(int64_t)path[0] * V + obs[0]];
  for (int t = 1; t < T; ++t) {
    d = d + a[(int64_t)path[t - 1] * N + path[t]];
    d = d + b[(int64_t)path[t] * V + obs[t]];
  }
  return d;
}

/* cvo_rescore_f64 over a CSR batch (test infrastructure: full-size property checks). */
void cvo_rescore_batch_f64(int N, int V, const double* pi, const double* a, const double* b, int64_t nseq,
                           const int64_t* offsets, const int32_t* obs, const int32_t* path, double* out) {
  for (int64_t s = 0; s < nseq; ++s)
    out[s] = cvo_rescore_f64(N, V, pi, a, b, (int)(offsets[s + 1] - offsets[s]), obs + offsets[s], path + offsets[s]);
}

double cvo_cp_superseq_f64(int N, int V, const double* pi, const double* a, const double* b,
                           int64_t nseq, const int64_t* offsets, const int32_t* obs,
                           int32_t* path) {
  const int64_t L = offsets[nseq] - offsets[0];
  if (L <= 0) return 0.0;
  double* arr = (double*)malloc(sizeof(double) * (size_t)L * (size_t)N);
  int32_t* bt = (int32_t*)calloc((size_t)L * (size_t)N, sizeof(int32_t));
  /* per-element "t == 0" flag: first element of each sequence (utils.rs:24-38) */
  unsigned char* first = (unsigned char*)calloc((size_t)L, 1);
  for (int64_t s = 0; s < nseq; ++s)
    if (offsets[s + 1] > offsets[s]) first[offsets[s] - offsets[0]] = 1;
  const int32_t* ob = obs + offsets[0];
  /* element 0: init_probs (cp.rs:66-68) */
  for (int j = 0; j < N; ++j) arr[j] = pi[j] + b[(int64_t)j * V + ob[0]];
  for (int64_t t = 1; t < L; ++t) {
    const double* prevr = arr + (t - 1) * N;
    double* row = arr + t * N;
    const int64_t o = ob[t];
    for (int j = 0; j < N; ++j) {
      /* transitions(): constant pi[j] vector at t==0, else column a[:,j] (utils.rs:32-38) */
      double m, s;
      int arg = 0;
      if (first[t]) {
        m = prevr[0] + pi[j];
        for (int i = 1; i < N; ++i) {
          s = prevr[i] + pi[j];
          if (s > m) { m = s; arg = i; }
        }
        /* arc_p at t==0 = init_prob (utils.rs:24-27, hmm.rs:211-213) */
        row[j] = prevr[arg] + (pi[j] + b[(int64_t)j * V + o]);
      } else {
        m = prevr[0] + a[j];
        for (int i = 1; i < N; ++i) {
          s = prevr[i] + a[(int64_t)i * N + j];
          if (s > m) { m = s; arg = i; }
        }
        row[j] = prevr[arg] + (a[(int64_t)arg * N + j] + b[(int64_t)j * V + o]);
      }
      bt[t * N + j] = arg;
    }
  }
  const double* last = arr + (L - 1) * N;
  int cs = 0;
  double obj = last[0];
  for (int j = 1; j < N; ++j)
    if (last[j] > obj) { obj = last[j]; cs = j; }
  for (int64_t t = L - 1; t >= 0; --t) {
    path[t] = cs;
    cs = bt[t * N + cs];
  }
  free(arr);
  free(bt);
  free(first);
  return obj;
}

/* Last delta row of the row-A0 forward recurrence over obs[0..T) with an arbitrary
 * transition matrix m[from*N + to] (pass a^T and pi = 0 over reversed observations for
 * the backward max-plus pass of the constrained decode spec, np_oracle.py). */
#define CVO_DEFINE_ROW(NAME, REAL)                                                              \
  void NAME(int N, int V, const REAL* pi, const REAL* m, const REAL* b, int T, const int32_t* obs, \
            REAL* out) {                                                                        \
    REAL* prev = (REAL*)malloc(sizeof(REAL) * (size_t)N);                                       \
    REAL* cur = (REAL*)malloc(sizeof(REAL) * (size_t)N);                                        \
    for (int j = 0; j < N; ++j) prev[j] = pi[j] + b[(int64_t)j * V + obs[0]];                   \
    for (int t = 1; t < T; ++t) {                                                               \
      for (int j = 0; j < N; ++j) {                                                             \
        REAL mx = prev[0] + m[j];                                                               \
        for (int i = 1; i < N; ++i) {                                                           \
          const REAL s = prev[i] + m[(int64_t)i * N + j];                                       \
          if (s > mx) mx = s;                                                                   \
        }                                                                                       \
        cur[j] = mx + b[(int64_t)j * V + obs[t]];                                               \
      }                                                                                         \
      REAL* tmp = prev;                                                                         \
      prev = cur;                                                                               \
      cur = tmp;                                                                                \
    }                                                                                           \
    for (int j = 0; j < N; ++j) out[j] = prev[j];                                               \
    free(prev);                                                                                 \
    free(cur);                                                                                  \
  }
CVO_DEFINE_ROW(cvo_forward_row_f64, double)
CVO_DEFINE_ROW(cvo_forward_row_f32, float)
